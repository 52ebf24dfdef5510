set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/adamab; mkdir -p $O; cd $R
for lib in ${ADAM_LIBS:-sel2 adaminc}; do
  export F110_LIB=$R/ab_libs/$lib.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$lib -o run -- python3 bench.py --workload ddpg --steps 100 --warmup 20 --no-cpu-baseline > $O/$lib.out 2> $O/$lib.err || exit 1
done
unset F110_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_ddpg_heads.py tests/test_gpu_learner_gemm.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1
