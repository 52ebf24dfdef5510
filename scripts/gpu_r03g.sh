set -o pipefail
mkdir -p gpurun_out/r03g
for v in ${VARIANTS:-calls inl}; do
  export F110_LIB=$PWD/f110_gymnasium_ros2_jazzy_amd/libf110_$v.so
  timeout -k 10 200 python -u -m pytest tests/test_gpu_batch.py -k "step1_matches" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03g/test_$v.log 2>&1 || { echo "tests failed $v"; tail -40 gpurun_out/r03g/test_$v.log; exit 1; }
  tail -1 gpurun_out/r03g/test_$v.log
  FA_ENVS=65536,8192,4096 FA_STEPS=200 FA_CHUNK=50 FA_ROUNDS=2 timeout -k 10 300 python scripts/fused_ab.py > gpurun_out/r03g/fused_ab_$v.json 2> gpurun_out/r03g/fused_ab_$v.err || { echo "fused ab failed $v"; tail -20 gpurun_out/r03g/fused_ab_$v.err; exit 1; }
  echo "$v"; tail -1 gpurun_out/r03g/fused_ab_$v.json
done
