# Round 5 (c4l): two-agent stream sub-shards (C4's runner) on the LDS theta-table kernel
# (k_rays_fxs<true, true>) against HEAD (one-wave blocks): GPU batch tests, then the C4 bench
# per build (interleaved, twice).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05c4l
mkdir -p "$OUT"
cd "$R"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "step $name failed rc=$?" >&2; tail -30 "$OUT/$name.err" >&2; exit 1; }
}
step tests 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for k in 1 2; do
    F110_LIB=$R/ab_libs/head.so step c4_head_$k 600 python -u bench.py --agents 2 --global-envs 8192 --no-cpu-baseline
    step c4_cur_$k 600 python -u bench.py --agents 2 --global-envs 8192 --no-cpu-baseline
done
echo "[$(date +%T)] done" >&2
