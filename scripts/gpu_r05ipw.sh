# Round 5 (ipw): k_rays_fxs (single-agent LDS kernel) with several cars per wave (F110_FXS_ITEMS:
# a grid of 1/K the blocks, each wave striding over K work items, the block's LDS table loaded
# once) against HEAD: the GPU batch tests at K = 2, then the bench per build / K, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05ipw
mkdir -p "$OUT"
cd "$R"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "step $name failed rc=$?" >&2; tail -30 "$OUT/$name.err" >&2; exit 1; }
}
F110_FXS_ITEMS=2 step tests 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for k in 1 2; do
    F110_LIB=$R/ab_libs/head.so step bench_head_$k 600 python -u bench.py --no-cpu-baseline
    for ipw in 1 2 4; do
        F110_FXS_ITEMS=$ipw step bench_ipw${ipw}_$k 600 python -u bench.py --no-cpu-baseline
    done
done
echo "[$(date +%T)] done" >&2
