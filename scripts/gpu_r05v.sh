# Round 5 (v): single-agent k_rays_fxs with its work items ordered by the last launch's trips
# (k_item_order) against HEAD: GPU batch tests, bench (interleaved, twice), shard sizes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05v
mkdir -p "$OUT"
cd "$R"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "step $name failed rc=$?" >&2; tail -30 "$OUT/$name.err" >&2; exit 1; }
}
step quick 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_gpu_env.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for k in 1 2; do
    for v in head order; do
        F110_LIB=$R/ab_libs/$v.so step bench_${v}_$k 600 python -u bench.py --no-cpu-baseline
    done
done
echo "[$(date +%T)] done" >&2
