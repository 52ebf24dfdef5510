# Round 5 (q): 8-wave blocks of k_rays_fxs with / without the LDS theta table, against HEAD:
# bench (stream shards; the roofline's profiled one-context pass) per build, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05r
mkdir -p "$OUT"
cd "$R"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "step $name failed rc=$?" >&2; tail -30 "$OUT/$name.err" >&2; exit 1; }
}
step suite 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
for k in 1 2; do
    for v in head lds8 q16; do
        F110_LIB=$R/ab_libs/$v.so step bench_${v}_$k 600 python -u bench.py --no-cpu-baseline
    done
done
echo "[$(date +%T)] done" >&2
