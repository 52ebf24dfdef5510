# Round 5 (b8): where the 8-wave blocks' one-context cost comes from: 8-wave blocks without the
# LDS table or its barrier (b8n) against the kept LDS build (cur); bench per build, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05b8
mkdir -p "$OUT"
cd "$R"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "step $name failed rc=$?" >&2; tail -30 "$OUT/$name.err" >&2; exit 1; }
}
for k in 1 2; do
    for v in cur b8n; do
        F110_LIB=$R/ab_libs/$v.so step bench_${v}_$k 600 python -u bench.py --no-cpu-baseline
    done
done
echo "[$(date +%T)] done" >&2
