# Round 5 (p): k_rays_fxs with the theta table in LDS (8-wave blocks) against HEAD's build
# (ab_libs/head.so): GPU suite, bench (head / new interleaved, twice), the 65536-car PMC pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05p
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
    F110_LIB=$R/ab_libs/head.so step bench_head_$k 600 python -u bench.py --no-cpu-baseline
    step bench_new_$k 600 python -u bench.py --no-cpu-baseline
done
step pmc 900 python -u scripts/profile_round.py r05p
echo "[$(date +%T)] done" >&2
