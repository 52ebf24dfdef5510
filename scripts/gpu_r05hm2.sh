# Round 5 (hm2): the hand-off mask variant against HEAD: k_agents per launch (one and two agents),
# the default bench (single-agent path, must not move) and the C4 / C5 benches.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05hm2
mkdir -p "$OUT"
cd "$R"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "step $name failed rc=$?" >&2; tail -30 "$OUT/$name.err" >&2; exit 1; }
}
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for k in 1 2; do
    step post_cur_$k 300 python -u scripts/post_probe.py
    F110_LIB=$R/ab_libs/head.so step post_head_$k 300 python -u scripts/post_probe.py
done
step agents_cur 300 python -u scripts/agents_probe.py
F110_LIB=$R/ab_libs/head.so step agents_head 300 python -u scripts/agents_probe.py
for k in 1 2; do
    F110_LIB=$R/ab_libs/head.so step bench_head_$k 600 python -u bench.py --no-cpu-baseline
    step bench_cur_$k 600 python -u bench.py --no-cpu-baseline
    F110_LIB=$R/ab_libs/head.so step c4_head_$k 600 python -u bench.py --agents 2 --global-envs 8192 --no-cpu-baseline
    step c4_cur_$k 600 python -u bench.py --agents 2 --global-envs 8192 --no-cpu-baseline
done
echo "[$(date +%T)] done" >&2
