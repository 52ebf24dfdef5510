# Round 5 (i): replay select A/B -- the probe per build (kernel stats), replay tests, C5 bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05i
mkdir -p "$OUT"
cd "$R"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "step $name failed rc=$?" >&2; tail -30 "$OUT/$name.err" >&2; exit 1; }
}
step tests 600 python -u -m pytest tests/test_gpu_replay.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
for v in r5_head r5_noplace cur; do
    if [ $v = cur ]; then unset F110_LIB; else export F110_LIB=$R/ab_libs/$v.so; fi
    step rp_$v 200 python -u scripts/replay_probe.py
    step prof_$v 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$v" -o run --output-format csv -- python3 scripts/replay_probe.py
done
unset F110_LIB
step c5 600 python -u bench.py --workload ddpg --steps 200 --warmup 20
echo "[$(date +%T)] done" >&2
