# Round 5 (x): the replay select as keys -> hist1 (+ candidates) -> sel (one block) -> mark -> finish
# against HEAD: replay GPU tests, scripts/replay_probe.py per build (digest and per-kernel time
# under rocprofv3), the C5 bench per build (interleaved).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05x
mkdir -p "$OUT"
cd "$R"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "step $name failed rc=$?" >&2; tail -30 "$OUT/$name.err" >&2; exit 1; }
}
step tests 600 python -u -m pytest tests/test_gpu_replay.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step probe_cur 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cur" -o run -- python -u scripts/replay_probe.py
F110_LIB=$R/ab_libs/head.so step probe_head 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_head" -o run -- python -u scripts/replay_probe.py
for k in 1 2; do
    step c5_cur_$k 600 python -u bench.py --workload ddpg --steps 200 --warmup 20
    F110_LIB=$R/ab_libs/head.so step c5_head_$k 600 python -u bench.py --workload ddpg --steps 200 --warmup 20
done
echo "[$(date +%T)] done" >&2
