# Round 5 (h): the replay changes -- replay GPU tests, the replay probe serial / overlapped
# (kernel stats), the C5 bench with and without the overlap.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05h
mkdir -p "$OUT"
cd "$R"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "step $name failed rc=$?" >&2; tail -30 "$OUT/$name.err" >&2; exit 1; }
}
step tests 600 python -u -m pytest tests/test_gpu_replay.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
step rp0 200 python -u scripts/replay_probe.py
RP_OVERLAP=1 step rp1 200 python -u scripts/replay_probe.py
RP_OVERLAP=1 step rp1prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/rp1prof" -o run --output-format csv -- python3 scripts/replay_probe.py
step c5 600 python -u bench.py --workload ddpg --steps 200 --warmup 20
F110_REPLAY_OVERLAP=0 step c5serial 600 python -u bench.py --workload ddpg --steps 200 --warmup 20
echo "[$(date +%T)] done" >&2
