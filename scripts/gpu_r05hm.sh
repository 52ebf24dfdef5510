# Round 5 (hm): two-agent k_rays_fxs writing the f64 scan hand-off only for the chunks k_post_multi's
# agent ray_cast may read (handoff_chunks) against HEAD: GPU suite, scripts/post_probe.py per build,
# C4 (stream shards and one context) and C5 benches per build, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05hm
mkdir -p "$OUT"
cd "$R"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "step $name failed rc=$?" >&2; tail -30 "$OUT/$name.err" >&2; exit 1; }
}
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for k in 1 2; do
    step post_cur_$k 300 python -u scripts/post_probe.py
    F110_LIB=$R/ab_libs/head.so step post_head_$k 300 python -u scripts/post_probe.py
done
for k in 1 2; do
    F110_LIB=$R/ab_libs/head.so step c4_head_$k 600 python -u bench.py --agents 2 --global-envs 8192 --no-cpu-baseline
    step c4_cur_$k 600 python -u bench.py --agents 2 --global-envs 8192 --no-cpu-baseline
    F110_LIB=$R/ab_libs/head.so step c5_head_$k 600 python -u bench.py --workload ddpg --steps 200 --warmup 20
    step c5_cur_$k 600 python -u bench.py --workload ddpg --steps 200 --warmup 20
done
echo "[$(date +%T)] done" >&2
