# Round 5 (w): k_post_multi with the sin / cos table in LDS against HEAD: GPU env / parity /
# config tests, then scripts/post_probe.py per build (interleaved, twice).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05w
mkdir -p "$OUT"
cd "$R"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "step $name failed rc=$?" >&2; tail -30 "$OUT/$name.err" >&2; exit 1; }
}
step tests 600 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for k in 1 2; do
    step probe_cur_$k 300 python -u scripts/post_probe.py
    F110_LIB=$R/ab_libs/head.so step probe_head_$k 300 python -u scripts/post_probe.py
done
echo "[$(date +%T)] done" >&2
