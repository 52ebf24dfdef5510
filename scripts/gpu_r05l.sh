# Round 5 (l): k_lwgrad two-deep prefetch A/B (learner_gemm_mb per build), learner tests, C5;
# k_post_multi phase probes (timing-only builds: no agent ray_cast / no GJK / no env epilogue).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05l
mkdir -p "$OUT"
cd "$R"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "step $name failed rc=$?" >&2; tail -30 "$OUT/$name.err" >&2; exit 1; }
}
for v in wg320 wgpf2; do F110_LIB=$R/ab_libs/$v.so step lg_$v 300 python -u scripts/learner_gemm_mb.py; done
step lgemm 600 python -u -m pytest tests/test_gpu_learner_gemm.py tests/test_gpu_replay.py tests/test_gpu_ddpg_heads.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
step c5 600 python -u bench.py --workload ddpg --steps 200 --warmup 20
step post_cur 300 python -u scripts/post_probe.py
for v in nrc ngjk nepi; do F110_LIB=$R/ab_libs/post_$v.so step post_$v 300 python -u scripts/post_probe.py; done
echo "[$(date +%T)] done" >&2
