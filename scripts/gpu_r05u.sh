# Round 5 (u): single-agent k_rays_fxs (8-wave LDS blocks) with car-major items (a car's waves in
# one block) against HEAD (wave-major), waves per car 1 / 2 / 4 / 8: scripts/shard_rules.py per build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05u
mkdir -p "$OUT"
cd "$R"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "step $name failed rc=$?" >&2; tail -30 "$OUT/$name.err" >&2; exit 1; }
}
step quick 600 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for v in head carmajor; do
    F110_LIB=$R/ab_libs/$v.so SR_ENVS=65536 SR_STREAMS=1,2 SR_CHOICES=2:1,2:2,2:4,2:8 SR_STEPS=200 SR_ROUNDS=2 \
        step rules65536_$v 600 python -u scripts/shard_rules.py
    F110_LIB=$R/ab_libs/$v.so SR_ENVS=8192,4096 SR_STREAMS=4 SR_CHOICES=2:1,2:2,2:3,2:4,2:8 SR_STEPS=300 SR_ROUNDS=2 \
        step rulessmall_$v 600 python -u scripts/shard_rules.py
done
echo "[$(date +%T)] done" >&2
