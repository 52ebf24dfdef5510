# k_rays_fxs with software-pipelined slots (F110_FXS_PIPE=1): identity + A/B; then the 2-rank rehearsal and lone-ray probe
set -o pipefail
mkdir -p gpurun_out/r03ai
export F110_FXS_PIPE=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_parity.py -k "refill_kernel_identical or fixed_point_cell_index_adversarial" > gpurun_out/r03ai/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03ai/tests.log; exit 1; }
unset F110_FXS_PIPE
tail -1 gpurun_out/r03ai/tests.log
AB_ENVS=65536,32768,8192 AB_STEPS=200 AB_ROUNDS=3 AB_VARIANTS='fxs:F110_FX_REFILL=1,F110_FX_PAD=1;pipe:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FXS_PIPE=1' timeout -k 10 300 python scripts/ray_ab.py > gpurun_out/r03ai/ab.json 2> gpurun_out/r03ai/ab.err || { echo "ab failed"; tail -30 gpurun_out/r03ai/ab.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03ai/ab.json'))
for E,v in d['by_envs'].items(): print(E, v['identical'], {n: round(v[n]['k_rays_ms'],4) for n in ('fxs','pipe')})
PY
bash scripts/gpu_r03ah.sh
