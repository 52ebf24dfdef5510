# k_rays_fxq (lean lane-level refill, one car per wave): identity + A/B against k_rays_fxs by size and threshold
set -o pipefail
mkdir -p gpurun_out/r03ae
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_parity.py -k "refill_kernel_identical or fixed_point_cell_index_adversarial" > gpurun_out/r03ae/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03ae/tests.log; exit 1; }
tail -1 gpurun_out/r03ae/tests.log
AB_ENVS=65536,32768,8192 AB_STEPS=200 AB_ROUNDS=3 AB_VARIANTS='fxs:F110_FX_REFILL=1,F110_FX_PAD=1;q64:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FX_LPOOL=1,F110_FX_POOL_T=64;q80:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FX_LPOOL=1,F110_FX_POOL_T=80;q96:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FX_LPOOL=1,F110_FX_POOL_T=96;q112:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FX_LPOOL=1,F110_FX_POOL_T=112' timeout -k 10 300 python scripts/ray_ab.py > gpurun_out/r03ae/ab.json 2> gpurun_out/r03ae/ab.err || { echo "ab failed"; tail -30 gpurun_out/r03ae/ab.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03ae/ab.json'))
for E,v in d['by_envs'].items(): print(E, v['identical'], {n: round(v[n]['k_rays_ms'],4) for n in ('fxs','q64','q80','q96','q112')})
PY
