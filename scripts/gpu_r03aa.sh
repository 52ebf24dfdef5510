# k_rays_fxs with the gathers issued before the guard-band test: identity + A/B
set -o pipefail
mkdir -p gpurun_out/r03aa
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_parity.py -k "refill_kernel_identical or fixed_point_cell_index_adversarial" > gpurun_out/r03aa/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03aa/tests.log; exit 1; }
tail -1 gpurun_out/r03aa/tests.log
AB_ENVS=65536,32768,16384 AB_STEPS=200 AB_ROUNDS=3 AB_VARIANTS='fxr:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FXR_LEAN=0;fxs:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FXR_LEAN=1' timeout -k 10 400 python scripts/ray_ab.py > gpurun_out/r03aa/ab.json 2> gpurun_out/r03aa/ab.err || { echo "ab failed"; tail -30 gpurun_out/r03aa/ab.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03aa/ab.json'))
for E,v in d['by_envs'].items(): print(E, v['identical'], {n: round(v[n]['k_rays_ms'],4) for n in ('fxr','fxs')})
PY
