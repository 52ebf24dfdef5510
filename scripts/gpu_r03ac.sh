# k_rays_fxs long-ray prefetch (F110_FXS_PF = trips before the touches start): identity + A/B by size
set -o pipefail
mkdir -p gpurun_out/r03ac
export F110_FXS_PF=16
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_parity.py -k "refill_kernel_identical or fixed_point_cell_index_adversarial" > gpurun_out/r03ac/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03ac/tests.log; exit 1; }
unset F110_FXS_PF
tail -1 gpurun_out/r03ac/tests.log
AB_ENVS=65536,32768,16384,8192 AB_STEPS=200 AB_ROUNDS=3 AB_VARIANTS='dflt:F110_FXR_LEAN=1;fxs:F110_FX_REFILL=1,F110_FX_PAD=1;pf32:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FXS_PF=32;pf64:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FXS_PF=64;pf128:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FXS_PF=128' timeout -k 10 500 python scripts/ray_ab.py > gpurun_out/r03ac/ab.json 2> gpurun_out/r03ac/ab.err || { echo "ab failed"; tail -30 gpurun_out/r03ac/ab.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03ac/ab.json'))
for E,v in d['by_envs'].items(): print(E, all(v['identical'].values()), {n: round(v[n]['k_rays_ms'],4) for n in ('dflt','fxs','pf32','pf64','pf128')})
PY
