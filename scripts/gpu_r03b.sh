set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -k "pool_kernel_identical or refill_kernel_identical" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03b/pooltest.log 2>&1 || { echo "pool test failed"; tail -40 gpurun_out/r03b/pooltest.log; exit 1; }
tail -2 gpurun_out/r03b/pooltest.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "adversarial_vs_oracle" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03b/advtest.log 2>&1 || { echo "adv test failed"; tail -40 gpurun_out/r03b/advtest.log; exit 1; }
tail -2 gpurun_out/r03b/advtest.log
AB_ENVS=65536,32768 AB_STEPS=100 AB_ROUNDS=3 AB_VARIANTS='fxr:F110_FX_REFILL=1;p1:F110_FX_POOL=1,F110_FX_PAD=1;p2:F110_FX_POOL=2,F110_FX_PAD=1;p2t48:F110_FX_POOL=2,F110_FX_POOL_T=48,F110_FX_PAD=1;p2t112:F110_FX_POOL=2,F110_FX_POOL_T=112,F110_FX_PAD=1' timeout -k 10 400 python scripts/ray_ab.py > gpurun_out/r03b/ab_pool.json 2> gpurun_out/r03b/ab_pool.err || { echo "ab failed"; tail -20 gpurun_out/r03b/ab_pool.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03b/ab_pool.json'))
for E,l in d['by_envs'].items():
    print(E, l['identical'], {k:round(v['k_rays_ms'],4) for k,v in l.items() if isinstance(v,dict) and 'k_rays_ms' in v})
PY
