set -o pipefail
mkdir -p gpurun_out/r03d
F110_RECORD_NONEXACT=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d/gputest.log 2>&1 || { echo "gputests failed"; tail -40 gpurun_out/r03d/gputest.log; exit 1; }
tail -3 gpurun_out/r03d/gputest.log
cat gpurun_out/nonexact_beams.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03d/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r03d/smoke.log; exit 1; }
tail -1 gpurun_out/r03d/smoke.log
export F110_SIMT=1
AB_ENVS=65536 AB_STEPS=100 AB_ROUNDS=3 AB_VARIANTS='fxr:F110_FX_REFILL=1;fxr_n0:F110_FX_REFILL=1,NOISE=0;p2t112:F110_FX_POOL=2,F110_FX_POOL_T=112,F110_FX_PAD=1;p2t112_n0:F110_FX_POOL=2,F110_FX_POOL_T=112,F110_FX_PAD=1,NOISE=0;p2t128:F110_FX_POOL=2,F110_FX_POOL_T=128,F110_FX_PAD=1;p1t112:F110_FX_POOL=1,F110_FX_POOL_T=112,F110_FX_PAD=1;p2t96:F110_FX_POOL=2,F110_FX_POOL_T=96,F110_FX_PAD=1' timeout -k 10 400 python scripts/ray_ab.py > gpurun_out/r03d/ab_pool.json 2> gpurun_out/r03d/ab_pool.err || { echo "ab failed"; tail -20 gpurun_out/r03d/ab_pool.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03d/ab_pool.json'))
for E,l in d['by_envs'].items():
    print(E, l['identical'])
    for k,v in l.items():
        if isinstance(v,dict) and 'k_rays_ms' in v:
            print(k, round(v['k_rays_ms'],4), {a:round(b,3) for a,b in l['diag'].get(k,{}).items()})
PY
