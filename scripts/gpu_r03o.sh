set -o pipefail
mkdir -p gpurun_out/r03o
AB_ENVS=16384,8192,4096 AB_STEPS=100 AB_ROUNDS=3 AB_VARIANTS='fxn2:F110_FX_REFILL=0,F110_FX_ILP=2;fxn2p:F110_FX_REFILL=0,F110_FX_ILP=2,F110_FX_PAD=1;fxn3p:F110_FX_REFILL=0,F110_FX_ILP=3,F110_FX_PAD=1;fxn3:F110_FX_REFILL=0,F110_FX_ILP=3;fxn4:F110_FX_REFILL=0,F110_FX_ILP=4;fxr1:F110_FX_REFILL=1,F110_FX_PAD=1,F110_HEAVY_T=0;fxr2:F110_FX_REFILL=2,F110_FX_PAD=1,F110_HEAVY_T=0;fxr3:F110_FX_REFILL=3,F110_FX_PAD=1,F110_HEAVY_T=0;fxr1s3:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FX_SLOTS=3,F110_HEAVY_T=0;h0:F110_HEAVY_T=0' timeout -k 10 500 python scripts/ray_ab.py > gpurun_out/r03o/ab_small.json 2> gpurun_out/r03o/ab_small.err || { echo "ab failed"; tail -20 gpurun_out/r03o/ab_small.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03o/ab_small.json'))
for E,l in d['by_envs'].items():
    print(E, l.get('identical'), {k: round(v['k_rays_ms'],4) for k,v in l.items() if isinstance(v,dict) and 'k_rays_ms' in v})
PY
AB_AGENTS=2 AB_ENVS=8192 AB_STEPS=100 AB_ROUNDS=3 AB_VARIANTS='fxn2:F110_FX_REFILL=0,F110_FX_ILP=2;fxn2p:F110_FX_REFILL=0,F110_FX_ILP=2,F110_FX_PAD=1;fxn3p:F110_FX_REFILL=0,F110_FX_ILP=3,F110_FX_PAD=1;fxr1:F110_FX_REFILL=1,F110_FX_PAD=1,F110_HEAVY_T=0;h0:F110_HEAVY_T=0' timeout -k 10 300 python scripts/ray_ab.py > gpurun_out/r03o/ab_c4.json 2> gpurun_out/r03o/ab_c4.err || { echo "ab c4 failed"; tail -20 gpurun_out/r03o/ab_c4.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03o/ab_c4.json'))
for E,l in d['by_envs'].items():
    print('C4', E, l.get('identical'), {k: round(v['k_rays_ms'],4) for k,v in l.items() if isinstance(v,dict) and 'k_rays_ms' in v}, {k: round(v.get('ms_per_step',0),4) for k,v in l.items() if isinstance(v,dict) and 'k_rays_ms' in v})
PY
