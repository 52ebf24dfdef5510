set -o pipefail
mkdir -p gpurun_out/r03r
AB_ENVS=8192,4096 AB_STEPS=100 AB_ROUNDS=3 AB_VARIANTS='def:F110_HEAVY_T=0;fx1:F110_FX_ILP=1,F110_HEAVY_T=0;tiled1:F110_FX_ILP=1,F110_FX_TABLE=tiled,F110_HEAVY_T=0;fxr1:F110_FX_REFILL=1,F110_FX_PAD=1,F110_HEAVY_T=0' timeout -k 10 400 python scripts/ray_ab.py > gpurun_out/r03r/ab_table.json 2> gpurun_out/r03r/ab_table.err || { echo "ab failed"; tail -20 gpurun_out/r03r/ab_table.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03r/ab_table.json'))
for E,l in d['by_envs'].items():
    print(E, all(v for k,v in l['identical'].items() if not k.endswith('_diff')), {k: round(v['k_rays_ms'],4) for k,v in l.items() if isinstance(v,dict) and 'k_rays_ms' in v})
PY
