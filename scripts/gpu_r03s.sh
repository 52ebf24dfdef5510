set -o pipefail
mkdir -p gpurun_out/r03s
AB_ENVS=16384,8192,4096 AB_STEPS=100 AB_ROUNDS=3 AB_VARIANTS='pf0:F110_PF_T=0;pf4:F110_PF_T=4;pf8:F110_PF_T=8;pf16:F110_PF_T=16;pf32:F110_PF_T=32' timeout -k 10 400 python scripts/ray_ab.py > gpurun_out/r03s/ab_pf.json 2> gpurun_out/r03s/ab_pf.err || { echo "ab failed"; tail -20 gpurun_out/r03s/ab_pf.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03s/ab_pf.json'))
for E,l in d['by_envs'].items():
    print(E, all(v for k,v in l['identical'].items() if not k.endswith('_diff')), {k: round(v['k_rays_ms'],4) for k,v in l.items() if isinstance(v,dict) and 'k_rays_ms' in v})
PY
