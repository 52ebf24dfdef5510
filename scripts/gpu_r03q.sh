set -o pipefail
mkdir -p gpurun_out/r03q
AB_ENVS=65536,16384,8192,4096 AB_STEPS=100 AB_ROUNDS=3 AB_VARIANTS='p0:F110_PRIO_T=0;p16:F110_PRIO_T=16;p32:F110_PRIO_T=32;p64:F110_PRIO_T=64;p128:F110_PRIO_T=128' timeout -k 10 500 python scripts/ray_ab.py > gpurun_out/r03q/ab_prio.json 2> gpurun_out/r03q/ab_prio.err || { echo "ab failed"; tail -20 gpurun_out/r03q/ab_prio.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03q/ab_prio.json'))
for E,l in d['by_envs'].items():
    print(E, all(v for k,v in l['identical'].items() if not k.endswith('_diff')), {k: round(v['k_rays_ms'],4) for k,v in l.items() if isinstance(v,dict) and 'k_rays_ms' in v})
PY
