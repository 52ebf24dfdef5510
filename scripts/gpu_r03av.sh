# k_rays_fxs occupancy probe at 65536 cars (dynamic LDS per one-wave block caps waves per CU)
set -o pipefail
mkdir -p gpurun_out/r03av
AB_ENVS=65536 AB_VARIANTS='l0:F110_FX_LDS=0;l5632:F110_FX_LDS=5632;l6656:F110_FX_LDS=6656;l8192:F110_FX_LDS=8192;l10240:F110_FX_LDS=10240' timeout -k 10 400 python scripts/ray_ab.py > gpurun_out/r03av/ab.json 2> gpurun_out/r03av/ab.err || { tail -20 gpurun_out/r03av/ab.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r03av/ab.json').read().strip().splitlines()[-1])
for E, r in d['by_envs'].items():
    print(E, {k: round(v['k_rays_ms'], 4) for k, v in r.items() if isinstance(v, dict) and 'k_rays_ms' in v}, r.get('identical'))
PY
