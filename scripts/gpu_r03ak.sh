# small shards: k_rays_fxn (default below 32768 cars) vs k_rays_fxs with 1-3 waves per car, and fxn's rays per lane
set -o pipefail
mkdir -p gpurun_out/r03ak
AB_ENVS=8192,16384,32768 AB_STEPS=200 AB_ROUNDS=3 AB_VARIANTS='fxn2:F110_FX_REFILL=0;fxn1:F110_FX_REFILL=0,F110_FX_ILP=1;fxn3:F110_FX_REFILL=0,F110_FX_ILP=3;fxs1:F110_FX_REFILL=1,F110_FX_PAD=1;fxs2:F110_FX_REFILL=2,F110_FX_PAD=1;fxs3:F110_FX_REFILL=3,F110_FX_PAD=1' timeout -k 10 400 python scripts/ray_ab.py > gpurun_out/r03ak/ab.json 2> gpurun_out/r03ak/ab.err || { echo "ab failed"; tail -30 gpurun_out/r03ak/ab.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03ak/ab.json'))
for E,v in d['by_envs'].items(): print(E, all(v['identical'].values()), {n: round(v[n]['k_rays_ms'],4) for n in ('fxn2','fxn1','fxn3','fxs1','fxs2','fxs3')})
PY
