# TA-bound check: k_rays_fx (1 ray per lane) on the row-major vs the 4x4-tiled EDT at 65536 cars, time + TA busy
set -o pipefail
mkdir -p gpurun_out/r03am
AB_ENVS=65536 AB_STEPS=100 AB_ROUNDS=2 AB_VARIANTS='rm:F110_FX_REFILL=0,F110_FX_ILP=1,F110_FX_TABLE=rm;tl:F110_FX_REFILL=0,F110_FX_ILP=1,F110_FX_TABLE=tiled;fxs:F110_FXR_LEAN=1' timeout -k 10 300 python scripts/ray_ab.py > gpurun_out/r03am/ab.json 2> gpurun_out/r03am/ab.err || { echo "ab failed"; tail -30 gpurun_out/r03am/ab.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03am/ab.json'))
for E,v in d['by_envs'].items(): print(E, v['identical'], {n: round(v[n]['k_rays_ms'],4) for n in ('rm','tl','fxs')})
PY
cd /tmp && export TMPDIR=/tmp
for T in rm tiled; do
  F110_FX_REFILL=0 F110_FX_ILP=1 F110_FX_TABLE=$T MB_ENVS=65536 timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03am/ta_$T -o run -- python3 $GRAFT_REPO_ROOT/scripts/ray_pmc.py > $GRAFT_REPO_ROOT/gpurun_out/r03am/ta_$T.log 2>&1 || { echo "pmc $T failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/r03am/ta_$T.log; exit 1; }
done
echo ok
