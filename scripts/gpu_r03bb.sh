# timing probe: do 4-byte gathers cost the TA fewer cycles than 8-byte ones? (F110_FXS_MASKLD=4, not exact)
# (the MASKLD=4 probe build was removed after this run; DESIGN §3.9 has the result)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03bb
mkdir -p $OUT
AB_ENVS=65536 AB_VARIANTS='m0:F110_FXS_MASKLD=0;m4:F110_FXS_MASKLD=4;m0b:F110_FXS_MASKLD=0;m4b:F110_FXS_MASKLD=4' timeout -k 10 300 python scripts/ray_ab.py > $OUT/ab.json 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
python - <<PY
import json
d = json.loads(open('$OUT/ab.json').read().strip().splitlines()[-1])
for E, r in d['by_envs'].items():
    print(E, {k: (round(v['k_rays_ms'], 4), round(r.get('mean_lookups', {}).get(k, 0), 4)) for k, v in r.items() if isinstance(v, dict) and 'k_rays_ms' in v})
PY
cd /tmp && export TMPDIR=/tmp
for M in 0 4; do
  F110_FXS_MASKLD=$M MB_ENVS=65536 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD TA_BUSY_avr GRBM_GUI_ACTIVE --output-format csv -d $OUT/ta_m$M -o run -- python3 $R/scripts/ray_pmc.py > $OUT/ta_m$M.log 2>&1 || { echo "pmc failed"; tail -8 $OUT/ta_m$M.log; exit 1; }
done
