# k_rays_fxs at 65536 cars, zero-cell gathers vs range-checked buffer gathers: TA / TD busy and L1 accesses
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03ax
mkdir -p $OUT
for M in 0 1; do
  F110_FXS_MASKLD=$M MB_ENVS=65536 timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max TD_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/ta_m$M -o run -- python3 $R/scripts/ray_pmc.py > $OUT/ta_m$M.log 2>&1 || { echo "pmc $M failed"; tail -5 $OUT/ta_m$M.log; exit 1; }
done
python3 - <<PY
import csv, glob, json
res = {}
for M in (0, 1):
    f = glob.glob('$OUT/ta_m%d/**/*counter_collection.csv' % M, recursive=True)[0]
    vals = {}
    for row in csv.DictReader(open(f)):
        if 'k_rays' in row.get('Kernel_Name', ''):
            vals.setdefault(row['Counter_Name'], []).append(float(row['Counter_Value']))
    m = {k: sum(v) / len(v) for k, v in vals.items()}
    cyc = m['GRBM_GUI_ACTIVE'] / 8.0
    m['ta_busy_frac'] = m['TA_BUSY_avr'] / cyc
    m['ta_busy_max_frac'] = m['TA_BUSY_max'] / cyc
    m['td_busy_frac'] = m['TD_BUSY_avr'] / cyc
    m['l1_hit'] = 1 - m['TCP_TCC_READ_REQ_sum'] / max(1, m['TCP_TOTAL_CACHE_ACCESSES_sum'])
    res['maskld_%d' % M] = m
print(json.dumps(res))
json.dump(res, open('$OUT/summary.json', 'w'), indent=1)
PY
