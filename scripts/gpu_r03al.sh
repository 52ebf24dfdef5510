# is k_rays bound by the vector-memory address / data path? TA / TD busy and L1 traffic at 65536 and 8192 cars
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03al
mkdir -p $OUT
for E in 65536 8192; do
  MB_ENVS=$E timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max TD_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/ta_$E -o run -- python3 $R/scripts/ray_pmc.py > $OUT/ta_$E.log 2>&1 || { echo "pmc $E failed"; tail -5 $OUT/ta_$E.log; exit 1; }
done
python3 - <<PY
import csv, glob, json
res = {}
for E in (65536, 8192):
    f = glob.glob('$OUT/ta_%d/**/*counter_collection.csv' % E, recursive=True)[0]
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
    res[E] = m
print(json.dumps(res))
json.dump(res, open('$OUT/summary.json', 'w'), indent=1)
PY
