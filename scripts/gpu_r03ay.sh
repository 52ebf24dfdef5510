# k_rays_fxs gathers for ended lanes: zero cell (0) / range-checked buffer load (1) / none, exec mask (2):
# parity, kernel A/B, TA busy and L1 accesses per launch at 65536 cars
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03ay
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_batch.py::test_refill_kernel_identical tests/test_gpu_parity.py::test_fixed_point_cell_index_adversarial_vs_oracle > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
AB_ENVS=65536,32768 AB_VARIANTS='m0:F110_FXS_MASKLD=0;m1:F110_FXS_MASKLD=1;m2:F110_FXS_MASKLD=2;m0b:F110_FXS_MASKLD=0;m2b:F110_FXS_MASKLD=2' timeout -k 10 400 python scripts/ray_ab.py > $OUT/ab.json 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
python - <<PY
import json
d = json.loads(open('$OUT/ab.json').read().strip().splitlines()[-1])
for E, r in d['by_envs'].items():
    print(E, {k: round(v['k_rays_ms'], 4) for k, v in r.items() if isinstance(v, dict) and 'k_rays_ms' in v}, r.get('identical'))
PY
cd /tmp && export TMPDIR=/tmp
for M in 0 2; do
  F110_FXS_MASKLD=$M MB_ENVS=65536 timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/ta_m$M -o run -- python3 $R/scripts/ray_pmc.py > $OUT/ta_m$M.log 2>&1 || { echo "pmc $M failed"; tail -5 $OUT/ta_m$M.log; exit 1; }
done
