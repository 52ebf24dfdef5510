# k_rays_fxs with interleaved (cos, sin) / (side, beam_cos) tables: one 16-byte load each (F110_FXS_PACK)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03be
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_batch.py::test_refill_kernel_identical tests/test_gpu_parity.py::test_fixed_point_cell_index_adversarial_vs_oracle > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
AB_ENVS=65536,32768 AB_VARIANTS='p0:F110_FXS_PACK=0;p1:F110_FXS_PACK=1;p0b:F110_FXS_PACK=0;p1b:F110_FXS_PACK=1' timeout -k 10 300 python scripts/ray_ab.py > $OUT/ab.json 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
python - <<PY
import json
d = json.loads(open('$OUT/ab.json').read().strip().splitlines()[-1])
for E, r in d['by_envs'].items():
    print(E, {k: round(v['k_rays_ms'], 4) for k, v in r.items() if isinstance(v, dict) and 'k_rays_ms' in v}, r.get('identical'))
PY
cd /tmp && export TMPDIR=/tmp
F110_FXS_PACK=1 MB_ENVS=65536 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD TA_BUSY_avr GRBM_GUI_ACTIVE --output-format csv -d $OUT/ta_p1 -o run -- python3 $R/scripts/ray_pmc.py > $OUT/ta_p1.log 2>&1 || { echo "pmc failed"; tail -8 $OUT/ta_p1.log; exit 1; }
