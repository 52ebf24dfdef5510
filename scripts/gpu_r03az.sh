# k_rays_fxs lock-step slots sharing one gather when no lane has both rays active (F110_FXS_PIPE=0 F110_FXS_MASKLD=3)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03az
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_batch.py::test_refill_kernel_identical tests/test_gpu_parity.py::test_fixed_point_cell_index_adversarial_vs_oracle > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
AB_ENVS=65536,32768,8192 AB_VARIANTS='pipe:F110_FXS_PIPE=1;lock:F110_FXS_PIPE=0;merge:F110_FXS_PIPE=0,F110_FXS_MASKLD=3;pipeb:F110_FXS_PIPE=1;mergeb:F110_FXS_PIPE=0,F110_FXS_MASKLD=3' timeout -k 10 400 python scripts/ray_ab.py > $OUT/ab.json 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
python - <<PY
import json
d = json.loads(open('$OUT/ab.json').read().strip().splitlines()[-1])
for E, r in d['by_envs'].items():
    print(E, {k: round(v['k_rays_ms'], 4) for k, v in r.items() if isinstance(v, dict) and 'k_rays_ms' in v}, r.get('identical'))
PY
