# k_rays_fxs (lean pass, fminf clamp, scalar lane count) identity + A/B; kernel-attached profiling events; short bench
set -o pipefail
mkdir -p gpurun_out/r03y
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_parity.py -k "refill_kernel_identical or fixed_point_cell_index_adversarial" > gpurun_out/r03y/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03y/tests.log; exit 1; }
tail -2 gpurun_out/r03y/tests.log
AB_ENVS=65536,32768,16384 AB_STEPS=200 AB_ROUNDS=3 AB_VARIANTS='fxr:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FXR_LEAN=0;fxs:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FXR_LEAN=1' timeout -k 10 400 python scripts/ray_ab.py > gpurun_out/r03y/ab.json 2> gpurun_out/r03y/ab.err || { echo "ab failed"; tail -30 gpurun_out/r03y/ab.err; exit 1; }
cat gpurun_out/r03y/ab.json
timeout -k 10 400 python bench.py --steps 1000 --no-cpu-baseline --no-secondary > gpurun_out/r03y/bench.json 2> gpurun_out/r03y/bench.err || { echo "bench failed"; tail -30 gpurun_out/r03y/bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r03y/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print(d['value'], d['ms_per_step'], d.get('single_stream'), r['kernel_le_step'], r['step_kernels_ms'], r['frac'], r.get('simt_efficiency'))
PY
