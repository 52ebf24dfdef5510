# k_rays_fxs (alignbit-free fixed-point offsets, branchless slot steps, padded rows of 511 mod 512 cells):
# full GPU suite, A/B against k_rays_fxr, bench with the interleaved profile
set -o pipefail
mkdir -p gpurun_out/r03z
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03z/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03z/tests.log; exit 1; }
tail -2 gpurun_out/r03z/tests.log
AB_ENVS=65536,32768 AB_STEPS=200 AB_ROUNDS=3 AB_VARIANTS='fxr:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FXR_LEAN=0;fxs:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FXR_LEAN=1' timeout -k 10 400 python scripts/ray_ab.py > gpurun_out/r03z/ab.json 2> gpurun_out/r03z/ab.err || { echo "ab failed"; tail -30 gpurun_out/r03z/ab.err; exit 1; }
cat gpurun_out/r03z/ab.json
timeout -k 10 400 python bench.py --steps 1000 --no-cpu-baseline --no-secondary > gpurun_out/r03z/bench.json 2> gpurun_out/r03z/bench.err || { echo "bench failed"; tail -30 gpurun_out/r03z/bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r03z/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print(d['value'], d['ms_per_step'], d.get('single_stream'), r['kernel_le_step'], r['step_kernels_ms'], r['frac'], r.get('simt_efficiency'))
PY
