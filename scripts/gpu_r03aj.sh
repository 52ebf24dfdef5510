# HEAD with k_rays_fxs<.., PIPE> as the default: full GPU suite, smoke, default bench, lone-ray probe, rocprof + PMC
set -o pipefail
mkdir -p gpurun_out/r03aj
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03aj/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03aj/tests.log; exit 1; }
tail -1 gpurun_out/r03aj/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03aj/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r03aj/smoke.log; exit 1; }
tail -1 gpurun_out/r03aj/smoke.log
timeout -k 10 500 python bench.py > gpurun_out/r03aj/bench.json 2> gpurun_out/r03aj/bench.err || { echo "bench failed"; tail -30 gpurun_out/r03aj/bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r03aj/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print(d['value'], d['ms_per_step'], d['single_stream']['value'], r['kernel_le_step'], r['frac'], {k: v['value'] for k, v in d.get('secondary', {}).items()}, d['scan_check']['bit_exact_fraction'])
PY
timeout -k 10 300 python scripts/lone_ray.py > gpurun_out/r03aj/lone.json 2> gpurun_out/r03aj/lone.err || { echo lone failed; tail -20 gpurun_out/r03aj/lone.err; exit 1; }
cat gpurun_out/r03aj/lone.json
timeout -k 10 600 python scripts/profile_round.py r03d > gpurun_out/r03aj/prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/r03aj/prof.log; exit 1; }
tail -1 gpurun_out/r03aj/prof.log | cut -c1-300
