# HEAD after the TILE revert: full GPU suite, smoke, default bench (gather roofline field)
set -o pipefail
mkdir -p gpurun_out/r03ao
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03ao/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03ao/tests.log; exit 1; }
tail -1 gpurun_out/r03ao/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03ao/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r03ao/smoke.log; exit 1; }
tail -1 gpurun_out/r03ao/smoke.log
timeout -k 10 500 python bench.py > gpurun_out/r03ao/bench.json 2> gpurun_out/r03ao/bench.err || { echo "bench failed"; tail -30 gpurun_out/r03ao/bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r03ao/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print(d['value'], d['ms_per_step'], d['single_stream']['value'], r['kernel_le_step']['ok'], r['kernel_ms'], r['frac'], r.get('gather_roofline'), {k: v['value'] for k, v in d.get('secondary', {}).items()})
PY
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r03ao/bench_short.json 2> gpurun_out/r03ao/bench_short.err || { echo "bench short failed"; tail -30 gpurun_out/r03ao/bench_short.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03ao/bench_short.json').read().strip().splitlines()[-1]); print('short', d['value'], d['roofline']['kernel_le_step'])"
