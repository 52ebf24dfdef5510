# HEAD with packed tables on by default: full GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out/r03bf
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03bf/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03bf/tests.log; exit 1; }
tail -1 gpurun_out/r03bf/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03bf/smoke.log 2>&1 || { tail -20 gpurun_out/r03bf/smoke.log; exit 1; }
tail -1 gpurun_out/r03bf/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r03bf/bench.json 2> gpurun_out/r03bf/bench.err || { tail -20 gpurun_out/r03bf/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03bf/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['ray_kernel'], d['roofline']['kernel_le_step'])"
