# round-3 final state (k_rays_fxs default): full GPU suite, smoke, default bench, C4 / C5 lines, rocprof + PMC
set -o pipefail
mkdir -p gpurun_out/r03af
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03af/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03af/tests.log; exit 1; }
tail -1 gpurun_out/r03af/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03af/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r03af/smoke.log; exit 1; }
tail -1 gpurun_out/r03af/smoke.log
timeout -k 10 500 python bench.py > gpurun_out/r03af/bench.json 2> gpurun_out/r03af/bench.err || { echo "bench failed"; tail -30 gpurun_out/r03af/bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r03af/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print(d['value'], d['ms_per_step'], d['single_stream']['value'], r['kernel_le_step'], r['frac'], d['secondary'] if 'secondary' in d else None, d['cpu_baseline']['value'] if d.get('cpu_baseline') else None, d['scan_check']['bit_exact_fraction'])
PY
timeout -k 10 300 python bench.py --agents 2 --global-envs 8192 --no-cpu-baseline --no-secondary > gpurun_out/r03af/bench_c4.json 2> gpurun_out/r03af/bench_c4.err || { echo "bench c4 failed"; tail -30 gpurun_out/r03af/bench_c4.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03af/bench_c4.json').read().strip().splitlines()[-1]); print('C4', d['value'], d['metric'])"
timeout -k 10 300 python bench.py --workload ddpg --agents 2 --global-envs 4096 --no-cpu-baseline --no-secondary > gpurun_out/r03af/bench_c5.json 2> gpurun_out/r03af/bench_c5.err || { echo "bench c5 failed"; tail -30 gpurun_out/r03af/bench_c5.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03af/bench_c5.json').read().strip().splitlines()[-1]); print('C5', d['value'], d['metric'])"
timeout -k 10 600 python scripts/profile_round.py r03c > gpurun_out/r03af/prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/r03af/prof.log; exit 1; }
tail -2 gpurun_out/r03af/prof.log | cut -c1-400
