# final round-3 evidence at HEAD: rocprofv3 trace + PMC (profile_round r03f), config 4 / 5 lines
set -o pipefail
mkdir -p gpurun_out/r03aq
timeout -k 10 300 python bench.py --agents 2 --global-envs 8192 --no-cpu-baseline --no-secondary > gpurun_out/r03aq/bench_c4.json 2> gpurun_out/r03aq/bench_c4.err || { echo "bench c4 failed"; tail -30 gpurun_out/r03aq/bench_c4.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03aq/bench_c4.json').read().strip().splitlines()[-1]); print('C4', d['value'], d['roofline']['kernel_le_step']['ok'])"
timeout -k 10 300 python bench.py --workload ddpg --agents 2 --global-envs 4096 --no-cpu-baseline --no-secondary > gpurun_out/r03aq/bench_c5.json 2> gpurun_out/r03aq/bench_c5.err || { echo "bench c5 failed"; tail -30 gpurun_out/r03aq/bench_c5.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03aq/bench_c5.json').read().strip().splitlines()[-1]); print('C5', d['value'])"
timeout -k 10 600 python scripts/profile_round.py r03f > gpurun_out/r03aq/prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/r03aq/prof.log; exit 1; }
tail -1 gpurun_out/r03aq/prof.log | cut -c1-200
