# 32768 cars per context: refill kernel with heavy-first off (one context) and S = 4 sub-shards; GPU suite
set -o pipefail
mkdir -p gpurun_out/r03as
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03as/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03as/tests.log; exit 1; }
tail -1 gpurun_out/r03as/tests.log
for E in 32768 16384; do
  timeout -k 10 200 python bench.py --steps 500 --no-cpu-baseline --no-secondary --no-full-outputs --global-envs $E > gpurun_out/r03as/e$E.json 2> gpurun_out/r03as/e$E.err || { tail -20 gpurun_out/r03as/e$E.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r03as/e$E.json').read().strip().splitlines()[-1]); print('$E', d['value'], d['config']['streams_per_gpu'], d['single_stream']['value'], d['roofline']['ray_kernel'], d['roofline']['kernel_le_step']['ok'])"
done
