set -o pipefail
mkdir -p gpurun_out/r03w
timeout -k 10 400 python bench.py --steps 1000 --no-cpu-baseline --no-secondary > gpurun_out/r03w/bench.json 2> gpurun_out/r03w/bench.err || { echo "bench failed"; tail -30 gpurun_out/r03w/bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r03w/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print(d['value'], r['kernel_le_step'], r['step_kernels_ms'], r['frac'])
PY
