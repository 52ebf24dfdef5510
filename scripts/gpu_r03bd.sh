# bench at HEAD: the per-instruction gather roofline fields
set -o pipefail
mkdir -p gpurun_out/r03bd
timeout -k 10 400 python bench.py > gpurun_out/r03bd/bench.json 2> gpurun_out/r03bd/bench.err || { tail -20 gpurun_out/r03bd/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03bd/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['simt_efficiency'], d['roofline']['gather_roofline'], d['roofline']['bound'])"
