# 2-rank same-GPU gloo rehearsal of the N>1 bench path with the interleaved profile pass (digest must equal N=1's),
# and the lone-ray probe of the small-shard floor
set -o pipefail
mkdir -p gpurun_out/r03ah
F110_SAME_DEVICE=1 F110_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/r03ah/bench_2rank.json 2> gpurun_out/r03ah/bench_2rank.err || { echo bench2 failed; tail -20 gpurun_out/r03ah/bench_2rank.err; exit 1; }
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/r03ah/bench_1rank.json 2> gpurun_out/r03ah/bench_1rank.err || { echo bench1 failed; tail -20 gpurun_out/r03ah/bench_1rank.err; exit 1; }
python - <<'PY'
import json
a=json.loads(open('gpurun_out/r03ah/bench_2rank.json').read().strip().splitlines()[-1])
b=json.loads(open('gpurun_out/r03ah/bench_1rank.json').read().strip().splitlines()[-1])
print('2rank', a['value'], a['trajectory_digest'], a['roofline']['kernel_le_step'])
print('1rank', b['value'], b['trajectory_digest'])
print('digest equal', a['trajectory_digest']['sha256'] == b['trajectory_digest']['sha256'])
PY
timeout -k 10 300 python scripts/lone_ray.py > gpurun_out/r03ah/lone.json 2> gpurun_out/r03ah/lone.err || { echo lone failed; tail -20 gpurun_out/r03ah/lone.err; exit 1; }
cat gpurun_out/r03ah/lone.json
