set -o pipefail
mkdir -p gpurun_out/r03a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03a/gputest.log 2>&1 || { echo "gputests failed"; tail -30 gpurun_out/r03a/gputest.log; exit 1; }
tail -3 gpurun_out/r03a/gputest.log
timeout -k 10 400 python bench.py > gpurun_out/r03a/bench_n1.json 2> gpurun_out/r03a/bench_n1.err || { echo bench failed; tail -20 gpurun_out/r03a/bench_n1.err; exit 1; }
F110_SAME_DEVICE=1 F110_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --no-cpu-baseline > gpurun_out/r03a/bench_2rank.json 2> gpurun_out/r03a/bench_2rank.err || { echo bench2 failed; tail -20 gpurun_out/r03a/bench_2rank.err; exit 1; }
python -c "
import json
a=json.load(open('gpurun_out/r03a/bench_n1.json')); b=json.load(open('gpurun_out/r03a/bench_2rank.json'))
print('n1', a['value'], a['trajectory_digest'], a['roofline']['kernel_le_step'], a['roofline']['frac'], a['roofline']['simt_efficiency'])
print('n2', b['value'], b['trajectory_digest'])
"
