# bench at the driver's short settings and edge step counts (the interleaved profile pass), and the default run
set -o pipefail
mkdir -p gpurun_out/r03ap
for KW in "20 5" "1 1" "7 0" "120 10"; do
  set -- $KW
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu-baseline > gpurun_out/r03ap/bench_$1_$2.json 2> gpurun_out/r03ap/bench_$1_$2.err || { echo "bench $1 $2 failed"; tail -20 gpurun_out/r03ap/bench_$1_$2.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r03ap/bench_$1_$2.json').read().strip().splitlines()[-1]); print('K=$1 W=$2', round(d['value']/1e6,2), d['roofline']['kernel_le_step']['ok'], round(d['roofline']['kernel_ms'],4), round(d['single_stream']['ms_per_step'],4))"
done
F110_SAME_DEVICE=1 F110_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/r03ap/bench_2rank_short.json 2> gpurun_out/r03ap/bench_2rank_short.err || { echo bench2 failed; tail -20 gpurun_out/r03ap/bench_2rank_short.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03ap/bench_2rank_short.json').read().strip().splitlines()[-1]); print('2rank short', round(d['value']/1e6,2), d['roofline']['kernel_le_step']['ok'])"
timeout -k 10 500 python bench.py > gpurun_out/r03ap/bench.json 2> gpurun_out/r03ap/bench.err || { echo "bench failed"; tail -30 gpurun_out/r03ap/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03ap/bench.json').read().strip().splitlines()[-1]); print('default', round(d['value']/1e6,2), d['roofline']['kernel_le_step'], d['roofline']['frac'], d['roofline']['gather_roofline']['frac'])"
