# small shards: stream sub-shards beyond HIP's default 4 hardware queues per process (GPU_MAX_HW_QUEUES)
set -o pipefail
mkdir -p gpurun_out/r03ad
for Q in 4 8 16; do
  for E in 8192 16384 4096; do
    for S in 4 8 16; do
      if [ $S -gt $Q ] && [ $S -gt 4 ]; then continue; fi
      GPU_MAX_HW_QUEUES=$Q timeout -k 10 120 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --no-secondary --no-full-outputs --global-envs $E --streams $S > gpurun_out/r03ad/q${Q}_e${E}_s${S}.json 2> gpurun_out/r03ad/q${Q}_e${E}_s${S}.err || { echo "bench failed q$Q e$E s$S"; tail -20 gpurun_out/r03ad/q${Q}_e${E}_s${S}.err; exit 1; }
      python -c "
import json,sys
d=json.loads(open('gpurun_out/r03ad/q${Q}_e${E}_s${S}.json').read().strip().splitlines()[-1])
print('Q=$Q E=$E S=$S', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],4), 'ms; one ctx', round(d['single_stream']['value']/1e6,2) if d.get('single_stream') else None)
"
    done
  done
done
