# the stream-count / refill rules at the scaling shard sizes and C4, against the previous choices
set -e
mkdir -p gpurun_out/refill_rules
timeout -k 10 120 python bench.py --global-envs 16384 --no-cpu-baseline --no-secondary > gpurun_out/refill_rules/e16384.json 2>/dev/null
timeout -k 10 120 python bench.py --global-envs 32768 --no-cpu-baseline --no-secondary > gpurun_out/refill_rules/e32768.json 2>/dev/null
timeout -k 10 120 python bench.py --global-envs 32768 --streams 4 --no-cpu-baseline --no-secondary > gpurun_out/refill_rules/e32768_s4.json 2>/dev/null
timeout -k 10 150 python bench.py --agents 2 --global-envs 8192 --no-cpu-baseline --no-secondary --steps 300 --warmup 30 > gpurun_out/refill_rules/c4.json 2>/dev/null
F110_FX_REFILL=0 timeout -k 10 150 python bench.py --agents 2 --global-envs 8192 --streams 2 --no-cpu-baseline --no-secondary --steps 300 --warmup 30 > gpurun_out/refill_rules/c4_prev.json 2>/dev/null
F110_FX_REFILL=0 timeout -k 10 150 python bench.py --agents 2 --global-envs 8192 --streams 4 --no-cpu-baseline --no-secondary --steps 300 --warmup 30 > gpurun_out/refill_rules/c4_s4_norefill.json 2>/dev/null
