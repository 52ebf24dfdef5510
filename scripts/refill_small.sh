# k_rays_fxr on the small per-GPU shards (N = 4 / 8 scaling sizes) with 4 stream sub-shards
set -e
mkdir -p gpurun_out/refill_small
timeout -k 10 120 python bench.py --global-envs 16384 --streams 4 --no-cpu-baseline --no-secondary > gpurun_out/refill_small/e16384_s4.json 2>/dev/null
F110_FX_REFILL=1 F110_FX_PAD=1 timeout -k 10 120 python bench.py --global-envs 16384 --streams 4 --no-cpu-baseline --no-secondary > gpurun_out/refill_small/e16384_s4_refill.json 2>/dev/null
F110_FX_ILP=2 F110_FX_REFILL=1 F110_FX_PAD=1 timeout -k 10 120 python bench.py --global-envs 8192 --streams 4 --no-cpu-baseline --no-secondary > gpurun_out/refill_small/e8192_s4_refill.json 2>/dev/null
F110_FX_ILP=2 F110_FX_REFILL=1 F110_FX_PAD=1 timeout -k 10 120 python bench.py --global-envs 8192 --streams 2 --no-cpu-baseline --no-secondary > gpurun_out/refill_small/e8192_s2_refill.json 2>/dev/null
