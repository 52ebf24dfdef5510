# bench lines at the per-GPU shard sizes of the N = 2 / 4 scaling runs: default kernel choice vs
# k_rays_fxr (+ padded EDT) forced on for the stream sub-shards (DESIGN 3.4 size rule)
set -e
mkdir -p gpurun_out/refill_sizes
for E in 32768 16384; do
  timeout -k 10 150 python bench.py --global-envs $E --no-cpu-baseline --no-secondary > gpurun_out/refill_sizes/e${E}_default.json 2>/dev/null
  F110_FX_REFILL=1 F110_FX_PAD=1 timeout -k 10 150 python bench.py --global-envs $E --no-cpu-baseline --no-secondary > gpurun_out/refill_sizes/e${E}_refill.json 2>/dev/null
done
