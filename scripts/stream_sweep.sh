set -e
mkdir -p gpurun_out/sweep
for cfg in "8192 4" "8192 8" "8192 6" "4096 4" "4096 8"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --global-envs $1 --streams $2 --no-cpu-baseline --no-secondary --steps 1000 --warmup 100 > gpurun_out/sweep/e$1_s$2.json 2> gpurun_out/sweep/e$1_s$2.err
done
