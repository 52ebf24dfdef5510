# rocprofv3 kernel stats of the default bench at HEAD (packed tables)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03bg
cd $R && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03bg/prof -o run -- python3 bench.py --steps 300 --no-cpu-baseline --no-secondary --no-full-outputs > $R/gpurun_out/r03bg/bench.json 2> $R/gpurun_out/r03bg/bench.err || { tail -20 $R/gpurun_out/r03bg/bench.err; exit 1; }
find $R/gpurun_out/r03bg/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $R/gpurun_out/r03bg/kernel_stats.csv
