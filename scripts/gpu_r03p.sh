set -o pipefail
mkdir -p gpurun_out/r03p
timeout -k 10 600 python bench.py > gpurun_out/r03p/bench.json 2> gpurun_out/r03p/bench.err || { echo "bench failed"; tail -30 gpurun_out/r03p/bench.err; exit 1; }
tail -c 1500 gpurun_out/r03p/bench.json
