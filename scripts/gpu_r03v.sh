set -o pipefail
mkdir -p gpurun_out/r03v
timeout -k 10 600 python bench.py > gpurun_out/r03v/bench.json 2> gpurun_out/r03v/bench.err || { echo "bench failed"; tail -30 gpurun_out/r03v/bench.err; exit 1; }
tail -c 600 gpurun_out/r03v/bench.json
timeout -k 10 900 python scripts/profile_round.py r03 > gpurun_out/r03v/profile_round.log 2>&1 || { echo "profile_round failed"; tail -30 gpurun_out/r03v/profile_round.log; exit 1; }
tail -5 gpurun_out/r03v/profile_round.log
