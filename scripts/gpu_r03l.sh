set -o pipefail
mkdir -p gpurun_out/r03l
F110_RECORD_NONEXACT=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03l/gputest.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03l/gputest.log; exit 1; }
tail -3 gpurun_out/r03l/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03l/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r03l/smoke.log; exit 1; }
tail -2 gpurun_out/r03l/smoke.log
