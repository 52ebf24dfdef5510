set -o pipefail
mkdir -p gpurun_out/r03f
timeout -k 10 200 python -u -m pytest tests/test_gpu_batch.py -k "step1_matches" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03f/test.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03f/test.log; exit 1; }
tail -2 gpurun_out/r03f/test.log
FA_ENVS=65536,16384,8192,4096 FA_STEPS=200 FA_CHUNK=50 timeout -k 10 500 python scripts/fused_ab.py > gpurun_out/r03f/fused_ab.json 2> gpurun_out/r03f/fused_ab.err || { echo "fused ab failed"; tail -20 gpurun_out/r03f/fused_ab.err; exit 1; }
head -4 gpurun_out/r03f/fused_ab.json
