set -o pipefail
mkdir -p gpurun_out/r03j
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -k "step1_matches" -x -v --timeout 120 --timeout-method thread > gpurun_out/r03j/test.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03j/test.log; exit 1; }
tail -6 gpurun_out/r03j/test.log
for c in ${CPWS:-8 4 2}; do
F110_FUSED_CPW=$c FA_MODES=three,fused,fused_n FA_ENVS=65536,8192,4096 FA_STEPS=200 FA_CHUNK=50 FA_ROUNDS=2 timeout -k 10 300 python scripts/fused_ab.py > gpurun_out/r03j/fused_ab_$c.json 2> gpurun_out/r03j/fused_ab_$c.err || { echo "fused ab failed"; tail -20 gpurun_out/r03j/fused_ab_$c.err; exit 1; }
echo "cpw $c"; tail -1 gpurun_out/r03j/fused_ab_$c.json
done
