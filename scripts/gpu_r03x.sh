# round 3 (second session): k_rays_fxs (lean refill pass) identity tests + A/B against k_rays_fxr
set -o pipefail
mkdir -p gpurun_out/r03x
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_parity.py -k "refill_kernel_identical or fixed_point_cell_index_adversarial" > gpurun_out/r03x/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03x/tests.log; exit 1; }
tail -3 gpurun_out/r03x/tests.log
AB_ENVS=65536,32768 AB_STEPS=200 AB_ROUNDS=3 AB_VARIANTS='fxr:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FXR_LEAN=0;fxs:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FXR_LEAN=1' timeout -k 10 400 python scripts/ray_ab.py > gpurun_out/r03x/ab.json 2> gpurun_out/r03x/ab.err || { echo "ab failed"; tail -30 gpurun_out/r03x/ab.err; exit 1; }
cat gpurun_out/r03x/ab.json
