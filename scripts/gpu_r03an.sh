# k_rays_fxs on the 4x4-tiled padded table (F110_FXS_TILE=1): identity + A/B + TA busy
set -o pipefail
mkdir -p gpurun_out/r03an
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_parity.py -k "refill_kernel_identical or fixed_point_cell_index_adversarial" > gpurun_out/r03an/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03an/tests.log; exit 1; }
tail -1 gpurun_out/r03an/tests.log
AB_ENVS=65536,32768,8192 AB_STEPS=200 AB_ROUNDS=3 AB_VARIANTS='fxs:F110_FX_REFILL=1,F110_FX_PAD=1;tile:F110_FX_REFILL=1,F110_FX_PAD=1,F110_FXS_TILE=1' timeout -k 10 300 python scripts/ray_ab.py > gpurun_out/r03an/ab.json 2> gpurun_out/r03an/ab.err || { echo "ab failed"; tail -30 gpurun_out/r03an/ab.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03an/ab.json'))
for E,v in d['by_envs'].items(): print(E, v['identical'], {n: round(v[n]['k_rays_ms'],4) for n in ('fxs','tile')})
PY
cd /tmp && export TMPDIR=/tmp
for T in 0 1; do
  F110_FXS_TILE=$T MB_ENVS=65536 timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03an/ta_$T -o run -- python3 $GRAFT_REPO_ROOT/scripts/ray_pmc.py > $GRAFT_REPO_ROOT/gpurun_out/r03an/ta_$T.log 2>&1 || { echo "pmc $T failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/r03an/ta_$T.log; exit 1; }
done
echo ok
