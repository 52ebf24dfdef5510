# k_rays_fxs with range-checked buffer gathers (F110_FXS_MASKLD): parity, kernel A/B at 65536 / 32768 cars, bench
set -o pipefail
mkdir -p gpurun_out/r03aw
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_batch.py::test_refill_kernel_identical tests/test_gpu_parity.py::test_fixed_point_cell_index_adversarial_vs_oracle > gpurun_out/r03aw/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03aw/tests.log; exit 1; }
tail -1 gpurun_out/r03aw/tests.log
AB_ENVS=65536,32768 AB_VARIANTS='g:F110_FXS_MASKLD=0;b:F110_FXS_MASKLD=1;g2:F110_FXS_MASKLD=0;b2:F110_FXS_MASKLD=1' timeout -k 10 400 python scripts/ray_ab.py > gpurun_out/r03aw/ab.json 2> gpurun_out/r03aw/ab.err || { tail -20 gpurun_out/r03aw/ab.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r03aw/ab.json').read().strip().splitlines()[-1])
for E, r in d['by_envs'].items():
    print(E, {k: round(v['k_rays_ms'], 4) for k, v in r.items() if isinstance(v, dict) and 'k_rays_ms' in v}, r.get('identical'))
PY
for M in 0 1; do
  F110_FXS_MASKLD=$M timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/r03aw/bench_m$M.json 2> gpurun_out/r03aw/bench_m$M.err || { tail -20 gpurun_out/r03aw/bench_m$M.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r03aw/bench_m$M.json').read().strip().splitlines()[-1]); print('m$M', d['value'], d['roofline']['frac'], d['roofline']['kernel_le_step'])"
done
