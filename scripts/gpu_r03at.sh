# k_rays_fx speculative tail step (F110_FX_SPEC): parity tests, kernel A/B at the small shards, bench at 8192 envs
set -o pipefail
mkdir -p gpurun_out/r03at
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_batch.py -k spec_step tests/test_gpu_parity.py::test_fixed_point_cell_index_adversarial_vs_oracle > gpurun_out/r03at/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03at/tests.log; exit 1; }
tail -1 gpurun_out/r03at/tests.log
AB_ENVS=2048,8192 AB_VARIANTS='base:F110_FX_SPEC=1:0;s2t64:F110_FX_SPEC=2:64;s4t64:F110_FX_SPEC=4:64;s2t8:F110_FX_SPEC=2:8;s4t8:F110_FX_SPEC=4:8;s4t16:F110_FX_SPEC=4:16;s4t32:F110_FX_SPEC=4:32' timeout -k 10 300 python scripts/ray_ab.py > gpurun_out/r03at/ab.json 2> gpurun_out/r03at/ab.err || { tail -20 gpurun_out/r03at/ab.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r03at/ab.json').read().strip().splitlines()[-1])
for E, r in d['by_envs'].items():
    print(E, {k: round(v['k_rays_ms'], 4) for k, v in r.items() if isinstance(v, dict) and 'k_rays_ms' in v}, r.get('identical'))
PY
for S in 1:0 4:8 4:16 2:8; do
  F110_FX_SPEC=$S timeout -k 10 200 python bench.py --steps 500 --no-cpu-baseline --no-secondary --no-full-outputs --global-envs 8192 > gpurun_out/r03at/e8192_$S.json 2> gpurun_out/r03at/e8192_$S.err || { tail -20 gpurun_out/r03at/e8192_$S.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r03at/e8192_$S.json').read().strip().splitlines()[-1]); print('$S', d['value'], d['config']['streams_per_gpu'], d['roofline']['ray_kernel'])"
done
