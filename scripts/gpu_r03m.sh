set -o pipefail
mkdir -p gpurun_out/r03m
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -k "refill or adversarial or dispatch_variants" -x -q --timeout 200 --timeout-method thread > gpurun_out/r03m/test.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03m/test.log; exit 1; }
tail -2 gpurun_out/r03m/test.log
for v in base new; do
  if [ $v = base ]; then export F110_LIB=$PWD/f110_gymnasium_ros2_jazzy_amd/libf110_base.so; else unset F110_LIB; fi
  AB_ENVS=65536,32768 AB_STEPS=100 AB_ROUNDS=3 AB_VARIANTS='fxr:F110_FX_REFILL=1,F110_FX_PAD=1;fxn:F110_FX_REFILL=0' timeout -k 10 300 python scripts/ray_ab.py > gpurun_out/r03m/ab_$v.json 2> gpurun_out/r03m/ab_$v.err || { echo "ab failed $v"; tail -20 gpurun_out/r03m/ab_$v.err; exit 1; }
  echo $v; python - $v <<'PY'
import json,sys
d=json.load(open(f'gpurun_out/r03m/ab_{sys.argv[1]}.json'))
for E,l in d['by_envs'].items():
    print(E, l.get('identical'), {k: round(v['k_rays_ms'],4) for k,v in l.items() if isinstance(v,dict) and 'k_rays_ms' in v})
PY
done
