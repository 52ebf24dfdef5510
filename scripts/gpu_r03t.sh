set -o pipefail
mkdir -p gpurun_out/r03t
for v in base new; do
  if [ $v = base ]; then export F110_LIB=$PWD/f110_gymnasium_ros2_jazzy_amd/libf110_base.so; VARS='s0:F110_SPEC_T=0'; else unset F110_LIB; VARS='s0:F110_SPEC_T=0;s8:F110_SPEC_T=8;s16:F110_SPEC_T=16;s32:F110_SPEC_T=32;s64:F110_SPEC_T=64'; fi
  AB_ENVS=8192,4096 AB_STEPS=100 AB_ROUNDS=3 AB_VARIANTS="$VARS" timeout -k 10 300 python scripts/ray_ab.py > gpurun_out/r03t/ab_$v.json 2> gpurun_out/r03t/ab_$v.err || { echo "ab failed"; tail -20 gpurun_out/r03t/ab_$v.err; exit 1; }
  echo $v; python - $v <<'PY'
import json,sys
d=json.load(open(f'gpurun_out/r03t/ab_{sys.argv[1]}.json'))
for E,l in d['by_envs'].items():
    print(E, all(v for k,v in l['identical'].items() if not k.endswith('_diff')), {k: round(v['k_rays_ms'],4) for k,v in l.items() if isinstance(v,dict) and 'k_rays_ms' in v}, {k: round(v,3) for k,v in l['mean_lookups'].items()})
PY
done
