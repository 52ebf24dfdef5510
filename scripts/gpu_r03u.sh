set -o pipefail
mkdir -p gpurun_out/r03u
for v in base pm8; do
  if [ $v = pm8 ]; then export F110_LIB=$PWD/f110_gymnasium_ros2_jazzy_amd/libf110_pm8.so; else unset F110_LIB; fi
  for i in 1 2; do
  timeout -k 10 120 python scripts/c4_trace.py > gpurun_out/r03u/c4_$v$i.json 2> gpurun_out/r03u/c4_$v$i.err || { echo "c4 failed"; tail -20 gpurun_out/r03u/c4_$v$i.err; exit 1; }
  echo $v; cat gpurun_out/r03u/c4_$v$i.json
  done
done
