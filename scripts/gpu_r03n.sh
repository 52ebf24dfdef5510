set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03n
for R in 0 1; do
F110_HEAVY_T=$([ $R = 1 ] && echo 0 || echo 16) F110_FX_REFILL=$R timeout -k 10 120 python scripts/c4_trace.py > gpurun_out/r03n/c4_r$R.json 2> gpurun_out/r03n/c4_r$R.err || { echo "c4 failed"; tail -20 gpurun_out/r03n/c4_r$R.err; exit 1; }
cat gpurun_out/r03n/c4_r$R.json
F110_HEAVY_T=$([ $R = 1 ] && echo 0 || echo 16) F110_FX_REFILL=$R C4_STEPS=50 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r03n/kt_r$R -o kt -- python scripts/c4_trace.py > gpurun_out/r03n/kt_r$R.log 2>&1 || { echo "kt failed"; tail -20 gpurun_out/r03n/kt_r$R.log; exit 1; }
done
F110_MULTI_BLOCK=64 timeout -k 10 120 python scripts/c4_trace.py > gpurun_out/r03n/c4_mb64.json 2> gpurun_out/r03n/c4_mb64.err || { echo "c4 mb64 failed"; tail -20 gpurun_out/r03n/c4_mb64.err; exit 1; }
cat gpurun_out/r03n/c4_mb64.json
F110_MULTI_BLOCK=64 F110_FX_REFILL=1 F110_HEAVY_T=0 timeout -k 10 120 python scripts/c4_trace.py > gpurun_out/r03n/c4_mb64_r1.json 2> gpurun_out/r03n/c4_mb64_r1.err || { echo "c4 mb64 r1 failed"; tail -20 gpurun_out/r03n/c4_mb64_r1.err; exit 1; }
cat gpurun_out/r03n/c4_mb64_r1.json
