set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03i
for E in 8192 4096; do
FP_ENVS=$E FP_STEPS=40 FP_MODES=three timeout -s KILL 120 rocprofv3 --kernel-trace -d gpurun_out/r03i/kt$E -o kt -- python scripts/fused_pmc.py > gpurun_out/r03i/kt$E.log 2>&1 || { echo "kt failed"; tail -20 gpurun_out/r03i/kt$E.log; exit 1; }
done
