set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03k
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r03k/kt -o kt -- python scripts/fused_pmc.py > gpurun_out/r03k/kt.log 2>&1 || { echo "kt failed"; tail -20 gpurun_out/r03k/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/r03k/p1 -o p1 -- python scripts/fused_pmc.py > gpurun_out/r03k/p1.log 2>&1 || { echo "p1 failed"; tail -20 gpurun_out/r03k/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FP64 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_INSTS_FLAT SQ_WAIT_ANY -d gpurun_out/r03k/p2 -o p2 -- python scripts/fused_pmc.py > gpurun_out/r03k/p2.log 2>&1 || { echo "p2 failed"; tail -20 gpurun_out/r03k/p2.log; exit 1; }
find gpurun_out/r03k -name "*.csv" | head -20
