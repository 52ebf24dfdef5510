# k_rays_fxs at 65536 cars: vector-memory read instructions and TA wavefronts against TA busy cycles
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03ba
mkdir -p $OUT
MB_ENVS=65536 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_WAVES TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/ta -o run -- python3 $R/scripts/ray_pmc.py > $OUT/ta.log 2>&1 || { echo "pmc failed"; tail -8 $OUT/ta.log; exit 1; }
