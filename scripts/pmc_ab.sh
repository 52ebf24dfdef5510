#!/bin/bash
# PMC counter groups of the headline ray kernels, per variant (env assignments):
#   PMC_VARIANTS="F110_RAY_KERNEL=2 F110_EVICT=0" MB_ENVS=65536 bash scripts/pmc_ab.sh <tag>
# PMC_GROUPS="G1 counters;G2 counters" replaces the default groups
# one rocprofv3 --pmc pass per (variant, group), each under its own time limit
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-ab}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
for V in ${PMC_VARIANTS:-F110_RAY_KERNEL=2 F110_RAY_KERNEL=3}; do
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    ( export $V; timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/v${V}_g$i -o run -- python3 $R/scripts/ray_pmc.py > $OUT/v${V}_g$i.log 2>&1 ) || { echo "variant $V group $i failed"; exit 1; }
  done < <(if [ -n "$PMC_GROUPS" ]; then echo "$PMC_GROUPS" | tr ';' '\n'; else cat <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD
TA_BUSY_avr TD_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum
TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TA_FLAT_READ_WAVEFRONTS_sum TA_BUFFER_READ_WAVEFRONTS_sum
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
GROUPS
fi)
done
echo done
