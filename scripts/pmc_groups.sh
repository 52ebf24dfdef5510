#!/bin/bash
# counter groups for k_rays analysis; one rocprofv3 --pmc pass per group
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_groups${MB_AGENTS:+_a$MB_AGENTS}${PMC_TAG:+_$PMC_TAG}
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/g$i -o run -- python $R/scripts/ray_pmc.py > $OUT/g$i.log 2>&1
  echo "group $i ($grp): exit $?" >> $OUT/summary.txt
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
TA_BUSY_avr TD_BUSY_avr TCP_PENDING_STALL_CYCLES_sum
SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT
GROUPS
