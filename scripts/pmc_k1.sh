#!/bin/bash
# PMC passes of one 2^24-record batch verified by a single launch and by a one-batch service
# grid (same records, same duration, so comparable clocks): the service-vs-launch loop gap.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
groups=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES"
)
for mode in launch svcrun; do
  OUT=gpurun_out/pmc_k1_$mode
  mkdir -p $OUT
  i=0
  for g in "${groups[@]}"; do
    i=$((i+1))
    reps=3; [[ $mode == svcrun ]] && reps=1
    timeout -k 10 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
        python3 scripts/pmc_driver.py zero $reps 16777216 $mode > $OUT/p$i.log 2>&1 || { echo "$mode pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
  done
done
