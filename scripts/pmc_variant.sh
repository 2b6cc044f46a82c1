#!/bin/bash
# SQ counter passes for one verify-kernel variant (HFV_KVARIANT=$1) at the sizes in $2
# (default 2^24): issue/wait/VALU/LDS counters, one rocprofv3 run per group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=$1; SIZES=${2:-16777216}
tag=$(echo "$V" | tr ',=' '_-')
OUT=gpurun_out/pmcv_$tag
mkdir -p $OUT
groups=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES"
  "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
)
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  echo "=== pass $i: $g"
  HFV_KVARIANT="$V" timeout -k 10 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python3 scripts/pmc_driver.py zero 5 $SIZES > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $OUT $SIZES k_verify
