#!/bin/bash
# PMC passes over scripts/pmc_driver.py, one rocprofv3 run per counter group (never
# combined with tracing domains).  Output: gpurun_out/pmc/<group>/...counter_collection.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
KS=${1:-zero}
SVC=${2:-}          # "svc": batches through the resident service (10 per grid); "bat": 10 per hfv_verify_batches call
ROT=${3:-rot1}      # "rot8": 8 resident 2^20 batches rotated, as in bench.py's headline
OUT=gpurun_out/pmc_$KS${SVC:+_$SVC}_$ROT
mkdir -p $OUT
groups=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum"
  "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_REQ_sum"
)
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  echo "=== pass $i: $g"
  timeout -k 10 300 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python3 scripts/pmc_driver.py $KS 10 1048576,16777216 ${SVC:-launch} $ROT > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
if [[ $SVC == bat ]]; then
    python3 scripts/pmc_summary.py $OUT 1048576,16777216 k_verify_batches 10
elif [[ $SVC == svc ]]; then
    python3 scripts/pmc_summary.py $OUT 1048576,16777216 k_verify_service 10
elif [[ $KS == br* ]]; then
    python3 scripts/pmc_summary.py $OUT 1048576 k_br_process
else
    python3 scripts/pmc_summary.py $OUT
fi
