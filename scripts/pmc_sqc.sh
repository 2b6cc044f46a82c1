#!/bin/bash
# Scalar/instruction cache PMC of the service (one-batch run grids) and of the launch kernel on
# the same 2^24 records: does the service's loop miss in the SQC caches?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for mode in launch svcrun; do
  OUT=gpurun_out/pmc_sqc_$mode
  mkdir -p $OUT
  i=0
  for g in "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQC_DCACHE_MISSES SQC_DCACHE_HITS"; do
    i=$((i+1))
    reps=3; [[ $mode == svcrun ]] && reps=1
    timeout -s KILL 90 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
        python3 scripts/pmc_driver.py zero $reps 16777216 $mode > $OUT/p$i.log 2>&1 || { echo "$mode pass $i failed"; grep -v "^[EW]2026" $OUT/p$i.log | tail -3; exit 1; }
  done
done
