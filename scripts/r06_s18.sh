#!/bin/bash
# round 6 session 18: PMC passes of the batch-list kernel with 256 IFID keys (config 3), for the
# line's config-3 ceilings on the batch-list path
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s18
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 bash scripts/pmc_round.sh ifid bat rot8 > $OUT/pmc_ifid_bat.log 2>&1 || { tail $OUT/pmc_ifid_bat.log; exit 1; }
mv gpurun_out/pmc_ifid_bat_rot8 $OUT/pmc_ifid_bat
tail -20 $OUT/pmc_ifid_bat.log
exit 0
