#!/bin/bash
# round 6 session 23: router PMC on a one-template batch (no divergence) beside the bench mix's
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s23
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 bash scripts/pmc_round.sh br1t > $OUT/pmc_br1t.log 2>&1 || { tail $OUT/pmc_br1t.log; exit 1; }
mv gpurun_out/pmc_br1t_rot1 $OUT/pmc_br1t
tail -5 $OUT/pmc_br1t.log
exit 0
