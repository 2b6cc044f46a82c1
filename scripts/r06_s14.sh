#!/bin/bash
# round 6 session 14: the router's account -- PMC of the config-4 kernel at HEAD and
# of the variant that only adds one unused 8-byte load of each frame's second line (w128xl), and
# the per-phase cycle split of the diagnostic build (HFV_BR_PROF)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s14
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/scion-xdp-br_amd/lib
timeout -k 10 600 bash scripts/pmc_round.sh br > $OUT/pmc_head.log 2>&1 || { tail $OUT/pmc_head.log; exit 1; }
mv gpurun_out/pmc_br_rot1 $OUT/pmc_br_head
HFV_LIB=$L/ab/libscionhfv_w128xl.so timeout -k 10 600 bash scripts/pmc_round.sh br > $OUT/pmc_xl.log 2>&1 || { tail $OUT/pmc_xl.log; exit 1; }
mv gpurun_out/pmc_br_rot1 $OUT/pmc_br_xl
HFV_LIB=$L/ab/libscionhfv_brprof.so timeout -k 10 300 python3 -u scripts/br_phase_probe.py > $OUT/phase.log 2>&1 || { tail $OUT/phase.log; exit 1; }
tail -3 $OUT/pmc_head.log $OUT/pmc_xl.log; cat $OUT/phase.log
exit 0
