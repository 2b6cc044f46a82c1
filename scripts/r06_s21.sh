#!/bin/bash
# round 6 session 21: router -- slot-0 round keys from a 192-byte LDS copy by broadcast
# (HFV_BR_LDSKEY=1: 90 instead of 124 spilled SGPRs) against SGPR-held keys, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s21
mkdir -p $OUT
export TMPDIR=/tmp
L=scion-xdp-br_amd/lib/ab
timeout -k 10 600 bash scripts/ab_br.sh 4 $L/libscionhfv_head0.so $L/libscionhfv_ldskey.so > $OUT/ab.log 2>&1
rc=$?
cat $OUT/ab.log
exit $rc
