#!/bin/bash
# round 6 session 13: what makes the 136-byte router window slower -- the tail store, the row pitch
# and AES copies, or the extra per-frame load -- interleaved config-4 A/B of the variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s13
mkdir -p $OUT
export TMPDIR=/tmp
L=scion-xdp-br_amd/lib
timeout -k 10 900 bash scripts/ab_br.sh 3 $L/libscionhfv.so $L/ab/libscionhfv_w128v.so $L/ab/libscionhfv_w136.so \
    $L/ab/libscionhfv_w136nost.so $L/ab/libscionhfv_w128r35c4.so $L/ab/libscionhfv_w128xl.so > $OUT/ab.log 2>&1
rc=$?
cat $OUT/ab.log
exit $rc
