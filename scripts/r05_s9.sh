#!/bin/bash
# round 5, session 9: config 3 (256 IFID keys) with the round issue order pinned in the IFID
# AES body (-DHFV_IFID_PIN=1) against the same build without: parity, interleaved A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_s9
mkdir -p $OUT
export TMPDIR=/tmp
L=scion-xdp-br_amd/lib/ab
HFV_LIB=$(readlink -f $L/libscionhfv_ifpin.so) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_service.py \
    -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/parity_ifpin.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $OUT/parity_ifpin.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 900 python3 scripts/ab_libs.py 4 $L/libscionhfv_pinhead.so $L/libscionhfv_ifpin.so -- --keysel ifid --steps 20 --warmup 5 \
    > $OUT/ab_ifpin.log 2>&1
rc=$?; echo "ab rc=$rc"; cat $OUT/ab_ifpin.log; exit $rc
