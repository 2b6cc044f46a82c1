#!/bin/bash
# round 5, session 11: the max-ilp machine scheduler (raises the IFID service body's LDS reads in
# flight at each wait from 4.0 to 5.8 in the ISA) against the default, config 3 then config 2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_s11
mkdir -p $OUT
L=scion-xdp-br_amd/lib/ab
HFV_LIB=$(readlink -f $L/libscionhfv_maxilp.so) timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/parity_maxilp.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $OUT/parity_maxilp.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 600 python3 scripts/ab_libs.py 4 $L/libscionhfv_head.so $L/libscionhfv_maxilp.so -- --keysel ifid --steps 20 --warmup 5 \
    > $OUT/ab_maxilp_ifid.log 2>&1
rc=$?; echo "ab ifid rc=$rc"; cat $OUT/ab_maxilp_ifid.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 400 python3 scripts/ab_libs.py 3 $L/libscionhfv_head.so $L/libscionhfv_maxilp.so > $OUT/ab_maxilp_zero.log 2>&1
rc=$?; echo "ab zero rc=$rc"; cat $OUT/ab_maxilp_zero.log; exit $rc
