#!/bin/bash
# round 5, session 19: config 3 with the lane range check formed after the rounds in the service
# (-DHFV_SVC_LATE_IN=1: the IFID body then drains its LDS reads far less often in the ISA)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_s19
mkdir -p $OUT
L=scion-xdp-br_amd/lib/ab
HFV_LIB=$(readlink -f $L/libscionhfv_latein.so) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_service.py \
    -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/parity_latein.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $OUT/parity_latein.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 900 python3 scripts/ab_libs.py 4 $L/libscionhfv_head.so $L/libscionhfv_latein.so -- --keysel ifid --steps 20 --warmup 5 \
    > $OUT/ab_latein_ifid.log 2>&1
rc=$?; echo "ab ifid rc=$rc"; cat $OUT/ab_latein_ifid.log; exit $rc
