#!/bin/bash
# round 5, session 20: round 9's 16 lookups through the vector L1 (a 4 KiB global table,
# -DHFV_VMEM_ROUND=9) instead of LDS, against HEAD: parity, interleaved headline A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_s20
mkdir -p $OUT
L=scion-xdp-br_amd/lib/ab
HFV_LIB=$(readlink -f $L/libscionhfv_vm9.so) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_service.py \
    -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/parity_vm9.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $OUT/parity_vm9.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 900 python3 scripts/ab_libs.py 4 $L/libscionhfv_head.so $L/libscionhfv_vm9.so > $OUT/ab_vm9.log 2>&1
rc=$?; echo "ab rc=$rc"; cat $OUT/ab_vm9.log; exit $rc
