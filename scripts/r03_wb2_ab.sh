#!/bin/bash
# Round 3: router next-tile loads between the parse and the MAC check (HFV_BR_WB=2) against
# before the write-back stores (1, the default) and stores first (0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_wb2}
mkdir -p $OUT
export TMPDIR=/tmp
L=scion-xdp-br_amd/lib/ab
HFV_LIB=$PWD/$L/libscionhfv_wb2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_br.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_br_wb2.log 2>&1
rc=$?; tail -3 $OUT/pytest_br_wb2.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 900 bash scripts/ab_br.sh 4 $L/libscionhfv_wb0.so $L/libscionhfv_wb1.so $L/libscionhfv_wb2.so > $OUT/ab.log 2>&1
rc=$?; cat $OUT/ab.log; exit $rc
