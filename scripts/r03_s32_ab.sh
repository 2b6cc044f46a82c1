#!/bin/bash
# Round 3: router verdict counters in 32-bit LDS words with 8 AES table copies (the build under
# test), 32-bit counters with 4 copies, and 64-bit counters with 4 copies: br + loop parity, A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_s32}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_br.py tests/test_gpu_loop.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_br.log 2>&1
rc=$?; tail -3 $OUT/pytest_br.log; [[ $rc -ne 0 ]] && exit $rc
L=scion-xdp-br_amd/lib/ab
timeout -k 10 900 bash scripts/ab_br.sh 4 $L/libscionhfv_s64.so $L/libscionhfv_s32c4.so $L/libscionhfv_s32c8.so > $OUT/ab.log 2>&1
rc=$?; cat $OUT/ab.log; exit $rc
