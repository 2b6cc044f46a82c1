#!/bin/bash
# Round 3: the router's past-window branches marked unlikely (rare blocks out of line: the hot path
# falls through instead of jumping) against HEAD: br + loop parity (HEAD build), interleaved A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_expect}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_br.py tests/test_gpu_loop.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_br.log 2>&1
rc=$?; tail -3 $OUT/pytest_br.log; [[ $rc -ne 0 ]] && exit $rc
L=scion-xdp-br_amd/lib/ab
timeout -k 10 900 bash scripts/ab_br.sh 4 $L/libscionhfv_base.so $L/libscionhfv_expect.so > $OUT/ab.log 2>&1
rc=$?; cat $OUT/ab.log; exit $rc
