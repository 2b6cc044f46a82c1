#!/bin/bash
# Round 3: router with the ingress interface's table reads issued before the parse
# (HFV_BR_EARLY_IF=1) against after it (0): br parity on 1, then an interleaved A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_eif}
mkdir -p $OUT
export TMPDIR=/tmp
L=scion-xdp-br_amd/lib/ab
HFV_LIB=$PWD/$L/libscionhfv_eif1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_br.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_br_eif1.log 2>&1
rc=$?; tail -3 $OUT/pytest_br_eif1.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 900 bash scripts/ab_br.sh 4 $L/libscionhfv_eif0.so $L/libscionhfv_eif1.so > $OUT/ab.log 2>&1
rc=$?; cat $OUT/ab.log; exit $rc
