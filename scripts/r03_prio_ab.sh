#!/bin/bash
# Round 3: router waves at raised issue priority from the end of the MAC checks until the next
# tile's loads are issued (HFV_BR_PRIO=1) against no priority change: br parity, then an A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_prio}
mkdir -p $OUT
export TMPDIR=/tmp
L=scion-xdp-br_amd/lib/ab
HFV_LIB=$PWD/$L/libscionhfv_prio1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_br.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_br_prio1.log 2>&1
rc=$?; tail -3 $OUT/pytest_br_prio1.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 900 bash scripts/ab_br.sh 4 $L/libscionhfv_prio0.so $L/libscionhfv_prio1.so > $OUT/ab.log 2>&1
rc=$?; cat $OUT/ab.log; exit $rc
