#!/bin/bash
# Round 3: router AES tables as T0 only with 16 lane copies and T1 = rotl8(T0) (HFV_TAB3_T1ROT=1)
# against T0/T1 with 8 copies (the default): br parity on the variant, then an interleaved A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_t1rot}
mkdir -p $OUT
export TMPDIR=/tmp
L=scion-xdp-br_amd/lib/ab
HFV_LIB=$PWD/$L/libscionhfv_t1rot.so timeout -k 10 600 python -u -m pytest tests/test_gpu_br.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_br_t1rot.log 2>&1
rc=$?; tail -3 $OUT/pytest_br_t1rot.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 900 bash scripts/ab_br.sh 4 $L/libscionhfv_c8.so $L/libscionhfv_t1rot.so > $OUT/ab.log 2>&1
rc=$?; cat $OUT/ab.log; exit $rc
