#!/bin/bash
# Round 3: router write-back ordering (HFV_BR_WB): parity of the default build, then an
# interleaved A/B of the config-4 kernel against the stores-first build and a no-write-back probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_wb}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_br.py tests/test_gpu_loop.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_br.log 2>&1
rc=$?; tail -3 $OUT/pytest_br.log; [[ $rc -ne 0 ]] && exit $rc
L=scion-xdp-br_amd/lib/ab
timeout -k 10 900 bash scripts/ab_br.sh 4 $L/libscionhfv_wb0.so $L/libscionhfv_wb1.so $L/libscionhfv_wb9.so > $OUT/ab.log 2>&1
rc=$?; cat $OUT/ab.log; exit $rc
