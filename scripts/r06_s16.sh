#!/bin/bash
# round 6 session 16: router -- reads past the window behind a wave-uniform ballot test (HFV_BR_UNI)
# instead of a divergent branch per accessor: router + loop GPU tests, then interleaved A/B
# against the build without it (uni0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s16
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300; return $rc; }
step pytest_br 600 python -u -m pytest tests/test_gpu_br.py tests/test_gpu_loop.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf || exit $?
L=scion-xdp-br_amd/lib
step ab_uni 600 bash scripts/ab_br.sh 4 $L/libscionhfv.so $L/ab/libscionhfv_uni0.so || exit $?
cat $OUT/ab_uni.log
exit 0
