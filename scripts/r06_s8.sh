#!/bin/bash
# round 6 session 8: the batch-list loop unrolled over fixed record slots (no loop-carried copy of
# in-flight loads), prefetch depth 1 (HEAD) and 2, against the round's earlier loop (interleaved A/B)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s8
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 14 "$OUT/$name.log" | cut -c1-330; return $rc; }
step pytest_u1 300 python -u -m pytest tests/test_gpu_batches.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
HFV_LIB=scion-xdp-br_amd/lib/ab/libscionhfv_u2.so step pytest_u2 300 python -u -m pytest tests/test_gpu_batches.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
step ab_unroll 900 python -u scripts/ab_libs.py 4 scion-xdp-br_amd/lib/ab/libscionhfv_base.so scion-xdp-br_amd/lib/ab/libscionhfv_u1.so scion-xdp-br_amd/lib/ab/libscionhfv_u2.so -- --steps 20 --warmup 5 --mode batches || exit $?
exit 0
