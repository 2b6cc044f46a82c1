#!/bin/bash
# round 6 session 2: batch-list kernel with clock stamps; prefetch depth 1 vs 2 (interleaved A/B)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s2
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 8 "$OUT/$name.log" | cut -c1-400; return $rc; }
step pytest_batches 300 python -u -m pytest tests/test_gpu_batches.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
HFV_LIB=scion-xdp-br_amd/lib/ab/libscionhfv_d2.so step pytest_batches_d2 300 python -u -m pytest tests/test_gpu_batches.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
step ab_depth 600 python -u scripts/ab_libs.py 4 scion-xdp-br_amd/lib/ab/libscionhfv_d1.so scion-xdp-br_amd/lib/ab/libscionhfv_d2.so -- --steps 20 --warmup 5 --mode batches || exit $?
exit 0
