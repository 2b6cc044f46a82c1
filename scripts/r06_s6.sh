#!/bin/bash
# round 6 session 6: the batch-list kernel's last AES round through the vector L1
# (HFV_BATCH_GLAST=1) against HEAD's all-LDS round (interleaved A/B), after its parity tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s6
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 12 "$OUT/$name.log" | cut -c1-330; return $rc; }
HFV_LIB=scion-xdp-br_amd/lib/ab/libscionhfv_glast.so step pytest_glast 300 python -u -m pytest tests/test_gpu_batches.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
step ab_glast 600 python -u scripts/ab_libs.py 4 scion-xdp-br_amd/lib/ab/libscionhfv_base.so scion-xdp-br_amd/lib/ab/libscionhfv_glast.so -- --steps 20 --warmup 5 --mode batches || exit $?
exit 0
