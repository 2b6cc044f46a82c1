#!/bin/bash
# round 6 session 5: the whole GPU suite after the test-hook split (hook tests rerun on the test
# build), then the batch-list kernel's round issue order pinned or not (interleaved A/B)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s5
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 12 "$OUT/$name.log" | cut -c1-330; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread -rf
rc=$?; [[ $rc -gt 1 ]] && exit $rc
step ab_pin 600 python -u scripts/ab_libs.py 4 scion-xdp-br_amd/lib/ab/libscionhfv_pin1.so scion-xdp-br_amd/lib/ab/libscionhfv_pin0.so -- --steps 20 --warmup 5 --mode batches || exit $?
exit 0
