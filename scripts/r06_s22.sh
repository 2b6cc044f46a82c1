#!/bin/bash
# round 6 session 22: batch-list soak, 60 s per key mode (random lists, ragged sizes, two strides,
# side stream, timed and plain calls, hfv_verify_records interleaved), against the generator truth
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s22
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 150 python3 -u scripts/batches_soak.py 60 7 zero > $OUT/soak_zero.log 2>&1 || { tail -5 $OUT/soak_zero.log; exit 1; }
timeout -k 10 150 python3 -u scripts/batches_soak.py 60 8 ifid > $OUT/soak_ifid.log 2>&1 || { tail -5 $OUT/soak_ifid.log; exit 1; }
tail -2 $OUT/soak_zero.log $OUT/soak_ifid.log
exit 0
