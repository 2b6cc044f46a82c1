#!/bin/bash
# round 6 session 24: batch-list kernel over HBM-resident (R = 8) against Infinity-Cache-resident
# (R = 1, 2) batches, interleaved: back to back, then with 50 ms of idle before every call
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s24
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u scripts/batches_rot_probe.py 8 > $OUT/rot.log 2>&1 && timeout -k 10 200 python3 -u scripts/batches_rot_probe.py 8 0.05 >> $OUT/rot.log 2>&1
rc=$?
grep -v amdgpu.ids $OUT/rot.log
exit $rc
