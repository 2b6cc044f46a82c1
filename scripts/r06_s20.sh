#!/bin/bash
# round 6 session 20: the router's divergence cost at HEAD (the bench mix in arrival order against
# the same frames sorted by template / ifindex / (ifindex, PathMeta), one template)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s20
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/br_divergence.py > $OUT/divergence.log 2>&1
rc=$?
grep -v amdgpu.ids $OUT/divergence.log
exit $rc
