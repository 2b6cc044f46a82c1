#!/bin/bash
# round 6 session 19: the default batch-list headline with two ranks on one GPU (new launcher test)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s19
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_launcher.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread -rf > $OUT/pytest_launcher.log 2>&1
rc=$?
tail -5 $OUT/pytest_launcher.log
exit $rc
