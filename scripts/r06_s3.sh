#!/bin/bash
# round 6 session 3: where a batch-list launch's time goes (block fill/finish stamps)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s3
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 12 "$OUT/$name.log" | cut -c1-300; return $rc; }
step pytest_batches 300 python -u -m pytest tests/test_gpu_batches.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
step span20 200 python -u scripts/batches_span.py 20 6 || exit $?
step span64 200 python -u scripts/batches_span.py 64 4 || exit $?
exit 0
