#!/bin/bash
# round 6 session 9: hfv_verify_records on the batch-list kernel (one batch): the whole GPU suite,
# then the headline command's quick line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s9
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-300; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread -rf
rc=$?; [[ $rc -gt 1 ]] && exit $rc
step bench_quick 300 python -u bench.py --steps 20 --warmup 5 --no-extras --cpu-budget 0 --no-host-e2e || exit $?
exit 0
