#!/bin/bash
# round 6 session 1: the stream-ordered batch-list launch -- its GPU tests, then the headline
# command's legs side by side (service grid vs one hfv_verify_batches call over the K batches)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s1
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-400; return $rc; }
step pytest_batches 300 python -u -m pytest tests/test_gpu_batches.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
for i in 1 2; do
  step bench_svc_$i 300 python -u bench.py --steps 20 --warmup 5 --no-extras --cpu-budget 0 --no-host-e2e || exit $?
  step bench_bat_$i 300 python -u bench.py --steps 20 --warmup 5 --no-extras --cpu-budget 0 --no-host-e2e --mode batches || exit $?
done
exit 0
