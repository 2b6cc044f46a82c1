#!/bin/bash
# round 6 session 10: per-XCD block weights for hfv_verify_batches -- the batch tests (incl. the
# forced-skew partition test), then an interleaved A/B of the headline line (learned weights vs
# equal shares), 3 runs each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s10
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400; return $rc; }
step pytest_batches 400 python -u -m pytest tests/test_gpu_batches.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf || exit $?
for i in 1 2 3; do
  HFV_BENCH_XCD_WEIGHTS=1 step bench_w1_$i 240 python -u bench.py --steps 20 --warmup 5 --no-extras --cpu-budget 0 --no-host-e2e || exit $?
  HFV_BENCH_XCD_WEIGHTS=0 step bench_w0_$i 240 python -u bench.py --steps 20 --warmup 5 --no-extras --cpu-budget 0 --no-host-e2e || exit $?
done
exit 0
