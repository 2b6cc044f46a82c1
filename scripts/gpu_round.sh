#!/bin/bash
# One GPU-box session: parity tests, bench, rocprof kernel-trace summary.
# Each GPU step has its own time limit; a crash/abort/timeout (status >= 2 other than a
# plain pytest failure) stops the script so nothing else touches the GPU afterwards.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step <name> <timeout-s> <cmd...>
    local name=$1 t=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 25 "$OUT/$name.log"
    return $rc
}
MODE=${1:-all}
if [[ $MODE == all || $MODE == test ]]; then
    step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
    rc=$?
    # 1 = some test failed (read the log); anything else non-zero = crash/timeout: stop here
    if [[ $rc -gt 1 ]]; then exit $rc; fi
fi
if [[ $MODE == sweep ]]; then
    step sweep 600 python scripts/sweep.py ${SWEEP_ARGS:-} || exit $?
fi
if [[ $MODE == all || $MODE == bench ]]; then
    step bench 600 python bench.py || exit $?
fi
if [[ $MODE == all || $MODE == bench || $MODE == br ]]; then
    step bench_br 600 python bench.py --workload br || exit $?
    step bench_brhost 600 python bench.py --workload br-host || exit $?
    step bench_brhost_dma 600 python bench.py --workload br-host --no-register || exit $?
fi
if [[ $MODE == all || $MODE == prof ]]; then
    # the same command as the bench step, under the kernel tracer
    step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
        python3 bench.py || exit $?
    python3 scripts/prof_summary.py $OUT/prof/run_kernel_trace.csv $OUT/prof/verify_by_batch.json
fi
if [[ $MODE == all || $MODE == prof || $MODE == br ]]; then
    step rocprof_br 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_br -o run -- \
        python3 bench.py --workload br --cpu-budget 0 || exit $?
fi
exit 0
