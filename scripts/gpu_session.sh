#!/bin/bash
# One GPU-box session: a list of named steps, each under its own time limit; a crash, abort or
# timeout (any status but 0, and 1 for pytest) ends the session so nothing else touches the
# GPU afterwards.  Logs: gpurun_out/<tag>/<step>.log.
#   scripts/gpu_session.sh <tag> step [step ...]
# steps: test | smoke | bench | bench_quick | prof | pmc_zero | pmc_ifid | pmc_br | br | brhost | loop | looptest |
#        ubench_<name>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {   # run <name> <timeout-s> <cmd...>
    local name=$1 t=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 4 "$OUT/$name.log"
    return $rc
}
for s in "$@"; do
    case $s in
    test)
        run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
        rc=$?; [[ $rc -gt 1 ]] && exit $rc ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5 || exit $? ;;
    bench_quick) run bench_quick 300 python bench.py --steps 20 --warmup 5 --no-extras --cpu-budget 0 --no-host-e2e || exit $? ;;
    prof)
        run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
            python3 bench.py --steps 20 --warmup 5 || exit $?
        python3 scripts/prof_summary.py "$OUT"/prof/run_kernel_trace.csv "$OUT"/prof/verify_by_batch.json > /dev/null ;;
    pmc_zero) run pmc_zero 1100 bash scripts/pmc_round.sh zero svc rot8 || exit $? ;;
    pmc_ifid) run pmc_ifid 1100 bash scripts/pmc_round.sh ifid svc rot8 || exit $? ;;
    pmc_br) run pmc_br 1100 bash scripts/pmc_round.sh br || exit $? ;;
    br) run bench_br 600 python bench.py --workload br || exit $? ;;
    brhost) run bench_brhost 600 python bench.py --workload br-host || exit $? ;;
    loop) run bench_loop 300 python bench.py --workload loop || exit $? ;;
    looptest) run pytest_loop 300 python -u -m pytest tests/test_gpu_loop.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread || exit $? ;;
    ubench_*) run "$s" 300 "./build_ub/${s#ubench_}" || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
exit 0
