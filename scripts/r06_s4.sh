#!/bin/bash
# round 6 session 4: the whole GPU suite, smoke, the driver's command (headline = batch list),
# the rocprofv3 kernel trace of the headline command and the PMC passes of the batch-list kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06_s4}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300; return $rc; }
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
rc=$?; [[ $rc -gt 1 ]] && exit $rc
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench_1 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
step rocprof_head 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_head -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-host-e2e --cpu-budget 0 || exit $?
step pmc_zero_bat 900 bash scripts/pmc_round.sh zero bat rot8 || exit $?
exit 0
