#!/bin/bash
# round 6 session 7: the whole GPU suite, smoke, the driver's command twice and the rocprofv3
# kernel trace of the headline command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06_s7}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300; return $rc; }
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
rc=$?; [[ $rc -gt 1 ]] && exit $rc
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench_1 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
step bench_2 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
step rocprof_head 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_head -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-host-e2e --cpu-budget 0 || exit $?

exit 0
