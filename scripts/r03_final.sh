#!/bin/bash
# Round-3 closing GPU session at HEAD: GPU tests, smoke, the driver's bench command three times,
# the config-4 bench, rocprofv3 kernel-trace stats of both, and the 2-rank same-GPU rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_final}
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step <name> <timeout-s> <cmd...>: stops the script on any failure
    local name=$1 t=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
    [[ $rc -ne 0 ]] && exit $rc
    return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do step bench_$i 240 python bench.py --steps 20 --warmup 5; done
step bench_br 240 python bench.py --workload br
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-host-e2e --loop-n 0 --cpu-budget 0
python3 scripts/prof_summary.py $OUT/prof/run_kernel_trace.csv $OUT/prof/verify_by_batch.json > $OUT/prof_summary.log 2>&1
step rocprof_br 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_br -o run -- python3 bench.py --workload br --cpu-budget 0
step same_device_n2 300 python bench.py --gpus 2 --same-device --steps 20 --warmup 5 --no-extras --no-host-e2e --cpu-budget 0 --loop-n 0
exit 0
