#!/bin/bash
# round 5, session 5: GPU tests, smoke, the driver's command twice, rocprofv3 of the headline-only
# command (+ per-grid summary of its kernel trace), a 2-rank same-GPU run of the full line, soaks
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_s5
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
python3 scripts/prof_summary.py $OUT/prof_head/run_kernel_trace.csv $OUT/prof_head_grids.json > /dev/null 2>&1
step same_device_2 400 python -u bench.py --gpus 2 --same-device --steps 20 --warmup 5 --big-n 0 --br-n 0 --loop-n 0 || exit $?
step soak_zero 120 python -u scripts/svc_soak.py 45 5 zero || exit $?
step soak_ifid 120 python -u scripts/svc_soak.py 45 6 ifid || exit $?
