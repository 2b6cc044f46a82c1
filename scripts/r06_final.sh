#!/bin/bash
# round 6, closing session: GPU tests, smoke, the driver's command twice, rocprofv3 kernel trace
# of the headline command (+ per-launch summary), PMC passes of the headline batch-list kernel and
# of the router at HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${FINAL_TAG:-r06_final}
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
if [[ -z "${SKIP_PMC:-}" ]]; then
    step pmc_bat 900 bash scripts/pmc_round.sh zero bat rot8 || exit $?
    mv gpurun_out/pmc_zero_bat_rot8 $OUT/pmc_zero_bat
    step pmc_br 600 bash scripts/pmc_round.sh br || exit $?
    mv gpurun_out/pmc_br_rot1 $OUT/pmc_br
fi
exit 0
