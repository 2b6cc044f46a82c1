#!/bin/bash
# round 5, session 3: the driver's command (all legs), its rocprofv3 kernel trace, config-3 PMC
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_s3
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -c 3000 "$OUT/$name.log" | tail -n 3; return $rc; }
step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
step rocprof 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
step pmc_ifid 600 bash scripts/pmc_round.sh ifid svc rot8 || exit $?
