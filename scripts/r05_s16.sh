#!/bin/bash
# round 5, session 16: the router's verdict-counter cost (counters on / off, HF check on / off),
# and the router GPU tests with HEAD's library
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_s16
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_br.py tests/test_gpu_loop.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $OUT/pytest_br.log 2>&1
rc=$?; echo "router tests rc=$rc"; tail -2 $OUT/pytest_br.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 300 python -u scripts/br_stats_probe.py 3 > $OUT/br_stats.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/br_stats.log; exit $rc
