#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r1b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r1b/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r1b/pytest_gpu.log
[[ $rc -gt 1 ]] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r1b/bench.log 2>&1 || { tail gpurun_out/r1b/bench.log; exit 1; }
tail -1 gpurun_out/r1b/bench.log | cut -c1-600
exit $rc
