#!/bin/bash
# round 5, session 18: the N > 1 path at HEAD -- launcher GPU tests and a full line from two
# ranks sharing GPU 0 (service legs, cpu_baseline on rank 0 after both ranks' GPU legs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_s18
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_launcher.py -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $OUT/launcher.log 2>&1
rc=$?; echo "launcher rc=$rc"; tail -2 $OUT/launcher.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 400 python -u bench.py --gpus 2 --same-device --steps 20 --warmup 5 --big-n 0 --br-n 0 --loop-n 0 \
    > $OUT/same_device_2.log 2>&1
rc=$?; echo "same-device rc=$rc"; tail -c 400 $OUT/same_device_2.log; exit $rc
