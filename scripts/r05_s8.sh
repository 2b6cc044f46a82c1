#!/bin/bash
# round 5, session 8: GPU tests with the pinned launch-kernel schedule, interleaved A/B of the
# product library against the pre-change build (launch kernel and service), the driver's command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_s8
mkdir -p $OUT
bash scripts/gpu_session.sh r05_s8 test smoke || exit $?
L=scion-xdp-br_amd/lib
timeout -k 10 900 python3 scripts/ab_libs.py 4 $L/ab/libscionhfv_head.so $L/libscionhfv.so > $OUT/ab_pin.log 2>&1
rc=$?; echo "ab rc=$rc"; cat $OUT/ab_pin.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 $OUT/bench.log; exit $rc
