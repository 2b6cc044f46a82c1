#!/bin/bash
# round 5, session 7: interleaved A/B against HEAD of (a) the per-round issue order pinned by
# sched_group_barrier (groups of 4 and 16 lookups) and (b) the headline key rows 10/11 held in
# VGPRs (the service's AES body then compiles to the launch loop's wait sequence,
# profiles/r05/isa_census.txt): service parity with (b), headline A/B, sustained A/B of (b)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_s7
mkdir -p $OUT
export TMPDIR=/tmp
L=scion-xdp-br_amd/lib/ab
HFV_LIB=$(readlink -f $L/libscionhfv_vk.so) timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/parity_vk.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $OUT/parity_vk.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 900 python3 scripts/ab_libs.py 3 $L/libscionhfv_head.so $L/libscionhfv_sg4.so $L/libscionhfv_sg16.so \
    $L/libscionhfv_vk.so > $OUT/ab_sched_vk.log 2>&1
rc=$?; echo "ab rc=$rc"; cat $OUT/ab_sched_vk.log; [[ $rc -ne 0 ]] && exit $rc
for r in 1 2; do
  for lib in $L/libscionhfv_head.so $L/libscionhfv_vk.so; do
    echo "## $(basename $lib)" >> $OUT/sustained_vk.log
    HFV_LIB=$PWD/$lib timeout -k 10 120 python scripts/svc_sustained.py 3 >> $OUT/sustained_vk.log 2>&1 || { echo "sustained $lib failed"; tail -5 $OUT/sustained_vk.log; exit 1; }
    sleep 2
  done
done
grep -v amdgpu.ids $OUT/sustained_vk.log
timeout -k 10 300 python -u scripts/svc_feed_depth.py 2 > $OUT/feed_depth.log 2>&1
rc=$?; echo "feed depth rc=$rc"; grep -v amdgpu.ids $OUT/feed_depth.log; exit $rc
