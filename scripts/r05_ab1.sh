#!/bin/bash
# round 5, session 2: tests, smoke, headline, then an interleaved A/B of service-loop variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_session.sh r05_s2 test smoke bench_quick || exit $?
L=scion-xdp-br_amd/lib/ab
timeout -k 10 600 python3 scripts/ab_libs.py 3 $L/libscionhfv_head.so $L/libscionhfv_np2.so $L/libscionhfv_nt.so \
    $L/libscionhfv_np2nt.so $L/libscionhfv_b1.so > gpurun_out/r05_s2/ab1.log 2>&1
echo "ab rc=$?"; cat gpurun_out/r05_s2/ab1.log
