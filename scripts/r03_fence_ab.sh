#!/bin/bash
# Round 3: name the round-2 config-5 loop failure's cause.  The same tests against the build
# without the cross-stream publish fence (HFV_PUB_FENCE=0) and the product build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_fence}
mkdir -p $OUT
T="tests/test_gpu_parity.py::test_key_publish_visible_on_other_streams tests/test_gpu_loop.py::test_loop_single_block_chunks tests/test_gpu_loop.py::test_loop_publish_races_second_stream"
HFV_LIB=scion-xdp-br_amd/lib/libscionhfv_nofence.so timeout -k 10 300 python -u -m pytest $T -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $OUT/nofence.log 2>&1
rc=$?
echo "nofence rc=$rc"
[[ $rc -gt 1 ]] && exit $rc
timeout -k 10 300 python -u -m pytest $T -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/fence.log 2>&1
rc=$?
echo "fence rc=$rc"
exit $rc
