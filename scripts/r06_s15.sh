#!/bin/bash
# round 6 session 15: router -- frames whose SCION header runs past the 128-byte window get their
# next 8 bytes with one early load (HFV_BR_EXT): router + loop GPU tests, then interleaved A/B
# against the build without it (ext0) and round 6's HEAD build (w128)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s15
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300; return $rc; }
step pytest_br 600 python -u -m pytest tests/test_gpu_br.py tests/test_gpu_loop.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf || exit $?
L=scion-xdp-br_amd/lib
step ab_ext 600 bash scripts/ab_br.sh 4 $L/libscionhfv.so $L/ab/libscionhfv_ext0.so $L/ab/libscionhfv_w128.so || exit $?
cat $OUT/ab_ext.log
exit 0
