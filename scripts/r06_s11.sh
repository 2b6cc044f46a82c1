#!/bin/bash
# round 6 session 11: router staging window 136 B (HEAD) -- router + loop GPU tests, then an
# interleaved A/B of the config-4 kernel against the 128-byte window build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s11
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300; return $rc; }
step pytest_br 600 python -u -m pytest tests/test_gpu_br.py tests/test_gpu_loop.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf || exit $?
step ab_win 600 bash scripts/ab_br.sh 4 scion-xdp-br_amd/lib/libscionhfv.so scion-xdp-br_amd/lib/ab/libscionhfv_w128.so || exit $?
cat $OUT/ab_win.log
exit 0
