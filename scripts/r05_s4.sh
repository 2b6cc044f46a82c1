#!/bin/bash
# round 5, session 4: launcher GPU tests, fixed vs per-batch grid cost, byte-1 bitop3 at sustained clock
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_s4
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 6 "$OUT/$name.log" | cut -c1-400; return $rc; }
step launcher 400 python -u -m pytest tests/test_launcher.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
step marginal 300 python -u scripts/svc_marginal.py 4 || exit $?
L=scion-xdp-br_amd/lib/ab
for r in 1 2 3; do
  for lib in $L/libscionhfv_head.so $L/libscionhfv_b1.so; do
    HFV_LIB=$PWD/$lib timeout -k 10 120 python scripts/svc_sustained.py 3 >> $OUT/sustained_ab.log 2>&1 || { echo "sustained $lib failed"; tail -5 $OUT/sustained_ab.log; exit 1; }
    sleep 2
  done
done
cat $OUT/sustained_ab.log | grep -v amdgpu.ids
