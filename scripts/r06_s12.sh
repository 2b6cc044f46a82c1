#!/bin/bash
# round 6 session 12: config-4 kernel time against the frame slot stride (HBM channel placement of
# the headers), window 136 (HEAD) and 128 builds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s12
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; cat "$OUT/$name.log" | grep -v amdgpu.ids | cut -c1-300; return $rc; }
HFV_LIB=$PWD/scion-xdp-br_amd/lib/ab/libscionhfv_w128.so step slot_w128 300 python -u scripts/br_slot_probe.py || exit $?
step slot_w136 300 python -u scripts/br_slot_probe.py || exit $?
exit 0
