#!/bin/bash
# round 6 session 17: what the router's write-back costs now (diagnostic build HFV_BR_WB=9: no
# write-back, wrong output) against HEAD, config-4 kernel at the bench's 2 KiB stride, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_s17
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/scion-xdp-br_amd/lib/ab
for r in 1 2 3; do
  for v in head wb9; do
    echo "round $r $v: $(HFV_LIB=$L/libscionhfv_$v.so timeout -k 10 120 python3 scripts/br_slot_probe.py 2048 2>/dev/null | grep stride)" | tee -a $OUT/ab.log || exit 1
  done
done
exit 0
