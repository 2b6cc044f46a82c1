#!/bin/bash
# round 5, session 15: what the router's write-back costs (diagnostic build HFV_BR_WB=9: no
# write-back at all, wrong output, timing only) against HEAD, with the HF check on and off
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_s15
mkdir -p $OUT
L=scion-xdp-br_amd/lib/ab
for r in 1 2 3; do
  for lib in $L/libscionhfv_br_head.so $L/libscionhfv_br_wb9.so; do
    for hf in "" "--no-hf-check"; do
      out=$(HFV_LIB=$(readlink -f $lib) timeout -k 10 200 python3 bench.py --workload br --steps 10 --warmup 3 --cpu-budget 0 $hf 2>/dev/null | grep '^{') || { echo "$lib $hf failed"; exit 1; }
      echo "$r $(basename $lib) ${hf:-hf-on} $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); r=d["roofline"]; print("kernel_ms", r["kernel_ms_mean"], "median", r["kernel_ms_median"])')" | tee -a $OUT/ab_wb9.log
    done
  done
done
