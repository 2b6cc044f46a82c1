#!/bin/bash
# Config-5 loop, DMA in with each chunk's copy on one stream (HFV_LOOP_SPLIT=0) or in two halves
# on two streams (1, the default): scripts/loop_split_probe.sh ROUNDS
set -u
R=${1:-4}
for r in $(seq 1 $R); do
  for sp in 0 1; do
    out=$(HFV_LOOP_SPLIT=$sp timeout -k 10 200 python3 bench.py --workload loop 2>/dev/null | grep '^{') || { echo "run failed"; exit 1; }
    echo "$r split=$sp $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); l=d["loop"]; print("mpkts", d["value"], "router_busy", l["stage_busy_frac"]["router"])')"
  done
done
