#!/bin/bash
# Config-5 loop, run-to-run spread with the copy engines (SDMA) and with blit-kernel copies
# (HSA_ENABLE_SDMA=0): scripts/loop_sdma_probe.sh ROUNDS
set -u
R=${1:-4}
for r in $(seq 1 $R); do
  for sd in 1 0; do
    out=$(HSA_ENABLE_SDMA=$sd timeout -k 10 200 python3 bench.py --workload loop 2>/dev/null | grep '^{') || { echo "run failed"; exit 1; }
    echo "$r sdma=$sd $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); l=d["loop"]; print("mpkts", d["value"], "router_busy", l["stage_busy_frac"]["router"])')"
  done
done
