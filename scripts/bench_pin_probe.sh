#!/bin/bash
# Headline run-to-run spread with the launching thread pinned to the GPU's NUMA node
# (HFV_BENCH_PIN=1, default) or left where it starts (0).  scripts/bench_pin_probe.sh ROUNDS
# (The HFV_BENCH_PIN knob was removed after this A/B: no difference; profiles/r02/svc_ab/.)
set -u
R=${1:-5}
for r in $(seq 1 $R); do
  for pin in 0 1; do
    out=$(HFV_BENCH_PIN=$pin timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extras --cpu-budget 0 --no-host-e2e 2>/dev/null | grep '^{') || { echo "run failed"; exit 1; }
    echo "$r pin=$pin $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); s=d["service"]; print("value", d["value"], "regions", s["timed_regions_ms"], "grids", s["grids_ms"])')"
  done
done
