#!/bin/bash
# Headline timed regions with hfv_service_run (waits for the grid, then the region's device
# synchronize) or hfv_service_run_async (only the device synchronize): HFV_BENCH_ASYNC=0/1.
set -u
R=${1:-4}
for r in $(seq 1 $R); do
  for a in 0 1; do
    out=$(HFV_BENCH_ASYNC=$a timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extras --cpu-budget 0 --no-host-e2e 2>/dev/null | grep '^{') || { echo "run failed"; exit 1; }
    echo "$r async=$a $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); s=d["service"]; print("value", d["value"], "regions", s["timed_regions_ms"], "grids", s["grids_ms"])')"
  done
done
