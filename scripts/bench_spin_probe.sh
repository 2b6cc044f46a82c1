#!/bin/bash
# Headline timed regions with HIP's default device-synchronize wait or a spin wait
# (hipDeviceScheduleSpin via HFV_BENCH_SPIN=1).  scripts/bench_spin_probe.sh ROUNDS
set -u
R=${1:-4}
for r in $(seq 1 $R); do
  for sp in 0 1; do
    out=$(HFV_BENCH_SPIN=$sp timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extras --cpu-budget 0 --no-host-e2e 2>/tmp/spin_err.log | grep '^{') || { echo "run failed"; tail -3 /tmp/spin_err.log; exit 1; }
    echo "$r spin=$sp $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); s=d["service"]; print("value", d["value"], "regions", s["timed_regions_ms"], "grids", s["grids_ms"])') $(grep -c hipSetDeviceFlags /tmp/spin_err.log)"
  done
done
