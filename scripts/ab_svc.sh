#!/bin/bash
# Interleaved A/B of library builds on the headline (service, 8 rotated 2^20 batches, K = 20):
#   scripts/ab_svc.sh ROUNDS lib1.so lib2.so ...
set -u
R=$1; shift
for r in $(seq 1 $R); do
  for lib in "$@"; do
    out=$(HFV_LIB=$(readlink -f $lib) timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extras --cpu-budget 0 --no-host-e2e 2>/dev/null | grep '^{') || { echo "$lib failed"; exit 1; }
    echo "$r $(basename $lib) $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); s=d["service"]; print("value", d["value"], "grid_ms", s["grid_ms"], "grids", s["grids_ms"], "mhz", s["shader_mhz"])')"
  done
done
