#!/bin/bash
# Interleaved A/B of library builds on the config-5 loop:  scripts/ab_loop.sh ROUNDS lib1.so lib2.so ...
set -u
R=$1; shift
for r in $(seq 1 $R); do
  for lib in "$@"; do
    out=$(HFV_LIB=$(readlink -f $lib) timeout -k 10 200 python3 bench.py --workload loop 2>/dev/null | grep '^{') || { echo "$lib failed"; exit 1; }
    echo "$r $(basename $lib) $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); l=d["loop"]; print("mpkts", d["value"], "router_busy", l["stage_busy_frac"]["router"])')"
  done
done
