#!/bin/bash
# Interleaved A/B of library builds on the config-4 kernel:  scripts/ab_br.sh ROUNDS lib1.so lib2.so ...
set -u
R=$1; shift
for r in $(seq 1 $R); do
  for lib in "$@"; do
    out=$(HFV_LIB=$(readlink -f $lib) timeout -k 10 200 python3 bench.py --workload br --steps 10 --warmup 3 --cpu-budget 0 2>/dev/null | grep '^{') || { echo "$lib failed"; exit 1; }
    echo "$r $(basename $lib) $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); r=d["roofline"]; print("kernel_ms", r["kernel_ms_mean"], "median", r["kernel_ms_median"], "value", d["value"])')"
  done
done
