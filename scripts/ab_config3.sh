#!/bin/bash
# Interleaved A/B of library builds on the config-3 leg (256 IFID keys) of the full bench:
#   scripts/ab_config3.sh ROUNDS lib1.so lib2.so ...   (one bench.py process per run)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$1; shift
for r in $(seq 1 $R); do
  for lib in "$@"; do
    out=$(HFV_LIB=$lib timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-budget 0 --no-host-e2e 2>/dev/null | grep '^{') || { echo "$r $(basename $lib) FAILED"; exit 1; }
    echo "$out" | python -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config3']
print('$r %-24s config3 frac %.4f grid_ms %.4f mpkts %.0f | headline grid %.4f' % ('$(basename $lib)', c['frac'], c['grid_ms'], c['mpkts'], d['service']['grid_ms']))"
  done
done
