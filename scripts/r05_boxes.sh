#!/bin/bash
# round 5: the driver's command three times on one box (run once per fresh box to see the spread)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-b1}
OUT=gpurun_out/r05_boxes_$TAG
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$i.log 2>&1 || { echo "bench $i failed"; tail -5 $OUT/bench_$i.log; exit 1; }
  grep '^{' $OUT/bench_$i.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); s=d['service']
print('$i value %.1f frac %.4f grid_ms %s mhz %s per_call %.3f config3 %.3f sustained %.3f@%s' % (d['value'], d['roofline']['frac'], s['grid_ms'], s['shader_mhz'], d['per_call']['frac'], d['config3']['frac'], d['sustained']['frac'], d['sustained']['shader_mhz']))"
done
