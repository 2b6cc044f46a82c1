#!/bin/bash
# round 5, session 14: the round-4 closing tree (commit c3ddbb7, built in r04tree/) against HEAD on
# one box, headline only, interleaved -- does round 5's service grid run slower than round 4's?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_s14
mkdir -p $OUT
ROOT=$PWD
for r in 1 2 3 4; do
  for t in head r04; do
    d=$ROOT; [[ $t == r04 ]] && d=$ROOT/r04tree
    out=$(cd $d && timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --cpu-budget 0 --no-host-e2e 2>/dev/null | grep '^{') \
        || { echo "$r $t FAILED"; exit 1; }
    echo "$out" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); s=d['service']
print('$r $t value %.1f grid_ms %s grids %s mhz %s launch_us %.2f' % (d['value'], s['grid_ms'], s['grids_ms'], s.get('shader_mhz'), d['per_launch']['kernel_ms_mean']*1e3))" | tee -a $OUT/ab_r04.log
  done
done
