#!/bin/bash
# Round 3: look for the occasional slow service grid (0.45-1.1 ms instead of 0.24-0.29 ms in the
# event-timed regions): the driver's bench command with 9 regions per leg, four times; per grid
# its shader clock and the block weights it left (bench.py service.grids_mhz / weights).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_slowgrid}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3 4; do
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-host-e2e --cpu-budget 0 --loop-n 0 --svc-reps 9 > $OUT/bench_$i.log 2>&1
    rc=$?; [[ $rc -ne 0 ]] && { tail -5 $OUT/bench_$i.log; exit $rc; }
    python - "$OUT/bench_$i.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
s, c = d["service"], d["config3"]
print("headline grids", s["grids_ms"], "mhz", s["grids_mhz"])
print("  weights", s["weights"][-1])
print("config3  grids", c["grids_ms"], "mhz", c["grids_mhz"])
PY
done
