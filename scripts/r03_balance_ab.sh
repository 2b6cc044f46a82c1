#!/bin/bash
# Round 3: weighted block shares (SvcWeights, re-derived after every hfv_service_run grid) against
# equal shares (HFV_SVC_BALANCE=0): the span probe on both, then the headline leg interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_balance}
mkdir -p $OUT
export TMPDIR=/tmp
SPAN=scion-xdp-br_amd/lib/ab/libscionhfv_span.so
for b in 0 1; do
    HFV_SVC_BALANCE=$b HFV_LIB=$PWD/$SPAN timeout -k 10 200 python scripts/svc_span.py 8 20 > $OUT/span_bal$b.log 2>&1 || { tail -5 $OUT/span_bal$b.log; exit 1; }
    echo "== span balance=$b"; grep -v amdgpu.ids $OUT/span_bal$b.log | tail -6
done
ARGS="--steps 20 --warmup 5 --no-extras --no-host-e2e --cpu-budget 0 --loop-n 0"
for i in 1 2 3 4; do
    for b in 0 1; do
        HFV_SVC_BALANCE=$b timeout -k 10 120 python bench.py $ARGS > $OUT/bench_bal${b}_$i.log 2>&1
        rc=$?; [[ $rc -ne 0 ]] && { echo "bal$b $i rc=$rc"; tail -5 $OUT/bench_bal${b}_$i.log; exit $rc; }
        python - "$OUT/bench_bal${b}_$i.log" "balance=$b" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["service"]
print(f"{sys.argv[2]:10s} value {d['value']:9.1f} ms/step {d['ms_per_step']*1e3:6.2f}us grid/batch {d['roofline']['kernel_ms_per_batch']*1e3:6.2f}us "
      f"frac {d['roofline']['frac']:.4f} regions {s['timed_regions_ms']} grids {s['grids_ms']} mhz {s['shader_mhz']}")
PY
    done
done
