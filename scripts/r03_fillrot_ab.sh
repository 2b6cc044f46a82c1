#!/bin/bash
# Round 3: service table fill with the chunk order rotated per block (HFV_SVC_FILLROT=1) against
# every block reading the image in the same order: span probe (fill time, K = 1 / 20), then
# the headline leg interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_fillrot}
mkdir -p $OUT
export TMPDIR=/tmp
L=scion-xdp-br_amd/lib/ab
for r in 0 1; do
    HFV_LIB=$PWD/$L/libscionhfv_span_rot$r.so timeout -k 10 200 python scripts/svc_span.py 4 > $OUT/span_rot$r.log 2>&1 || { tail -5 $OUT/span_rot$r.log; exit 1; }
    echo "== span rot=$r"; grep -v amdgpu.ids $OUT/span_rot$r.log | grep "^K"
done
ARGS="--steps 20 --warmup 5 --no-extras --no-host-e2e --cpu-budget 0 --loop-n 0"
for i in 1 2 3 4; do
    for r in 0 1; do
        HFV_LIB=$PWD/$L/libscionhfv_rot$r.so timeout -k 10 120 python bench.py $ARGS > $OUT/bench_rot${r}_$i.log 2>&1
        rc=$?; [[ $rc -ne 0 ]] && { echo "rot$r $i rc=$rc"; tail -5 $OUT/bench_rot${r}_$i.log; exit $rc; }
        python - "$OUT/bench_rot${r}_$i.log" "rot=$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["service"]
print(f"{sys.argv[2]:8s} value {d['value']:9.1f} ms/step {d['ms_per_step']*1e3:6.2f}us grid/batch {d['roofline']['kernel_ms_per_batch']*1e3:6.2f}us "
      f"frac {d['roofline']['frac']:.4f} grids {s['grids_ms']} mhz {s['shader_mhz']}")
PY
    done
done
