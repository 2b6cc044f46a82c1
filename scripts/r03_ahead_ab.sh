#!/bin/bash
# Round 3: service tile claims one iteration ahead (HFV_SVC_AHEAD=1) against at the top of the
# iteration that loads the tile (0): span probe (block / wave exit spread), then the headline leg
# interleaved; the service tests on the build under test first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_ahead}
mkdir -p $OUT
export TMPDIR=/tmp
L=scion-xdp-br_amd/lib/ab
HFV_LIB=$PWD/$L/libscionhfv_ahead0.so timeout -k 10 600 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_svc_ahead0.log 2>&1
rc=$?; tail -2 $OUT/pytest_svc_ahead0.log; [[ $rc -ne 0 ]] && exit $rc
for r in 0 1; do
    HFV_LIB=$PWD/$L/libscionhfv_span_ahead$r.so timeout -k 10 200 python scripts/svc_span.py 4 > $OUT/span_ahead$r.log 2>&1 || { tail -5 $OUT/span_ahead$r.log; exit 1; }
    echo "== span ahead=$r"; grep -v amdgpu.ids $OUT/span_ahead$r.log | grep "^K"
done
ARGS="--steps 20 --warmup 5 --no-extras --no-host-e2e --cpu-budget 0 --loop-n 0"
for i in 1 2 3 4; do
    for r in 0 1; do
        HFV_LIB=$PWD/$L/libscionhfv_ahead$r.so timeout -k 10 120 python bench.py $ARGS > $OUT/bench_ahead${r}_$i.log 2>&1
        rc=$?; [[ $rc -ne 0 ]] && { echo "ahead$r $i rc=$rc"; tail -5 $OUT/bench_ahead${r}_$i.log; exit $rc; }
        python - "$OUT/bench_ahead${r}_$i.log" "ahead=$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["service"]
print(f"{sys.argv[2]:8s} value {d['value']:9.1f} ms/step {d['ms_per_step']*1e3:6.2f}us grid/batch {d['roofline']['kernel_ms_per_batch']*1e3:6.2f}us "
      f"frac {d['roofline']['frac']:.4f} grids {s['grids_ms']} mhz {s['shader_mhz']}")
PY
    done
done
