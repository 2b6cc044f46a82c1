#!/bin/bash
# Round 3: service round tables written into LDS by the block's threads (HFV_SVC_FILL=2) against
# LDS-DMA from the global image (1): service + parity tests on 2, span probe, headline leg interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_fill}
mkdir -p $OUT
export TMPDIR=/tmp
L=scion-xdp-br_amd/lib/ab
HFV_LIB=$PWD/$L/libscionhfv_fill2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_svc_fill2.log 2>&1
rc=$?; tail -2 $OUT/pytest_svc_fill2.log; [[ $rc -ne 0 ]] && exit $rc
for r in 1 2; do
    HFV_LIB=$PWD/$L/libscionhfv_span_fill$r.so timeout -k 10 200 python scripts/svc_span.py 4 > $OUT/span_fill$r.log 2>&1 || { tail -5 $OUT/span_fill$r.log; exit 1; }
    echo "== span fill=$r"; grep -v amdgpu.ids $OUT/span_fill$r.log | grep "^K"
done
ARGS="--steps 20 --warmup 5 --no-extras --no-host-e2e --cpu-budget 0 --loop-n 0"
for i in 1 2 3 4; do
    for r in 1 2; do
        HFV_LIB=$PWD/$L/libscionhfv_fill$r.so timeout -k 10 120 python bench.py $ARGS > $OUT/bench_fill${r}_$i.log 2>&1
        rc=$?; [[ $rc -ne 0 ]] && { echo "fill$r $i rc=$rc"; tail -5 $OUT/bench_fill${r}_$i.log; exit $rc; }
        python - "$OUT/bench_fill${r}_$i.log" "fill=$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["service"]
print(f"{sys.argv[2]:8s} value {d['value']:9.1f} ms/step {d['ms_per_step']*1e3:6.2f}us grid/batch {d['roofline']['kernel_ms_per_batch']*1e3:6.2f}us "
      f"frac {d['roofline']['frac']:.4f} grids {s['grids_ms']} mhz {s['shader_mhz']}")
PY
    done
done
