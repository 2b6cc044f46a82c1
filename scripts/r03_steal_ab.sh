#!/bin/bash
# Round 3: tail stealing in the resident service (HFV_SVC_STEAL, one build, host switch):
# service + parity GPU tests with stealing on, then the headline leg interleaved on/off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_steal}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_parity.py tests/test_launcher.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_svc.log 2>&1
rc=$?; tail -2 $OUT/pytest_svc.log; [[ $rc -ne 0 ]] && exit $rc
ARGS="--steps 20 --warmup 5 --no-extras --no-host-e2e --cpu-budget 0 --loop-n 0"
for i in 1 2 3 4; do
    for st in 0 1; do
        HFV_SVC_STEAL=$st timeout -k 10 120 python bench.py $ARGS > $OUT/bench_steal${st}_$i.log 2>&1
        rc=$?; [[ $rc -ne 0 ]] && { echo "steal$st $i rc=$rc"; tail -5 $OUT/bench_steal${st}_$i.log; exit $rc; }
        python - "$OUT/bench_steal${st}_$i.log" "steal=$st" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["service"]
print(f"{sys.argv[2]:8s} value {d['value']:9.1f} ms/step {d['ms_per_step']*1e3:6.2f}us grid/batch {d['roofline']['kernel_ms_per_batch']*1e3:6.2f}us "
      f"frac {d['roofline']['frac']:.4f} grids {s['grids_ms']} mhz {s['shader_mhz']}")
PY
    done
done
