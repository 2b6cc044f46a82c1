#!/bin/bash
# Round 3: config 3 (256 IFID keys) service variants (HFV_SVC_IFID=lds|sched|gather) against each
# other: parity of the variant first, then the bench's config-3 leg, interleaved.
# usage: r03_ifid_ab.sh <outdir> <variant> [<variant>...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_ifid}
mkdir -p $OUT
shift
VARS="${@:-lds}"
for v in $VARS; do
    HFV_SVC_IFID=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_parity.py -x -q \
        --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_$v.log 2>&1
    rc=$?; echo "pytest $v rc=$rc"; [[ $rc -ne 0 ]] && exit $rc
done
for i in 1 2; do
    for v in $VARS; do
        export HFV_SVC_IFID=$v
        timeout -k 10 300 python bench.py --keysel ifid --steps 20 --warmup 5 --no-extras --no-host-e2e --cpu-budget 0 \
            --loop-n 0 > $OUT/bench_${v}_$i.log 2>&1
        rc=$?; echo "bench $v $i rc=$rc"; [[ $rc -ne 0 ]] && exit $rc
        python - "$OUT/bench_${v}_$i.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r, s = d["roofline"], d["service"]
print(sys.argv[1], "config3", d["value"], "frac", r["frac"], "grid_ms", r["grid_ms"], "mhz", s["shader_mhz"])
PY
    done
done
exit 0
