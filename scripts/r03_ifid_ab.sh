#!/bin/bash
# Round 3: config 3 (256 IFID keys) -- key rows gathered into VGPRs beside the 4 LDS round tables
# (default) against the round-2 LDS key image (HFV_SVC_IFID_LDS=1).  Parity first, then the
# bench's config-3 leg, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_ifid}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_parity.py -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [[ $rc -ne 0 ]] && exit $rc
for i in 1 2; do
    for v in gather lds; do
        if [[ $v == lds ]]; then export HFV_SVC_IFID_LDS=1; else unset HFV_SVC_IFID_LDS; fi
        timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_${v}_$i.log 2>&1
        rc=$?; echo "bench $v $i rc=$rc"; [[ $rc -ne 0 ]] && exit $rc
        python - "$OUT/bench_${v}_$i.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config3"]
print(sys.argv[1], "headline", d["value"], "frac", d["roofline"]["frac"], "| config3", c["mpkts"], "frac", c["frac"], "grid_ms", c["grid_ms"], "mhz", c.get("shader_mhz"))
PY
    done
done
exit 0
