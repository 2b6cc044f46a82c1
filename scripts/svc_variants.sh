#!/bin/bash
# A/B of the resident service's cache-coherence variants (HFV_SVC_ACQ / HFV_SVC_REL builds
# under scratch/lib_a*): correctness of the rewritten-buffer test + bench service rates.
set -o pipefail
mkdir -p gpurun_out/svcvar
for d in scratch/lib_a*; do
    v=$(basename $d)
    HFV_LIB=$PWD/$d/libscionhfv.so timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread \
        tests/test_gpu_service.py -k "rewritten or ragged or golden" > gpurun_out/svcvar/${v}_pytest.log 2>&1
    echo "$v pytest rc=$?"
    HFV_LIB=$PWD/$d/libscionhfv.so timeout -k 10 200 python -u bench.py --cpu-budget 0 --no-host-e2e \
        > gpurun_out/svcvar/${v}_bench.log 2>&1 || { echo "$v bench failed"; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/svcvar/${v}_bench.log').read().strip().splitlines()[-1])
h=d['hbm_resident']
print('$v', 'svc', d['service']['mpkts'], 'grid_ms', d['service']['grid_ms'], 'launch', d['per_launch']['mpkts'], '2^24 svc', h['service_mpkts'], 'launch', h['mpkts'])
"
done
