#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r1c}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $D/pytest_gpu.log 2>&1; rc=$?
tail -3 $D/pytest_gpu.log
[[ $rc -ne 0 ]] && exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --cpu-budget 0 --no-host-e2e > $D/bench$i.log 2>&1 || { tail $D/bench$i.log; exit 1; }
python3 -c "
import json
d=json.loads(open('$D/bench$i.log').read().strip().splitlines()[-1]); h=d['hbm_resident']
print('value', d['value'], d['service'], 'launch', d['per_launch']['mpkts'], d['per_launch']['kernel_ms_mean'], '2^24 svc', h['service_mpkts'], h['service_ms_per_batch'], 'launch', h['mpkts'], h['kernel_ms_mean'])"
done
timeout -k 10 300 python -u bench.py --cpu-budget 0 --no-host-e2e --keysel ifid > $D/bench_ifid.log 2>&1 || { tail $D/bench_ifid.log; exit 1; }
python3 -c "
import json
d=json.loads(open('$D/bench_ifid.log').read().strip().splitlines()[-1]); h=d['hbm_resident']
print('ifid value', d['value'], d['service'], 'launch', d['per_launch']['mpkts'], d['per_launch']['kernel_ms_mean'], '2^24 svc', h['service_mpkts'], h['service_ms_per_batch'], 'launch', h['mpkts'], h['kernel_ms_mean'])"
