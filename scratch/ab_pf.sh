#!/bin/bash
set -o pipefail
D=gpurun_out/abpf
mkdir -p $D
HFV_KVARIANT=pf=2 HFV_KVARIANT_IFID=pf=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $D/pytest_pf2.log 2>&1 || { tail -20 $D/pytest_pf2.log; exit 1; }
tail -1 $D/pytest_pf2.log
show() { python3 -c "
import json
d=json.loads(open('$1').read().strip().splitlines()[-1]); h=d['hbm_resident']; p=d['per_launch']
print('$2', 'svc', d['service']['mpkts'], 'launch', p['mpkts'], 'kern_us', round(p['kernel_ms_mean']*1e3,2), '2^24 launch us', round(h['kernel_ms_mean']*1e3,1), h['mpkts'], 'svc2^24', h['service_mpkts'])"; }
for r in 1 2; do
  for v in 1 2; do
    HFV_KVARIANT=pf=$v HFV_KVARIANT_IFID=pf=$v timeout -k 10 200 python -u bench.py --cpu-budget 0 --no-host-e2e > $D/b_pf${v}_$r.log 2>&1 || { tail $D/b_pf${v}_$r.log; exit 1; }
    show $D/b_pf${v}_$r.log "pf=$v run $r"
  done
done
for v in 1 2; do
  HFV_KVARIANT_IFID=pf=$v timeout -k 10 200 python -u bench.py --cpu-budget 0 --no-host-e2e --keysel ifid > $D/bi_pf$v.log 2>&1 || exit 1
  show $D/bi_pf$v.log "ifid pf=$v"
done
