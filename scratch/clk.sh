#!/bin/bash
set -o pipefail
D=gpurun_out/clk; mkdir -p $D
timeout -k 10 100 python -u scripts/svc_probe.py > $D/p1m.log 2>&1 || { tail $D/p1m.log; exit 1; }
timeout -k 10 100 python -u scripts/svc_probe.py 16777216 20 > $D/p16m.log 2>&1 || exit 1
HFV_SVC_GRID=32 timeout -k 10 100 python -u scripts/svc_probe.py 1048576 16 > $D/p1m_g32.log 2>&1 || exit 1
HFV_SVC_GRID=128 timeout -k 10 100 python -u scripts/svc_probe.py 1048576 32 > $D/p1m_g128.log 2>&1 || exit 1
for f in $D/*.log; do echo $f; grep '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    d=json.loads(l); print(d['n'], d['K'], 'grid_ms', d['grid_ms'], 'MHz', d['shader_mhz'], 'gap_us', d['done_gap_us_median'])"; done
