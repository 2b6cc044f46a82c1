#!/bin/bash
# Headline timed regions with the service grid's timing events attached to the launch
# (hipExtLaunchKernel, default) or recorded around a plain launch (HFV_SVC_EVREC=1).
# (The HFV_SVC_EVREC knob was removed after this A/B: no difference; profiles/r02/svc_ab/.)
set -u
R=${1:-4}
for r in $(seq 1 $R); do
  for e in 0 1; do
    out=$(HFV_SVC_EVREC=$e HFV_SVC_TRACE=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extras --cpu-budget 0 --no-host-e2e 2>/tmp/evrec_err.log | grep '^{') || { echo "run failed"; exit 1; }
    echo "$r evrec=$e $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); s=d["service"]; print("value", d["value"], "regions", s["timed_regions_ms"], "grids", s["grids_ms"], "calls", s["service_run_call_us"])') launch_us $(grep -o 'launch call [0-9.]*' /tmp/evrec_err.log | tail -3 | awk '{print $3}' | tr '\n' ' ')"
  done
done
