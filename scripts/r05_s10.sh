#!/bin/bash
# round 5, session 10: host-side phases of the headline service call (VERDICT r04 #1b)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05_s10
timeout -k 10 240 python -u scripts/svc_call_probe.py 12 > gpurun_out/r05_s10/call_probe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r05_s10/call_probe.log; exit $rc
