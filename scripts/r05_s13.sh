#!/bin/bash
# round 5, session 13: where the router kernel's waves spend their cycles (HFV_BR_PROF build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05_s13
HFV_LIB=$(readlink -f scion-xdp-br_amd/lib/ab/libscionhfv_brprof.so) timeout -k 10 240 python -u scripts/br_phase_probe.py \
    > gpurun_out/r05_s13/br_phase.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r05_s13/br_phase.log; exit $rc
