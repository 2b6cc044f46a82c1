#!/bin/bash
# GPU-box A/B of router-kernel library variants: scripts/ab_br_session.sh TAG ROUNDS lib...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out/$TAG
timeout -k 10 900 bash scripts/ab_br.sh $R "$@" > gpurun_out/$TAG/ab.log 2>&1
rc=$?; cat gpurun_out/$TAG/ab.log; exit $rc
