#!/bin/bash
# A/B of router-kernel builds on one box: bench.py --workload br with each library in
# scion-xdp-br_amd/lib/ab/ (HFV_LIB override), two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2; do
  for so in scion-xdp-br_amd/lib/ab/*.so; do
    tag=$(basename $so .so)
    echo "=== $round $tag"
    HFV_LIB=$PWD/$so timeout -k 10 180 python bench.py --workload br --cpu-budget 0 --steps 5 > gpurun_out/ab_${tag}_$round.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['roofline']['kernel_ms_mean'], d['value'])" gpurun_out/ab_${tag}_$round.log
  done
done
