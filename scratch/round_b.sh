#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r1b
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1b/prof -o run -- python3 bench.py > gpurun_out/r1b/rocprof_bench.log 2>&1 || { tail gpurun_out/r1b/rocprof_bench.log; exit 1; }
python3 scripts/prof_summary.py gpurun_out/r1b/prof/run_kernel_trace.csv gpurun_out/r1b/prof/verify_by_batch.json
tail -1 gpurun_out/r1b/rocprof_bench.log | cut -c1-300
./scripts/pmc_round.sh zero svc > gpurun_out/r1b/pmc_svc.log 2>&1 || { tail -20 gpurun_out/r1b/pmc_svc.log; exit 1; }
tail -40 gpurun_out/r1b/pmc_svc.log
