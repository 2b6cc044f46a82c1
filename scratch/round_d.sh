#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r1d
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py > $D/rocprof_bench.log 2>&1 || { tail $D/rocprof_bench.log; exit 1; }
python3 scripts/prof_summary.py $D/prof/run_kernel_trace.csv $D/prof/verify_by_batch.json > /dev/null
tail -1 $D/rocprof_bench.log | cut -c1-200
./scripts/pmc_round.sh br > $D/pmc_br.log 2>&1 || { tail -20 $D/pmc_br.log; exit 1; }
tail -45 $D/pmc_br.log
