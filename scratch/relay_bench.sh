#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/relay
run() {  # run <tag> <lib or empty>
    if [[ -n $2 ]]; then export HFV_LIB=$2; else unset HFV_LIB; fi
    timeout -k 10 200 python -u bench.py --cpu-budget 0 --no-host-e2e > gpurun_out/relay/bench_$1.log 2>&1 || { tail -20 gpurun_out/relay/bench_$1.log; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/relay/bench_$1.log').read().strip().splitlines()[-1]); h=d['hbm_resident']
print('$1', d['service'], 'launch', d['per_launch']['mpkts'], d['per_launch']['kernel_ms_mean'], '2^24 svc', h['service_mpkts'], h['service_ms_per_batch'], 'launch', h['mpkts'], h['kernel_ms_mean'])"
}
for v in ${VARIANTS:-a1 a0 a1b a0b}; do
    case $v in a1*) run $v "";; *) run $v $PWD/scratch/lib_relay_${v%b}/libscionhfv.so;; esac
done
