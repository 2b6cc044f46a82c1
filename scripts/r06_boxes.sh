#!/bin/bash
# round 6: the driver's command three times on one box (run once per gpurun call, i.e. per box),
# then the HBM- vs cache-resident probe of the headline kernel at the burst clock
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_boxes/${BOX_TAG:-a}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$i.log 2>&1 || { tail -5 $OUT/bench_$i.log; exit 1; }
  grep '^{' $OUT/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$i', d['value'], r['frac'], r['kernel_ms'], d['batches']['shader_mhz'], d['sustained_batches']['frac'], d['config4']['kernel_ms_mean'])"
done
timeout -k 10 200 python3 -u scripts/batches_rot_probe.py 8 0.1 > $OUT/rot.log 2>&1 || { tail -5 $OUT/rot.log; exit 1; }
grep -v amdgpu.ids $OUT/rot.log
exit 0
