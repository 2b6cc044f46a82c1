#!/bin/bash
# Round 3: where do the ~35 us around a K = 20 service region go?  The headline leg only, under
# runtime knobs that change the launch / completion path, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03_overhead}
mkdir -p $OUT
ARGS="--steps 20 --warmup 5 --no-extras --no-host-e2e --cpu-budget 0 --loop-n 0 --svc-reps 5"
for i in 1 2 3; do
    for v in untimed timed; do
        case $v in
            untimed) E="HFV_BENCH_TIMED_VALUE=0" ;;
            timed) E="HFV_BENCH_TIMED_VALUE=1" ;;
            devkernarg) E="HIP_FORCE_DEV_KERNARG=1" ;;
            skipargcopy) E="ROC_SKIP_KERNEL_ARG_COPY=1" ;;
            nodirect) E="AMD_DIRECT_DISPATCH=0" ;;
        esac
        env $E timeout -k 10 120 python bench.py $ARGS > $OUT/${v}_$i.log 2>&1
        rc=$?; [[ $rc -ne 0 ]] && { echo "$v $i rc=$rc"; tail -5 $OUT/${v}_$i.log; exit $rc; }
        python - "$OUT/${v}_$i.log" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["service"]
ov = [round((r - g) * 1e3, 1) for r, g in zip(s["timed_regions_ms"], s["grids_ms"])]
ovt = [round((r - g) * 1e3, 1) for r, g in zip(s["event_timed_regions_ms"], s["grids_ms"])]
print(f"{sys.argv[2]:12s} value {d['value']:9.1f} ms/step {d['ms_per_step']*1e3:6.2f}us grid/batch {d['roofline']['kernel_ms_per_batch']*1e3:6.2f}us "
      f"value-region - grid us {ov} event-region - grid us {ovt} launch us {s['service_run_call_us']} mhz {s['shader_mhz']}")
PY
    done
done
