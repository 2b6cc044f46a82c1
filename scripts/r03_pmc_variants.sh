#!/bin/bash
# Round 3: SQ/LDS counters of the resident service, config 2 and the config-3 variants
# (HFV_SVC_IFID=lds|sched), 2^20 rotated batches as in the bench.  One rocprofv3 run per
# counter group, never with a tracing domain.  usage: r03_pmc_variants.sh <outdir> <ks:variant>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_pmc}
shift
groups=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES"
)
for kv in "$@"; do
  ks=${kv%%:*}; var=${kv#*:}
  D=$OUT/${ks}_$var
  mkdir -p $D
  i=0
  for g in "${groups[@]}"; do
    i=$((i+1))
    HFV_SVC_IFID=$var timeout -k 10 -s KILL 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $D/p$i -o run -- \
        python3 scripts/pmc_driver.py $ks 10 1048576 svc rot8 > $D/p$i.log 2>&1 || { echo "$kv pass $i failed"; tail -5 $D/p$i.log; exit 1; }
  done
  python3 scripts/pmc_summary.py $D 1048576 k_verify_service 10 > /dev/null
  python3 - $D/summary.json $kv <<'PY'
import json, sys
o = json.load(open(sys.argv[1]))["1048576"]
g = lambda k: o.get(k, float("nan"))
print(sys.argv[2], "LDS instr/pkt %.1f" % (g("SQ_INSTS_LDS") / 16384 * 64 / 64),
      "IDX_ACTIVE %.3gM" % (g("SQ_LDS_IDX_ACTIVE") / 1e6), "BANK_CONFLICT %.3gM" % (g("SQ_LDS_BANK_CONFLICT") / 1e6),
      "WAIT_INST_LDS %.3gM" % (g("SQ_WAIT_INST_LDS") / 1e6), "VALU/pkt %.1f" % (g("SQ_INSTS_VALU") / 16384),
      "WAVE_CYCLES %.3gM" % (g("SQ_WAVE_CYCLES") / 1e6), "WAIT_ANY %.3gM" % (g("SQ_WAIT_ANY") / 1e6),
      "BUSY %.3gM" % (g("SQ_BUSY_CYCLES") / 1e6), "GUI %.3gK" % (g("GRBM_GUI_ACTIVE") / 1e3))
PY
done
