#!/bin/bash
# Parity tests + a short bench for each KEYSEL_ZERO verify-kernel variant named on the
# command line (HFV_KVARIANT strings), e.g.
#   bash scripts/variants.sh "bs=99,block=256" "bs=4" "bs=0"
# Each GPU step has its own time limit; a crash/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_gpu_parity.py}
for v in "$@"; do
    tag=$(echo "$v" | tr ',=' '_-')
    echo "=== $v parity"
    HFV_KVARIANT="$v" timeout -k 10 300 python -m pytest $TESTS -x -q -p no:cacheprovider \
        > gpurun_out/var_${tag}_pytest.log 2>&1
    rc=$?
    tail -n 3 gpurun_out/var_${tag}_pytest.log
    if [[ $rc -gt 1 ]]; then exit $rc; fi
    echo "=== $v bench"
    HFV_KVARIANT="$v" timeout -k 10 300 python bench.py --cpu-budget 0 --no-host-e2e --steps ${STEPS:-100} \
        > gpurun_out/var_${tag}_bench.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; h=d.get('hbm_resident',{}); print('value', d['value'], 'kern_ms', r['kernel_ms_mean'], 'frac', r['frac'], 'hbm', h.get('kernel_ms_mean'), h.get('frac'), r.get('variant'))" gpurun_out/var_${tag}_bench.log
done
