#!/bin/bash
# GPU-box check of verify-kernel variants: service and parity tests with each library, then an
# interleaved headline A/B.   scripts/svc_variant_session.sh TAG ROUNDS lib...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest tests/test_gpu_service.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
for lib in "$@"; do
  n=$(basename $lib .so)
  HFV_LIB=$(readlink -f $lib) timeout -k 10 400 $T > $OUT/tests_$n.log 2>&1; rc=$?; echo "$n tests rc=$rc"; tail -2 $OUT/tests_$n.log
  [[ $rc -ne 0 ]] && exit $rc
done
timeout -k 10 900 bash scripts/ab_svc.sh $R "$@" > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; exit $rc
