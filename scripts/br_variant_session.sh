#!/bin/bash
# GPU-box check of router-kernel variants: config-4/5 parity tests with the default library and
# with each variant, then an interleaved A/B.   scripts/br_variant_session.sh TAG ROUNDS lib...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest tests/test_gpu_br.py tests/test_gpu_loop.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 400 $T > $OUT/parity_default.log 2>&1; rc=$?; echo "default parity rc=$rc"; tail -2 $OUT/parity_default.log
[[ $rc -gt 1 ]] && exit $rc
for lib in "$@"; do
  n=$(basename $lib .so)
  HFV_LIB=$(readlink -f $lib) timeout -k 10 400 $T > $OUT/parity_$n.log 2>&1; rc=$?; echo "$n parity rc=$rc"; tail -2 $OUT/parity_$n.log
  [[ $rc -gt 1 ]] && exit $rc
done
timeout -k 10 900 bash scripts/ab_br.sh $R "$@" > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; exit $rc
