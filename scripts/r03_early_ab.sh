#!/bin/bash
# Round 3: A/B of library builds on the service grid's fixed cost (region_floor: K = 1 and
# K = 20 grids) and on the headline (ab_libs), interleaved.  Usage: r03_early_ab.sh OUT lib...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_service.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_service.log 2>&1 || { tail -20 $OUT/pytest_service.log; exit 1; }
tail -2 $OUT/pytest_service.log
for i in 1 2; do
    for lib in "$@"; do
        echo "== $lib $i"
        HFV_LIB=$PWD/$lib timeout -k 10 200 python scripts/region_floor.py 10 > $OUT/floor_$(basename $lib .so)_$i.log 2>&1 || { tail -5 $OUT/floor_$(basename $lib .so)_$i.log; exit 1; }
        grep svc $OUT/floor_$(basename $lib .so)_$i.log
    done
done
timeout -k 10 600 python scripts/ab_libs.py 3 "$@" > $OUT/ab.log 2>&1; rc=$?
cat $OUT/ab.log
exit $rc
