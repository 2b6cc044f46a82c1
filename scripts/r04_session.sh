#!/bin/bash
# Round-4 closing GPU session, in two parts (each under gpurun's 20-minute limit):
#   part 1: the GPU tests, smoke, the driver's bench command twice, the config-4 bench
#   part 2: rocprofv3 kernel-trace stats of the driver's command, PMC passes of the service
#           headline (config 2) and config 3
# Output: gpurun_out/r04_final/.  Every GPU step has its own time limit; a crash, abort or
# time-out stops the script (nothing else touches the GPU afterwards).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R04_OUT:-r04_final}
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step <name> <timeout-s> <cmd...>
    local name=$1 t=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 4 "$OUT/$name.log"
    return $rc
}
PART=${1:-1}
if [[ $PART == 1 ]]; then
    step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
    rc=$?; if [[ $rc -gt 1 ]]; then exit $rc; fi
    step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
    step bench_1 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
    step bench_2 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
fi
if [[ $PART == 2 ]]; then
    step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o run -- \
        python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
    step pmc_zero 400 bash scripts/pmc_round.sh zero svc rot8 || exit $?
    step pmc_ifid 400 bash scripts/pmc_round.sh ifid svc rot8 || exit $?
fi
if [[ $PART == br ]]; then   # where the router kernel's waves spend their cycles (diagnostic build)
    # (build it first, in this container: scripts/mkvar_br.sh brprof -DHFV_BR_PROF=1)
    HFV_LIB=$PWD/scion-xdp-br_amd/lib/ab/libscionhfv_brprof.so step br_phase 300 python scripts/br_phase_probe.py || exit $?
fi
