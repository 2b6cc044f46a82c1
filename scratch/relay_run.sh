#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/relay
timeout -k 10 150 python -u -m pytest -x -v --timeout 60 --timeout-method thread tests/test_gpu_service.py > gpurun_out/relay/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/relay/pytest.log; exit 1; }
tail -1 gpurun_out/relay/pytest.log
VARIANTS="${VARIANTS:-a1 a1b}" ./scratch/relay_bench.sh
