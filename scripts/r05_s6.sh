#!/bin/bash
# round 5, session 6: router header-extension registers (HFV_BR_EXT) -- parity with both builds, A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=scion-xdp-br_amd/lib/ab
timeout -k 10 1000 bash scripts/br_variant_session.sh r05_s6 4 $L/libscionhfv_br_ext0.so $L/libscionhfv_br_ext1.so
