#!/bin/bash
# round 5, session 12: machine-scheduler strategies for the router kernel (config 4), parity + A/B
L=scion-xdp-br_amd/lib/ab
timeout -k 10 1000 bash scripts/br_variant_session.sh r05_s12 3 $L/libscionhfv_br_head.so $L/libscionhfv_br_max-ilp.so \
    $L/libscionhfv_br_max-memory-clause.so
