#!/bin/bash
# round 5, session 17: the router with 16-bit header accessors (even offsets, -DHFV_BR_EVEN=1)
# against HEAD: parity (router + loop GPU tests) with both builds, then an interleaved A/B
L=scion-xdp-br_amd/lib/ab
timeout -k 10 1000 bash scripts/br_variant_session.sh r05_s17 4 $L/libscionhfv_br_head.so $L/libscionhfv_br_even.so
