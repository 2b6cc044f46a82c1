#!/bin/bash
# mkvar_k.sh <name> <flags...>: library variant with the verify kernels built with extra flags
set -e
cd "$(dirname "$0")/../scion-xdp-br_amd"
name=$1; shift
mkdir -p build/obj/vark_$name lib/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wextra -Werror -Wno-unused-parameter -mllvm -amdgpu-atomic-optimizer-strategy=None "$@" -c -o build/obj/vark_$name/hfv_kernels.hip.o csrc/hfv_kernels.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o lib/ab/libscionhfv_$name.so build/obj/vark_$name/hfv_kernels.hip.o build/obj/hfv_br_kernel.hip.o build/obj/hfv_api.cpp.o build/obj/hfv_aes_host.cpp.o build/obj/hfv_keymap.cpp.o build/obj/hfv_statsmap.cpp.o build/obj/hfv_config.cpp.o build/obj/hfv_loop.cpp.o
