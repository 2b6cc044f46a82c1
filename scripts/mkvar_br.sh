#!/bin/bash
# mkvar.sh <name> <flags...>: library variant with the router kernel built with extra flags
set -e
cd /root/repo/scion-xdp-br_amd
name=$1; shift
mkdir -p build/obj/var_$name lib/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wextra -Werror -Wno-unused-parameter -mllvm -amdgpu-atomic-optimizer-strategy=None "$@" -c -o build/obj/var_$name/hfv_br_kernel.hip.o csrc/hfv_br_kernel.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o lib/ab/libscionhfv_$name.so build/obj/hfv_kernels.hip.o build/obj/var_$name/hfv_br_kernel.hip.o build/obj/hfv_api.cpp.o build/obj/hfv_aes_host.cpp.o build/obj/hfv_keymap.cpp.o build/obj/hfv_statsmap.cpp.o build/obj/hfv_config.cpp.o build/obj/hfv_loop.cpp.o
