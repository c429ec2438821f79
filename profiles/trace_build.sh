#!/bin/bash
# Build an instrumented variant of the library (profiling only, never shipped):
#   profiles/trace_build.sh sph   NAME -DLPE_FTRACE   -> per-block phase stamps in k_forces_couple
#   profiles/trace_build.sh rigid NAME -DLPE_PTRACE   -> per-colour-step stamps in k_pgs_colour / k_pos_colour
# The variant links the other objects of build/ (run `make` first) and lands in
# profiles/_var/liblpe_NAME.so; run the matching script with LPE_LIB pointing at it.
set -e
which=$1; n=$2; shift 2
d=/tmp/lpe_var_$n; mkdir -p $d profiles/_var
src=little-physics-engine_amd/csrc/lpe_$which.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
    -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -Wall -Wno-unused-function \
    "$@" -c $src -o $d/lpe_$which.o
objs=$(ls build/*.o | grep -v "lpe_$which.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o profiles/_var/liblpe_$n.so $objs $d/lpe_$which.o \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo profiles/_var/liblpe_$n.so
