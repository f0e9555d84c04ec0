#!/bin/bash
# Link an A/B variant of the kernel library: one source recompiled with extra
# flags, every other object from the last in-tree build.
#   tools/build_variant.sh <name> <source.hip> [hipcc flags...]  ->  ops/_hip_kernels_<name>.so
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
obj=build/kernels/$(basename "$src").o
vobj=build/kernels/$(basename "$src").$name.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-result \
  -Icsrc/kernels "$@" -c "$src" -o "$vobj"
objs=$(ls build/kernels/*.hip.o | grep -v "^$obj\$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs "$vobj" -o kubeflow_controller_amd/ops/_hip_kernels_$name.so
echo built kubeflow_controller_amd/ops/_hip_kernels_$name.so
