#!/bin/bash
# Variant kernel library for same-box A/Bs and diagnostic builds:
#   tools/build_kernel_variant.sh NAME SRC.hip "-DMACRO=V ..."
# recompiles csrc/kernels/SRC.hip with the extra flags and links it with the other
# objects of the last regular build into kubeflow_controller_amd/ops/_hip_kernels_NAME.so
# (select it with KFA_KERNELS_SO=_hip_kernels_NAME.so; delete it after the A/B).
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; src=$2; flags=$3
python3 -c "from kubeflow_controller_amd import _build; _build.build_kernels()"
obj=build/variant/$name; mkdir -p $obj
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
$HIPCC -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-result -Icsrc/kernels $flags \
  -c csrc/kernels/$src -o $obj/$src.o
objs=$(ls build/kernels/*.o | grep -v "/$src.o$")
$HIPCC -shared -fPIC --offload-arch=gfx950 $objs $obj/$src.o -o kubeflow_controller_amd/ops/_hip_kernels_$name.so
echo kubeflow_controller_amd/ops/_hip_kernels_$name.so
