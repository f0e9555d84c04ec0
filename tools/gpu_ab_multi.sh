set -o pipefail
for v in ${AB_VARIANTS:-wdy wx wpart}; do echo "== $v"; bash tools/gpu_ab_env.sh KFA_KERNELS_SO=_hip_kernels.so KFA_KERNELS_SO=_hip_kernels_$v.so || exit 1; done
