set -o pipefail
for v in s18 s3 el2 bnld; do echo "== $v"; bash tools/gpu_ab_env.sh KFA_KERNELS_SO=_hip_kernels.so KFA_KERNELS_SO=_hip_kernels_$v.so || exit 1; done
