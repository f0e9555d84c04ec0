// Diagnostic kernels for the GPU tests (not on any training path).
//
// kfa_cu_hog: `blocks` workgroups that each hold 96 KB of LDS (so no 128 KB
// gemm_ppp block can share their CU) and sleep-spin for `usec` microseconds of
// wall clock (s_memrealtime, 100 MHz), then write one word each.  Launched on
// one stream while a kernel under test runs on another, it takes most of the CUs
// away for a known time: a kernel whose blocks wait on other blocks of the same
// launch (co-residency assumptions) stalls until the hog ends; one whose blocks
// never wait finishes on the CUs that are left.  Every wave exits after `usec`.
#include "common.h"

namespace {

constexpr int kHogLds = 96 * 1024;

__global__ __launch_bounds__(64) void cu_hog_kernel(unsigned long long ticks, int* out) {
  __shared__ int pad[kHogLds / 4];
  pad[threadIdx.x] = (int)threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = pad[(blockIdx.x * 7) & 63] + 1;
}

}  // namespace

// out: int32 [blocks]; each element becomes (its index * 7 mod 64) + 1 when its block ends
KFA_API int kfa_cu_hog(int blocks, long usec, int* out, hipStream_t st) {
  if (blocks <= 0 || usec <= 0 || usec > 5000000 || out == nullptr) return -1;
  hipLaunchKernelGGL(cu_hog_kernel, dim3(blocks), dim3(64), 0, st, (unsigned long long)usec * 100ull, out);
  return kfa_status();
}
