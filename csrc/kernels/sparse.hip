// Sparse (row-wise) embedding optimizers for the parameter-server tables of
// Wide&Deep (SURVEY §2.6 K6 "sparse Adam/SGD row update on the owner", §7.3 H6).
//
// Gradients arrive as (row id, dense row) pairs — duplicates allowed, from all
// workers after the all-to-all push.  Step 1 (``kfa_embed_bwd``'s scatter
// kernel, transformer.hip) adds them into a self-cleaning fp32 scratch table.
// Step 2 (here) walks the same id list: for each element, an atomic exchange
// hands the summed gradient to exactly one occurrence, which applies the
// optimizer to that element of the master table and its moments in place and
// leaves the scratch zeroed.  Rows that were not looked up are never touched
// (lazy Adam semantics, as TF's sparse apply on the PS).
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void sparse_adam_kernel(const long* __restrict__ ids, float* __restrict__ scratch,
                                                          float* __restrict__ w, float* __restrict__ m,
                                                          float* __restrict__ v, long n, int D, float lr, float b1,
                                                          float b2, float eps, float wd, float c1, float c2,
                                                          float gscale) {
  const long total = n * (long)D;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / D;
    const int c = (int)(i - r * D);
    const long e = ids[r] * D + c;
    float g = __hip_atomic_exchange(scratch + e, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (g == 0.f) continue;
    g *= gscale;
    const float mm = b1 * m[e] + (1.f - b1) * g;
    const float vv = b2 * v[e] + (1.f - b2) * g * g;
    m[e] = mm;
    v[e] = vv;
    const float upd = (mm * c1) / (sqrtf(vv * c2) + eps) + wd * w[e];
    w[e] -= lr * upd;
  }
}

__global__ __launch_bounds__(256) void sparse_sgd_kernel(const long* __restrict__ ids, float* __restrict__ scratch,
                                                         float* __restrict__ w, long n, int D, float lr,
                                                         float gscale) {
  const long total = n * (long)D;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / D;
    const int c = (int)(i - r * D);
    const long e = ids[r] * D + c;
    const float g = __hip_atomic_exchange(scratch + e, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (g != 0.f) w[e] -= lr * g * gscale;
  }
}

__global__ __launch_bounds__(256) void scatter_add_rows_kernel(const long* __restrict__ ids,
                                                               const bf16_t* __restrict__ g, float* __restrict__ scratch,
                                                               long n, int D) {
  const long total = n * (long)D;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / D;
    const int c = (int)(i - r * D);
    atomicAdd(scratch + ids[r] * D + c, bf2f(g[i]));
  }
}

int grid_for(long n) {
  long g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

}  // namespace

// scratch[ids[r]] += g[r]  (g: bf16 [n, D], any D)
KFA_API int kfa_scatter_add_rows(const long* ids, const void* g, float* scratch, long n, int D, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(scatter_add_rows_kernel, dim3(grid_for(n * D)), dim3(256), 0, s, ids, (const bf16_t*)g, scratch,
                     n, D);
  return kfa_status();
}

// Adam on the looked-up rows; c1 = 1/(1-b1^t), c2 = 1/(1-b2^t); decoupled decay (AdamW) wd.
KFA_API int kfa_sparse_adam(const long* ids, float* scratch, float* w, float* m, float* v, long n, int D, float lr,
                            float b1, float b2, float eps, float wd, float c1, float c2, float gscale, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(sparse_adam_kernel, dim3(grid_for(n * D)), dim3(256), 0, s, ids, scratch, w, m, v, n, D, lr, b1,
                     b2, eps, wd, c1, c2, gscale);
  return kfa_status();
}

KFA_API int kfa_sparse_sgd(const long* ids, float* scratch, float* w, long n, int D, float lr, float gscale,
                           hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(sparse_sgd_kernel, dim3(grid_for(n * D)), dim3(256), 0, s, ids, scratch, w, n, D, lr, gscale);
  return kfa_status();
}
