// Fused optimizer apply over FLAT parameter buckets (SURVEY §2.6 K4 Adam, K5 SGD).
//
// One launch updates a whole bucket (every parameter of a dtype group lives in
// one contiguous buffer, see parallel/flat.py), instead of one launch per
// tensor.  Mixed precision: the fp32 master copy is updated and the bf16
// compute copy (if any) is rewritten in the same pass; grads may be bf16
// (the all-reduced bucket) or fp32.  8 elements per lane, 16-B loads for
// bf16, 2x16-B for fp32.
#include "common.h"

namespace {

template <bool GBF16>
__device__ __forceinline__ void load_grad8(const void* g, long i, float out[8], float scale) {
  if (GBF16) {
    unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(g) + i), out);
  } else {
    const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(g) + i);
    const float4 b = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(g) + i + 4);
    out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w; out[4] = b.x; out[5] = b.y; out[6] = b.z; out[7] = b.w;
  }
#pragma unroll
  for (int j = 0; j < 8; j++) out[j] *= scale;
}

__device__ __forceinline__ void load8(const float* p, float o[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
__device__ __forceinline__ void store8(float* p, const float o[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(o[4], o[5], o[6], o[7]);
}

template <bool GBF16>
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ w, bf16_t* __restrict__ wb,
                                                  const void* __restrict__ g, float* __restrict__ mom, long n8,
                                                  float lr, float momentum, float dampening, float wd, int nesterov,
                                                  float gscale, int first) {
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < n8; v += (long)gridDim.x * blockDim.x) {
    const long i = v * 8;
    float gr[8], p[8];
    load_grad8<GBF16>(g, i, gr, gscale);
    load8(w + i, p);
#pragma unroll
    for (int j = 0; j < 8; j++) gr[j] = fmaf(wd, p[j], gr[j]);
    if (mom) {
      float m[8];
      if (first) {
#pragma unroll
        for (int j = 0; j < 8; j++) m[j] = gr[j];
      } else {
        load8(mom + i, m);
#pragma unroll
        for (int j = 0; j < 8; j++) m[j] = fmaf(momentum, m[j], (1.f - dampening) * gr[j]);
      }
      store8(mom + i, m);
#pragma unroll
      for (int j = 0; j < 8; j++) gr[j] = nesterov ? fmaf(momentum, m[j], gr[j]) : m[j];
    }
#pragma unroll
    for (int j = 0; j < 8; j++) p[j] = fmaf(-lr, gr[j], p[j]);
    store8(w + i, p);
    if (wb) *reinterpret_cast<uint4*>(wb + i) = pack8(p);
  }
}

// AdamW (decoupled weight decay; wd = 0 gives Adam).  bc1 = 1 - b1^t, bc2 = 1 - b2^t.
template <bool GBF16>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ w, bf16_t* __restrict__ wb,
                                                   const void* __restrict__ g, float* __restrict__ m_,
                                                   float* __restrict__ v_, long n8, float lr, float b1, float b2,
                                                   float eps, float wd, float bc1, float bc2, float gscale,
                                                   const float* __restrict__ dbc) {
  if (dbc) {  // bias corrections produced on the device (adam_bc_kernel): replayable in a HIP graph
    bc1 = dbc[0];
    bc2 = dbc[1];
  }
  const float step = lr / bc1;
  const float rbc2 = rsqrtf(bc2);
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < n8; v += (long)gridDim.x * blockDim.x) {
    const long i = v * 8;
    float gr[8], p[8], m[8], s[8];
    load_grad8<GBF16>(g, i, gr, gscale);
    load8(w + i, p);
    load8(m_ + i, m);
    load8(v_ + i, s);
#pragma unroll
    for (int j = 0; j < 8; j++) {
      m[j] = fmaf(b1, m[j], (1.f - b1) * gr[j]);
      s[j] = fmaf(b2, s[j], (1.f - b2) * gr[j] * gr[j]);
      const float denom = sqrtf(s[j]) * rbc2 + eps;
      p[j] = p[j] * (1.f - lr * wd) - step * m[j] / denom;
    }
    store8(m_ + i, m);
    store8(v_ + i, s);
    store8(w + i, p);
    if (wb) *reinterpret_cast<uint4*>(wb + i) = pack8(p);
  }
}

// t += 1; bc = (1 - b1^t, 1 - b2^t): the per-step scalars of Adam kept on the
// device, so a captured step needs no host value that changes per step
// seed >= 0 (an eager step): the host's step count replaces the device one first — the
// re-seed that used to be a separate fill launch; seed < 0 (graph replay): t advances
__global__ void adam_bc_kernel(int* __restrict__ t, float* __restrict__ bc, float b1, float b2, int seed) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const int s = (seed >= 0 ? seed : t[0]) + 1;
    t[0] = s;
    bc[0] = 1.f - powf(b1, (float)s);
    bc[1] = 1.f - powf(b2, (float)s);
  }
}

// master fp32 -> bf16 copy (initial sync / after broadcast)
__global__ void f32_to_bf16_kernel(const float* __restrict__ a, bf16_t* __restrict__ b, long n8) {
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < n8; v += (long)gridDim.x * blockDim.x) {
    float p[8];
    load8(a + v * 8, p);
    *reinterpret_cast<uint4*>(b + v * 8) = pack8(p);
  }
}

// sum of squares for grad-norm clipping: per-block partials -> atomicAdd
template <bool GBF16>
__global__ __launch_bounds__(256) void sumsq_kernel(const void* __restrict__ g, long n8, float* __restrict__ out) {
  float acc = 0.f;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < n8; v += (long)gridDim.x * blockDim.x) {
    float gr[8];
    load_grad8<GBF16>(g, v * 8, gr, 1.f);
#pragma unroll
    for (int j = 0; j < 8; j++) acc = fmaf(gr[j], gr[j], acc);
  }
  acc = wave_sum(acc);
  __shared__ float sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, sh[0] + sh[1] + sh[2] + sh[3]);
}

int grid_for(long n8) {
  long b = (n8 + 255) / 256;
  return (int)(b < 2048 ? (b < 1 ? 1 : b) : 2048);
}

}  // namespace

// n must be a multiple of 8 (flat buckets are padded); pointers 16-B aligned.
KFA_API int kfa_sgd_step(float* w, bf16_t* wb, const void* g, int g_is_bf16, float* mom, long n, float lr,
                         float momentum, float dampening, float wd, int nesterov, float gscale, int first,
                         hipStream_t s) {
  if (n % 8) return -1;
  const long n8 = n / 8;
  if (g_is_bf16)
    hipLaunchKernelGGL(sgd_kernel<true>, dim3(grid_for(n8)), dim3(256), 0, s, w, wb, g, mom, n8, lr, momentum,
                       dampening, wd, nesterov, gscale, first);
  else
    hipLaunchKernelGGL(sgd_kernel<false>, dim3(grid_for(n8)), dim3(256), 0, s, w, wb, g, mom, n8, lr, momentum,
                       dampening, wd, nesterov, gscale, first);
  return kfa_status();
}

// dbc: nullptr (bc1 / bc2 as given) or the device pair written by kfa_adam_bc
KFA_API int kfa_adam_step(float* w, bf16_t* wb, const void* g, int g_is_bf16, float* m, float* v, long n, float lr,
                          float b1, float b2, float eps, float wd, float bc1, float bc2, float gscale, const float* dbc,
                          hipStream_t s) {
  if (n % 8) return -1;
  const long n8 = n / 8;
  if (g_is_bf16)
    hipLaunchKernelGGL(adam_kernel<true>, dim3(grid_for(n8)), dim3(256), 0, s, w, wb, g, m, v, n8, lr, b1, b2, eps,
                       wd, bc1, bc2, gscale, dbc);
  else
    hipLaunchKernelGGL(adam_kernel<false>, dim3(grid_for(n8)), dim3(256), 0, s, w, wb, g, m, v, n8, lr, b1, b2, eps,
                       wd, bc1, bc2, gscale, dbc);
  return kfa_status();
}

KFA_API int kfa_adam_bc(int* t, float* bc, float b1, float b2, hipStream_t s) {
  hipLaunchKernelGGL(adam_bc_kernel, dim3(1), dim3(64), 0, s, t, bc, b1, b2, -1);
  return kfa_status();
}

// the same, the device count first set to `seed` when seed >= 0 (eager steps, resumes)
KFA_API int kfa_adam_bc_seed(int* t, float* bc, float b1, float b2, int seed, hipStream_t s) {
  hipLaunchKernelGGL(adam_bc_kernel, dim3(1), dim3(64), 0, s, t, bc, b1, b2, seed);
  return kfa_status();
}

KFA_API int kfa_f32_to_bf16(const float* a, bf16_t* b, long n, hipStream_t s) {
  if (n % 8) return -1;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid_for(n / 8)), dim3(256), 0, s, a, b, n / 8);
  return kfa_status();
}

// out must be zeroed by the caller (accumulates)
KFA_API int kfa_sumsq(const void* g, int g_is_bf16, long n, float* out, hipStream_t s) {
  if (n % 8) return -1;
  if (g_is_bf16)
    hipLaunchKernelGGL(sumsq_kernel<true>, dim3(grid_for(n / 8)), dim3(256), 0, s, g, n / 8, out);
  else
    hipLaunchKernelGGL(sumsq_kernel<false>, dim3(grid_for(n / 8)), dim3(256), 0, s, g, n / 8, out);
  return kfa_status();
}
