// Softmax cross-entropy, forward + backward fused, and
// row argmax / accuracy (K3).
//
// One 256-thread block per row.  Pass 1: online (max, sum-exp) over the row
// with 16-B loads; pass 2 writes dlogits = (softmax - onehot) * gscale / B
// directly in the forward, so backward is a scalar multiply (usually 1.0,
// skipped).  Row loss is written per row and reduced by the caller.
// Rows whose label is < 0 (ignore_index) get loss 0 and zero gradient.
#include "common.h"

namespace {

__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
  const float mm = fmaxf(m, m2);
  s = (m == -INFINITY ? 0.f : s * __expf(m - mm)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mm));
  m = mm;
}

template <bool BF16>
__global__ __launch_bounds__(256) void xent_kernel(const void* __restrict__ logits, const long* __restrict__ labels,
                                                   const float* __restrict__ bias, float* __restrict__ row_loss,
                                                   void* __restrict__ dlogits, int V, float gscale, float smoothing) {
  const long row = blockIdx.x;
  const int t = threadIdx.x;
  const long lab = labels[row];
  const bf16_t* lb = reinterpret_cast<const bf16_t*>(logits) + row * V;
  const float* lf = reinterpret_cast<const float*>(logits) + row * V;
  // optional per-column bias (e.g. the MLM decoder bias) is added on the fly
  auto ld = [&](int i) -> float { return (BF16 ? bf2f(lb[i]) : lf[i]) + (bias ? bias[i] : 0.f); };
  auto ldv = [&](int i, float f[8]) {
    unpack8(*reinterpret_cast<const uint4*>(lb + i), f);
    if (bias) {
      const float4 b0 = *reinterpret_cast<const float4*>(bias + i), b1 = *reinterpret_cast<const float4*>(bias + i + 4);
      f[0] += b0.x; f[1] += b0.y; f[2] += b0.z; f[3] += b0.w; f[4] += b1.x; f[5] += b1.y; f[6] += b1.z; f[7] += b1.w;
    }
  };

  float m = -INFINITY, s = 0.f, sum_z = 0.f;
  const bool vec = BF16 && (V % 8 == 0);
  if (vec) {
    for (int i = t * 8; i < V; i += 256 * 8) {
      float f[8];
      ldv(i, f);
      float lm = f[0];
#pragma unroll
      for (int j = 1; j < 8; j++) lm = fmaxf(lm, f[j]);
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 8; j++) { ls += __expf(f[j] - lm); sum_z += f[j]; }
      online_merge(m, s, lm, ls);
    }
  } else {
    for (int i = t; i < V; i += 256) {
      const float z = ld(i);
      sum_z += z;
      online_merge(m, s, z, 1.f);
    }
  }
  // wave then block merge
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    online_merge(m, s, m2, s2);
    sum_z += __shfl_xor(sum_z, o, 64);
  }
  __shared__ float shm[4], shs[4], shz[4];
  if ((t & 63) == 0) { shm[t >> 6] = m; shs[t >> 6] = s; shz[t >> 6] = sum_z; }
  __syncthreads();
  m = shm[0]; s = shs[0]; sum_z = shz[0];
  for (int w = 1; w < 4; w++) { online_merge(m, s, shm[w], shs[w]); sum_z += shz[w]; }
  const float lse = m + __logf(s);
  const bool ignore = lab < 0 || lab >= V;
  if (t == 0) {
    float loss = 0.f;
    if (!ignore) {
      const float zl = ld((int)lab);
      loss = (1.f - smoothing) * (lse - zl) + smoothing * (lse - sum_z / (float)V);
    }
    row_loss[row] = loss;
  }
  if (!dlogits) return;
  bf16_t* dl = reinterpret_cast<bf16_t*>(dlogits) + row * V;
  float* dlf = reinterpret_cast<float*>(dlogits) + row * V;
  const float off = smoothing / (float)V;
  if (vec) {
    for (int i = t * 8; i < V; i += 256 * 8) {
      float f[8];
      ldv(i, f);
#pragma unroll
      for (int j = 0; j < 8; j++) {
        float p = __expf(f[j] - lse) - off;
        if (i + j == lab) p -= (1.f - smoothing);
        f[j] = ignore ? 0.f : p * gscale;
      }
      *reinterpret_cast<uint4*>(dl + i) = pack8(f);
    }
  } else {
    for (int i = t; i < V; i += 256) {
      float p = __expf(ld(i) - lse) - off;
      if (i == lab) p -= (1.f - smoothing);
      const float gv = ignore ? 0.f : p * gscale;
      if (BF16) dl[i] = (bf16_t)f2bf(gv); else dlf[i] = gv;
    }
  }
}

template <bool BF16>
__global__ __launch_bounds__(256) void argmax_kernel(const void* __restrict__ logits, long* __restrict__ out, int V) {
  const long row = blockIdx.x;
  const int t = threadIdx.x;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = t; i < V; i += 256) {
    const float z = BF16 ? bf2f(reinterpret_cast<const bf16_t*>(logits)[row * V + i])
                         : reinterpret_cast<const float*>(logits)[row * V + i];
    if (z > best || (z == best && i < bi)) { best = z; bi = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float b2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    if (b2 > best || (b2 == best && i2 < bi)) { best = b2; bi = i2; }
  }
  __shared__ float sb[4];
  __shared__ int si[4];
  if ((t & 63) == 0) { sb[t >> 6] = best; si[t >> 6] = bi; }
  __syncthreads();
  if (t == 0) {
    for (int w = 1; w < 4; w++)
      if (sb[w] > best || (sb[w] == best && si[w] < bi)) { best = sb[w]; bi = si[w]; }
    out[row] = bi;
  }
}

}  // namespace

KFA_API int kfa_softmax_xent(const void* logits, int logits_bf16, const long* labels, const float* bias,
                             float* row_loss, void* dlogits, long rows, int V, float gscale, float smoothing,
                             hipStream_t s) {
  if (rows <= 0 || V <= 0) return -1;
  if (logits_bf16)
    hipLaunchKernelGGL(xent_kernel<true>, dim3(rows), dim3(256), 0, s, logits, labels, bias, row_loss, dlogits, V,
                       gscale, smoothing);
  else
    hipLaunchKernelGGL(xent_kernel<false>, dim3(rows), dim3(256), 0, s, logits, labels, bias, row_loss, dlogits, V,
                       gscale, smoothing);
  return kfa_status();
}

KFA_API int kfa_argmax(const void* logits, int logits_bf16, long* out, long rows, int V, hipStream_t s) {
  if (rows <= 0 || V <= 0) return -1;
  if (logits_bf16)
    hipLaunchKernelGGL(argmax_kernel<true>, dim3(rows), dim3(256), 0, s, logits, out, V);
  else
    hipLaunchKernelGGL(argmax_kernel<false>, dim3(rows), dim3(256), 0, s, logits, out, V);
  return kfa_status();
}
