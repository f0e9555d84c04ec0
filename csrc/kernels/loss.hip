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

// ---- small classifier head + softmax cross-entropy (BERT's NSP: [B, H] x [2, H]ᵀ):
//   logits[b][c] = x_b . W_c + bias_c,  loss = mean_b (logsumexp_c logits[b] - logits[b][y_b])
// forward saves p = softmax(logits); backward with g[b][c] = dloss (p - [c == y_b]) / B:
//   dx_b = Σ_c g[b][c] W_c (bf16),  dW_c = Σ_b g[b][c] x_b,  db_c = Σ_b g[b][c]
// One 32-lane half-wave per row; per-block partials reduced in a fixed order.  C <= 8,
// H % 8 == 0, H <= 1024.  Replaces an N = 2 hipBLASLt GEMM per direction + the loss chain.
constexpr int kClsMaxC = 8, kClsMaxPieces = 4;  // H <= 32 lanes x 4 pieces x 8

__device__ __forceinline__ int cls_blocks(int B) {
  const int b = (B + 7) / 8;
  return b < 256 ? b : 256;
}

template <int CM>
__global__ __launch_bounds__(256) void cls_head_fwd(const bf16_t* __restrict__ x, const float* __restrict__ W,
                                                    const float* __restrict__ bias, const long* __restrict__ y,
                                                    float* __restrict__ prob, float* __restrict__ part, int B, int H,
                                                    int C) {
  __shared__ float red[8];
  const int hw = threadIdx.x >> 5, l = threadIdx.x & 31, npc = H / 8;
  float lsum = 0.f;
  for (long b = (long)blockIdx.x * 8 + hw; b < B; b += (long)gridDim.x * 8) {
    float z[CM];
#pragma unroll
    for (int c = 0; c < CM; c++) z[c] = 0.f;
    for (int j = l; j < npc; j += 32) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + b * H + j * 8), f);
#pragma unroll
      for (int c = 0; c < CM; c++) {
        if (c < C) {
          const float4 w0 = *reinterpret_cast<const float4*>(W + (long)c * H + j * 8);
          const float4 w1 = *reinterpret_cast<const float4*>(W + (long)c * H + j * 8 + 4);
          z[c] += f[0] * w0.x + f[1] * w0.y + f[2] * w0.z + f[3] * w0.w + f[4] * w1.x + f[5] * w1.y + f[6] * w1.z +
                  f[7] * w1.w;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < CM; c++)
#pragma unroll
      for (int o = 16; o; o >>= 1) z[c] += __shfl_xor(z[c], o, 32);
    if (l == 0) {
      float mx = -3.0e38f;
#pragma unroll
      for (int c = 0; c < CM; c++)
        if (c < C) {
          z[c] += bias[c];
          mx = fmaxf(mx, z[c]);
        }
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < CM; c++)
        if (c < C) se += expf(z[c] - mx);
      const float lse = mx + logf(se);
      const long yy = y[b];
      float zy = 0.f;
#pragma unroll
      for (int c = 0; c < CM; c++)
        if (c < C) {
          prob[b * C + c] = expf(z[c] - lse);
          if (c == yy) zy = z[c];
        }
      lsum += lse - zy;
    }
  }
  if (l == 0) red[hw] = lsum;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < 8; i++) t += red[i];
    part[blockIdx.x] = t;
  }
}

// loss[0] = sum(part[0..n)) / B, fixed order (one block)
__global__ __launch_bounds__(256) void cls_head_loss(const float* __restrict__ part, int n, int B,
                                                     float* __restrict__ loss) {
  __shared__ float red[256];
  float t = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) t += part[i];
  red[threadIdx.x] = t;
  __syncthreads();
  for (int o = 128; o; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = red[0] / (float)B;
}

// part: [gridDim.x][C * H + C] = per-block (dW | db)
template <int CM>
__global__ __launch_bounds__(256) void cls_head_bwd(const bf16_t* __restrict__ x, const float* __restrict__ W,
                                                    const long* __restrict__ y, const float* __restrict__ prob,
                                                    const float* __restrict__ dloss, bf16_t* __restrict__ dx,
                                                    float* __restrict__ part, int B, int H, int C) {
  extern __shared__ float sh[];  // [8][C * H + C]
  const int hw = threadIdx.x >> 5, l = threadIdx.x & 31, npc = H / 8, WC = C * H + C;
  const float gs = dloss[0] / (float)B;
  float acc[CM][kClsMaxPieces][8] = {};
  float bacc[CM] = {};
  for (long b = (long)blockIdx.x * 8 + hw; b < B; b += (long)gridDim.x * 8) {
    const long yy = y[b];
    float g[CM];
#pragma unroll
    for (int c = 0; c < CM; c++) {
      g[c] = c < C ? gs * (prob[b * C + c] - (c == yy ? 1.f : 0.f)) : 0.f;
      bacc[c] += g[c];
    }
#pragma unroll
    for (int q = 0; q < kClsMaxPieces; q++) {
      const int j = l + 32 * q;
      if (j < npc) {
        float f[8], o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        unpack8(*reinterpret_cast<const uint4*>(x + b * H + j * 8), f);
#pragma unroll
        for (int c = 0; c < CM; c++) {
          if (c < C) {
#pragma unroll
            for (int e = 0; e < 8; e++) {
              acc[c][q][e] += g[c] * f[e];
              o[e] += g[c] * W[(long)c * H + j * 8 + e];
            }
          }
        }
        *reinterpret_cast<uint4*>(dx + b * H + j * 8) = pack8(o);
      }
    }
  }
  float* mine = sh + hw * WC;
#pragma unroll
  for (int c = 0; c < CM; c++) {
    if (c < C) {
#pragma unroll
      for (int q = 0; q < kClsMaxPieces; q++) {
        const int j = l + 32 * q;
        if (j < npc)
#pragma unroll
          for (int e = 0; e < 8; e++) mine[c * H + j * 8 + e] = acc[c][q][e];
      }
      if (l == 0) mine[C * H + c] = bacc[c];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < WC; i += 256) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; k++) t += sh[k * WC + i];
    part[(long)blockIdx.x * WC + i] = t;
  }
}

// out[c] = sum over n partial rows of part[i][c], fixed order (16 columns x 16 row groups per block)
__global__ __launch_bounds__(256) void cls_head_reduce(const float* __restrict__ part, int n, int W,
                                                       float* __restrict__ out) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float t = 0.f;
  if (c < W)
    for (int i = g; i < n; i += 16) t += part[(long)i * W + c];
  red[g][cl] = t;
  __syncthreads();
  if (g == 0 && c < W) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; k++) s += red[k][cl];
    out[c] = s;
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

// blocks of the classifier-head kernels for B rows (partial rows of the backward)
KFA_API int kfa_cls_head_blocks(int B) { return (B + 7) / 8 < 256 ? (B + 7) / 8 : 256; }

// x [B][H] bf16, W [C][H] fp32, bias [C] fp32, labels [B] int64 -> prob [B][C] fp32, loss (one float);
// part: kfa_cls_head_blocks(B) floats.  C <= 8, H % 8 == 0, H <= 1024.
KFA_API int kfa_cls_head_fwd(const bf16_t* x, const float* W, const float* bias, const long* y, float* prob, float* part,
                             float* loss, int B, int H, int C, hipStream_t st) {
  if (B <= 0 || C <= 0 || C > kClsMaxC || H % 8 || H > 8 * 32 * kClsMaxPieces) return -1;
  const int nb = kfa_cls_head_blocks(B);
  if (C <= 2) hipLaunchKernelGGL(cls_head_fwd<2>, dim3(nb), dim3(256), 0, st, x, W, bias, y, prob, part, B, H, C);
  else hipLaunchKernelGGL(cls_head_fwd<kClsMaxC>, dim3(nb), dim3(256), 0, st, x, W, bias, y, prob, part, B, H, C);
  hipLaunchKernelGGL(cls_head_loss, dim3(1), dim3(256), 0, st, part, nb, B, loss);
  return kfa_status();
}

// dx [B][H] bf16 (written); grads [C * H + C] fp32 = (dW | db) (written); part: blocks x (C*H + C) floats.
// C * H <= 4096 (the per-block LDS image of 8 half-waves' partials: 8 x (C·H + C) floats <= 131 KB)
KFA_API int kfa_cls_head_bwd(const bf16_t* x, const float* W, const long* y, const float* prob, const float* dloss,
                             bf16_t* dx, float* part, float* grads, int B, int H, int C, hipStream_t st) {
  if (B <= 0 || C <= 0 || C > kClsMaxC || H % 8 || H > 8 * 32 * kClsMaxPieces || C * H > 4096) return -1;
  const int nb = kfa_cls_head_blocks(B), WC = C * H + C;
  const size_t lds = (size_t)8 * WC * 4;
  if (lds > 65536) {
    // the attribute is per function AND per device: both instances (C <= 2 reaches 65,600 B at
    // H = 1024, BERT-large NSP), raised once on every device this process launches on
    static unsigned long long done = 0;  // bit d: device d has both attributes
    int dev = 0;
    (void)hipGetDevice(&dev);
    const unsigned long long bit = 1ull << (dev & 63);
    if (!(__atomic_load_n(&done, __ATOMIC_ACQUIRE) & bit)) {
      const int cap = 8 * (4096 + kClsMaxC) * 4;
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&cls_head_bwd<kClsMaxC>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, cap);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&cls_head_bwd<2>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, cap);
      __atomic_fetch_or(&done, bit, __ATOMIC_RELEASE);
    }
  }
  if (C <= 2) hipLaunchKernelGGL(cls_head_bwd<2>, dim3(nb), dim3(256), lds, st, x, W, y, prob, dloss, dx, part, B, H, C);
  else hipLaunchKernelGGL(cls_head_bwd<kClsMaxC>, dim3(nb), dim3(256), lds, st, x, W, y, prob, dloss, dx, part, B, H, C);
  hipLaunchKernelGGL(cls_head_reduce, dim3((WC + 15) / 16), dim3(256), 0, st, part, nb, WC, grads);
  return kfa_status();
}
