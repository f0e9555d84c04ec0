// The ResNet stem (7x7 / stride 2 / pad 3 conv over 3 channels) on the
// implicit-GEMM MFMA kernels — SURVEY §2.6 K7.
//
// A 3-channel input cannot feed a BK = 64 (r, s, c) tap slice.  Space-to-depth
// turns the strided conv into a stride-1 one with enough channels:
//   xs[n][i][j][(di*2 + dj)*4 + c] = x[n][2i + di - pad][2j + dj - pad][c]   (c < 3, else 0)
//   ws[co][r'][s'][(di*2 + dj)*4 + c] = w[co][2r' + di][2s' + dj][c]        (in range, else 0)
//   y[n][p][q][co] = sum_{r',s'} xs[n][p + r'][q + s'][:] . ws[co][r'][s'][:]
// — a 4x4 / stride 1 / pad 0 conv over 16 channels whose 4 taps of one row are
// ONE contiguous 64-element (128-B) run of xs: exactly one BK slice of
// conv_igemm_kernel (kfa_conv_igemm accepts C = 16 when S*C = 64, pad 0).
// K = 256 instead of 147 (zero weights), but every operand load is a full
// 16-B, 128-B-coalesced LDS-DMA and the BatchNorm statistics stay fused.
// The weight gradient is the same conv's wgrad over xs (wgrad_kernel, C = 16),
// folded back onto the 7x7x3 taps.
#include "common.h"

namespace {

// one thread per xs pixel (16 channels = 32 B written as two 16-B stores)
__global__ void stem_s2d_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ xs, int Nb, int H, int W, int C,
                                int Hs, int Ws, int pad) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)Nb * Hs * Ws;
  if (idx >= total) return;
  const int j = (int)(idx % Ws);
  const long t = idx / Ws;
  const int i = (int)(t % Hs);
  const int n = (int)(t / Hs);
  uint32_t v[8];
#pragma unroll
  for (int d = 0; d < 4; d++) {
    const int h = 2 * i + (d >> 1) - pad, w = 2 * j + (d & 1) - pad;
    const bool ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
    const bf16_t* src = x + (((long)n * H + (ok ? h : 0)) * W + (ok ? w : 0)) * C;
    uint32_t e[4];
#pragma unroll
    for (int c = 0; c < 4; c++) e[c] = (ok && c < C) ? (uint32_t)src[c] : 0u;
    v[2 * d] = e[0] | (e[1] << 16);
    v[2 * d + 1] = e[2] | (e[3] << 16);
  }
  uint4* dst = reinterpret_cast<uint4*>(xs + idx * 16);
  dst[0] = make_uint4(v[0], v[1], v[2], v[3]);
  dst[1] = make_uint4(v[4], v[5], v[6], v[7]);
}

// w [Co][R][S][C] -> ws [Co][Rs][Ss][16]
__global__ void stem_weight_s2d_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ ws, int Co, int R, int S,
                                       int C, int Rs, int Ss) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = Co * Rs * Ss * 16;
  if (idx >= total) return;
  const int e = idx & 15, c = e & 3, d = e >> 2;
  int t = idx >> 4;
  const int s2 = t % Ss;
  t /= Ss;
  const int r2 = t % Rs, co = t / Rs;
  const int r = 2 * r2 + (d >> 1), s = 2 * s2 + (d & 1);
  ws[idx] = (r < R && s < S && c < C) ? w[((co * R + r) * S + s) * C + c] : (bf16_t)0;
}

// dW [Co][R][S][C] (+)= fold(dWs [Co][Rs][Ss][16] fp32)
__global__ void stem_wgrad_fold_kernel(const float* __restrict__ dws, void* __restrict__ dw, int f32, int accumulate,
                                       int Co, int R, int S, int C, int Rs, int Ss) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = Co * R * S * C;
  if (idx >= total) return;
  const int c = idx % C;
  int t = idx / C;
  const int s = t % S;
  t /= S;
  const int r = t % R, co = t / R;
  const float g = dws[((co * Rs + (r >> 1)) * Ss + (s >> 1)) * 16 + ((r & 1) * 2 + (s & 1)) * 4 + c];
  if (f32) {
    float* o = reinterpret_cast<float*>(dw) + idx;
    *o = accumulate ? *o + g : g;
  } else {
    bf16_t* o = reinterpret_cast<bf16_t*>(dw) + idx;
    *o = (bf16_t)f2bf(accumulate ? bf2f(*o) + g : g);
  }
}

}  // namespace

KFA_API int kfa_stem_s2d(const bf16_t* x, bf16_t* xs, int Nb, int H, int W, int C, int pad, hipStream_t st) {
  if (C > 4 || (H + 2 * pad) % 2 || (W + 2 * pad) % 2) return -1;
  const int Hs = (H + 2 * pad) / 2, Ws = (W + 2 * pad) / 2;
  const long total = (long)Nb * Hs * Ws;
  hipLaunchKernelGGL(stem_s2d_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, xs, Nb, H, W, C, Hs,
                     Ws, pad);
  return kfa_status();
}

KFA_API int kfa_stem_weight_s2d(const bf16_t* w, bf16_t* ws, int Co, int R, int S, int C, hipStream_t st) {
  if (C > 4) return -1;
  const int Rs = (R + 1) / 2, Ss = (S + 1) / 2;
  const int total = Co * Rs * Ss * 16;
  hipLaunchKernelGGL(stem_weight_s2d_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w, ws, Co, R, S, C, Rs, Ss);
  return kfa_status();
}

KFA_API int kfa_stem_wgrad_fold(const float* dws, void* dw, int f32, int accumulate, int Co, int R, int S, int C,
                                hipStream_t st) {
  if (C > 4) return -1;
  const int Rs = (R + 1) / 2, Ss = (S + 1) / 2;
  const int total = Co * R * S * C;
  hipLaunchKernelGGL(stem_wgrad_fold_kernel, dim3((total + 255) / 256), dim3(256), 0, st, dws, dw, f32, accumulate, Co,
                     R, S, C, Rs, Ss);
  return kfa_status();
}
