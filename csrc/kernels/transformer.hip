// Transformer building blocks for BERT / Wide&Deep (SURVEY §2.6 K1 epilogues,
// K6 embedding, K10 LayerNorm, K11 attention softmax).
//
// Everything here is bandwidth-bound, so every kernel is one streaming pass
// with 16-byte (8 x bf16) accesses, and the pieces an unfused graph would run
// as separate elementwise kernels are folded in:
//
//  * LayerNorm fwd: y = LN(res + dropout(x + bias)) — the residual add, the
//    bias of the producing GEMM and the hidden dropout ride along; the summed
//    input is stored (bf16) for backward.
//  * LayerNorm bwd: dx, the dropout-masked branch gradient, dgamma/dbeta and
//    the producing GEMM's dbias in one pass (column sums reduced in LDS per
//    block, then one fp32 atomic per column per block into the flat gradient).
//  * bias+activation fwd/bwd (GELU-erf / tanh / ReLU / identity) with fused
//    dbias column sums.
//  * QKV split (bias add + head split + 1/sqrt(d) scaling) and its inverse
//    (head merge + dbias), context head merge/split.
//  * masked, scaled softmax over attention scores with counter-hash dropout
//    (mask recomputed in backward, never stored) and its backward.
//  * multi-table embedding gather-sum and the sparse backward (fp32
//    scatter-add into a self-cleaning scratch, then a fold into the bf16/fp32
//    gradient that touches only the looked-up rows).
//
// Dropout RNG: keep(seed, i) = hash(seed, i) >= p * 2^32 — a stateless
// counter hash (drop_hash, common.h), so forward and backward regenerate the
// same mask from (seed, element index).
#include <cstdlib>

#include "common.h"

namespace {

constexpr int kRowsPerBlock = 4;  // one wave per row

__device__ __forceinline__ bool keep(uint64_t seed, uint64_t i, uint32_t thresh) {
  return drop_hash(seed, i) >= thresh;
}

#ifndef KFA_TF_LD_NT
#define KFA_TF_LD_NT 1  // BERT-base +0.8 % (docs/kernels.md)
#endif
__device__ __forceinline__ uint4 ld16(const bf16_t* p) {  // activation-sized inputs, read once per pass
#if KFA_TF_LD_NT
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v[0], v[1], v[2], v[3]);
#else
  return *reinterpret_cast<const uint4*>(p);
#endif
}
__device__ __forceinline__ void load8(const bf16_t* p, float f[8]) { unpack8(ld16(p), f); }
__device__ __forceinline__ void store8(bf16_t* p, const float f[8]) { *reinterpret_cast<uint4*>(p) = pack8(f); }
__device__ __forceinline__ void load8f(const float* p, float f[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// ----------------------------------------------------------------------------- LayerNorm
template <int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                     const float* __restrict__ bias, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, bf16_t* __restrict__ y,
                                                     bf16_t* __restrict__ xsum, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, long rows, int H, float eps,
                                                     uint32_t thresh, float dscale, uint64_t seed) {
  const long row = (long)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const long base = row * (long)H;
  float v[NV][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; j++) {
    const int c = (j * 64 + lane) * 8;
    if (c < H) {
      load8(x + base + c, v[j]);
      if (bias) {
        float b[8];
        load8f(bias + c, b);
#pragma unroll
        for (int e = 0; e < 8; e++) v[j][e] += b[e];
      }
      if (thresh) {
#pragma unroll
        for (int e = 0; e < 8; e++) v[j][e] = keep(seed, base + c + e, thresh) ? v[j][e] * dscale : 0.f;
      }
      if (res) {
        float r[8];
        load8(res + base + c, r);
#pragma unroll
        for (int e = 0; e < 8; e++) v[j][e] += r[e];
      }
#pragma unroll
      for (int e = 0; e < 8; e++) s += v[j][e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; e++) v[j][e] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)H;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NV; j++) {
    const int c = (j * 64 + lane) * 8;
    if (c < H) {
#pragma unroll
      for (int e = 0; e < 8; e++) { const float d = v[j][e] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)H + eps);
#pragma unroll
  for (int j = 0; j < NV; j++) {
    const int c = (j * 64 + lane) * 8;
    if (c < H) {
      if (xsum) store8(xsum + base + c, v[j]);
      float g[8], b[8], o[8];
      load8f(gamma + c, g);
      load8f(beta + c, b);
#pragma unroll
      for (int e = 0; e < 8; e++) o[e] = (v[j][e] - mean) * rstd * g[e] + b[e];
      store8(y + base + c, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Backward. Each block walks a contiguous chunk of rows, one wave per row;
// per-lane column accumulators are reduced across the 4 waves through LDS and
// each block adds its column sums to dgamma / dbeta / dbias (sum of the branch
// gradient) with one fp32 atomic per column (no partial buffer, no finalize
// launch).
// dy2 (nullable): a second gradient summed into dy on the fly — a residual join
// (dres + dbranch·W) whose GEMM then needs no addend epilogue (ops/transformer.py).
// DEEP: rows of the wave in flight ahead of the one being reduced (1 or 2):
// one row ahead leaves 8 waves x 1 row = ~36 KB of loads in flight per CU,
// about half of what hides an HBM miss (MI355X_MICROARCH.md); two rows ahead
// doubles it at +48 VGPRs (KFA_LN_BWD_DEEP).
// floats per (wave, column half) region of ln_bwd_kernel's block reduction: H / 2 plus a
// 16-dword shift (the column reads are ds_read_b32: bank = dword mod 32, so the two
// halves land on disjoint banks), dropped at H = 4096 to stay within 64 KB of LDS
__host__ __device__ __forceinline__ int ln_red_stride(int H) { return H / 2 + (H < 4096 ? 16 : 0); }

template <int NV, bool TWO, int DEEP>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ dy2,
                                                     const bf16_t* __restrict__ xs,
                                                     const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                                     const float* __restrict__ gamma, bf16_t* __restrict__ dx,
                                                     bf16_t* __restrict__ dbranch, float* __restrict__ o_gamma,
                                                     float* __restrict__ o_beta, float* __restrict__ o_bias, long rows,
                                                     int H, long rows_per_block, uint32_t thresh, float dscale,
                                                     uint64_t seed) {
  static_assert(DEEP == 1 || DEEP == 2, "rows in flight");
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4 waves][2 halves][H / 2 + 32]
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = min(rows, r0 + rows_per_block);
  float ag[NV][8], ab[NV][8], ad[NV][8];
#pragma unroll
  for (int j = 0; j < NV; j++)
#pragma unroll
    for (int e = 0; e < 8; e++) ag[j][e] = ab[j][e] = ad[j][e] = 0.f;

  // gamma is per column: in registers for the whole chunk (was re-read every row)
  float gm[NV][8];
#pragma unroll
  for (int j = 0; j < NV; j++) {
    const int c = (j * 64 + lane) * 8;
    if (c < H) load8f(gamma + c, gm[j]);
  }
  // software pipeline: the next DEEP rows' dy / x AND their mean / rstd are in
  // flight while this row reduces (slot S holds the rows row0 + S·4, + DEEP·4, ...)
  uint4 nd[DEEP][NV], nx[DEEP][NV], ne[DEEP][NV];
  float nmean[DEEP], nrstd[DEEP];
  auto fetch = [&](auto sc, long row) __attribute__((always_inline)) {
    constexpr int S = decltype(sc)::value;
    if (row < r1) {
      nmean[S] = mean_in[row];
      nrstd[S] = rstd_in[row];
    }
#pragma unroll
    for (int j = 0; j < NV; j++) {
      const int c = (j * 64 + lane) * 8;
      if (c < H && row < r1) {
        nd[S][j] = ld16(dy + row * (long)H + c);
        if constexpr (TWO) ne[S][j] = ld16(dy2 + row * (long)H + c);
        nx[S][j] = ld16(xs + row * (long)H + c);
      }
    }
  };
  auto process = [&](auto sc, long row) __attribute__((always_inline)) {
    constexpr int S = decltype(sc)::value;
    const long base = row * (long)H;
    const float mean = nmean[S], rstd = nrstd[S];
    uint4 cd[NV], cx[NV], ce[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) { cd[j] = nd[S][j]; cx[j] = nx[S][j]; ce[j] = ne[S][j]; }
    fetch(sc, row + DEEP * kRowsPerBlock);
    float xh[NV][8], g[NV][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NV; j++) {
      const int c = (j * 64 + lane) * 8;
      if (c < H) {
        float d[8], xv[8];
        unpack8(cd[j], d);
        if constexpr (TWO) {
          float d2[8];
          unpack8(ce[j], d2);
#pragma unroll
          for (int e = 0; e < 8; e++) d[e] += d2[e];
        }
        unpack8(cx[j], xv);
#pragma unroll
        for (int e = 0; e < 8; e++) {
          xh[j][e] = (xv[e] - mean) * rstd;
          g[j][e] = d[e] * gm[j][e];
          ag[j][e] += d[e] * xh[j][e];
          ab[j][e] += d[e];
          s1 += g[j][e] * xh[j][e];
          s2 += g[j][e];
        }
      }
    }
    const float c1 = wave_sum(s1) / (float)H, c2 = wave_sum(s2) / (float)H;
#pragma unroll
    for (int j = 0; j < NV; j++) {
      const int c = (j * 64 + lane) * 8;
      if (c < H) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; e++) o[e] = rstd * (g[j][e] - c2 - xh[j][e] * c1);
        store8(dx + base + c, o);
        if (thresh) {
#pragma unroll
          for (int e = 0; e < 8; e++) o[e] = keep(seed, base + c + e, thresh) ? o[e] * dscale : 0.f;
          if (dbranch) store8(dbranch + base + c, o);
        }
#pragma unroll
        for (int e = 0; e < 8; e++) ad[j][e] += o[e];
      }
    }
  };
  fetch(std::integral_constant<int, 0>{}, r0 + w);
  if constexpr (DEEP == 2) fetch(std::integral_constant<int, 1>{}, r0 + w + kRowsPerBlock);
  for (long row = r0 + w; row < r1; row += DEEP * kRowsPerBlock) {
    process(std::integral_constant<int, 0>{}, row);
    if constexpr (DEEP == 2)
      if (row + kRowsPerBlock < r1) process(std::integral_constant<int, 1>{}, row + kRowsPerBlock);
  }
  // block-reduce the three column accumulators
  auto reduce_out = [&](float (&acc)[NV][8], float* out) {
    if (!out) return;  // block-uniform
    // [wave][column half][8-column group][4]: lane-contiguous 16-B writes (the earlier
    // [wave][column] rows put 8 lanes on every bank), halves HS floats apart (see
    // ln_red_stride: the two halves' column reads land on disjoint banks)
    const int HS = ln_red_stride(H);
#pragma unroll
    for (int j = 0; j < NV; j++) {
      const int gi = j * 64 + lane;
      if (gi * 8 < H) {
        *reinterpret_cast<float4*>(red + (w * 2) * HS + gi * 4) = make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
        *reinterpret_cast<float4*>(red + (w * 2 + 1) * HS + gi * 4) = make_float4(acc[j][4], acc[j][5], acc[j][6], acc[j][7]);
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < H; c += 256) {
      const int o = ((c & 7) >> 2) * HS + (c >> 3) * 4 + (c & 3);
      atomicAdd(out + c, red[o] + red[2 * HS + o] + red[4 * HS + o] + red[6 * HS + o]);
    }
    __syncthreads();
  };
  reduce_out(ag, o_gamma);
  reduce_out(ab, o_beta);
  reduce_out(ad, o_bias);
}

// ----------------------------------------------------------------------------- bias + activation
enum Act { kNone = 0, kGelu = 1, kTanh = 2, kRelu = 3 };

__device__ __forceinline__ float act_f(float z, int act) {
  switch (act) {
    case kGelu: return gelu_f(z);
    case kTanh: return tanhf(z);
    case kRelu: return fmaxf(z, 0.f);
    default: return z;
  }
}

__device__ __forceinline__ float act_grad(float z, int act) {
  switch (act) {
    case kGelu: return gelu_grad(z);
    case kTanh: { const float t = tanhf(z); return 1.f - t * t; }
    case kRelu: return z > 0.f ? 1.f : 0.f;
    default: return 1.f;
  }
}

// y[r, c] = act(x[r, c] + b[c]); one thread per 8 columns, grid-stride rows,
// two 8-column groups per iteration with both loads issued before either is
// used; the activation is a template parameter (no per-element switch).
template <int ACT>
__global__ __launch_bounds__(256) void bias_act_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ b,
                                                           bf16_t* __restrict__ y, long rows, int N,
                                                           uint32_t thresh, float dscale, uint64_t seed) {
  const long nv = rows * (N / 8), stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nv; i += 2 * stride) {
    long idx[2] = {i, i + stride};
    float f[2][8];
#pragma unroll
    for (int u = 0; u < 2; u++) {
      if (idx[u] >= nv) break;
      const long r = idx[u] / (N / 8);
      const int c = (int)(idx[u] - r * (N / 8)) * 8;
      load8(x + r * N + c, f[u]);
      if (b) {
        float bb[8];
        load8f(b + c, bb);
#pragma unroll
        for (int e = 0; e < 8; e++) f[u][e] += bb[e];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; u++) {
      if (idx[u] >= nv) break;
      const long r = idx[u] / (N / 8);
      const int c = (int)(idx[u] - r * (N / 8)) * 8;
#pragma unroll
      for (int e = 0; e < 8; e++) f[u][e] = act_f(f[u][e], ACT);
      if (thresh)
#pragma unroll
        for (int e = 0; e < 8; e++) f[u][e] = keep(seed, r * N + c + e, thresh) ? f[u][e] * dscale : 0.f;
      store8(y + r * N + c, f[u]);
    }
  }
}

// dx = dy * act'(x + b), dbias partials.  Block = CL column-lanes (8 columns
// each) x 256/CL row-lanes; grid = (ceil(N / (8 CL)), row chunks).  CL = 16 for
// wide N keeps >= 2048 blocks in flight (memory-bound: 8 waves/CU are not enough
// outstanding loads) while each row still reads 256 contiguous bytes.
template <int CL>
__global__ __launch_bounds__(256) void bias_act_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                           const float* __restrict__ b, bf16_t* __restrict__ dx,
                                                           float* __restrict__ dbias, long rows, int N, int act,
                                                           long rows_per_block, uint32_t thresh, float dscale,
                                                           uint64_t seed, const float* __restrict__ gscale) {
  constexpr int RL = 256 / CL, W = CL * 8;
  constexpr int RS = CL * 4 + 16;  // [row-lane][column half][column-lane][4], halves 16 banks apart (see ln_red_stride)
  __shared__ __attribute__((aligned(16))) float red[RL * 2 * RS];
  const int cl = threadIdx.x % CL, rl = threadIdx.x / CL;
  const int c = blockIdx.x * W + cl * 8;
  const long r0 = (long)blockIdx.y * rows_per_block;
  const long r1 = min(rows, r0 + rows_per_block);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const float gs = gscale ? *gscale : 1.f;  // upstream gradient scalar (device-resident)
  if (c < N) {
    float bb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (b) load8f(b + c, bb);
#pragma unroll 2
    for (long r = r0 + rl; r < r1; r += RL) {
      float d[8], z[8];
      load8(dy + r * N + c, d);
      if (gscale)
#pragma unroll
        for (int e = 0; e < 8; e++) d[e] *= gs;
      if (thresh)
#pragma unroll
        for (int e = 0; e < 8; e++) d[e] = keep(seed, r * N + c + e, thresh) ? d[e] * dscale : 0.f;
      if (act != kNone) {
        load8(x + r * N + c, z);
#pragma unroll
        for (int e = 0; e < 8; e++) d[e] *= act_grad(z[e] + bb[e], act);
      }
      if (dx) store8(dx + r * N + c, d);
#pragma unroll
      for (int e = 0; e < 8; e++) acc[e] += d[e];
    }
  }
  *reinterpret_cast<float4*>(red + (rl * 2) * RS + cl * 4) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  *reinterpret_cast<float4*>(red + (rl * 2 + 1) * RS + cl * 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  __syncthreads();
  if (dbias)
    for (int k = threadIdx.x; k < W; k += 256) {
      const int cc = blockIdx.x * W + k;
      const int o = ((k & 7) >> 2) * RS + (k >> 3) * 4 + (k & 3);
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < RL; ++j) sum += red[j * 2 * RS + o];
      if (cc < N) atomicAdd(dbias + cc, sum);
    }
}

// ----------------------------------------------------------------------------- attention layout
// qkv [T, 3H] (+ bias) -> q, k, v  [B, h, S, d]; q scaled by `qscale`.
__global__ __launch_bounds__(256) void qkv_split_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ bias,
                                                        bf16_t* __restrict__ q, bf16_t* __restrict__ k,
                                                        bf16_t* __restrict__ v, long T, int S, int heads, int d,
                                                        float qscale) {
  const int H = heads * d, W = 3 * H;
  const long nv = T * (W / 8);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nv; i += (long)gridDim.x * 256) {
    const long t = i / (W / 8);
    const int c = (int)(i - t * (W / 8)) * 8;
    const int which = c / H, cc = c - which * H, hh = cc / d, dd = cc - hh * d;
    const long b = t / S, s = t - b * S;
    float f[8];
    load8(qkv + t * W + c, f);
    if (bias) {
      float bb[8];
      load8f(bias + c, bb);
#pragma unroll
      for (int e = 0; e < 8; e++) f[e] += bb[e];
    }
    if (which == 0)
#pragma unroll
      for (int e = 0; e < 8; e++) f[e] *= qscale;
    bf16_t* dst = which == 0 ? q : (which == 1 ? k : v);
    store8(dst + ((b * heads + hh) * S + s) * d + dd, f);
  }
}

// inverse: dq, dk, dv [B,h,S,d] -> dqkv [T, 3H] (dq scaled by qscale) + dbias partials
__global__ __launch_bounds__(256) void qkv_merge_bwd_kernel(const bf16_t* __restrict__ dq, const bf16_t* __restrict__ dk,
                                                            const bf16_t* __restrict__ dv, bf16_t* __restrict__ dqkv,
                                                            float* __restrict__ dbias, long T, int S, int heads, int d,
                                                            float qscale, long rows_per_block) {
  __shared__ float red[4][512];
  const int H = heads * d, W = 3 * H;
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 512 + cl * 8;
  const long r0 = (long)blockIdx.y * rows_per_block;
  const long r1 = min(T, r0 + rows_per_block);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c < W) {
    const int which = c / H, cc = c - which * H, hh = cc / d, dd = cc - hh * d;
    const bf16_t* src = which == 0 ? dq : (which == 1 ? dk : dv);
    const float sc = which == 0 ? qscale : 1.f;
    for (long t = r0 + rl; t < r1; t += 4) {
      const long b = t / S, s = t - b * S;
      float f[8];
      load8(src + ((b * heads + hh) * S + s) * d + dd, f);
#pragma unroll
      for (int e = 0; e < 8; e++) { f[e] *= sc; acc[e] += f[e]; }
      store8(dqkv + t * W + c, f);
    }
  }
#pragma unroll
  for (int e = 0; e < 8; e++) red[rl][cl * 8 + e] = acc[e];
  __syncthreads();
  if (dbias)
    for (int k = threadIdx.x; k < 512; k += 256) {
      const int cc = blockIdx.x * 512 + k;
      if (cc < W) atomicAdd(dbias + cc, red[0][k] + red[1][k] + red[2][k] + red[3][k]);
    }
}

// [B,h,S,d] <-> [T, H]  (to_rows=1: heads -> rows)
__global__ __launch_bounds__(256) void heads_permute_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                            long T, int S, int heads, int d, int to_rows) {
  const int H = heads * d;
  const long nv = T * (H / 8);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nv; i += (long)gridDim.x * 256) {
    const long t = i / (H / 8);
    const int c = (int)(i - t * (H / 8)) * 8;
    const int hh = c / d, dd = c - hh * d;
    const long b = t / S, s = t - b * S;
    const long hi = ((b * heads + hh) * S + s) * d + dd, ri = t * H + c;
    *reinterpret_cast<uint4*>(dst + (to_rows ? ri : hi)) = *reinterpret_cast<const uint4*>(src + (to_rows ? hi : ri));
  }
}

// ----------------------------------------------------------------------------- attention softmax
// rows of S scores (bf16, q pre-scaled); key_bias [B, S] additive (nullable).
// G = lanes per row (S/8 clamped to 64), 64/G rows per wave.
template <int G, int NV>
__global__ __launch_bounds__(256) void attn_softmax_fwd_kernel(bf16_t* __restrict__ sc, const float* __restrict__ key_bias,
                                                               bf16_t* __restrict__ pdrop, long rows, int S, int heads,
                                                               uint32_t thresh, float dscale, uint64_t seed) {
  constexpr int RPW = 64 / G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long row = ((long)blockIdx.x * 4 + w) * RPW + lane / G;
  const int gl = lane % G;
  const bool valid = row < rows;
  const long b = valid ? row / ((long)heads * S) : 0;
  float m = -INFINITY;
  float f[NV][8];  // the row lives in registers: S == 8 * G * NV
#pragma unroll
  for (int j = 0; j < NV; j++) {
    if (valid) {
      const int c = (j * G + gl) * 8;
      load8(sc + row * S + c, f[j]);
      if (key_bias) {
        float kb[8];
        load8f(key_bias + b * S + c, kb);
#pragma unroll
        for (int e = 0; e < 8; e++) f[j][e] += kb[e];
      }
#pragma unroll
      for (int e = 0; e < 8; e++) m = fmaxf(m, f[j][e]);
    }
  }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; j++)
    if (valid)
#pragma unroll
      for (int e = 0; e < 8; e++) { f[j][e] = __expf(f[j][e] - m); s += f[j][e]; }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float inv = 1.f / s;
#pragma unroll
  for (int j = 0; j < NV; j++) {
    if (valid) {
      const int c = (j * G + gl) * 8;
#pragma unroll
      for (int e = 0; e < 8; e++) f[j][e] *= inv;
      store8(sc + row * S + c, f[j]);
      if (pdrop) {
#pragma unroll
        for (int e = 0; e < 8; e++) f[j][e] = keep(seed, row * S + c + e, thresh) ? f[j][e] * dscale : 0.f;
        store8(pdrop + row * S + c, f[j]);
      }
    }
  }
}

// dS = P * (dP - sum(P * dP)),  dP = keep ? dPdrop * dscale : 0.  In place on dp.
template <int G, int NV>
__global__ __launch_bounds__(256) void attn_softmax_bwd_kernel(const bf16_t* __restrict__ p, bf16_t* __restrict__ dp,
                                                               long rows, int S, uint32_t thresh, float dscale,
                                                               uint64_t seed) {
  constexpr int RPW = 64 / G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long row = ((long)blockIdx.x * 4 + w) * RPW + lane / G;
  const int gl = lane % G;
  const bool valid = row < rows;
  float pv[NV][8], dv[NV][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; j++) {
    if (valid) {
      const int c = (j * G + gl) * 8;
      load8(p + row * S + c, pv[j]);
      load8(dp + row * S + c, dv[j]);
#pragma unroll
      for (int e = 0; e < 8; e++) {
        if (thresh) dv[j][e] = keep(seed, row * S + c + e, thresh) ? dv[j][e] * dscale : 0.f;
        s += pv[j][e] * dv[j][e];
      }
    }
  }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
#pragma unroll
  for (int j = 0; j < NV; j++) {
    if (valid) {
      const int c = (j * G + gl) * 8;
#pragma unroll
      for (int e = 0; e < 8; e++) dv[j][e] = pv[j][e] * (dv[j][e] - s);
      store8(dp + row * S + c, dv[j]);
    }
  }
}

// ----------------------------------------------------------------------------- embeddings
// out[r] = sum_k tab_k[ids_k[r]] (k < 3, nullable), tables bf16 or fp32 (D % 8 == 0)
template <bool F32>
__device__ __forceinline__ void load_row8(const void* tab, long row, int D, int c, float f[8]) {
  if (F32) load8f(reinterpret_cast<const float*>(tab) + row * D + c, f);
  else load8(reinterpret_cast<const bf16_t*>(tab) + row * D + c, f);
}

__global__ __launch_bounds__(256) void embed_fwd_kernel(const long* __restrict__ i0, const void* __restrict__ t0,
                                                        const long* __restrict__ i1, const void* __restrict__ t1,
                                                        const long* __restrict__ i2, const void* __restrict__ t2,
                                                        int f32mask, bf16_t* __restrict__ out, long n, int D,
                                                        long ostride) {
  const long nv = n * (D / 8);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nv; i += (long)gridDim.x * 256) {
    const long r = i / (D / 8);
    const int c = (int)(i - r * (D / 8)) * 8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, f[8];
    const long* ids[3] = {i0, i1, i2};
    const void* tabs[3] = {t0, t1, t2};
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (!tabs[k]) continue;
      const long row = ids[k] ? ids[k][r] : r;
      if (f32mask & (1 << k)) load_row8<true>(tabs[k], row, D, c, f);
      else load_row8<false>(tabs[k], row, D, c, f);
#pragma unroll
      for (int e = 0; e < 8; e++) acc[e] += f[e];
    }
    store8(out + r * ostride + c, acc);
  }
}

// scratch[ids[r]] += dout[r]  (fp32 atomics; scratch is kept all-zero between calls)
// One element per lane: the 64 lanes of a wave touch 64 consecutive floats of one
// scratch row (one 256-B atomic wave-instruction).  (8 elements per lane made
// every atomic instruction span 2 KiB in 32-B steps: ~9x slower.)
__global__ __launch_bounds__(256) void embed_bwd_scatter_kernel(const long* __restrict__ ids,
                                                                const bf16_t* __restrict__ dout, long dstride,
                                                                float* __restrict__ scratch, long n, int D) {
  const long ne = n * D;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < ne; i += (long)gridDim.x * 256) {
    const long r = i / D;
    const int c = (int)(i - r * D);
    const long row = ids ? ids[r] : r;
    atomicAdd(scratch + row * D + c, bf2f(dout[r * dstride + c]));
  }
}

// grad[row] += exchange(scratch[row], 0) for every looked-up row; the atomic
// exchange hands each element's sum to exactly one occurrence, the others see
// 0 and skip the write, and the scratch is left zeroed for the next call.
// One element per lane (contiguous 256-B wave accesses), as the scatter.
__global__ __launch_bounds__(256) void embed_bwd_fold_kernel(const long* __restrict__ ids, float* __restrict__ scratch,
                                                             void* __restrict__ grad, int grad_f32, long n, int D,
                                                             int accumulate) {
  const long ne = n * D;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < ne; i += (long)gridDim.x * 256) {
    const long r = i / D;
    const int c = (int)(i - r * D);
    const long row = ids ? ids[r] : r;
    const float v = __hip_atomic_exchange(scratch + row * D + c, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == 0.f) continue;
    if (grad_f32) {
      float* g = reinterpret_cast<float*>(grad) + row * D + c;
      *g = accumulate ? *g + v : v;
    } else {
      bf16_t* g = reinterpret_cast<bf16_t*>(grad) + row * D + c;
      *g = (bf16_t)f2bf(accumulate ? bf2f(*g) + v : v);
    }
  }
}

// Gradient of a TINY table (R <= 8 rows: BERT's segment / token-type embedding)
// — grad[ids[r]] += dout[r] — where every token hits one of a few rows: global
// atomics serialise on them and the one-hot GEMM has M = R (hipBLASLt ran it at
// ~140 us for R = 2).  Two launches:
//  1. block (column group of 64, token chunk): a wave takes 8 rows x 64 columns per
//     step (lane = row lane / 8, 8 columns lane % 8: 16-B loads, 4 steps in flight)
//     and adds each row into register accumulators acc[R][8] (a select per table
//     row: no dynamic register indexing); then the 8 row-lanes and the 4 waves of
//     the block are summed (shuffles, LDS) and the block stores a partial [chunk][R][D];
//  2. grad[r][c] += Σ_chunk partial[chunk][r][c] in chunk order (deterministic),
//     into an fp32 or a bf16 gradient.
// (An LDS-atomic version for tables up to 512 rows ran 174 us per table — slower
// than the one-hot MFMA GEMM the position table keeps: 38 us.)
constexpr int kSmallTabMaxRows = 8;
constexpr int kSmallTabChunks = 32;

template <int RM>
__global__ __launch_bounds__(256) void embed_small_part_kernel(const long* __restrict__ ids,
                                                               const bf16_t* __restrict__ dout, long dstride,
                                                               float* __restrict__ part, long n, int D, int R,
                                                               long rows_per_block) {
  __shared__ float red[4][RM][64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int c0 = blockIdx.x * 64, rs = lane >> 3, cc = (lane & 7) * 8;
  float acc[RM][8];
#pragma unroll
  for (int q = 0; q < RM; q++)
#pragma unroll
    for (int e = 0; e < 8; e++) acc[q][e] = 0.f;
  const long r0 = (long)blockIdx.y * rows_per_block, r1 = min(n, r0 + rows_per_block);
  const bool live = c0 + cc < D;  // D % 8 == 0: a lane's 8 columns are all in or all out
  for (long r = r0 + w * 8 + rs; r < r1 + 96; r += 128) {
    long id[4];
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const long rr = r + 32 * j;
      const bool ok = rr < r1 && live;
      id[j] = ok ? ids[rr] : -1;
      v[j] = ok ? *reinterpret_cast<const uint4*>(dout + rr * dstride + c0 + cc) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      float f[8];
      unpack8(v[j], f);
#pragma unroll
      for (int q = 0; q < RM; q++) {
        const float m = id[j] == q ? 1.f : 0.f;
#pragma unroll
        for (int e = 0; e < 8; e++) acc[q][e] = fmaf(m, f[e], acc[q][e]);
      }
    }
  }
  // sum the 8 row-lanes sharing a column chunk (lane bits 3..5), then the 4 waves
#pragma unroll
  for (int q = 0; q < RM; q++)
#pragma unroll
    for (int e = 0; e < 8; e++) {
      float x = acc[q][e];
      x += __shfl_xor(x, 8, 64);
      x += __shfl_xor(x, 16, 64);
      x += __shfl_xor(x, 32, 64);
      acc[q][e] = x;
    }
  if (rs == 0)
#pragma unroll
    for (int q = 0; q < RM; q++)
#pragma unroll
      for (int e = 0; e < 8; e++) red[w][q][cc + e] = acc[q][e];
  __syncthreads();
  float* dst = part + (long)blockIdx.y * R * D;
  for (int i = t; i < R * 64; i += 256) {
    const int q = i >> 6, c = i & 63;
    if (c0 + c < D) dst[(long)q * D + c0 + c] = red[0][q][c] + red[1][q][c] + red[2][q][c] + red[3][q][c];
  }
}

__global__ __launch_bounds__(256) void embed_small_reduce_kernel(const float* __restrict__ part, int chunks, long RD,
                                                                 void* __restrict__ grad, int grad_f32) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < RD; i += (long)gridDim.x * 256) {
    float s = 0.f;
    for (int k = 0; k < chunks; k++) s += part[k * RD + i];
    if (grad_f32) {
      reinterpret_cast<float*>(grad)[i] += s;
    } else {
      bf16_t* g = reinterpret_cast<bf16_t*>(grad) + i;
      *g = (bf16_t)f2bf(bf2f(*g) + s);
    }
  }
}

int grid_for(long nvec) {
  long g = (nvec + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

uint32_t drop_thresh(float p) {
  if (p <= 0.f) return 0u;
  const double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 4294967295u : (uint32_t)t;
}

}  // namespace

// ============================================================================= C ABI
static long ln_bwd_blocks(long rows) { return rows < 2048 ? (rows + 3) / 4 : 512; }

KFA_API long kfa_ln_part_floats(long rows, int H) {  // no scratch needed any more (ABI stability)
  (void)rows; (void)H;
  return 0;
}

namespace {
template <int NV>
void launch_ln_fwd(dim3 g, hipStream_t s, const void* x, const void* res, const float* bias, const float* gamma,
                   const float* beta, void* y, void* xsum, float* mean, float* rstd, long rows, int H, float eps,
                   uint32_t th, float ds, uint64_t seed) {
  hipLaunchKernelGGL(ln_fwd_kernel<NV>, g, dim3(256), 0, s, (const bf16_t*)x, (const bf16_t*)res, bias, gamma, beta,
                     (bf16_t*)y, (bf16_t*)xsum, mean, rstd, rows, H, eps, th, ds, seed);
}
template <int NV>
void launch_ln_bwd(dim3 g, size_t lds, hipStream_t s, const void* dy, const void* dy2, const void* xs,
                   const float* mean, const float* rstd, const float* gamma, void* dx, void* dbranch, float* o0,
                   float* o1, float* o2, long rows, int H, long rpb, uint32_t th, float ds, uint64_t seed) {
  static int deep = -1;
  if (deep < 0) {
    const char* e = getenv("KFA_LN_BWD_DEEP");
    deep = (e && e[0] == '2') ? 2 : 1;
  }
#define KFA_LNB(TW, D)                                                                                              \
  hipLaunchKernelGGL((ln_bwd_kernel<NV, TW, D>), g, dim3(256), lds, s, (const bf16_t*)dy,                          \
                     TW ? (const bf16_t*)dy2 : nullptr, (const bf16_t*)xs, mean, rstd, gamma, (bf16_t*)dx,          \
                     (bf16_t*)dbranch, o0, o1, o2, rows, H, rpb, th, ds, seed)
  if (dy2 && deep == 2) KFA_LNB(true, 2);
  else if (dy2) KFA_LNB(true, 1);
  else if (deep == 2) KFA_LNB(false, 2);
  else KFA_LNB(false, 1);
#undef KFA_LNB
}
template <int G, int NV>
void launch_sm_fwd(hipStream_t s, void* scores, const float* key_bias, void* pdrop, long rows, int S, int heads,
                   uint32_t th, float ds, uint64_t seed) {
  const long rpb = 4 * (64 / G);
  hipLaunchKernelGGL((attn_softmax_fwd_kernel<G, NV>), dim3((unsigned)((rows + rpb - 1) / rpb)), dim3(256), 0, s,
                     (bf16_t*)scores, key_bias, th ? (bf16_t*)pdrop : nullptr, rows, S, heads, th, ds, seed);
}
template <int G, int NV>
void launch_sm_bwd(hipStream_t s, const void* probs, void* dp, long rows, int S, uint32_t th, float ds,
                   uint64_t seed) {
  const long rpb = 4 * (64 / G);
  hipLaunchKernelGGL((attn_softmax_bwd_kernel<G, NV>), dim3((unsigned)((rows + rpb - 1) / rpb)), dim3(256), 0, s,
                     (const bf16_t*)probs, (bf16_t*)dp, rows, S, th, ds, seed);
}
}  // namespace

KFA_API int kfa_ln_fwd(const void* x, const void* res, const float* bias, const float* gamma, const float* beta,
                       void* y, void* xsum, float* mean, float* rstd, long rows, int H, float eps, float p,
                       unsigned long long seed, hipStream_t s) {
  if (rows <= 0 || H % 8 || H > 4096) return -1;
  const uint32_t th = drop_thresh(p);
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  dim3 g((unsigned)((rows + kRowsPerBlock - 1) / kRowsPerBlock));
  if (H <= 512) launch_ln_fwd<1>(g, s, x, res, bias, gamma, beta, y, xsum, mean, rstd, rows, H, eps, th, ds, seed);
  else if (H <= 1024) launch_ln_fwd<2>(g, s, x, res, bias, gamma, beta, y, xsum, mean, rstd, rows, H, eps, th, ds, seed);
  else if (H <= 2048) launch_ln_fwd<4>(g, s, x, res, bias, gamma, beta, y, xsum, mean, rstd, rows, H, eps, th, ds, seed);
  else launch_ln_fwd<8>(g, s, x, res, bias, gamma, beta, y, xsum, mean, rstd, rows, H, eps, th, ds, seed);
  return kfa_status();
}

static void zero_if(float* p, int n, int accumulate, hipStream_t s) {
  if (p && !accumulate) (void)hipMemsetAsync(p, 0, (size_t)n * sizeof(float), s);
}

// dgamma/dbeta/dbias: fp32, (+)= when accumulate (else overwritten); any may be
// null.  `part` is unused (kept for ABI stability).
// dy2 (nullable): second gradient, the kernel's dy is dy + dy2.
KFA_API int kfa_ln_bwd2(const void* dy, const void* dy2, const void* xs, const float* mean, const float* rstd,
                        const float* gamma, void* dx, void* dbranch, float* part, float* dgamma, float* dbeta,
                        float* dbias, long rows, int H, float p, unsigned long long seed, int accumulate,
                        hipStream_t s) {
  (void)part;
  if (rows <= 0 || H % 8 || H > 4096) return -1;
  const long nblk = ln_bwd_blocks(rows);
  const long rpb = (rows + nblk - 1) / nblk;
  const uint32_t th = drop_thresh(p);
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const size_t lds = 8 * (size_t)ln_red_stride(H) * sizeof(float);  // ln_bwd_kernel's reduction layout
  zero_if(dgamma, H, accumulate, s);
  zero_if(dbeta, H, accumulate, s);
  zero_if(dbias, H, accumulate, s);
  dim3 g((unsigned)nblk);
#define LNB(NV) launch_ln_bwd<NV>(g, lds, s, dy, dy2, xs, mean, rstd, gamma, dx, dbranch, dgamma, dbeta, dbias, rows, \
                                  H, rpb, th, ds, seed)
  if (H <= 512) LNB(1);
  else if (H <= 1024) LNB(2);
  else if (H <= 2048) LNB(4);
  else LNB(8);
#undef LNB
  return kfa_status();
}

KFA_API int kfa_ln_bwd(const void* dy, const void* xs, const float* mean, const float* rstd, const float* gamma,
                       void* dx, void* dbranch, float* part, float* dgamma, float* dbeta, float* dbias, long rows,
                       int H, float p, unsigned long long seed, int accumulate, hipStream_t s) {
  return kfa_ln_bwd2(dy, nullptr, xs, mean, rstd, gamma, dx, dbranch, part, dgamma, dbeta, dbias, rows, H, p, seed,
                     accumulate, s);
}

KFA_API int kfa_bias_act_fwd(const void* x, const float* b, void* y, long rows, int N, int act, float p,
                             unsigned long long seed, hipStream_t s) {
  if (rows <= 0 || N % 8) return -1;
  const uint32_t th = drop_thresh(p);
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const dim3 g(grid_for((rows * (N / 8) + 1) / 2));  // two 8-column groups per thread per iteration
#define KFA_BAF(A) \
  hipLaunchKernelGGL(bias_act_fwd_kernel<A>, g, dim3(256), 0, s, (const bf16_t*)x, b, (bf16_t*)y, rows, N, th, ds, \
                     (uint64_t)seed)
  if (act == kGelu) KFA_BAF(kGelu);
  else if (act == kTanh) KFA_BAF(kTanh);
  else if (act == kRelu) KFA_BAF(kRelu);
  else KFA_BAF(kNone);
#undef KFA_BAF
  return kfa_status();
}

// row chunks of the column-sum producers: ~16 rows per block-lane pass, capped
static long colsum_chunks(long rows) { return rows < 1024 ? (rows + 15) / 16 : (rows < 8192 ? 64 : 256); }

KFA_API long kfa_colsum_part_floats(long rows, int N) {  // no scratch needed any more (ABI stability)
  (void)rows; (void)N;
  return 0;
}

// dx = dropout_mask(dy) * act'(x + b) (dx nullable: then only dbias is produced);
// dbias (+)= column sums of dx (fp32 atomics, one per column per block).
static int bias_act_bwd_launch(const void* dy, const void* x, const float* b, void* dx, float* dbias, long rows,
                               int N, int act, float p, unsigned long long seed, int accumulate, const float* gscale,
                               hipStream_t s);

KFA_API int kfa_bias_act_bwd(const void* dy, const void* x, const float* b, void* dx, float* part, float* dbias,
                             long rows, int N, int act, float p, unsigned long long seed, int accumulate,
                             hipStream_t s) {
  (void)part;
  return bias_act_bwd_launch(dy, x, b, dx, dbias, rows, N, act, p, seed, accumulate, nullptr, s);
}

// dx = dy * (*gscale) (dx must not alias dy) and dbias (+)= its column sums, one pass: the tied
// MLM decoder's backward scales the loss kernel's dlogits by the upstream gradient and
// takes the decoder-bias gradient in the same read (was a torch mul_ + a column-sum pass)
KFA_API int kfa_scale_colsum(const void* dy, void* dx, float* dbias, long rows, int N, const float* gscale,
                             int accumulate, hipStream_t s) {
  return bias_act_bwd_launch(dy, nullptr, nullptr, dx, dbias, rows, N, kNone, 0.f, 0ull, accumulate, gscale, s);
}

static int bias_act_bwd_launch(const void* dy, const void* x, const float* b, void* dx, float* dbias, long rows,
                               int N, int act, float p, unsigned long long seed, int accumulate, const float* gscale,
                               hipStream_t s) {
  if (rows <= 0 || N % 8) return -1;
  const long chunks = colsum_chunks(rows);
  const long rpb = (rows + chunks - 1) / chunks;
  const uint32_t th = drop_thresh(p);
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  zero_if(dbias, N, accumulate, s);
  static const int cl16 = [] { const char* e = getenv("KFA_BIAS_ACT_CL16"); return e ? atoi(e) : 1; }();
  // KFA_BIAS_ACT_RPB: minimum rows per block of the CL = 16 form (A/B override).  Default 64
  // (4 rows per thread) on wide N; 256 when N <= 512 (two to four column blocks), where
  // reaching 2048 blocks left each thread 4 rows and the block reduction + atomics
  // dominated: W&D 34.99-35.03 -> 35.49-35.67 M ex/s, BERT (N >= 768) 10,114-10,135 with
  // 64 vs 10,081-10,092 with 256 everywhere (tools/gpu_r6_barpb.sh)
  static const long rpb_env = [] { const char* e = getenv("KFA_BIAS_ACT_RPB"); return e && atol(e) > 0 ? atol(e) : 0L; }();
  if (N >= 128 && cl16) {
    // >= 2048 blocks, >= min_rpb / 16 rows per thread; the dbias atomics stay at <= max(chunks, 256) per column
    const long bx = (N + 127) / 128;
    const long min_rpb = rpb_env > 0 ? rpb_env : (bx <= 4 ? 256L : 64L);
    const long want = std::max(chunks, (2048 + bx - 1) / bx);
    const long ch = std::max(1L, std::min(want, (rows + min_rpb - 1) / min_rpb));
    const long rp = (rows + ch - 1) / ch;
    hipLaunchKernelGGL(bias_act_bwd_kernel<16>, dim3((unsigned)bx, (unsigned)ch), dim3(256), 0, s,
                       (const bf16_t*)dy, (const bf16_t*)x, b, (bf16_t*)dx, dbias, rows, N, act, rp, th, ds,
                       (uint64_t)seed, gscale);
    return kfa_status();
  }
  hipLaunchKernelGGL(bias_act_bwd_kernel<64>, dim3((N + 511) / 512, (unsigned)chunks), dim3(256), 0, s,
                     (const bf16_t*)dy, (const bf16_t*)x, b, (bf16_t*)dx, dbias, rows, N, act, rpb, th, ds,
                     (uint64_t)seed, gscale);
  return kfa_status();
}

KFA_API int kfa_qkv_split(const void* qkv, const float* bias, void* q, void* k, void* v, long T, int S, int heads,
                          int d, float qscale, hipStream_t s) {
  if (T <= 0 || T % S || d % 8) return -1;
  hipLaunchKernelGGL(qkv_split_kernel, dim3(grid_for(T * 3 * heads * d / 8)), dim3(256), 0, s, (const bf16_t*)qkv,
                     bias, (bf16_t*)q, (bf16_t*)k, (bf16_t*)v, T, S, heads, d, qscale);
  return kfa_status();
}

KFA_API int kfa_qkv_merge_bwd(const void* dq, const void* dk, const void* dv, void* dqkv, float* part, float* dbias,
                              long T, int S, int heads, int d, float qscale, int accumulate, hipStream_t s) {
  (void)part;
  if (T <= 0 || T % S || d % 8) return -1;
  const int W = 3 * heads * d;
  const long chunks = colsum_chunks(T);
  const long rpb = (T + chunks - 1) / chunks;
  zero_if(dbias, W, accumulate, s);
  hipLaunchKernelGGL(qkv_merge_bwd_kernel, dim3((W + 511) / 512, (unsigned)chunks), dim3(256), 0, s,
                     (const bf16_t*)dq, (const bf16_t*)dk, (const bf16_t*)dv, (bf16_t*)dqkv, dbias, T, S, heads, d,
                     qscale, rpb);
  return kfa_status();
}

KFA_API int kfa_heads_permute(const void* src, void* dst, long T, int S, int heads, int d, int to_rows,
                              hipStream_t s) {
  if (T <= 0 || T % S || d % 8) return -1;
  hipLaunchKernelGGL(heads_permute_kernel, dim3(grid_for(T * heads * d / 8)), dim3(256), 0, s, (const bf16_t*)src,
                     (bf16_t*)dst, T, S, heads, d, to_rows);
  return kfa_status();
}

static int sm_supported(int S) { return S == 64 || S == 128 || S == 256 || S == 512 || S == 1024 || S == 2048; }

KFA_API int kfa_attn_softmax_fwd(void* scores, const float* key_bias, void* pdrop, long rows, int S, int heads,
                                 float p, unsigned long long seed, hipStream_t s) {
  if (rows <= 0 || !sm_supported(S)) return -1;
  const uint32_t th = drop_thresh(p);
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  switch (S) {
    case 64: launch_sm_fwd<8, 1>(s, scores, key_bias, pdrop, rows, S, heads, th, ds, seed); break;
    case 128: launch_sm_fwd<16, 1>(s, scores, key_bias, pdrop, rows, S, heads, th, ds, seed); break;
    case 256: launch_sm_fwd<32, 1>(s, scores, key_bias, pdrop, rows, S, heads, th, ds, seed); break;
    case 512: launch_sm_fwd<64, 1>(s, scores, key_bias, pdrop, rows, S, heads, th, ds, seed); break;
    case 1024: launch_sm_fwd<64, 2>(s, scores, key_bias, pdrop, rows, S, heads, th, ds, seed); break;
    default: launch_sm_fwd<64, 4>(s, scores, key_bias, pdrop, rows, S, heads, th, ds, seed); break;
  }
  return kfa_status();
}

KFA_API int kfa_attn_softmax_bwd(const void* probs, void* dp, long rows, int S, float p, unsigned long long seed,
                                 hipStream_t s) {
  if (rows <= 0 || !sm_supported(S)) return -1;
  const uint32_t th = drop_thresh(p);
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  switch (S) {
    case 64: launch_sm_bwd<8, 1>(s, probs, dp, rows, S, th, ds, seed); break;
    case 128: launch_sm_bwd<16, 1>(s, probs, dp, rows, S, th, ds, seed); break;
    case 256: launch_sm_bwd<32, 1>(s, probs, dp, rows, S, th, ds, seed); break;
    case 512: launch_sm_bwd<64, 1>(s, probs, dp, rows, S, th, ds, seed); break;
    case 1024: launch_sm_bwd<64, 2>(s, probs, dp, rows, S, th, ds, seed); break;
    default: launch_sm_bwd<64, 4>(s, probs, dp, rows, S, th, ds, seed); break;
  }
  return kfa_status();
}

KFA_API int kfa_embed_fwd(const long* i0, const void* t0, const long* i1, const void* t1, const long* i2,
                          const void* t2, int f32mask, void* out, long n, int D, long ostride, hipStream_t s) {
  if (n <= 0 || D % 8 || ostride % 8) return -1;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(grid_for(n * (D / 8))), dim3(256), 0, s, i0, t0, i1, t1, i2, t2, f32mask,
                     (bf16_t*)out, n, D, ostride);
  return kfa_status();
}

// scratch: zero-initialised fp32 [rows_of_table, D], left zeroed on return.
// scratch floats kfa_embed_small_bwd needs (the per-chunk partial images)
KFA_API long kfa_embed_small_ws_floats(int R, int D) { return (long)kSmallTabChunks * R * D; }

// grad [R][D] (fp32 or bf16) += sum of dout rows by id, R <= 8, D % 8 == 0 (ids outside
// [0, R) skipped); part: kfa_embed_small_ws_floats(R, D) floats of scratch
KFA_API int kfa_embed_small_bwd(const long* ids, const void* dout, long dstride, void* grad, int grad_f32, long n,
                                int D, int R, float* part, hipStream_t s) {
  if (n <= 0) return 0;
  if (R <= 0 || R > kSmallTabMaxRows || D <= 0 || D % 8 || !ids || !part) return -1;
  const int cg = (D + 63) / 64;
  const long rpb = (n + kSmallTabChunks - 1) / kSmallTabChunks;
  if (R <= 2)
    hipLaunchKernelGGL(embed_small_part_kernel<2>, dim3(cg, kSmallTabChunks), dim3(256), 0, s, ids,
                       (const bf16_t*)dout, dstride, part, n, D, R, rpb);
  else
    hipLaunchKernelGGL(embed_small_part_kernel<kSmallTabMaxRows>, dim3(cg, kSmallTabChunks), dim3(256), 0, s, ids,
                       (const bf16_t*)dout, dstride, part, n, D, R, rpb);
  const long RD = (long)R * D, b = (RD + 255) / 256;
  hipLaunchKernelGGL(embed_small_reduce_kernel, dim3((unsigned)(b < 2048 ? b : 2048)), dim3(256), 0, s, part,
                     kSmallTabChunks, RD, grad, grad_f32);
  return kfa_status();
}

KFA_API int kfa_embed_bwd(const long* ids, const void* dout, long dstride, float* scratch, void* grad, int grad_f32,
                          long n, int D, int accumulate, hipStream_t s) {
  if (n <= 0 || D % 8 || dstride % 8) return -1;
  const int ge = grid_for(n * D);
  hipLaunchKernelGGL(embed_bwd_scatter_kernel, dim3(ge), dim3(256), 0, s, ids, (const bf16_t*)dout, dstride, scratch,
                     n, D);
  hipLaunchKernelGGL(embed_bwd_fold_kernel, dim3(ge), dim3(256), 0, s, ids, scratch, grad, grad_f32, n, D, accumulate);
  return kfa_status();
}

KFA_API int kfa_colsum(const void* x, float* part, float* out, long rows, int N, int accumulate, hipStream_t s) {
  return kfa_bias_act_bwd(x, nullptr, nullptr, nullptr, part, out, rows, N, kNone, 0.f, 0ull, accumulate, s);
}
