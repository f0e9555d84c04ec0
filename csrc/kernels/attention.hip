// Fused multi-head self-attention, sequence 128 x head dim 64 (BERT-base /
// BERT-large pre-training phase 1) — SURVEY §2.6 K11 ("GEMM + softmax;
// optionally a fused flash-style kernel").
//
// One workgroup per (sequence, head), 4 waves.  A head's whole 128 x 128 score
// tile fits on chip, so no online rescaling is needed.
//
// forward   Q, K, V are read straight from the QKV projection [T, 3H] (+ bias,
//           q scaled by 1/sqrt(d)) into LDS.  Wave w computes Sᵀ = K·Qᵀ for the
//           queries 32w..32w+31 on MFMA — swapped, so each lane owns one query
//           column and its keys sit in registers: the row softmax is an
//           in-register reduction plus two cross-lane steps.  Key mask,
//           softmax, counter-hash dropout, then Oᵀ = Vᵀ·Pᵀ with V read
//           transposed by ds_read_b64_tr_b16 (T10).  O goes straight into the
//           [T, H] context layout through a 16-B-per-lane LDS stage; only the
//           row log-sum-exp [B·h, S] is kept for the backward.
// backward  key-owner (FlashAttention-2) form, see attn_bwd_kernel: wave w
//           owns 32 keys, recomputes P = exp(S − lse) and dP = dO·Vᵀ for them
//           over all queries, dS = P∘(dP − D) with D = rowsum(dO∘O); P and dS
//           feed dVᵀ / dKᵀ straight from registers, only dSᵀ is staged in LDS
//           for dQ.  80 KiB of LDS -> two workgroups per CU.  dq / dk / dv go
//           straight into the [T, 3H] gradient of the QKV projection and the
//           QKV bias gradient (column sums) is added with one atomic per
//           column per wave.
// Replaces, per layer: head split / merge, 2 + 4 batched GEMMs, two softmax
// passes and the [B·h, S, S] probability + dropout tensors (2 x 100 MB per
// BERT-base layer at 256 x 128 tokens).
//
// LDS images: [rows][64] bf16 (128-B rows) keep 16-B chunk c of row r at
// c ^ m(r) (see off64: conflict-free for row AND transposed reads); [rows][128]
// (256-B rows) at c ^ (r & 15) (row reads conflict-free, transposed reads at
// most 2-way).
#include "common.h"

#include <stdlib.h>

namespace {

constexpr int AS = 128;  // sequence length
constexpr int AD = 64;   // head dim

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

// [rows][64] images: chunk c of row r at c ^ m(r), m(r) = 2·((r>>1)&1) + 4·(((r>>2)^(r>>3))&1) + ((r>>3)&1).
// Conflict-free for the 16x16x32 row reads (ds_read_b128, 16-row groups) AND for
// both transposed-read row sets (8 consecutive rows; rows R..R+3 with R+8..R+11):
// within a parity the 4 rows' masks differ in bits 1-2, so the two logical
// chunks of a transposed read land in 8 distinct 16-B slots.  (The plain
// c ^ ((r>>1)&7) swizzle is 2-way on the transposed reads.)
__device__ __forceinline__ int off64(int row, int col) {
  const int m = (((row >> 1) & 1) << 1) | ((((row >> 2) ^ (row >> 3)) & 1) << 2) | ((row >> 3) & 1);
  return row * 128 + ((((col >> 3) ^ m) & 7) << 4) + (col & 7) * 2;
}
__device__ __forceinline__ int off128(int row, int col) {
  return row * 256 + ((((col >> 3) ^ row) & 15) << 4) + (col & 7) * 2;
}
template <int W>
__device__ __forceinline__ int ioff(int row, int col) {
  if constexpr (W == 64) return off64(row, col);
  else return off128(row, col);
}

// 16x16x32 operand: columns k0..k0+7 of `row`
template <int W>
__device__ __forceinline__ short8 rd_row(const char* img, int row, int k0) {
  return *reinterpret_cast<const short8*>(img + ioff<W>(row, k0));
}

// 16x16x32 operand from 8 consecutive ROWS: lane (g = lane>>4, i = lane&15) gets
// column cb + i of rows kb + 8g .. kb + 8g + 7 (two ds_read_b64_tr_b16)
template <int W>
__device__ __forceinline__ short8 rd_tr(const char* img, int kb, int cb, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int col = cb + 4 * (i & 3), r0 = kb + 8 * g + (i >> 2);
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + ioff<W>(r0, col)));
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + ioff<W>(r0 + 4, col)));
  return short8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// D[i][j] += Σ_k A[i][k]·B[k][j]; lane l holds A[l&15][8(l>>4)+e], B[8(l>>4)+e][l&15],
// D[4(l>>4)+r][l&15]
__device__ __forceinline__ floatx4 mma(short8 a, short8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
  return make_uint2(pack2(a, b), pack2(c, d));
}

// NI [128 rows][64] images of one head: image i = columns col[i].. of rows
// row0.. of src[i] (row stride ld[i]), (+ bias[col]) (· scale[i]).  Thread t
// moves chunk t & 7 of rows (t >> 3) + 32k.  Split in two so that a kernel can
// issue every global load it needs (biases first, then the image rows, then
// its own register operands) before the first LDS store: the vmcnt counter is
// in order, so a load issued after a store's source would stall the store.
template <int NI>
struct ImageLoad {
  uint4 raw[NI][4];
  float bb[NI][8];
};

template <int NI>
__device__ __forceinline__ void images_issue(ImageLoad<NI>& L, const bf16_t* const (&src)[NI], const long (&ld)[NI],
                                             long row0, const int (&col)[NI], const float* __restrict__ bias,
                                             const bool (&use_bias)[NI], int tid) {
  const int r0 = tid >> 3, c = tid & 7;
#pragma unroll
  for (int i = 0; i < NI; i++) {
    if (use_bias[i]) {  // compile-time after unrolling
      const float4 b0 = *reinterpret_cast<const float4*>(bias + col[i] + c * 8);
      const float4 b1 = *reinterpret_cast<const float4*>(bias + col[i] + c * 8 + 4);
      L.bb[i][0] = b0.x; L.bb[i][1] = b0.y; L.bb[i][2] = b0.z; L.bb[i][3] = b0.w;
      L.bb[i][4] = b1.x; L.bb[i][5] = b1.y; L.bb[i][6] = b1.z; L.bb[i][7] = b1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; e++) L.bb[i][e] = 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < NI; i++)
#pragma unroll
    for (int k = 0; k < 4; k++)
      L.raw[i][k] = *reinterpret_cast<const uint4*>(src[i] + (row0 + r0 + 32 * k) * ld[i] + col[i] + c * 8);
}

template <int NI>
__device__ __forceinline__ void images_commit(const ImageLoad<NI>& L, const bool (&transform)[NI],
                                              const float (&scale)[NI], char* const (&img)[NI], int tid) {
  const int r0 = tid >> 3, c = tid & 7;
#pragma unroll
  for (int i = 0; i < NI; i++)
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint4 v = L.raw[i][k];
      if (transform[i]) {
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int e = 0; e < 8; e++) f[e] = (f[e] + L.bb[i][e]) * scale[i];
        v = pack8(f);
      }
      *reinterpret_cast<uint4*>(img[i] + off64(r0 + 32 * k, c * 8)) = v;
    }
}

// additive key mask of this lane's keys 16kt + 4fq + r
__device__ __forceinline__ void load_key_bias(const float* __restrict__ kbias, long row0, int fq, float kb[8][4]) {
#pragma unroll
  for (int kt = 0; kt < 8; kt++) {
    const float4 v = *reinterpret_cast<const float4*>(kbias + row0 + kt * 16 + 4 * fq);
    kb[kt][0] = v.x;
    kb[kt][1] = v.y;
    kb[kt][2] = v.z;
    kb[kt][3] = v.w;
  }
}

// Sᵀ for queries qb..qb+31: s[kt][qt][r] = score(q = qb + 16qt + fr, key = 16kt + 4fq + r)
__device__ __forceinline__ void scores_t(const char* Qi, const char* Ki, int qb, int fr, int fq, floatx4 s[8][2]) {
#pragma unroll
  for (int kt = 0; kt < 8; kt++) s[kt][0] = s[kt][1] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ks++) {
    const short8 b0 = rd_row<64>(Qi, qb + fr, ks * 32 + fq * 8);
    const short8 b1 = rd_row<64>(Qi, qb + 16 + fr, ks * 32 + fq * 8);
#pragma unroll
    for (int kt = 0; kt < 8; kt++) {
      const short8 a = rd_row<64>(Ki, kt * 16 + fr, ks * 32 + fq * 8);
      s[kt][0] = mma(a, b0, s[kt][0]);
      s[kt][1] = mma(a, b1, s[kt][1]);
    }
  }
}

// rows ra..ra+3 and rb..rb+3 (any two 4-row groups) of column cb + (lane & 15):
// the 16x16x32 operand whose k index runs over a PERMUTED row order.  Used where
// the other operand comes straight from an MFMA result held in registers (lane
// = column, 4 consecutive rows per 16-row tile): k order is free in a dot
// product, so only the two operands have to agree on it.
template <int W>
__device__ __forceinline__ short8 rd_tr2(const char* img, int ra, int rb, int cb, int lane) {
  const int i = lane & 15;
  const int col = cb + 4 * (i & 3);
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + ioff<W>(ra + (i >> 2), col)));
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + ioff<W>(rb + (i >> 2), col)));
  return short8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

__device__ __forceinline__ short8 pack_pair(floatx4 x, floatx4 y) {
  const uint2 lo = pack4(x[0], x[1], x[2], x[3]), hi = pack4(y[0], y[1], y[2], y[3]);
  const uint4 u = make_uint4(lo.x, lo.y, hi.x, hi.y);
  return *reinterpret_cast<const short8*>(&u);
}

__global__ __launch_bounds__(256, 3) void attn_fwd_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ bqkv,
                                                          const float* __restrict__ kbias, bf16_t* __restrict__ out,
                                                          float* __restrict__ lse, int heads, float qscale,
                                                          uint32_t thresh, float dscale, uint64_t seed) {
  // Q, K, V images only (48 KiB: three workgroups per CU): the probabilities
  // feed P·V straight from registers and O is staged in the Q image afterwards
  __shared__ __attribute__((aligned(16))) char sm[3 * 16384];
  char* Qi = sm;
  char* Ki = sm + 16384;
  char* Vi = sm + 32768;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int bh = blockIdx.x, b = bh / heads, h = bh - b * heads, H = heads * AD;
  const long row0 = (long)b * AS;
  const int qb = wave * 32;
  const int col[3] = {h * AD, H + h * AD, 2 * H + h * AD};
  const bool ub[3] = {true, true, true};
  const bool tf[3] = {true, true, true};
  const float sc[3] = {qscale, 1.f, 1.f};
  char* const img[3] = {Qi, Ki, Vi};
  const bf16_t* const src[3] = {qkv, qkv, qkv};
  const long ld[3] = {3L * H, 3L * H, 3L * H};
  ImageLoad<3> L;
  images_issue<3>(L, src, ld, row0, col, bqkv, ub, tid);
  float kb[8][4];
  load_key_bias(kbias, row0, fq, kb);
  images_commit<3>(L, tf, sc, img, tid);
  __syncthreads();

  floatx4 s[8][2];
  scores_t(Qi, Ki, qb, fr, fq, s);
#pragma unroll
  for (int qt = 0; qt < 2; qt++) {
    const int q = qb + qt * 16 + fr;
    float mx = -3.0e38f;
#pragma unroll
    for (int kt = 0; kt < 8; kt++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        s[kt][qt][r] += kb[kt][r];
        mx = fmaxf(mx, s[kt][qt][r]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 8; kt++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const float e = __expf(s[kt][qt][r] - mx);
        s[kt][qt][r] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    if (fq == 0) lse[(long)bh * AS + q] = mx + __logf(sum);
    const float inv = 1.f / sum;
#pragma unroll
    for (int kt = 0; kt < 8; kt++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        float v = s[kt][qt][r] * inv;
        if (thresh)
          v = drop_hash(seed, ((uint64_t)bh * AS + q) * AS + kt * 16 + 4 * fq + r) >= thresh ? v * dscale : 0.f;
        s[kt][qt][r] = v;
      }
  }

  // Oᵀ[d][q] = Σ_key V[key][d] · Pd[q][key]:  o[dt][qt][r] = O(q = qb + 16qt + fr, d = 16dt + 4fq + r).
  // The B operand (Pdᵀ, k = key) comes from the registers: tiles 2ks and 2ks+1 give this
  // lane keys {32ks + 4fq + r, 32ks + 16 + 4fq + r} — a permuted k order, matched by
  // reading V's rows in the same order (rd_tr2, as the backward's dVᵀ).
  floatx4 o[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; dt++) o[dt][0] = o[dt][1] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ks++) {
    const short8 b0 = pack_pair(s[2 * ks][0], s[2 * ks + 1][0]);
    const short8 b1 = pack_pair(s[2 * ks][1], s[2 * ks + 1][1]);
    const int ra = 32 * ks + 4 * fq;
#pragma unroll
    for (int dt = 0; dt < 4; dt++) {
      const short8 a = rd_tr2<64>(Vi, ra, ra + 16, dt * 16, lane);
      o[dt][0] = mma(a, b0, o[dt][0]);
      o[dt][1] = mma(a, b1, o[dt][1]);
    }
  }
  __syncthreads();  // every wave is done with the Q image: it becomes the O stage
  char* Pw = Qi + wave * 4096;  // this wave's [32 q][64] O stage
#pragma unroll
  for (int dt = 0; dt < 4; dt++)
#pragma unroll
    for (int qt = 0; qt < 2; qt++)
      *reinterpret_cast<uint2*>(Pw + off64(qt * 16 + fr, dt * 16 + 4 * fq)) =
          pack4(o[dt][qt][0], o[dt][qt][1], o[dt][qt][2], o[dt][qt][3]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int it = 0; it < 4; it++) {
    const int r = it * 8 + (lane >> 3), c = lane & 7;
    *reinterpret_cast<uint4*>(out + (row0 + qb + r) * H + h * AD + c * 8) =
        *reinterpret_cast<const uint4*>(Pw + off64(r, c * 8));
  }
}

// Backward, key-owner form (FlashAttention-2 style): wave w owns keys
// kw = 32w..32w+31 and streams the 128 queries in 4 steps of 32.  Per step the
// wave forms S and dP = dO·Vᵀ for its keys on MFMA (lane = key column, 4
// consecutive queries per 16-query tile), P = exp(S − lse), dS = P∘(dP − D)
// with D = rowsum(dO∘O) computed up front, and feeds P and dS STRAIGHT from
// registers into dVᵀ += dOᵀ·Pd and dKᵀ += Qᵀ·dS (the queries are the k index:
// rd_tr2 reads dO / Q in the matching permuted row order).  Only dS goes
// through LDS (as dSᵀ [key][q]) for dQᵀ = Kᵀ·dSᵀ, computed after one barrier
// by wave w for its queries 32w...  LDS = Q, K, dO images + dSᵀ = 80 KiB:
// two workgroups per CU, so one loads while the other multiplies.
// LDSD: D = rowsum(dO∘O) exchanged through the (not yet used) dSᵀ image instead of
// a global scratch row — no vmcnt(0) + memory round trip before phase A.
template <bool LDSD>
__global__ __launch_bounds__(256, 2) void attn_bwd_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ bqkv,
                                                          const float* __restrict__ kbias, const bf16_t* __restrict__ out,
                                                          const float* __restrict__ lse, const bf16_t* __restrict__ dout,
                                                          bf16_t* __restrict__ dqkv, float* __restrict__ dbqkv,
                                                          float* __restrict__ dwork, int heads, float qscale,
                                                          uint32_t thresh, float dscale, uint64_t seed) {
  __shared__ __attribute__((aligned(16))) char sm[3 * 16384 + 32768];  // 80 KiB
  char* Qi = sm;            // [128 q][64]      q·scale (+ bias)
  char* Ki = sm + 16384;    // [128 key][64]    k (+ bias)
  char* Gi = sm + 32768;    // [128 q][64]      dO
  char* dST = sm + 49152;   // [128 key][128 q] dL/dS, transposed
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int bh = blockIdx.x, b = bh / heads, h = bh - b * heads, H = heads * AD;
  const long row0 = (long)b * AS, W3 = 3L * H;
  const int kw = wave * 32;
  // every global load up front, in consumption order: biases, Q / K / dO image
  // rows, this lane's V operand pieces V[kw + 16kt + fr][32ks + 8fq ..] (+ bias),
  // the O rows 2·lane, 2·lane + 1 (for D) and their lse
  const int icol[3] = {h * AD, H + h * AD, h * AD};
  const bool iub[3] = {true, true, false};
  const bool itf[3] = {true, true, false};
  const float isc[3] = {qscale, 1.f, 1.f};
  char* const iimg[3] = {Qi, Ki, Gi};
  const bf16_t* const isrc[3] = {qkv, qkv, dout};
  const long ild[3] = {W3, W3, (long)H};
  ImageLoad<3> L;
  images_issue<3>(L, isrc, ild, row0, icol, bqkv, iub, tid);
  float vb[2][8];
#pragma unroll
  for (int ks = 0; ks < 2; ks++) {
    const int col = 2 * H + h * AD + ks * 32 + fq * 8;
    const float4 b0 = *reinterpret_cast<const float4*>(bqkv + col), b1 = *reinterpret_cast<const float4*>(bqkv + col + 4);
    vb[ks][0] = b0.x; vb[ks][1] = b0.y; vb[ks][2] = b0.z; vb[ks][3] = b0.w;
    vb[ks][4] = b1.x; vb[ks][5] = b1.y; vb[ks][6] = b1.z; vb[ks][7] = b1.w;
  }
  // D = rowsum(dO∘O) is formed ONCE per workgroup: wave w takes queries 32w..32w+31,
  // a lane half a row (32 d), the pair combines with one shuffle and D goes through
  // a global scratch row of this head (every wave then reads all 128) — each wave
  // used to load all 128 O rows itself (64 KiB of O per workgroup instead of 16)
  uint4 vraw[2][2], oraw[4];
#pragma unroll
  for (int kt = 0; kt < 2; kt++)
#pragma unroll
    for (int ks = 0; ks < 2; ks++)
      vraw[kt][ks] = *reinterpret_cast<const uint4*>(qkv + (row0 + kw + kt * 16 + fr) * W3 + 2 * H + h * AD +
                                                     ks * 32 + fq * 8);
  const int dq = wave * 32 + (lane >> 1), dh = (lane & 1) * 32;  // this lane's D row and half
#pragma unroll
  for (int c = 0; c < 4; c++) oraw[c] = *reinterpret_cast<const uint4*>(out + (row0 + dq) * H + h * AD + dh + c * 8);
  const float2 lse2 = *reinterpret_cast<const float2*>(lse + (long)bh * AS + 2 * lane);
  float kbv[2];
#pragma unroll
  for (int kt = 0; kt < 2; kt++) kbv[kt] = kbias[row0 + kw + kt * 16 + fr];
  images_commit<3>(L, itf, isc, iimg, tid);
  short8 vreg[2][2];
#pragma unroll
  for (int kt = 0; kt < 2; kt++)
#pragma unroll
    for (int ks = 0; ks < 2; ks++) {
      float f[8];
      unpack8(vraw[kt][ks], f);
#pragma unroll
      for (int e = 0; e < 8; e++) f[e] += vb[ks][e];
      const uint4 u = pack8(f);
      vreg[kt][ks] = *reinterpret_cast<const short8*>(&u);
    }
  __syncthreads();

  // D[q] = Σ_d dO[q][d]·O[q][d]: this wave's 32 queries -> the head's scratch row,
  // then every wave keeps q = 2·lane, 2·lane + 1
  {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      float g[8], o[8];
      unpack8(*reinterpret_cast<const uint4*>(Gi + off64(dq, dh + c * 8)), g);
      unpack8(oraw[c], o);
#pragma unroll
      for (int e = 0; e < 8; e++) acc += g[e] * o[e];
    }
    acc += __shfl_xor(acc, 1, 64);
    if (!(lane & 1)) {
      if constexpr (LDSD) reinterpret_cast<float*>(dST)[dq] = acc;
      else dwork[(long)bh * AS + dq] = acc;
    }
  }
  if constexpr (!LDSD) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float dd[2];
  {
    const float2 d2 = LDSD ? *reinterpret_cast<const float2*>(reinterpret_cast<const float*>(dST) + 2 * lane)
                           : *reinterpret_cast<const float2*>(dwork + (long)bh * AS + 2 * lane);
    dd[0] = d2.x;
    dd[1] = d2.y;
  }
  if constexpr (LDSD) __syncthreads();  // every wave has its D before phase A writes dSᵀ
  short8 kreg[2][2];
#pragma unroll
  for (int kt = 0; kt < 2; kt++)
#pragma unroll
    for (int ks = 0; ks < 2; ks++) kreg[kt][ks] = rd_row<64>(Ki, kw + kt * 16 + fr, ks * 32 + fq * 8);

  // ---- phase A: 4 steps of 32 queries; dvT / dkT[dt][kt][r] = dV / dK(key = kw + 16kt + fr, d = 16dt + 4fq + r)
  floatx4 dvT[4][2], dkT[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; dt++) dvT[dt][0] = dvT[dt][1] = dkT[dt][0] = dkT[dt][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < 4; j++) {
    // s / dp[qt][kt][r]: (q = 32j + 16qt + 4fq + r, key = kw + 16kt + fr)
    floatx4 s[2][2], dp[2][2];
#pragma unroll
    for (int qt = 0; qt < 2; qt++) s[qt][0] = s[qt][1] = dp[qt][0] = dp[qt][1] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ks++)
#pragma unroll
      for (int qt = 0; qt < 2; qt++) {
        const short8 aq = rd_row<64>(Qi, 32 * j + 16 * qt + fr, ks * 32 + fq * 8);
        const short8 ag = rd_row<64>(Gi, 32 * j + 16 * qt + fr, ks * 32 + fq * 8);
#pragma unroll
        for (int kt = 0; kt < 2; kt++) {
          s[qt][kt] = mma(aq, kreg[kt][ks], s[qt][kt]);
          dp[qt][kt] = mma(ag, vreg[kt][ks], dp[qt][kt]);
        }
      }
    floatx4 pd[2][2], ds[2][2];
#pragma unroll
    for (int qt = 0; qt < 2; qt++) {
      const int qb4 = 32 * j + 16 * qt + 4 * fq;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const float Dq = __shfl(dd[r & 1], (qb4 + r) >> 1, 64);
        const float lq = __shfl(r & 1 ? lse2.y : lse2.x, (qb4 + r) >> 1, 64);
#pragma unroll
        for (int kt = 0; kt < 2; kt++) {
          const float p = __expf(s[qt][kt][r] + kbv[kt] - lq);
          float g = dp[qt][kt][r], pv = p;
          if (thresh) {
            const bool keep =
                drop_hash(seed, ((uint64_t)bh * AS + qb4 + r) * AS + kw + kt * 16 + fr) >= thresh;
            pv = keep ? p * dscale : 0.f;
            g = keep ? g * dscale : 0.f;
          }
          pd[qt][kt][r] = pv;
          ds[qt][kt][r] = p * (g - Dq);
        }
      }
    }
    // dSᵀ -> LDS: row key, 4 consecutive queries
#pragma unroll
    for (int qt = 0; qt < 2; qt++)
#pragma unroll
      for (int kt = 0; kt < 2; kt++)
        *reinterpret_cast<uint2*>(dST + off128(kw + kt * 16 + fr, 32 * j + 16 * qt + 4 * fq)) =
            pack4(ds[qt][kt][0], ds[qt][kt][1], ds[qt][kt][2], ds[qt][kt][3]);
    // dVᵀ[d][key] += Σ_q dOᵀ[d][q]·Pd[q][key];  dKᵀ[d][key] += Σ_q Qᵀ[d][q]·dS[q][key]
    const int ra = 32 * j + 4 * fq, rb = ra + 16;
    short8 gtr[4], qtr[4];  // dO / Q columns, shared by both key tiles
#pragma unroll
    for (int dt = 0; dt < 4; dt++) {
      gtr[dt] = rd_tr2<64>(Gi, ra, rb, dt * 16, lane);
      qtr[dt] = rd_tr2<64>(Qi, ra, rb, dt * 16, lane);
    }
#pragma unroll
    for (int kt = 0; kt < 2; kt++) {
      const short8 bp = pack_pair(pd[0][kt], pd[1][kt]);
      const short8 bs = pack_pair(ds[0][kt], ds[1][kt]);
#pragma unroll
      for (int dt = 0; dt < 4; dt++) {
        dvT[dt][kt] = mma(gtr[dt], bp, dvT[dt][kt]);
        dkT[dt][kt] = mma(qtr[dt], bs, dkT[dt][kt]);
      }
    }
  }
  __syncthreads();

  // ---- phase B: dQᵀ[d][q] = Σ_key Kᵀ[d][key]·dSᵀ[key][q] for q = qw + 16qt + fr
  const int qw = wave * 32;
  floatx4 dqT[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; dt++) dqT[dt][0] = dqT[dt][1] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ks++) {
    const short8 b0 = rd_tr<128>(dST, ks * 32, qw, lane);
    const short8 b1 = rd_tr<128>(dST, ks * 32, qw + 16, lane);
#pragma unroll
    for (int dt = 0; dt < 4; dt++) {
      const short8 a = rd_tr<64>(Ki, ks * 32, dt * 16, lane);
      dqT[dt][0] = mma(a, b0, dqT[dt][0]);
      dqT[dt][1] = mma(a, b1, dqT[dt][1]);
    }
  }
  __syncthreads();  // every wave is done with the images: they become the output stage
  char* st = sm + wave * 12288;  // [dq | dk | dv] x [32 rows][64]
#pragma unroll
  for (int dt = 0; dt < 4; dt++)
#pragma unroll
    for (int t2 = 0; t2 < 2; t2++) {
      const int o = off64(t2 * 16 + fr, dt * 16 + 4 * fq);
      *reinterpret_cast<uint2*>(st + o) = pack4(dqT[dt][t2][0] * qscale, dqT[dt][t2][1] * qscale,
                                                dqT[dt][t2][2] * qscale, dqT[dt][t2][3] * qscale);
      *reinterpret_cast<uint2*>(st + 4096 + o) = pack4(dkT[dt][t2][0], dkT[dt][t2][1], dkT[dt][t2][2], dkT[dt][t2][3]);
      *reinterpret_cast<uint2*>(st + 8192 + o) = pack4(dvT[dt][t2][0], dvT[dt][t2][1], dvT[dt][t2][2], dvT[dt][t2][3]);
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int c = lane & 7;
#pragma unroll
  for (int jj = 0; jj < 3; jj++) {
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int it = 0; it < 4; it++) {
      const int r = it * 8 + (lane >> 3);
      const uint4 v = *reinterpret_cast<const uint4*>(st + jj * 4096 + off64(r, c * 8));
      *reinterpret_cast<uint4*>(dqkv + (row0 + kw + r) * W3 + jj * H + h * AD + c * 8) = v;
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int e = 0; e < 8; e++) cs[e] += f[e];
    }
    if (dbqkv) {
#pragma unroll
      for (int o = 8; o < 64; o <<= 1)
#pragma unroll
        for (int e = 0; e < 8; e++) cs[e] += __shfl_xor(cs[e], o, 64);
      if (lane < 8)
#pragma unroll
        for (int e = 0; e < 8; e++) atomicAdd(dbqkv + jj * H + h * AD + c * 8 + e, cs[e]);
    }
  }
}

// ============================================================================
// Long sequences, S = 128·n (BERT pre-training phase 2: S = 512).  The same
// lane layouts and LDS images as the S = 128 kernels, tiled over 128-key /
// 128-query blocks:
//   forward   one workgroup per (sequence, head, 128-query block); key blocks
//             streamed through LDS with an online softmax (running max / sum per
//             query, held by the lane that owns the query column; O rescaled in
//             registers), so no S x S tensor exists;
//   backward  D = rowsum(dO∘O) by a small pre-pass, then two kernels that both
//             recompute P and dS for their tiles (no atomics, no S x S buffer):
//             key-owner dK / dV (the S = 128 kernel's phase A over every query
//             block) and query-owner dQ = dS·K.
// Dropout uses the same counter hash of (bh, query, key) as the S = 128 path.
constexpr int BLK = 128;

__global__ __launch_bounds__(256, 2) void attn_fwd_long_kernel(const bf16_t* __restrict__ qkv,
                                                               const float* __restrict__ bqkv,
                                                               const float* __restrict__ kbias, bf16_t* __restrict__ out,
                                                               float* __restrict__ lse, int heads, int S, float qscale,
                                                               uint32_t thresh, float dscale, uint64_t seed) {
  __shared__ __attribute__((aligned(16))) char sm[3 * 16384 + 4 * 8192];  // 80 KiB
  char* Qi = sm;
  char* Ki = sm + 16384;
  char* Vi = sm + 32768;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  char* Pw = sm + 49152 + wave * 8192;
  const int nb = S / BLK;
  const int qblk = blockIdx.x % nb, bh = blockIdx.x / nb, b = bh / heads, h = bh - b * heads, H = heads * AD;
  const long seq0 = (long)b * S, q0 = seq0 + (long)qblk * BLK;
  const int qb = wave * 32;
  {
    const int col[1] = {h * AD};
    const bool ub[1] = {true}, tf[1] = {true};
    const float sc[1] = {qscale};
    char* const img[1] = {Qi};
    const bf16_t* const src[1] = {qkv};
    const long ld[1] = {3L * H};
    ImageLoad<1> L;
    images_issue<1>(L, src, ld, q0, col, bqkv, ub, tid);
    images_commit<1>(L, tf, sc, img, tid);
  }
  float m[2] = {-3.0e38f, -3.0e38f}, l[2] = {0.f, 0.f};
  floatx4 o[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; dt++) o[dt][0] = o[dt][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < nb; j++) {
    const long k0 = seq0 + (long)j * BLK;
    if (j > 0) __syncthreads();  // every wave is done with key block j-1
    const int col[2] = {H + h * AD, 2 * H + h * AD};
    const bool ub[2] = {true, true}, tf[2] = {true, true};
    const float sc[2] = {1.f, 1.f};
    char* const img[2] = {Ki, Vi};
    const bf16_t* const src[2] = {qkv, qkv};
    const long ld[2] = {3L * H, 3L * H};
    ImageLoad<2> L;
    images_issue<2>(L, src, ld, k0, col, bqkv, ub, tid);
    float kb[8][4];
    load_key_bias(kbias, k0, fq, kb);
    images_commit<2>(L, tf, sc, img, tid);
    __syncthreads();
    floatx4 s[8][2];
    scores_t(Qi, Ki, qb, fr, fq, s);
#pragma unroll
    for (int qt = 0; qt < 2; qt++) {
      const int q = qblk * BLK + qb + qt * 16 + fr;
      float mx = -3.0e38f;
#pragma unroll
      for (int kt = 0; kt < 8; kt++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          s[kt][qt][r] += kb[kt][r];
          mx = fmaxf(mx, s[kt][qt][r]);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m[qt], mx);
      const float alpha = __expf(m[qt] - mn);
      float sum = 0.f;
#pragma unroll
      for (int kt = 0; kt < 8; kt++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const float e = __expf(s[kt][qt][r] - mn);
          s[kt][qt][r] = e;
          sum += e;
        }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      l[qt] = l[qt] * alpha + sum;
      m[qt] = mn;
#pragma unroll
      for (int dt = 0; dt < 4; dt++)
#pragma unroll
        for (int r = 0; r < 4; r++) o[dt][qt][r] *= alpha;
#pragma unroll
      for (int kt = 0; kt < 8; kt++) {
        float pp[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
          float v = s[kt][qt][r];
          if (thresh)
            v = drop_hash(seed, ((uint64_t)bh * S + q) * S + j * BLK + kt * 16 + 4 * fq + r) >= thresh ? v * dscale
                                                                                                       : 0.f;
          pp[r] = v;
        }
        *reinterpret_cast<uint2*>(Pw + off128(qt * 16 + fr, kt * 16 + 4 * fq)) = pack4(pp[0], pp[1], pp[2], pp[3]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // only this wave reads its P rows
#pragma unroll
    for (int ks = 0; ks < 4; ks++) {
      const short8 b0 = rd_row<128>(Pw, fr, ks * 32 + fq * 8);
      const short8 b1 = rd_row<128>(Pw, 16 + fr, ks * 32 + fq * 8);
#pragma unroll
      for (int dt = 0; dt < 4; dt++) {
        const short8 a = rd_tr<64>(Vi, ks * 32, dt * 16, lane);
        o[dt][0] = mma(a, b0, o[dt][0]);
        o[dt][1] = mma(a, b1, o[dt][1]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // Pw is rewritten next block
  }
#pragma unroll
  for (int qt = 0; qt < 2; qt++) {
    const float inv = 1.f / l[qt];
    if (fq == 0) lse[(long)bh * S + qblk * BLK + qb + qt * 16 + fr] = m[qt] + __logf(l[qt]);
#pragma unroll
    for (int dt = 0; dt < 4; dt++)
#pragma unroll
      for (int r = 0; r < 4; r++) o[dt][qt][r] *= inv;
  }
#pragma unroll
  for (int dt = 0; dt < 4; dt++)
#pragma unroll
    for (int qt = 0; qt < 2; qt++)
      *reinterpret_cast<uint2*>(Pw + off64(qt * 16 + fr, dt * 16 + 4 * fq)) =
          pack4(o[dt][qt][0], o[dt][qt][1], o[dt][qt][2], o[dt][qt][3]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int it = 0; it < 4; it++) {
    const int r = it * 8 + (lane >> 3), c = lane & 7;
    *reinterpret_cast<uint4*>(out + (q0 + qb + r) * H + h * AD + c * 8) =
        *reinterpret_cast<const uint4*>(Pw + off64(r, c * 8));
  }
}

// D[bh][s] = Σ_d dO[token][h·64 + d]·O[token][h·64 + d]  (token = b·S + s), one thread per (token, head)
__global__ void attn_rowdot_kernel(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ out,
                                   float* __restrict__ D, long tokens, int heads, int S) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= tokens * heads) return;
  const long tok = t / heads;
  const int h = (int)(t - tok * heads), H = heads * AD;
  const uint4* g = reinterpret_cast<const uint4*>(dout + tok * H + h * AD);
  const uint4* o = reinterpret_cast<const uint4*>(out + tok * H + h * AD);
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < 8; c++) {
    float a[8], b[8];
    unpack8(g[c], a);
    unpack8(o[c], b);
#pragma unroll
    for (int e = 0; e < 8; e++) acc += a[e] * b[e];
  }
  const long b = tok / S;
  D[(b * heads + h) * S + (tok - b * S)] = acc;
}

// stage a wave's [32 rows][64] fp32 tiles t[dt][t2] (rows 16·t2 + fr, cols 16·dt + 4fq + r), scaled, as bf16
__device__ __forceinline__ void stage_tile(char* st, const floatx4 (&t)[4][2], float scale, int fr, int fq) {
#pragma unroll
  for (int dt = 0; dt < 4; dt++)
#pragma unroll
    for (int t2 = 0; t2 < 2; t2++)
      *reinterpret_cast<uint2*>(st + off64(t2 * 16 + fr, dt * 16 + 4 * fq)) =
          pack4(t[dt][t2][0] * scale, t[dt][t2][1] * scale, t[dt][t2][2] * scale, t[dt][t2][3] * scale);
}

// write a staged [32 rows][64] tile to rows row0.. of dqkv column block colb; column sums -> dbias[colb..]
__device__ __forceinline__ void store_tile(const char* st, bf16_t* __restrict__ dqkv, long row0, long W3, int colb,
                                           float* __restrict__ dbias, int lane) {
  const int c = lane & 7;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < 4; it++) {
    const int r = it * 8 + (lane >> 3);
    const uint4 v = *reinterpret_cast<const uint4*>(st + off64(r, c * 8));
    *reinterpret_cast<uint4*>(dqkv + (row0 + r) * W3 + colb + c * 8) = v;
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int e = 0; e < 8; e++) cs[e] += f[e];
  }
  if (dbias) {
#pragma unroll
    for (int o = 8; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; e++) cs[e] += __shfl_xor(cs[e], o, 64);
    if (lane < 8)
#pragma unroll
      for (int e = 0; e < 8; e++) atomicAdd(dbias + colb + c * 8 + e, cs[e]);
  }
}

// key-owner dK / dV: workgroup per (sequence, head, 128-key block); wave w owns keys 32w.. of the block
__global__ __launch_bounds__(256, 2) void attn_bwd_kv_long_kernel(
    const bf16_t* __restrict__ qkv, const float* __restrict__ bqkv, const float* __restrict__ kbias,
    const float* __restrict__ lse, const float* __restrict__ Dq, const bf16_t* __restrict__ dout,
    bf16_t* __restrict__ dqkv, float* __restrict__ dbqkv, int heads, int S, float qscale, uint32_t thresh,
    float dscale, uint64_t seed) {
  __shared__ __attribute__((aligned(16))) char sm[3 * 16384];  // Q, K, dO images (48 KiB)
  char* Qi = sm;
  char* Ki = sm + 16384;
  char* Gi = sm + 32768;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int nb = S / BLK;
  const int kblk = blockIdx.x % nb, bh = blockIdx.x / nb, b = bh / heads, h = bh - b * heads, H = heads * AD;
  const long seq0 = (long)b * S, k0 = seq0 + (long)kblk * BLK, W3 = 3L * H;
  const int kw = wave * 32;
  {
    const int col[1] = {H + h * AD};
    const bool ub[1] = {true}, tf[1] = {true};
    const float sc[1] = {1.f};
    char* const img[1] = {Ki};
    const bf16_t* const src[1] = {qkv};
    const long ld[1] = {W3};
    ImageLoad<1> L;
    images_issue<1>(L, src, ld, k0, col, bqkv, ub, tid);
    images_commit<1>(L, tf, sc, img, tid);
  }
  short8 vreg[2][2];
#pragma unroll
  for (int ks = 0; ks < 2; ks++) {
    const int col = 2 * H + h * AD + ks * 32 + fq * 8;
    const float4 b0 = *reinterpret_cast<const float4*>(bqkv + col), b1 = *reinterpret_cast<const float4*>(bqkv + col + 4);
    const float vb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int kt = 0; kt < 2; kt++) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(qkv + (k0 + kw + kt * 16 + fr) * W3 + col), f);
#pragma unroll
      for (int e = 0; e < 8; e++) f[e] += vb[e];
      const uint4 u = pack8(f);
      vreg[kt][ks] = *reinterpret_cast<const short8*>(&u);
    }
  }
  float kbv[2];
#pragma unroll
  for (int kt = 0; kt < 2; kt++) kbv[kt] = kbias[k0 + kw + kt * 16 + fr];
  __syncthreads();
  short8 kreg[2][2];
#pragma unroll
  for (int kt = 0; kt < 2; kt++)
#pragma unroll
    for (int ks = 0; ks < 2; ks++) kreg[kt][ks] = rd_row<64>(Ki, kw + kt * 16 + fr, ks * 32 + fq * 8);
  floatx4 dvT[4][2], dkT[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; dt++) dvT[dt][0] = dvT[dt][1] = dkT[dt][0] = dkT[dt][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < nb; i++) {
    const long qrow0 = seq0 + (long)i * BLK;
    if (i > 0) __syncthreads();  // every wave is done with the previous Q / dO images
    const int col[2] = {h * AD, h * AD};
    const bool ub[2] = {true, false}, tf[2] = {true, false};
    const float sc[2] = {qscale, 1.f};
    char* const img[2] = {Qi, Gi};
    const bf16_t* const src[2] = {qkv, dout};
    const long ld[2] = {W3, (long)H};
    ImageLoad<2> L;
    images_issue<2>(L, src, ld, qrow0, col, bqkv, ub, tid);
    const float2 lse2 = *reinterpret_cast<const float2*>(lse + (long)bh * S + i * BLK + 2 * lane);
    const float2 dd2 = *reinterpret_cast<const float2*>(Dq + (long)bh * S + i * BLK + 2 * lane);
    images_commit<2>(L, tf, sc, img, tid);
    __syncthreads();
    for (int j = 0; j < 4; j++) {
      floatx4 s[2][2], dp[2][2];
#pragma unroll
      for (int qt = 0; qt < 2; qt++) s[qt][0] = s[qt][1] = dp[qt][0] = dp[qt][1] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ks++)
#pragma unroll
        for (int qt = 0; qt < 2; qt++) {
          const short8 aq = rd_row<64>(Qi, 32 * j + 16 * qt + fr, ks * 32 + fq * 8);
          const short8 ag = rd_row<64>(Gi, 32 * j + 16 * qt + fr, ks * 32 + fq * 8);
#pragma unroll
          for (int kt = 0; kt < 2; kt++) {
            s[qt][kt] = mma(aq, kreg[kt][ks], s[qt][kt]);
            dp[qt][kt] = mma(ag, vreg[kt][ks], dp[qt][kt]);
          }
        }
      floatx4 pd[2][2], ds[2][2];
#pragma unroll
      for (int qt = 0; qt < 2; qt++) {
        const int qb4 = 32 * j + 16 * qt + 4 * fq;  // query within the block
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const float D = __shfl(r & 1 ? dd2.y : dd2.x, (qb4 + r) >> 1, 64);
          const float lq = __shfl(r & 1 ? lse2.y : lse2.x, (qb4 + r) >> 1, 64);
#pragma unroll
          for (int kt = 0; kt < 2; kt++) {
            const float p = __expf(s[qt][kt][r] + kbv[kt] - lq);
            float g = dp[qt][kt][r], pv = p;
            if (thresh) {
              const bool keep = drop_hash(seed, ((uint64_t)bh * S + i * BLK + qb4 + r) * S + kblk * BLK + kw +
                                                    kt * 16 + fr) >= thresh;
              pv = keep ? p * dscale : 0.f;
              g = keep ? g * dscale : 0.f;
            }
            pd[qt][kt][r] = pv;
            ds[qt][kt][r] = p * (g - D);
          }
        }
      }
      const int ra = 32 * j + 4 * fq, rb = ra + 16;
      short8 gtr[4], qtr[4];
#pragma unroll
      for (int dt = 0; dt < 4; dt++) {
        gtr[dt] = rd_tr2<64>(Gi, ra, rb, dt * 16, lane);
        qtr[dt] = rd_tr2<64>(Qi, ra, rb, dt * 16, lane);
      }
#pragma unroll
      for (int kt = 0; kt < 2; kt++) {
        const short8 bp = pack_pair(pd[0][kt], pd[1][kt]);
        const short8 bs = pack_pair(ds[0][kt], ds[1][kt]);
#pragma unroll
        for (int dt = 0; dt < 4; dt++) {
          dvT[dt][kt] = mma(gtr[dt], bp, dvT[dt][kt]);
          dkT[dt][kt] = mma(qtr[dt], bs, dkT[dt][kt]);
        }
      }
    }
  }
  __syncthreads();  // the images become the output stage
  char* st = sm + wave * 8192;
  stage_tile(st, dkT, 1.f, fr, fq);
  stage_tile(st + 4096, dvT, 1.f, fr, fq);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  store_tile(st, dqkv, k0 + kw, W3, H + h * AD, dbqkv, lane);
  store_tile(st + 4096, dqkv, k0 + kw, W3, 2 * H + h * AD, dbqkv, lane);
}

// query-owner dQ = dS·K: workgroup per (sequence, head, 128-query block); wave w owns queries 32w..
__global__ __launch_bounds__(256, 2) void attn_bwd_q_long_kernel(
    const bf16_t* __restrict__ qkv, const float* __restrict__ bqkv, const float* __restrict__ kbias,
    const float* __restrict__ lse, const float* __restrict__ Dq, const bf16_t* __restrict__ dout,
    bf16_t* __restrict__ dqkv, float* __restrict__ dbqkv, int heads, int S, float qscale, uint32_t thresh,
    float dscale, uint64_t seed) {
  __shared__ __attribute__((aligned(16))) char sm[4 * 16384];  // Q, dO, K, V images (64 KiB)
  char* Qi = sm;
  char* Gi = sm + 16384;
  char* Ki = sm + 32768;
  char* Vi = sm + 49152;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int nb = S / BLK;
  const int qblk = blockIdx.x % nb, bh = blockIdx.x / nb, b = bh / heads, h = bh - b * heads, H = heads * AD;
  const long seq0 = (long)b * S, q0 = seq0 + (long)qblk * BLK, W3 = 3L * H;
  const int qb = wave * 32;
  {
    const int col[2] = {h * AD, h * AD};
    const bool ub[2] = {true, false}, tf[2] = {true, false};
    const float sc[2] = {qscale, 1.f};
    char* const img[2] = {Qi, Gi};
    const bf16_t* const src[2] = {qkv, dout};
    const long ld[2] = {W3, (long)H};
    ImageLoad<2> L;
    images_issue<2>(L, src, ld, q0, col, bqkv, ub, tid);
    images_commit<2>(L, tf, sc, img, tid);
  }
  float lq[2], Dv[2];
#pragma unroll
  for (int qt = 0; qt < 2; qt++) {
    const long qi = (long)bh * S + qblk * BLK + qb + qt * 16 + fr;
    lq[qt] = lse[qi];
    Dv[qt] = Dq[qi];
  }
  floatx4 dqT[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; dt++) dqT[dt][0] = dqT[dt][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < nb; j++) {
    const long k0 = seq0 + (long)j * BLK;
    if (j > 0) __syncthreads();  // every wave is done with key block j-1
    const int col[2] = {H + h * AD, 2 * H + h * AD};
    const bool ub[2] = {true, true}, tf[2] = {true, true};
    const float sc[2] = {1.f, 1.f};
    char* const img[2] = {Ki, Vi};
    const bf16_t* const src[2] = {qkv, qkv};
    const long ld[2] = {W3, W3};
    ImageLoad<2> L;
    images_issue<2>(L, src, ld, k0, col, bqkv, ub, tid);
    float kb[8][4];
    load_key_bias(kbias, k0, fq, kb);
    images_commit<2>(L, tf, sc, img, tid);
    __syncthreads();
    floatx4 s[8][2], dp[8][2];
    scores_t(Qi, Ki, qb, fr, fq, s);   // (q = qb + 16qt + fr, key = 16kt + 4fq + r)
    scores_t(Gi, Vi, qb, fr, fq, dp);  // dP(q, key) = dO[q]·V[key]
#pragma unroll
    for (int qt = 0; qt < 2; qt++) {
      const int q = qblk * BLK + qb + qt * 16 + fr;
#pragma unroll
      for (int kt = 0; kt < 8; kt++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const float p = __expf(s[kt][qt][r] + kb[kt][r] - lq[qt]);
          float g = dp[kt][qt][r];
          if (thresh)
            g = drop_hash(seed, ((uint64_t)bh * S + q) * S + j * BLK + kt * 16 + 4 * fq + r) >= thresh ? g * dscale
                                                                                                       : 0.f;
          s[kt][qt][r] = p * (g - Dv[qt]);  // dS
        }
    }
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int ra = 32 * c + 4 * fq, rb = ra + 16;
      short8 ktr[4];
#pragma unroll
      for (int dt = 0; dt < 4; dt++) ktr[dt] = rd_tr2<64>(Ki, ra, rb, dt * 16, lane);
#pragma unroll
      for (int qt = 0; qt < 2; qt++) {
        const short8 bs = pack_pair(s[2 * c][qt], s[2 * c + 1][qt]);
#pragma unroll
        for (int dt = 0; dt < 4; dt++) dqT[dt][qt] = mma(ktr[dt], bs, dqT[dt][qt]);
      }
    }
  }
  __syncthreads();
  char* st = sm + wave * 4096;
  stage_tile(st, dqT, qscale, fr, fq);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  store_tile(st, dqkv, q0 + qb, W3, h * AD, dbqkv, lane);
}

uint32_t attn_drop_thresh(float p) {
  if (p <= 0.f) return 0u;
  const double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 4294967295u : (uint32_t)t;
}

}  // namespace

// KFA_ATTN_PF=0: the S = 128 backward exchanges D through global scratch (the
// pre-round-4 form) instead of LDS.  (A persistent forward that prefetched the
// next (sequence, head)'s Q / K / V into registers measured 96.5 vs 80 us per
// BERT-base layer: its 72 prefetch VGPRs cost the third workgroup per CU and
// spilled — not kept.)
static bool attn_pf() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("KFA_ATTN_PF");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

static bool attn_long_forced() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("KFA_ATTN_LONG");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  return v == 1;
}

// ctx [B*S, heads*64] = attention(qkv [B*S, 3*heads*64] (+ bqkv), key_bias [B, S]); lse [B*heads, S]
// S = 128: one workgroup per (sequence, head); S = 128·n: per 128-query block, online softmax.
KFA_API int kfa_attn_fwd(const void* qkv, const float* bqkv, const float* key_bias, void* out, float* lse, int B, int S,
                         int heads, int d, float qscale, float p, unsigned long long seed, hipStream_t st) {
  if (!bqkv || !key_bias) return -1;  // the caller passes zeros: no branches around the prologue loads
  if (B <= 0 || heads <= 0 || S <= 0 || S % BLK || S > 8192 || d != AD || (long)B * heads * (S / BLK) >= (1L << 31))
    return -1;
  const uint32_t th = attn_drop_thresh(p);
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  if (S == AS && !attn_long_forced())
    hipLaunchKernelGGL(attn_fwd_kernel, dim3((unsigned)(B * heads)), dim3(256), 0, st, (const bf16_t*)qkv, bqkv,
                       key_bias, (bf16_t*)out, lse, heads, qscale, th, ds, (uint64_t)seed);
  else
    hipLaunchKernelGGL(attn_fwd_long_kernel, dim3((unsigned)((long)B * heads * (S / BLK))), dim3(256), 0, st,
                       (const bf16_t*)qkv, bqkv, key_bias, (bf16_t*)out, lse, heads, S, qscale, th, ds, (uint64_t)seed);
  return kfa_status();
}

// dqkv [B*S, 3H] (overwritten); dbqkv [3H] fp32 (+)= bias gradient (nullable)
// (out = the forward's ctx: D = rowsum(dO∘O) is formed from it).  work: B*heads*S floats (D of every query)
KFA_API int kfa_attn_bwd(const void* qkv, const float* bqkv, const float* key_bias, const void* out, const float* lse,
                         const void* dout, void* dqkv, float* dbqkv, int B, int S, int heads, int d, float qscale,
                         float p, unsigned long long seed, float* work, hipStream_t st) {
  if (!bqkv || !key_bias) return -1;
  if (B <= 0 || heads <= 0 || S <= 0 || S % BLK || S > 8192 || d != AD || (long)B * heads * (S / BLK) >= (1L << 31))
    return -1;
  const uint32_t th = attn_drop_thresh(p);
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  if (S == AS && !attn_long_forced()) {
    if (!work) return -3;
    if (attn_pf())
      hipLaunchKernelGGL(attn_bwd_kernel<true>, dim3((unsigned)(B * heads)), dim3(256), 0, st, (const bf16_t*)qkv,
                         bqkv, key_bias, (const bf16_t*)out, lse, (const bf16_t*)dout, (bf16_t*)dqkv, dbqkv, work, heads,
                         qscale, th, ds, (uint64_t)seed);
    else
      hipLaunchKernelGGL(attn_bwd_kernel<false>, dim3((unsigned)(B * heads)), dim3(256), 0, st, (const bf16_t*)qkv,
                         bqkv, key_bias, (const bf16_t*)out, lse, (const bf16_t*)dout, (bf16_t*)dqkv, dbqkv, work, heads,
                         qscale, th, ds, (uint64_t)seed);
    return kfa_status();
  }
  if (!work) return -3;
  const long tokens = (long)B * S;
  hipLaunchKernelGGL(attn_rowdot_kernel, dim3((unsigned)((tokens * heads + 255) / 256)), dim3(256), 0, st,
                     (const bf16_t*)dout, (const bf16_t*)out, work, tokens, heads, S);
  const dim3 grid((unsigned)((long)B * heads * (S / BLK)));
  hipLaunchKernelGGL(attn_bwd_kv_long_kernel, grid, dim3(256), 0, st, (const bf16_t*)qkv, bqkv, key_bias, lse, work,
                     (const bf16_t*)dout, (bf16_t*)dqkv, dbqkv, heads, S, qscale, th, ds, (uint64_t)seed);
  hipLaunchKernelGGL(attn_bwd_q_long_kernel, grid, dim3(256), 0, st, (const bf16_t*)qkv, bqkv, key_bias, lse, work,
                     (const bf16_t*)dout, (bf16_t*)dqkv, dbqkv, heads, S, qscale, th, ds, (uint64_t)seed);
  return kfa_status();
}
