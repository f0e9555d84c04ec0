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
#include <algorithm>

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

// Dropout of the attention probabilities (every kernel of this file): ONE 32-bit
// counter hash per PAIR of scores (q, k) and (q, k + 16), k with bit 4 clear, whose
// 16-bit halves decide the two keeps: keep iff half >= t16 = round(p·2^16) (drop
// probability t16 / 2^16, kept values scaled by 2^16 / (2^16 − t16)).  Every lane
// layout below holds both keys of a pair in one lane (key tiles kt and kt + 1 of 16),
// so a pair costs one hash — half the quarter-rate v_mul_lo_u32 work of a per-score
// hash, which was ~40 % of the forward's VALU cycles.
__device__ __forceinline__ uint32_t attn_pair_hash(uint64_t seed, uint64_t row, int S, int key_lo) {
  return drop_hash(seed, row * (uint64_t)S + (uint64_t)key_lo);
}
// S = 128: the index row·128 + key never carries across a 2^32 boundary, so
// drop_hash's 64-bit index splits into lo = (row << 7) ^ key and hi = row >> 25 —
// per row (lane) once; a pair is then one xor-add plus the 32-bit finaliser.
struct RowKey {
  uint32_t a, b;
};
__device__ __forceinline__ RowKey row_key128(uint64_t seed, uint64_t row) {
  return RowKey{(uint32_t)(row << 7) ^ (uint32_t)seed, (uint32_t)(seed >> 32) + __umul24((uint32_t)(row >> 25), 0x9E3779u)};
}
__device__ __forceinline__ uint32_t pair_hash128(RowKey k, uint32_t key_lo) {
  uint32_t x = (k.a ^ key_lo) + k.b;  // == drop_hash(seed, row·128 + key_lo)
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ bool keep_lo(uint32_t h, uint32_t t16) { return (h & 0xffffu) >= t16; }
__device__ __forceinline__ bool keep_hi(uint32_t h, uint32_t t16) { return (h >> 16) >= t16; }

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// Packed keep mask (S = 128): word [bh][c][q] (c = (key >> 2) & 3) holds bit
// (key >> 4)·4 + (key & 3) for the 32 keys with that c — exactly the 32 keys one
// forward lane (fq = c) owns for query q, so the forward stores one dword per lane
// and query, and a backward lane reads its 4 consecutive queries as one 16-B chunk.
// 2 KiB per head (6 MiB per BERT-base layer at 256 x 128): the backward reads bits
// instead of re-hashing every score.
//
// DROP: 0 no dropout, 1 pair hash, 2 pair hash + write the packed mask.
template <int DROP>
__global__ __launch_bounds__(256, 3) void attn_fwd_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ bqkv,
                                                          const float* __restrict__ kbias, bf16_t* __restrict__ out,
                                                          float* __restrict__ lse, uint32_t* __restrict__ mask, int heads,
                                                          float qscale, uint32_t thresh, float dscale, uint64_t seed) {
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
  // scores in log2 units: q is scaled by log2(e)/sqrt(d) and the key mask by log2(e),
  // so the softmax exponent is one subtraction + v_exp_f32 per score
  const float sc[3] = {qscale * kLog2e, 1.f, 1.f};
  char* const img[3] = {Qi, Ki, Vi};
  const bf16_t* const src[3] = {qkv, qkv, qkv};
  const long ld[3] = {3L * H, 3L * H, 3L * H};
  ImageLoad<3> L;
  images_issue<3>(L, src, ld, row0, col, bqkv, ub, tid);
  float kb[8][4];
  load_key_bias(kbias, row0, fq, kb);
  images_commit<3>(L, tf, sc, img, tid);
#pragma unroll
  for (int kt = 0; kt < 8; kt++)
#pragma unroll
    for (int r = 0; r < 4; r++) kb[kt][r] *= kLog2e;
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
        const float e = __builtin_amdgcn_exp2f(s[kt][qt][r] - mx);
        s[kt][qt][r] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    if (fq == 0) lse[(long)bh * AS + q] = (mx + __log2f(sum)) * kLn2;  // natural-log units
    const float inv = 1.f / sum;
    if constexpr (DROP == 0) {
#pragma unroll
      for (int kt = 0; kt < 8; kt++)
#pragma unroll
        for (int r = 0; r < 4; r++) s[kt][qt][r] *= inv;
    } else {
      const float invd = inv * dscale;
      RowKey rk = row_key128(seed, (uint64_t)bh * AS + q);
      rk.a ^= 4 * fq;  // this lane's keys 32kp + 4fq + r: the fq bits are disjoint from 32kp + r
      uint32_t bits = 0;
#pragma unroll
      for (int kp = 0; kp < 4; kp++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const uint32_t hh = pair_hash128(rk, 32 * kp + r);
          const bool k0 = keep_lo(hh, thresh), k1 = keep_hi(hh, thresh);
          s[2 * kp][qt][r] = k0 ? s[2 * kp][qt][r] * invd : 0.f;
          s[2 * kp + 1][qt][r] = k1 ? s[2 * kp + 1][qt][r] * invd : 0.f;
          if constexpr (DROP == 2) bits |= ((uint32_t)k0 << (8 * kp + r)) | ((uint32_t)k1 << (8 * kp + 4 + r));
        }
      if constexpr (DROP == 2) mask[((long)bh * 4 + fq) * AS + q] = bits;
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
//
// Per-query operands through the not-yet-written part of dSᵀ: step j's dS lands in
// the query columns 32j..32j+31 of the wave's own 32 key rows, so before phase A
// each wave parks, in THOSE columns of its rows kw..kw+11, what step j will read:
// D and lse·log2(e) of the step's 32 queries (rows kw..kw+3) and, with a forward
// mask (DROP 2), the step's keep-mask words (rows kw+4..kw+11).  A step reads its
// block (one ds_read_b128 per 4 queries) before it overwrites it with dS — the
// reads replace 64 ds_bpermute lane shuffles and 64 per-score hashes per lane.
// DROP: 0 no dropout, 1 pair hash (no mask), 2 packed mask from the forward (parked
// in LDS), 3 packed mask read from memory per step (one step ahead).
template <int DROP>
__global__ __launch_bounds__(256, 2) void attn_bwd_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ bqkv,
                                                          const float* __restrict__ kbias, const bf16_t* __restrict__ out,
                                                          const float* __restrict__ lse, const bf16_t* __restrict__ dout,
                                                          bf16_t* __restrict__ dqkv, float* __restrict__ dbqkv,
                                                          const uint32_t* __restrict__ mask, int heads, float qscale,
                                                          uint32_t thresh, float dscale, uint64_t seed) {
  __shared__ __attribute__((aligned(16))) char sm[3 * 16384 + 32768];  // 80 KiB
  char* Qi = sm;            // [128 q][64]      q·scale (+ bias)
  char* Ki = sm + 16384;    // [128 key][64]    k (+ bias)
  char* Gi = sm + 32768;    // [128 q][64]      dO
  char* dST = sm + 49152;   // [128 key][128 q] dL/dS, transposed
  float* Dx = reinterpret_cast<float*>(dST + 12 * 256);  // D exchange: rows 12-13 (no parked block there)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int bh = blockIdx.x, b = bh / heads, h = bh - b * heads, H = heads * AD;
  const long row0 = (long)b * AS, W3 = 3L * H;
  const int kw = wave * 32;
  // every global load up front, in consumption order: biases, Q / K / dO image
  // rows, this lane's V operand pieces V[kw + 16kt + fr][32ks + 8fq ..] (+ bias),
  // the O half-row for D, the lse / mask chunks this lane parks
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
  // a lane half a row (32 d), the pair combines with one shuffle
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
  // parked D / lse chunk of this lane: step cj, kind cw (0 D, 1 lse), queries cq..cq+3
  const int cj = lane >> 4, cw = (lane >> 3) & 1, cqt = (lane >> 2) & 1, cf = lane & 3;
  const int cq = 32 * cj + 16 * cqt + 4 * cf;
  const float4 lse4 = *reinterpret_cast<const float4*>(lse + (long)bh * AS + cq);
  // parked mask chunks: ids lane, lane + 64 -> (step, c, qt, f): words [bh][c][32 step + 16 qt + 4 f ..]
  uint4 mraw[2];
  if constexpr (DROP == 2) {
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const int id = lane + 64 * t, mj = id >> 5, mc = (id >> 3) & 3, mqt = (id >> 2) & 1, mf = id & 3;
      mraw[t] = *reinterpret_cast<const uint4*>(mask + ((long)bh * 4 + mc) * AS + 32 * mj + 16 * mqt + 4 * mf);
    }
  }
  // DROP 3: this lane's mask words straight from memory, one step ahead
  const uint32_t* const mlane = mask + ((long)bh * 4 + ((fr >> 2) & 3)) * AS + 4 * fq;
  uint4 mg[2] = {};
  if constexpr (DROP == 3) {
#pragma unroll
    for (int qt = 0; qt < 2; qt++) mg[qt] = *reinterpret_cast<const uint4*>(mlane + 16 * qt);
  }
  float kbv[2];
#pragma unroll
  for (int kt = 0; kt < 2; kt++) kbv[kt] = kbias[row0 + kw + kt * 16 + fr] * kLog2e;
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

  // D[q] = Σ_d dO[q][d]·O[q][d]: this wave's 32 queries -> the exchange row
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
    if (!(lane & 1)) Dx[dq] = acc;
  }
  if constexpr (DROP == 2) {
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const int id = lane + 64 * t, mj = id >> 5, mc = (id >> 3) & 3, mqt = (id >> 2) & 1, mf = id & 3;
      *reinterpret_cast<uint4*>(dST + off128(kw + 4 + 2 * mc + mqt, 32 * mj + 8 * mf)) = mraw[t];
    }
  }
  __syncthreads();
  {
    const float4 d4 = *reinterpret_cast<const float4*>(Dx + cq);
    const float4 v = cw ? make_float4(lse4.x * kLog2e, lse4.y * kLog2e, lse4.z * kLog2e, lse4.w * kLog2e) : d4;
    *reinterpret_cast<float4*>(dST + off128(kw + 2 * cw + cqt, 32 * cj + 8 * cf)) = v;
  }
  __syncthreads();  // every wave has read the D exchange row before phase A writes dSᵀ over it
  short8 kreg[2][2];
#pragma unroll
  for (int kt = 0; kt < 2; kt++)
#pragma unroll
    for (int ks = 0; ks < 2; ks++) kreg[kt][ks] = rd_row<64>(Ki, kw + kt * 16 + fr, ks * 32 + fq * 8);
  const int mbit = 8 * wave + (fr & 3), mrow = kw + 4 + 2 * ((fr >> 2) & 3);  // mask bit of key tile 0 / parked row
  const int dsbits = __float_as_int(dscale);

  // ---- phase A: 4 steps of 32 queries; dvT / dkT[dt][kt][r] = dV / dK(key = kw + 16kt + fr, d = 16dt + 4fq + r)
  floatx4 dvT[4][2], dkT[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; dt++) dvT[dt][0] = dvT[dt][1] = dkT[dt][0] = dkT[dt][1] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; j++) {
    // this step's parked operands (read before the step's dS overwrites them)
    float4 Dv[2], Lv[2];
    uint4 mw[2] = {};
#pragma unroll
    for (int qt = 0; qt < 2; qt++) {
      Dv[qt] = *reinterpret_cast<const float4*>(dST + off128(kw + qt, 32 * j + 8 * fq));
      Lv[qt] = *reinterpret_cast<const float4*>(dST + off128(kw + 2 + qt, 32 * j + 8 * fq));
      if constexpr (DROP == 2) mw[qt] = *reinterpret_cast<const uint4*>(dST + off128(mrow + qt, 32 * j + 8 * fq));
      if constexpr (DROP == 3) {
        mw[qt] = mg[qt];
        if (j < 3) mg[qt] = *reinterpret_cast<const uint4*>(mlane + 32 * (j + 1) + 16 * qt);
      }
    }
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
      const float Dr[4] = {Dv[qt].x, Dv[qt].y, Dv[qt].z, Dv[qt].w};
      const float Lr[4] = {Lv[qt].x, Lv[qt].y, Lv[qt].z, Lv[qt].w};
      const uint32_t Mr[4] = {mw[qt].x, mw[qt].y, mw[qt].z, mw[qt].w};
#pragma unroll
      for (int r = 0; r < 4; r++) {
        uint32_t hh = 0;
        if constexpr (DROP == 1)
          hh = pair_hash128(row_key128(seed, (uint64_t)bh * AS + 32 * j + 16 * qt + 4 * fq + r), kw + fr);
#pragma unroll
        for (int kt = 0; kt < 2; kt++) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[qt][kt][r], kLog2e, kbv[kt]) - Lr[r]);
          const float g = dp[qt][kt][r];
          if constexpr (DROP == 0) {
            pd[qt][kt][r] = p;
            ds[qt][kt][r] = p * (g - Dr[r]);
          } else {
            float m;
            if constexpr (DROP == 1) m = (kt ? keep_hi(hh, thresh) : keep_lo(hh, thresh)) ? dscale : 0.f;
            else m = __int_as_float(__builtin_amdgcn_sbfe((int)Mr[r], mbit + 4 * kt, 1) & dsbits);
            pd[qt][kt][r] = p * m;
            ds[qt][kt][r] = p * fmaf(g, m, -Dr[r]);
          }
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
  bf16_t* const drow = dqkv + (row0 + kw) * W3 + h * AD + c * 8;
#pragma unroll
  for (int jj = 0; jj < 3; jj++)
#pragma unroll
    for (int it = 0; it < 4; it++) {
      const int r = it * 8 + (lane >> 3);
      *reinterpret_cast<uint4*>(drow + r * W3 + jj * H) = *reinterpret_cast<const uint4*>(st + jj * 4096 + off64(r, c * 8));
    }
  if (dbqkv) {  // bias-gradient column sums of this wave's 32 rows
    // dbqkv here is the PARTIAL buffer [B * 4][3H]: row (b, wave) gets this wave's sums
    // of its head's 3 x 64 columns — every element written once, no atomics (the per-wave
    // atomics into [3H] serialised 1024 adds per element at L2: +160 us / layer);
    // kfa_attn_bwd sums the rows into the bias gradient afterwards
    float* const prow = dbqkv + ((long)b * 4 + wave) * W3 + h * AD + c * 8;
#pragma unroll
    for (int jj = 0; jj < 3; jj++) {
      float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int it = 0; it < 4; it++) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(st + jj * 4096 + off64(it * 8 + (lane >> 3), c * 8)), f);
#pragma unroll
        for (int e = 0; e < 8; e++) cs[e] += f[e];
      }
#pragma unroll
      for (int o = 8; o < 64; o <<= 1)
#pragma unroll
        for (int e = 0; e < 8; e++) cs[e] += __shfl_xor(cs[e], o, 64);
      if (lane < 8) {
        *reinterpret_cast<float4*>(prow + jj * H) = make_float4(cs[0], cs[1], cs[2], cs[3]);
        *reinterpret_cast<float4*>(prow + jj * H + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
      }
    }
  }
}

// out[c] (+)= sum over the R partial rows part[r][c] (attn_bwd_kernel's per-(sequence,
// wave) bias-gradient rows): block = 64 columns x 4 row lanes, grid.y row chunks, one
// fp32 atomic per column per block
__global__ __launch_bounds__(256) void attn_dbias_reduce(const float* __restrict__ part, long R, int C,
                                                         float* __restrict__ out, long rows_per_block) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6;
  const long r0 = (long)blockIdx.y * rows_per_block, r1 = min(R, r0 + rows_per_block);
  float s = 0.f;
  if (c < C)
    for (long r = r0 + rl; r < r1; r += 4) s += part[r * C + c];
  red[rl][threadIdx.x & 63] = s;
  __syncthreads();
  if (rl == 0 && c < C) atomicAdd(out + c, (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]));
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
      for (int kp = 0; kp < 4; kp++) {
        float pp[2][4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
          float v0 = s[2 * kp][qt][r], v1 = s[2 * kp + 1][qt][r];
          if (thresh) {
            const uint32_t hh = attn_pair_hash(seed, (uint64_t)bh * S + q, S, j * BLK + 32 * kp + 4 * fq + r);
            v0 = keep_lo(hh, thresh) ? v0 * dscale : 0.f;
            v1 = keep_hi(hh, thresh) ? v1 * dscale : 0.f;
          }
          pp[0][r] = v0;
          pp[1][r] = v1;
        }
#pragma unroll
        for (int u = 0; u < 2; u++)
          *reinterpret_cast<uint2*>(Pw + off128(qt * 16 + fr, (2 * kp + u) * 16 + 4 * fq)) =
              pack4(pp[u][0], pp[u][1], pp[u][2], pp[u][3]);
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
          const uint32_t hh =
              thresh ? attn_pair_hash(seed, (uint64_t)bh * S + i * BLK + qb4 + r, S, kblk * BLK + kw + fr) : 0u;
#pragma unroll
          for (int kt = 0; kt < 2; kt++) {
            const float p = __expf(s[qt][kt][r] + kbv[kt] - lq);
            float g = dp[qt][kt][r], pv = p;
            if (thresh) {
              const bool keep = kt ? keep_hi(hh, thresh) : keep_lo(hh, thresh);
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
      for (int kp = 0; kp < 4; kp++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const uint32_t hh =
              thresh ? attn_pair_hash(seed, (uint64_t)bh * S + q, S, j * BLK + 32 * kp + 4 * fq + r) : 0u;
#pragma unroll
          for (int u = 0; u < 2; u++) {
            const int kt = 2 * kp + u;
            const float p = __expf(s[kt][qt][r] + kb[kt][r] - lq[qt]);
            float g = dp[kt][qt][r];
            if (thresh) g = (u ? keep_hi(hh, thresh) : keep_lo(hh, thresh)) ? g * dscale : 0.f;
            s[kt][qt][r] = p * (g - Dv[qt]);  // dS
          }
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

// t16 = round(p·2^16) (0: no dropout) and the keep scale 2^16 / (2^16 − t16)
uint32_t attn_drop_t16(float p) {
  if (!(p > 0.f)) return 0u;
  const double t = (double)p * 65536.0 + 0.5;
  return t >= 65536.0 ? 65536u : (uint32_t)t;
}
float attn_drop_scale(uint32_t t16) { return t16 >= 65536u ? 0.f : 65536.f / (float)(65536u - t16); }

}  // namespace

// (A persistent forward that prefetched the next (sequence, head)'s Q / K / V into
// registers measured 96.5 vs 80 us per BERT-base layer: its 72 prefetch VGPRs cost
// the third workgroup per CU and spilled — not kept.)
// KFA_ATTN_MASK_LDS=0: the backward reads the forward's keep mask from memory per
// step instead of parking it in LDS (A/B)
static bool attn_mask_lds() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("KFA_ATTN_MASK_LDS");
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

// words of the packed keep mask the S = 128 forward can write (0 when it writes none)
KFA_API long kfa_attn_mask_words(int B, int S, int heads) {
  return (S == AS && !attn_long_forced()) ? (long)B * heads * 4 * AS : 0L;
}

// ctx [B*S, heads*64] = attention(qkv [B*S, 3*heads*64] (+ bqkv), key_bias [B, S]); lse [B*heads, S]
// S = 128: one workgroup per (sequence, head); S = 128·n: per 128-query block, online softmax.
// mask (nullable; kfa_attn_mask_words words): the S = 128 kernel stores its dropout keep bits there.
KFA_API int kfa_attn_fwd(const void* qkv, const float* bqkv, const float* key_bias, void* out, float* lse, int B, int S,
                         int heads, int d, float qscale, float p, unsigned long long seed, unsigned* mask,
                         hipStream_t st) {
  if (!bqkv || !key_bias) return -1;  // the caller passes zeros: no branches around the prologue loads
  if (B <= 0 || heads <= 0 || S <= 0 || S % BLK || S > 8192 || d != AD || (long)B * heads * (S / BLK) >= (1L << 31))
    return -1;
  const uint32_t th = attn_drop_t16(p);
  const float ds = attn_drop_scale(th);
  if (S == AS && !attn_long_forced()) {
    const dim3 grid((unsigned)(B * heads));
    if (!th)
      hipLaunchKernelGGL(attn_fwd_kernel<0>, grid, dim3(256), 0, st, (const bf16_t*)qkv, bqkv, key_bias, (bf16_t*)out,
                         lse, (uint32_t*)nullptr, heads, qscale, th, ds, (uint64_t)seed);
    else if (!mask)
      hipLaunchKernelGGL(attn_fwd_kernel<1>, grid, dim3(256), 0, st, (const bf16_t*)qkv, bqkv, key_bias, (bf16_t*)out,
                         lse, (uint32_t*)nullptr, heads, qscale, th, ds, (uint64_t)seed);
    else
      hipLaunchKernelGGL(attn_fwd_kernel<2>, grid, dim3(256), 0, st, (const bf16_t*)qkv, bqkv, key_bias, (bf16_t*)out,
                         lse, (uint32_t*)mask, heads, qscale, th, ds, (uint64_t)seed);
  } else {
    hipLaunchKernelGGL(attn_fwd_long_kernel, dim3((unsigned)((long)B * heads * (S / BLK))), dim3(256), 0, st,
                       (const bf16_t*)qkv, bqkv, key_bias, (bf16_t*)out, lse, heads, S, qscale, th, ds, (uint64_t)seed);
  }
  return kfa_status();
}

// dqkv [B*S, 3H] (overwritten); dbqkv [3H] fp32 (+)= bias gradient (nullable)
// (out = the forward's ctx: D = rowsum(dO∘O) is formed from it).  work: B*heads*S floats (D of every query,
// S > 128).  mask: the S = 128 forward's keep bits (nullable: the kernel re-hashes).
KFA_API long kfa_attn_dbias_part_floats(int B, int heads) { return (long)B * 4 * 3 * heads * AD; }

KFA_API int kfa_attn_bwd(const void* qkv, const float* bqkv, const float* key_bias, const void* out, const float* lse,
                         const void* dout, void* dqkv, float* dbqkv, int B, int S, int heads, int d, float qscale,
                         float p, unsigned long long seed, const unsigned* mask, float* work, float* dbpart,
                         hipStream_t st) {
  if (!bqkv || !key_bias) return -1;
  if (B <= 0 || heads <= 0 || S <= 0 || S % BLK || S > 8192 || d != AD || (long)B * heads * (S / BLK) >= (1L << 31))
    return -1;
  const uint32_t th = attn_drop_t16(p);
  const float ds = attn_drop_scale(th);
  if (S == AS && !attn_long_forced()) {
    const dim3 grid((unsigned)(B * heads));
    float* const dbias_out = dbqkv;
    if (dbqkv) {  // the kernel writes per-(sequence, wave) partial rows; summed below
      if (!dbpart) return -3;
      dbqkv = dbpart;
    }
    if (!th)
      hipLaunchKernelGGL(attn_bwd_kernel<0>, grid, dim3(256), 0, st, (const bf16_t*)qkv, bqkv, key_bias,
                         (const bf16_t*)out, lse, (const bf16_t*)dout, (bf16_t*)dqkv, dbqkv, (const uint32_t*)nullptr,
                         heads, qscale, th, ds, (uint64_t)seed);
    else if (!mask)
      hipLaunchKernelGGL(attn_bwd_kernel<1>, grid, dim3(256), 0, st, (const bf16_t*)qkv, bqkv, key_bias,
                         (const bf16_t*)out, lse, (const bf16_t*)dout, (bf16_t*)dqkv, dbqkv, (const uint32_t*)nullptr,
                         heads, qscale, th, ds, (uint64_t)seed);
    else if (attn_mask_lds())
      hipLaunchKernelGGL(attn_bwd_kernel<2>, grid, dim3(256), 0, st, (const bf16_t*)qkv, bqkv, key_bias,
                         (const bf16_t*)out, lse, (const bf16_t*)dout, (bf16_t*)dqkv, dbqkv, (const uint32_t*)mask,
                         heads, qscale, th, ds, (uint64_t)seed);
    else
      hipLaunchKernelGGL(attn_bwd_kernel<3>, grid, dim3(256), 0, st, (const bf16_t*)qkv, bqkv, key_bias,
                         (const bf16_t*)out, lse, (const bf16_t*)dout, (bf16_t*)dqkv, dbqkv, (const uint32_t*)mask,
                         heads, qscale, th, ds, (uint64_t)seed);
    if (dbias_out) {
      const long R = (long)B * 4;
      const int C = 3 * heads * AD;
      const long chunks = std::min<long>(16, (R + 63) / 64);
      hipLaunchKernelGGL(attn_dbias_reduce, dim3((unsigned)((C + 63) / 64), (unsigned)chunks), dim3(256), 0, st,
                         dbpart, R, C, dbias_out, (R + chunks - 1) / chunks);
    }
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
