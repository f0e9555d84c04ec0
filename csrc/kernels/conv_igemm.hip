// Implicit-GEMM convolution on MFMA (bf16 in, fp32 accumulate), NHWC.
// SURVEY §2.6 K7 (ResNet-50 conv2d fwd + dgrad) and K1 (plain GEMM = 1x1 conv).
//
// One kernel computes  D[m][n] = sum_k A[m][k] * B[n][k]  (+ E[m][n])  where
// (with bnb.emb: + E[m][n] * bit(emb, m*N + n), the residual gradient of a
// BN + residual + ReLU output formed from its raw gradient and ReLU bit mask)
//   A = implicit im2col of an NHWC tensor T[Nb][H][W][C]:
//         m = (nb, p, q) in [Nb][P][Q],  k = (r, s, c) in [R][S][C]
//         A[m][k] = T[nb][p*sa + r*ra + oa][q*sa + s*ra + ob][c]   (0 outside)
//   B = [N][K] row-major bf16 (K contiguous) — conv weights in [Cout][R][S][Cin]
//   D = bf16 rows, row m written at pixel (nb, p*os + oph, q*os + opw) of an
//       [Nb][OH][OW][ldd] tensor.
// Forward conv:   sa = stride, ra = +1, oa = -pad, os = 1.
// Dgrad stride 1: T = dY, ra = -1, oa = +pad, B = W transposed to [Cin][R][S][Cout].
// Dgrad stride 2: one launch per output parity class (ph, pw) over its tap subset
//                 (os = 2), B = the class's tap-subset weights (see conv.py).
//
// Tiling for CDNA4: 256 threads = 4 waves, each wave owns a 64x64 output tile
// (4x4 MFMA 16x16x32 bf16 tiles, 64 fp32 accumulator VGPRs).  Block tiles
// 128x128 (2x2 waves) or 256x64 (4x1, for Cout = 64 layers).  BK = 64 = one
// (r, s) tap slice (C % 64 == 0).  Global->register prefetch of tile k+1 is
// issued before the MFMAs of tile k (T14) — across tile boundaries too: the
// blocks are persistent (2 per CU) and sweep an XCD-local tile range, so the
// next tile's first slice loads under the current tile's last MFMAs and
// epilogue.  LDS is double-buffered (one barrier
// per k-tile) and XOR-swizzled (chunk ^= (row>>1)&7) so the 16-lane groups of
// each ds_read_b128 hit 16 distinct 16-B slots.  Operand roles are chosen so
// each lane's 4 accumulator rows are 4 CONSECUTIVE output channels (8-B stores).
#include <cstdlib>

#include "common.h"

namespace {

#ifndef KFA_CONV_STORE_AUX
#define KFA_CONV_STORE_AUX 2  // output stores non-temporal (streamed; +1.7 % ResNet-50 vs 0, docs/kernels.md)
#endif

constexpr int BK = 64;
constexpr int kBnSlots = 64;  // must match batchnorm.hip kSlots (fused statistics land in its slots)

// Backward BatchNorm statistics fused into a dgrad epilogue: the dgrad output is
// dL/dy of a BatchNorm(+ReLU) whose input x / output y / batch mean are given;
// the epilogue accumulates sum(dz) and sum(dz * (x - mean)), dz = dy * (y > 0),
// into the BN slots (what bn_bwd_partial computes), so the BN backward skips
// that pass.  x == nullptr: forward statistics (sum, sum of squares) instead.
struct BnBwd {
  const bf16_t* x;
  const bf16_t* y;   // ReLU mask source (forward output), or nullptr: mask from x with ss
  const float* ss;   // the BN forward's [scale | shift] (used when relu && !y && !mb)
  const uint8_t* mb; // the BN forward's output ReLU bit mask (BN + residual; used when relu && !y)
  const float* mean;
  int relu;
  const uint8_t* emb;  // addend E masked by these ReLU bits (E = a block output's raw gradient), or nullptr
};

// BatchNorm-apply + ReLU prologue (PRO): T is a BatchNorm's RAW input x and the
// A operand is relu(x * scale[c] + shift[c]) (bf16, rounded exactly as bn_apply
// rounds it), applied on the register path between the global load and the LDS
// store; padding taps stay 0.  The blocks of tile column 0 also write the
// normalised value of every centre-tap slice to y (which then covers each input
// pixel once — stride 1, P == H, Q == W, host-checked), so the backward's weight
// gradient reads y as before and the BatchNorm's own apply pass is gone.
struct Pro {
  const float* ss;  // [scale | shift], 2C floats
  bf16_t* y;        // normalised activation (same layout as T), or nullptr
};

struct Geo {
  int Nb, H, W, C;   // gathered tensor T
  int P, Q;          // GEMM row space (m = nb*P*Q + p*Q + q)
  int R, S;          // taps
  int sa, ra, oa, ob;  // gather: ih = p*sa + r*ra + oa, iw = q*sa + s*ra + ob
  int M, N, K;       // GEMM sizes (K = R*S*C)
  int OH, OW, os, oph, opw, ldd;  // output pixel mapping / row stride (elements)
  unsigned t_bytes, b_bytes, d_bytes;  // buffer extents: out-of-range lanes read 0 / drop stores
};

// Buffer-resource loads/stores (T8): the hardware range check turns padding
// taps and tile tails into zero loads / dropped stores with NO branch, so hipcc
// can keep counted vmcnt waits instead of draining to vmcnt(0) around each
// guarded load (cdna_hip_programming.md §5 'Three .s-level traps' (c)).
constexpr unsigned kOOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
#ifndef KFA_CONV_EPI_LOAD_AUX
#define KFA_CONV_EPI_LOAD_AUX 2  // epilogue addend / BN-input loads non-temporal (read once; +0.2 %)
#endif
__device__ __forceinline__ uint4 bload16(__amdgpu_buffer_rsrc_t r, unsigned off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, KFA_CONV_EPI_LOAD_AUX);
  return *reinterpret_cast<uint4*>(&v);
}

// 16 B per lane buffer -> LDS DMA (buffer_load_dwordx4 ... lds): voff per lane,
// soff wave-uniform.  A plain device function: the builtin named directly inside
// the templated kernel's lambdas stops clang's host pass from emitting the
// kernels' launch stubs.
__device__ __forceinline__ void buf_dma16(__amdgpu_buffer_rsrc_t r, bf16_t* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}
#ifndef KFA_CONV_LOAD_AUX
#define KFA_CONV_LOAD_AUX 0
#endif
// the gathered activation operand (each element used by one tile column only)
__device__ __forceinline__ void buf_dma16_act(__amdgpu_buffer_rsrc_t r, bf16_t* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0,
                                           KFA_CONV_LOAD_AUX);
}

// x / d for 0 <= x < 2^24 via an fp32 reciprocal + one correction step
// (hipcc's int32 division is a ~40-instruction sequence; these run per row).
__device__ __forceinline__ int fdiv(int x, int d, float rcp) {
  int q = (int)((float)x * rcp);
  const int r = x - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

// Workgroup barrier for LDS hand-off only.  __syncthreads() is a workgroup
// release fence too, which makes hipcc drain vmcnt(0) for the epilogue's
// global stores — and with them the prefetch loads in flight.  Nothing in this
// kernel needs global-memory ordering between waves, only LDS.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int N>
__device__ __forceinline__ void lgkm_wait() {
  if constexpr (N == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
  else static_assert(N < 0, "lgkm_wait: add the literal");
}

__device__ __forceinline__ int swz(int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3); }

// WM x WN waves, each owning TM x TN MFMA 16x16 tiles (wave tile 16TM x 16TN)
// (8 waves: 256 x 256 tiles of 128 x 64 per wave, one block per CU — half the
// operand bytes per MFMA of the 4-wave 128 x 128 tile; the epilogue then stages
// the wave tile in NHALF passes so it fits the one ring buffer it may use.)
// EPI: epilogue features compiled in (kEpiE addend, kEpiStats fused BN statistics,
// kEpiBnBwd backward statistics of the BN this dgrad feeds, kEpiEmb ReLU-bit-masked
// addend).  A feature's runtime pointer may still be null; features not compiled in
// cost no registers — the all-features build spilled (256 VGPRs) and serialised the
// main loop's LDS fragment reads on a reused register.
constexpr unsigned kEpiE = 1, kEpiStats = 2, kEpiBnBwd = 4, kEpiEmb = 8, kEpiYMask = 16, kEpiAll = 31;

struct EpiRes {  // buffer resources of the epilogue's output / addend / BN input / BN output
  __amdgpu_buffer_rsrc_t d, e, bx, by;
};

// Epilogue of one wave tile through LDS: MFMA leaves each lane 4 consecutive
// channels of one pixel (acc[ni][mi][r] = D(m = mw + 16 mi + fr, n = nw + 16 ni
// + 4 fq + r)); staging the wave's tile in LDS (XOR-swizzled 16-B chunks,
// conflict-free both ways) lets every lane store 16 B and a wave cover 128-B row
// segments, so the HBM writes of the memory-bound layers (K = 64..256) coalesce.
// NHALF staging passes over the wave's rows (1 for 64-row wave tiles; 4 for the
// 128-row ones, keeping the epilogue's in-flight loads at 48 VGPRs).  `stage`:
// this wave's 256 * (TM / NHALF) * TN staged elements; `first_barrier`: the
// first pass waits at a workgroup barrier before its LDS writes (the stage
// aliases an operand buffer other waves may still be reading).  Also: the
// residual-gradient addend (kEpiE, masked by ReLU bits with kEpiEmb) and the
// fused BatchNorm statistics (kEpiStats; kEpiBnBwd: backward statistics of the
// BN this dgrad feeds).  The accumulators are zeroed for the next tile.
template <int TM, int TN, int NHALF, unsigned EPI>
__device__ __forceinline__ void conv_epilogue(const Geo& g, floatx4 (&acc)[TN][TM], char* stage, bool first_barrier,
                                              int lane, int mw, int nw, int PQ, float rPQ, float rQ, bool lin_d,
                                              const bf16_t* E, float* stats, const BnBwd& bnb, const EpiRes& er) {
  constexpr int TMH = TM / NHALF;     // MFMA row tiles per pass
  constexpr int RB = 32 * TN;         // staged row bytes
  constexpr int CPR = 2 * TN;         // 16-B chunks per staged row
  constexpr int IT = (16 * TMH * CPR) / 64;  // 16-B row pieces per lane per pass
  const int fr = lane & 15, fq = lane >> 4;
  const int c = lane % CPR;
  const int n = nw + c * 8;
  float mu[8] = {0, 0, 0, 0, 0, 0, 0, 0}, msc[8], msf[8];
  constexpr bool kE = EPI & kEpiE, kST = EPI & kEpiStats, kBS = EPI & kEpiBnBwd, kEM = EPI & kEpiEmb;
  constexpr bool kYM = EPI & kEpiYMask;  // ReLU mask read from the BN output (else bits / recomputed from x)
  const bool bstat = kBS && kST && stats && bnb.x;
  const bool ymask = kYM && bnb.relu && bnb.y;       // mask from the output y
  const bool bmask = bnb.relu && !bnb.y && bnb.mb;   // from the output bit mask
  // else (relu) recomputed from x with the saved scale / shift
  if (bstat)
#pragma unroll
    for (int j = 0; j < 8; j++) {
      mu[j] = n + j < g.N ? bnb.mean[n + j] : 0.f;
      msc[j] = (bnb.relu && !ymask && !bmask && n + j < g.N) ? bnb.ss[n + j] : 0.f;
      msf[j] = (bnb.relu && !ymask && !bmask && n + j < g.N) ? bnb.ss[g.N + n + j] : 0.f;
    }
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // fused BN statistics
#pragma unroll
  for (int hh = 0; hh < NHALF; hh++) {
    // output offsets first, so the epilogue's global loads (residual-grad addend,
    // BN input / output for the fused backward statistics) are all in flight
    // while the tile is staged through LDS
    unsigned offs[IT];
#pragma unroll
    for (int it = 0; it < IT; it++) {
      const int m = mw + hh * TMH * 16 + it * (64 / CPR) + lane / CPR;
      unsigned orow;  // byte offset of output row m
      if (lin_d) {
        orow = (unsigned)m * (unsigned)g.ldd * 2u;
      } else {
        const int nb = fdiv(m, PQ, rPQ), rem = m - nb * PQ;
        const int p = fdiv(rem, g.Q, rQ), q = rem - p * g.Q;
        orow = (unsigned)((nb * g.OH + p * g.os + g.oph) * g.OW + (q * g.os + g.opw)) * (unsigned)g.ldd * 2u;
      }
      offs[it] = (m >= g.M || n >= g.N) ? kOOB : orow + (unsigned)n * 2u;
    }
    uint4 ev[IT], bx[IT], by[IT];
    unsigned mbits[IT], ebits[IT];
    if (kE && E)
#pragma unroll
      for (int it = 0; it < IT; it++) {
        ev[it] = bload16(er.e, offs[it]);
        if (kEM && bnb.emb) ebits[it] = offs[it] != kOOB ? (unsigned)bnb.emb[offs[it] >> 4] : 0u;
      }
    if (bstat)
#pragma unroll
      for (int it = 0; it < IT; it++) {
        bx[it] = bload16(er.bx, offs[it]);
        if (ymask) by[it] = bload16(er.by, offs[it]);
        if (bmask) mbits[it] = offs[it] != kOOB ? (unsigned)bnb.mb[offs[it] >> 4] : 0u;  // 8 bf16 = 16 B per bit byte
      }

    if (hh == 0 && first_barrier) lds_barrier();  // every wave is done reading the operand buffer under `stage`
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave read back its previous pass
#pragma unroll
    for (int mj = 0; mj < TMH; mj++)
#pragma unroll
      for (int ni = 0; ni < TN; ni++) {
        const int mi = hh * TMH + mj;
        const int row = mj * 16 + fr, col = ni * 16 + fq * 4;
        const uint2 o = make_uint2(pack2(acc[ni][mi][0], acc[ni][mi][1]), pack2(acc[ni][mi][2], acc[ni][mi][3]));
        *reinterpret_cast<uint2*>(stage + row * RB + (((col >> 3) ^ (row & (CPR - 1))) << 4) + (col & 7) * 2) = o;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < IT; it++) {
      const int r = it * (64 / CPR) + lane / CPR;
      const uint4 v = *reinterpret_cast<const uint4*>(stage + r * RB + ((c ^ (r & (CPR - 1))) << 4));
      const unsigned off = offs[it];
      uint4 o = v;
      if (kE && E) {  // wave-uniform branch
        float f[8], h[8];
        unpack8(v, f);
        unpack8(ev[it], h);
        if (kEM && bnb.emb) {  // residual gradient dz = dy * relu-mask, formed here instead of by the BN backward
#pragma unroll
          for (int j = 0; j < 8; j++) f[j] += ((ebits[it] >> j) & 1u) ? h[j] : 0.f;
        } else {
#pragma unroll
          for (int j = 0; j < 8; j++) f[j] += h[j];
        }
        o = pack8(f);
      }
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<decltype(__builtin_amdgcn_raw_buffer_load_b128(er.d, 0, 0, 0))*>(&o), er.d, off, 0, KFA_CONV_STORE_AUX);
      if (kST && stats && off != kOOB) {  // wave-uniform pointer test; per-lane row mask
        float f[8];
        unpack8(o, f);  // the bf16-rounded values the BatchNorm will see
        if (bstat) {    // backward statistics of the BN this dgrad feeds
          float xf[8];
          unpack8(bx[it], xf);
          if (ymask) {
            float yf[8];
            unpack8(by[it], yf);
#pragma unroll
            for (int j = 0; j < 8; j++) f[j] = yf[j] > 0.f ? f[j] : 0.f;
          } else if (bmask) {
#pragma unroll
            for (int j = 0; j < 8; j++) f[j] = ((mbits[it] >> j) & 1u) ? f[j] : 0.f;
          } else if (bnb.relu) {  // y = relu(fma(x, sc, sh)) exactly as bn_apply evaluated it
#pragma unroll
            for (int j = 0; j < 8; j++) f[j] = fmaf(xf[j], msc[j], msf[j]) > 0.f ? f[j] : 0.f;
          }
#pragma unroll
          for (int j = 0; j < 8; j++) { s1[j] += f[j]; s2[j] += f[j] * (xf[j] - mu[j]); }
        } else {
#pragma unroll
          for (int j = 0; j < 8; j++) { s1[j] += f[j]; s2[j] += f[j] * f[j]; }
        }
      }
    }
  }
  if (kST && stats) {
    // Butterfly-reduce over the lanes sharing channel chunk c = lane % CPR (xor
    // 8, 16, 32): every lane ends with its chunk's wave totals.  Lane L then
    // publishes channel (L % 8) * 8 + L / 8 — its own chunk, register L / 8
    // (a select chain, no shuffles) — so ONE 64-lane atomic instruction per
    // statistic covers the wave's 64 channels (CPR == 8: TN == 4).
    static_assert(CPR == 8, "fused BN statistics assume 64-channel wave tiles");
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
      for (int j = 0; j < 8; j++) { s1[j] += __shfl_xor(s1[j], o, 64); s2[j] += __shfl_xor(s2[j], o, 64); }
    const int jj = lane >> 3;
    float a = s1[0], b = s2[0];
#pragma unroll
    for (int j = 1; j < 8; j++) {
      a = jj == j ? s1[j] : a;
      b = jj == j ? s2[j] : b;
    }
    const int nc = n + jj;
    if (nc < g.N) {
      float* slot = stats + (long)(blockIdx.x % kBnSlots) * 2 * g.N;
      __hip_atomic_fetch_add(slot + nc, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(slot + g.N + nc, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
#pragma unroll
  for (int i = 0; i < TN; i++)
#pragma unroll
    for (int j = 0; j < TM; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
}

template <int WM, int WN, int TM, int TN, unsigned EPI, bool PRO = false>
__global__ __launch_bounds__(64 * WM * WN, 2) void conv_igemm_kernel(const bf16_t* __restrict__ T,
                                                                     const bf16_t* __restrict__ B,
                                                                     bf16_t* __restrict__ D, const bf16_t* __restrict__ E,
                                                                     const bf16_t* __restrict__ Z,
                                                                     float* __restrict__ stats, BnBwd bnb, Geo g,
                                                                     Pro pro = Pro{nullptr, nullptr}) {
  constexpr int NW = WM * WN, RPP = 8 * NW;  // waves; tile rows per staging pass (8 per wave)
  constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
  constexpr int AR = BM / RPP, BR = BN / RPP;  // 16-B chunks per thread per k-tile
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* As = smem;                  // [2][BM][BK]
  bf16_t* Bs = smem + 2 * BM * BK;    // [2][BN][BK]
  float* ssl = reinterpret_cast<float*>(smem + 2 * (BM + BN) * BK);  // PRO: [scale | shift] (2C floats)

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS-DMA bases in SGPRs
  const int wm = wave % WM, wn = wave / WM;
  const int ntn = (g.N + BN - 1) / BN;
  const int ntiles = ((g.M + BM - 1) / BM) * ntn;

  // Persistent blocks.  XCD-aware assignment (T1): the blocks that share an
  // XCD (b % 8) sweep one contiguous range of tiles, so tiles in flight on an
  // XCD share A/B panels in its L2.
  const int nwg = gridDim.x;
  const int G = nwg < 8 ? nwg : 8;                        // XCD groups that have blocks
  const int xcd = blockIdx.x % G, slot = blockIdx.x / G;
  const int nslot = (nwg - xcd + G - 1) / G;               // blocks in this group
  const int t_lo = (int)((long)ntiles * xcd / G), t_hi = (int)((long)ntiles * (xcd + 1) / G);
  const int my_tiles = t_hi - t_lo > slot ? (t_hi - t_lo - slot + nslot - 1) / nslot : 0;
  auto tile_of = [&](int i) { return t_lo + slot + i * nslot; };

  const int kc = tid & 7;
  const int rbase = tid >> 3;  // 0..RPP-1
  const int PQ = g.P * g.Q;
  const float rPQ = 1.f / (float)PQ, rQ = 1.f / (float)g.Q;
  // pointwise fast paths: A row m is T[m] (1x1 / stride 1 / no pad) and/or D row m is D[m]
  const bool lin_a = g.R == 1 && g.S == 1 && g.sa == 1 && g.oa == 0 && g.ob == 0 && g.H == g.P && g.W == g.Q;
  const bool lin_d = g.os == 1 && g.oph == 0 && g.opw == 0 && g.OH == g.P && g.OW == g.Q;
  int a_hb[AR], a_wb[AR], a_vo[AR];  // a_vo: byte offset of the row at tap (0, 0) + swizzled chunk (< 2^31, host-checked)
  unsigned b_off[BR];
  const __amdgpu_buffer_rsrc_t rT = rsrc(T, g.t_bytes), rB = rsrc(B, g.b_bytes), rD = rsrc(D, g.d_bytes);
  const __amdgpu_buffer_rsrc_t rE = rsrc(E ? E : D, E ? g.d_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rBX = rsrc(bnb.x ? bnb.x : D, bnb.x ? g.d_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rBY = rsrc(bnb.y ? bnb.y : D, bnb.y ? g.d_bytes : 0u);
  auto setup = [&](int tile) {
    const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
#pragma unroll
    for (int i = 0; i < AR; i++) {
      const int m = m0 + rbase + RPP * i;
      const int cs = (kc ^ ((((i * RPP) + rbase) >> 1) & 7)) * 8;  // this lane's swizzled source chunk
      if (m < g.M && lin_a) {
        a_hb[i] = 0;
        a_wb[i] = 0;
        a_vo[i] = (m * g.C + cs) * 2;
      } else if (m < g.M) {  // a_vo: the row's offset at tap (0, 0) (may lie outside the image)
        const int nb = fdiv(m, PQ, rPQ), rem = m - nb * PQ;
        const int p = fdiv(rem, g.Q, rQ), q = rem - p * g.Q;
        a_hb[i] = p * g.sa + g.oa;
        a_wb[i] = q * g.sa + g.ob;
        a_vo[i] = ((nb * g.H * g.W + a_hb[i] * g.W + a_wb[i]) * g.C + cs) * 2;
      } else {
        a_hb[i] = -(1 << 28);  // forces out-of-range
        a_wb[i] = 0;
        a_vo[i] = (int)kOOB;
      }
    }
#pragma unroll
    for (int i = 0; i < BR; i++) {
      const int n = n0 + rbase + RPP * i;
      const int cs = (kc ^ ((((i * RPP) + rbase) >> 1) & 7)) * 8;
      b_off[i] = n < g.N ? (unsigned)(n * g.K + cs) * 2u : kOOB;
    }
  };

  // Operand staging: LDS-DMA (global_load_lds_dwordx4).  Each wave-instruction
  // writes 1 KiB = 8 tile rows lane-linearly; the XOR swizzle is applied on the
  // per-lane SOURCE address (rule 21); padding taps / tails read as zero (range check).
  // No staging VGPRs, no ds_write pass; waits are counted by hand.
  const int nk = g.K / BK;
  const int total = my_tiles * nk;
  int setup_tile = -1;
  const int l8 = lane >> 3, pos = lane & 7;
  // DMA sources as 32-bit buffer offsets (buffer_load ... lds): the per-lane part
  // is fixed per tile (the swizzled chunk included), the k-slice's channel offset
  // goes in the SCALAR offset, padding taps / tails get an offset past the
  // buffer (read as 0 by the range check).  1x1 stride-1 layers then issue
  // their DMAs with no per-step vector math at all.
  // issue() runs for st = 0, 1, 2, ... in order: the (tile, k-slice, channel
  // offset, tap) of the next slice is carried incrementally (wave-uniform) instead
  // of four scalar divisions per k-step
  int nx_ti = 0, nx_kt = 0, nx_c0 = 0, nx_r = 0, nx_s = 0;
  // PRO register-path state of the slice in flight: raw A chunks, their source
  // offsets (for the y write), valid-tap bits, the slice's scalar offset / channel base
  uint4 pr_a[PRO ? AR : 1];
  int pr_vo[PRO ? AR : 1];
  unsigned pr_ok = 0;
  int pr_soff = 0, pr_ch = 0;
  bool pr_y = false;
  const int pr_cs = (kc ^ ((rbase >> 1) & 7)) * 8;  // this lane's source chunk (the same for every i: RPP % 16 == 0)
  auto ti_col0 = [&](int ti) { return tile_of(ti) % ntn == 0; };
  const __amdgpu_buffer_rsrc_t rY = rsrc(pro.y ? pro.y : D, pro.y ? g.t_bytes : 0u);
  auto issue = [&](int st, int buf) {
    (void)st;
    const int ti = nx_ti, k0 = nx_kt * BK, c0 = nx_c0;
    if (ti != setup_tile) { setup(tile_of(ti)); setup_tile = ti; }
    const int dh = nx_r * g.ra, dw = nx_s * g.ra;
    const int ta_off = (dh * g.W + dw) * g.C * 2;  // the tap's offset: one scalar add per DMA, no per-lane multiply
    nx_c0 += BK;  // advance to the next slice: BK channels of one tap, or BK / C whole taps (C < BK)
    while (nx_c0 >= g.C) {
      nx_c0 -= g.C;
      if (++nx_s == g.S) { nx_s = 0; nx_r++; }
    }
    if (++nx_kt == nk) { nx_kt = 0; nx_ti++; nx_c0 = 0; nx_r = 0; nx_s = 0; }
    if constexpr (PRO) {  // register path: loads now, normalised + stored to LDS by pro_store
      pr_soff = (lin_a ? k0 : c0) * 2;
      pr_ch = lin_a ? k0 : c0;
      pr_y = pro.y && (ti_col0(ti) && (lin_a || (dh + g.oa == 0 && dw + g.ob == 0)));
      pr_ok = 0;
#pragma unroll
      for (int i = 0; i < AR; i++) {
        int vo = a_vo[i];
        if (!lin_a) {
          const int ih = a_hb[i] + dh, iw = a_wb[i] + dw;
          const bool ok = (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
          vo = ok ? a_vo[i] + ta_off : (int)kOOB;
          pr_ok |= ok ? (1u << i) : 0u;
        } else {
          pr_ok |= 1u << i;
        }
        pr_vo[i] = vo;
        auto v = __builtin_amdgcn_raw_buffer_load_b128(rT, (unsigned)vo, (unsigned)pr_soff, KFA_CONV_LOAD_AUX);
        pr_a[i] = *reinterpret_cast<uint4*>(&v);
      }
    } else if (lin_a) {  // the whole offset but the slice's is fixed per tile (a_vo, setup)
#pragma unroll
      for (int i = 0; i < AR; i++)
        buf_dma16_act(rT, As + buf * BM * BK + (i * RPP + wave * 8) * BK, a_vo[i], k0 * 2);
    } else {
#pragma unroll
      for (int i = 0; i < AR; i++) {
        const int ih = a_hb[i] + dh, iw = a_wb[i] + dw;
        const bool ok = (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        const int vo = ok ? a_vo[i] + ta_off : (int)kOOB;  // selects, no branch
        buf_dma16_act(rT, As + buf * BM * BK + (i * RPP + wave * 8) * BK, vo, c0 * 2);
      }
    }
#pragma unroll
    for (int i = 0; i < BR; i++)
      buf_dma16(rB, Bs + buf * BN * BK + (i * RPP + wave * 8) * BK, (int)b_off[i], k0 * 2);
  };
  floatx4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; i++)
#pragma unroll
    for (int j = 0; j < TM; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  // Fragment reads ahead of the MFMAs that use them: k-half 0's A and B plus
  // k-half 1's B fragments are issued before k-half 0's MFMAs, k-half 1's A
  // fragments between the two MFMA groups, each group preceded by a counted
  // lgkmcnt.  The reads are inline asm: with compiler-visible ds_reads hipcc
  // re-used a few fragment registers and waited lgkmcnt(0) between small MFMA
  // groups (its wait pass does not count these reads exactly), exposing the LDS
  // latency several times per k-step.  sched_barrier after each wait keeps the
  // MFMAs behind it (rule 18).  TM + 2 TN <= 15 reads in flight (4-bit counter);
  // the 8-wave 256x256 variant keeps the plain form.
  auto compute = [&](int buf) {
    const bf16_t* Ab = As + buf * BM * BK;
    const bf16_t* Bb = Bs + buf * BN * BK;
    short8 af[2][TM], bf[2][TN];
    auto mfma = [&](int ks) {
#pragma unroll
      for (int ni = 0; ni < TN; ni++)
#pragma unroll
        for (int mi = 0; mi < TM; mi++)
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ks][ni], af[ks][mi], acc[ni][mi], 0, 0, 0);
    };
    auto rd = [&](const bf16_t* p) {
      short8 v;
      const unsigned la = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const bf16_t*)p;
      asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(la) : "memory");
      return v;
    };
    if constexpr (TM + 2 * TN <= 15) {
#pragma unroll
      for (int i = 0; i < TN; i++) bf[0][i] = rd(Bb + swz(wn * TN * 16 + i * 16 + fr, fq));
#pragma unroll
      for (int i = 0; i < TM; i++) af[0][i] = rd(Ab + swz(wm * TM * 16 + i * 16 + fr, fq));
#pragma unroll
      for (int i = 0; i < TN; i++) bf[1][i] = rd(Bb + swz(wn * TN * 16 + i * 16 + fr, 4 + fq));
      lgkm_wait<TN>();  // k-half 0's fragments landed; k-half 1's B reads may still be in flight
      __builtin_amdgcn_sched_barrier(0);
      mfma(0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; i++) af[1][i] = rd(Ab + swz(wm * TM * 16 + i * 16 + fr, 4 + fq));
      lgkm_wait<0>();
      __builtin_amdgcn_sched_barrier(0);
      mfma(1);
    } else if constexpr (PRO) {
      // 8-wave 256x256 tiles with the BatchNorm prologue: one k-half's 12 reads, wait,
      // its MFMAs.  Inline asm: with compiler-visible reads hipcc waited vmcnt(0) — the
      // NEXT slice's register loads and DMAs, issued at the top of the step — before
      // every step's first read (the plain variants keep the compiler's form below: no
      // such wait there, and its counted lgkmcnt interleave)
#pragma unroll
      for (int ks = 0; ks < 2; ks++) {
#pragma unroll
        for (int i = 0; i < TM; i++) af[ks][i] = rd(Ab + swz(wm * TM * 16 + i * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int i = 0; i < TN; i++) bf[ks][i] = rd(Bb + swz(wn * TN * 16 + i * 16 + fr, ks * 4 + fq));
        lgkm_wait<0>();
        __builtin_amdgcn_sched_barrier(0);
        mfma(ks);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ks++) {
#pragma unroll
        for (int i = 0; i < TM; i++)
          af[ks][i] = *reinterpret_cast<const short8*>(Ab + swz(wm * TM * 16 + i * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int i = 0; i < TN; i++)
          bf[ks][i] = *reinterpret_cast<const short8*>(Bb + swz(wn * TN * 16 + i * 16 + fr, ks * 4 + fq));
        mfma(ks);
      }
    }
  };
  // Epilogue: conv_epilogue (below the kernel) over this wave's tile, staged in
  // ring buffer `buf` once every wave is done reading it (its first pass's barrier)
  constexpr int NHALF = NW == 4 ? 1 : TM / 2;
  constexpr int WT = 256 * (TM / NHALF) * TN;  // staged elements per wave per pass
  static_assert(NW * WT <= (BM + BN) * BK, "conv epilogue stage must fit one ring buffer");
  const EpiRes er{rD, rE, rBX, rBY};
  auto epilogue = [&](int tile, int buf) {
    const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
    const int e = wave * WT;
    char* stage = reinterpret_cast<char*>(e < BM * BK ? As + buf * BM * BK + e : Bs + buf * BN * BK + (e - BM * BK));
    conv_epilogue<TM, TN, NHALF, EPI>(g, acc, stage, true, lane, m0 + wm * TM * 16, n0 + wn * TN * 16, PQ, rPQ, rQ,
                                      lin_d, E, stats, bnb, er);
  };

  // PRO: the slice's A chunks landed -> relu(x * sc + sh) (0 on padding taps) into
  // LDS `buf` at the positions the LDS-DMA would have filled; centre-tap slices of
  // tile column 0 also go to y.
  auto pro_store = [&](int buf) {
    if constexpr (PRO) {
      const int c = pr_ch + pr_cs;
      float sc[8], sh[8];
      {
        // inline-asm reads: compiler-visible ones got an s_waitcnt vmcnt(0) (draining the
        // next slice's B DMAs) in front of them
        typedef __attribute__((ext_vector_type(4))) float f32x4;
        f32x4 v[4];
        const unsigned la = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const float*)(ssl + c);
        const unsigned lb = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const float*)(ssl + g.C + c);
        asm volatile("ds_read_b128 %0, %1" : "=v"(v[0]) : "v"(la) : "memory");
        asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(v[1]) : "v"(la) : "memory");
        asm volatile("ds_read_b128 %0, %1" : "=v"(v[2]) : "v"(lb) : "memory");
        asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(v[3]) : "v"(lb) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]) :: "memory");
        const float4 a0 = make_float4(v[0][0], v[0][1], v[0][2], v[0][3]), a1 = make_float4(v[1][0], v[1][1], v[1][2], v[1][3]);
        const float4 b0 = make_float4(v[2][0], v[2][1], v[2][2], v[2][3]), b1 = make_float4(v[3][0], v[3][1], v[3][2], v[3][3]);
        sc[0] = a0.x; sc[1] = a0.y; sc[2] = a0.z; sc[3] = a0.w; sc[4] = a1.x; sc[5] = a1.y; sc[6] = a1.z; sc[7] = a1.w;
        sh[0] = b0.x; sh[1] = b0.y; sh[2] = b0.z; sh[3] = b0.w; sh[4] = b1.x; sh[5] = b1.y; sh[6] = b1.z; sh[7] = b1.w;
      }
#pragma unroll
      for (int i = 0; i < AR; i++) {
        float f[8];
        unpack8(pr_a[i], f);
        const bool ok = (pr_ok >> i) & 1u;
#pragma unroll
        for (int j = 0; j < 8; j++) f[j] = ok ? fmaxf(fmaf(f[j], sc[j], sh[j]), 0.f) : 0.f;
        uint4 o = pack8(f);
        {  // inline asm: a compiler-visible LDS store got an s_waitcnt vmcnt(0) for the DMAs in flight
          typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
          const u32x4 w = {o.x, o.y, o.z, o.w};
          const unsigned la = (unsigned)(uintptr_t)(__attribute__((address_space(3))) bf16_t*)(
              As + buf * BM * BK + (i * RPP + wave * 8) * BK + lane * 8);
          asm volatile("ds_write_b128 %0, %1" ::"v"(la), "v"(w) : "memory");
        }
        if (pr_y) {
          __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<decltype(__builtin_amdgcn_raw_buffer_load_b128(rY, 0, 0, 0))*>(&o),
                                                 rY, (unsigned)pr_vo[i], (unsigned)pr_soff, 0);
          // wait states for the store's data VGPRs before the next VALU write: hipcc's hazard
          // pass misses this store-data hazard across the branch join inside the k-loop (the
          // next chunk's first VALU op overwrote the 2nd data dword: tests/test_conv_gpu.py)
          asm volatile("s_nop 4" ::: "memory");
        }
      }
    }
  };
  auto pro_wait = [&]() {  // this slice's A loads retired (its BR B-operand DMAs may still be in flight)
    if constexpr (BR == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (BR == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  if (nk == 0) {  // no taps reach these outputs (strided dgrad parity class): D = 0 (+ E)
    for (int i = 0; i < my_tiles; i++) {
      epilogue(tile_of(i), 0);
      lds_barrier();
    }
    return;
  }
  if constexpr (PRO) {
    for (int i = tid; i < 2 * g.C; i += 64 * NW) ssl[i] = pro.ss[i];
    __syncthreads();
  }
  issue(0, 0);
  if constexpr (PRO) {
    if (total > 0) {
      pro_wait();
      pro_store(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the loop's first barrier publishes them
    }
  }
  for (int st = 0; st < total; st++) {
    const int buf = st & 1;
    if (st + 1 < total) {
      issue(st + 1, buf ^ 1);
      // slice st landed (and older stores retired); slice st+1 stays in flight
      if constexpr (AR + BR == 8) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
      else if constexpr (AR + BR == 6) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    compute(buf);
    if constexpr (PRO) {
      if (st + 1 < total) {
        pro_wait();
        pro_store(buf ^ 1);
      }
    }
    if ((st + 1) % nk == 0) epilogue(tile_of(st / nk), buf);
    lds_barrier();  // every wave is done reading `buf` before slice st+2 is DMA'd into it
  }
}

// ---------------------------------------------------------------------------
// Ping-pong implicit GEMM (256 x 256 tiles): gemm_pp_kernel's two-wave-group
// schedule (gemm.hip, "Ping-pong 256x256 kernel") with the A operand gathered
// from the NHWC activation as in conv_igemm_kernel.  512 threads = two wave
// GROUPS (waves 0-3: tile rows 0-127, waves 4-7: rows 128-255; wave w owns the
// 128 x 64 tile at (w >> 2, w & 3)), one block per CU, BK = 64 = one tap's 64
// channels.  Each k-tile is four 16 KB pieces ordered by first use
//   A0: A rows {0-63, 128-191}   B0: B rows {64c + 0..31}
//   B1: B rows {64c + 32..63}    A1: A rows {64-127, 192-255}
// consumed in four phases of 16 MFMAs per wave; group 1 runs one barrier
// behind group 0, so on every SIMD one wave's MFMAs run under the other's LDS
// fragment reads and DMA issue, and four pieces (8 DMAs per lane) stay in
// flight across the barriers (never vmcnt(0) in the main loop).  Compared
// with the 4-wave 128 x 128 conv_igemm_kernel (two blocks per CU, ONE k-step
// of prefetch, 19-24 % MFMA busy at 3.6-4.4 VALU per MFMA,
// profiles/pmc/r4_resnet50_step.md): 128 x 64 wave tiles read 0.375 LDS
// fragments per MFMA instead of 0.5, the tile moves half the L2 -> LDS bytes
// per FLOP, and the load latency is covered by ~a k-tile of work.
// Gather: the A piece of k-tile kt reads tap (r, s), channels c0..c0+63, at
// per-lane 32-bit offsets (rows past M and padding taps go past the buffer
// and read 0); the tap walk is carried incrementally (wave-uniform) — the A0
// piece of a k-tile advances it, its A1 piece (issued three phases later, no
// other A0 in between) reuses it.  Epilogue: conv_epilogue (LDS-staged 16-B
// stores + fused addend / BN statistics), 4 staging passes per 128-row wave tile.
#ifndef KFA_CONV_PP_NHALF
#define KFA_CONV_PP_NHALF 4  // epilogue staging passes over the 128-row wave tile (8 KB of LDS per wave per pass at 2)
#endif
// WR wave-rows x WC = 8 / WR wave-columns of 128 x 64 wave tiles: WR = 2 is the
// 256 x 256 tile above (one wave-row per group); WR = 4 the 512 x 128 tile of the
// 128-channel layers (two wave-rows per group, 2 x 2 waves), the SAME wave tile and
// phase schedule with A pieces of 256 rows (32 KB, 4 DMAs per lane) and B pieces of
// 64 rows (8 KB, 1 DMA): 2 x 80 KB = the whole 160 KB of LDS, 104 FLOP per operand
// byte (the 128 x 128 tile: 64).
template <int WR>
__device__ __forceinline__ void pp_vm_wait(int n) {  // s_waitcnt vmcnt(n), n in [0, 2*WR + 8/WR]
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
  }
}

template <unsigned EPI, int WR = 2>
__global__ __launch_bounds__(512, 1) void conv_pp_kernel(const bf16_t* __restrict__ T, const bf16_t* __restrict__ B,
                                                         bf16_t* __restrict__ D, const bf16_t* __restrict__ E,
                                                         float* __restrict__ stats, BnBwd bnb, Geo g) {
  constexpr int TM = 8, TN = 4, WC = 8 / WR, MT = 128 * WR, NT = 64 * WC;
  constexpr int AP = WR * 64 * 128, BP = WC * 32 * 128;  // A / B piece bytes (64-deep rows of 128 B)
  constexpr int KTB = 2 * (AP + BP);                     // one k-tile buffer: [A0][B0][B1][A1]
  constexpr int OFF[4] = {0, AP, AP + BP, AP + 2 * BP};
  constexpr int NDMA[4] = {WR, WC / 2, WC / 2, WR};      // DMA instructions per lane of each piece
  constexpr int STEADY = 2 * WR + WC;                    // DMAs of any four consecutive phases
  __shared__ __attribute__((aligned(16))) char smem[2 * KTB];  // 128 KB (WR 2) / 160 KB (WR 4)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = WR == 2 ? wave >> 2 : ((wave >> 2) << 1) | ((wave >> 1) & 1);  // group = wave >> 2
  const int wc = wave & (WC - 1);
  // T1 XCD remap + grouped raster (as gemm_pp_kernel): the blocks of one XCD take
  // consecutive tiles, GM row panels wide
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, x8 = bid & 7;
  const int wg = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (bid >> 3);
  const int ntn = (g.N + NT - 1) / NT, ntm = (g.M + MT - 1) / MT;
  constexpr int GM = 4;
  const int grp = wg / (GM * ntn), gm0 = grp * GM, gmn = min(GM, ntm - gm0), rem = wg - grp * GM * ntn;
  const int m0 = (gm0 + rem % gmn) * MT, n0 = (rem / gmn) * NT;

  const __amdgpu_buffer_rsrc_t rT = rsrc(T, g.t_bytes), rB = rsrc(B, g.b_bytes), rD = rsrc(D, g.d_bytes);
  const int PQ = g.P * g.Q;
  const float rPQ = 1.f / (float)PQ, rQ = 1.f / (float)g.Q;
  const bool lin_a = g.R == 1 && g.S == 1 && g.sa == 1 && g.oa == 0 && g.ob == 0 && g.H == g.P && g.W == g.Q;
  const bool lin_d = g.os == 1 && g.oph == 0 && g.opw == 0 && g.OH == g.P && g.OW == g.Q;
  // DMA plan: instruction j of wave w fills piece rows j*64 + w*8 + lane/8,
  // physical chunk lane&7 <- logical chunk (lane&7) ^ ((row >> 1) & 7).
  // A piece h, instruction j: wave-row j's rows h*64 + [0, 64);  B piece h,
  // instruction j: wave-columns 2j, 2j+1's columns h*32 + [0, 32).
  const int prow = wave * 8 + (lane >> 3);
  const int lc = (lane & 7) ^ ((prow >> 1) & 7);
  int a_hb[2][WR], a_wb[2][WR], a_vo[2][WR];  // [h: A0 / A1][j]
  int b_vo[2][WC / 2];                        // [h: B0 / B1][j]
#pragma unroll
  for (int h = 0; h < 2; h++) {
#pragma unroll
    for (int j = 0; j < WR; j++) {
      const int m = m0 + j * 128 + h * 64 + prow;
      if (m < g.M && lin_a) {
        a_hb[h][j] = 0;
        a_wb[h][j] = 0;
        a_vo[h][j] = (m * g.C + lc * 8) * 2;
      } else if (m < g.M) {  // a_vo: the row's offset at tap (0, 0) (may lie outside the image)
        const int nb = fdiv(m, PQ, rPQ), rm = m - nb * PQ;
        const int p = fdiv(rm, g.Q, rQ), q = rm - p * g.Q;
        a_hb[h][j] = p * g.sa + g.oa;
        a_wb[h][j] = q * g.sa + g.ob;
        a_vo[h][j] = ((nb * g.H * g.W + a_hb[h][j] * g.W + a_wb[h][j]) * g.C + lc * 8) * 2;
      } else {
        a_hb[h][j] = -(1 << 28);  // forces out-of-range
        a_wb[h][j] = 0;
        a_vo[h][j] = (int)kOOB;
      }
    }
#pragma unroll
    for (int j = 0; j < WC / 2; j++) {
      const int n = n0 + (2 * j + (prow >> 5)) * 64 + h * 32 + (prow & 31);
      b_vo[h][j] = n < g.N ? (n * g.K + lc * 8) * 2 : (int)kOOB;
    }
  }
  const int nk = g.K / BK;
  const int plast = 4 * nk - 7;  // last phase that issues a piece
  // tap walk of the A pieces (wave-uniform): next k-tile's (channel offset, r, s)
  int tw_c0 = 0, tw_r = 0, tw_s = 0;
  int ta_dh = 0, ta_dw = 0, ta_off = 0, ta_soff = 0;  // the tap of the last A0 piece issued
  auto issue = [&](int P, auto pc, auto steady) __attribute__((always_inline)) {
    constexpr int p = decltype(pc)::value;
    const int kt = (P + 6) >> 2;
    if (decltype(steady)::value || kt < nk) {
      char* dst = smem + (kt & 1) * KTB + OFF[p] + wave * 8 * 128;
      if constexpr (p == 0 || p == 3) {
        constexpr int h = p == 3;
        if constexpr (h == 0) {  // A0 of k-tile kt: advance the tap walk
          ta_dh = tw_r * g.ra;
          ta_dw = tw_s * g.ra;
          ta_off = (ta_dh * g.W + ta_dw) * g.C * 2;
          ta_soff = (lin_a ? kt * BK : tw_c0) * 2;
          tw_c0 += BK;
          if (tw_c0 >= g.C) {
            tw_c0 = 0;
            if (++tw_s == g.S) { tw_s = 0; tw_r++; }
          }
        }
#pragma unroll
        for (int j = 0; j < WR; j++) {
          int vo = a_vo[h][j];
          if (!lin_a) {  // selects, no branch: the tap offset is one scalar add
            const int ih = a_hb[h][j] + ta_dh, iw = a_wb[h][j] + ta_dw;
            const bool ok = (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
            vo = ok ? vo + ta_off : (int)kOOB;
          }
          buf_dma16_act(rT, reinterpret_cast<bf16_t*>(dst + j * 64 * 128), vo, ta_soff);
        }
      } else {
        constexpr int h = p == 2;
#pragma unroll
        for (int j = 0; j < WC / 2; j++)
          buf_dma16(rB, reinterpret_cast<bf16_t*>(dst + j * 64 * 128), b_vo[h][j], kt * BK * 2);
      }
    }
  };
  auto retire = [&](int P, auto steady) __attribute__((always_inline)) {
    if constexpr (decltype(steady)::value) {
      pp_vm_wait<WR>(STEADY);
    } else {  // keep the pieces of phases [P - 3, min(P, plast)] in flight
      int n = 0;
#pragma unroll
      for (int d = 0; d < 4; d++) {
        const int q = P - d;
        if (q <= plast) n += NDMA[(q + 2) & 3];  // phase q issues piece (q + 2) & 3
      }
      pp_vm_wait<WR>(n);
    }
  };

  // this lane's fragment read offsets in a piece: row fr, logical chunk 4 ks + fq
  const int fr = lane & 15, fq = lane >> 4;
  const int ro0 = fr * 128 + ((fq ^ (fr >> 1)) << 4), ro1 = fr * 128 + (((4 + fq) ^ (fr >> 1)) << 4);
  floatx4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; i++)
#pragma unroll
    for (int j = 0; j < TM; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  short8 a[4][2], b0[2][2], b1[2][2];

  // prologue: pieces of phases -6..-1 (A0 B0 B1 A1 of k-tile 0, A0 B0 of k-tile 1)
  issue(-6, std::integral_constant<int, 0>{}, std::false_type{});
  issue(-5, std::integral_constant<int, 1>{}, std::false_type{});
  issue(-4, std::integral_constant<int, 2>{}, std::false_type{});
  issue(-3, std::integral_constant<int, 3>{}, std::false_type{});
  issue(-2, std::integral_constant<int, 0>{}, std::false_type{});
  issue(-1, std::integral_constant<int, 1>{}, std::false_type{});
  retire(-1, std::false_type{});
  asm volatile("s_barrier" ::: "memory");
  if (wave >> 2) asm volatile("s_barrier" ::: "memory");  // group 1 runs one barrier behind

  auto mfma_q = [&](short8 (&bb)[2][2], int mh, int nh) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ks++)
#pragma unroll
      for (int ni = 0; ni < 2; ni++)
#pragma unroll
        for (int mi = 0; mi < 4; mi++)
          acc[nh * 2 + ni][mh * 4 + mi] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[ni][ks], a[mi][ks], acc[nh * 2 + ni][mh * 4 + mi], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto rd = [&](const char* p) -> short8 { return *reinterpret_cast<const short8*>(p); };

  // one k-tile = four phases (st: std::true_type when every phase of k-tile u
  // issues a piece, i.e. u + 2 < nk)
  auto ktile = [&](int u, auto st) __attribute__((always_inline)) {
    const char* buf = smem + (u & 1) * KTB;
    const int P = 4 * u;
    {  // s0: A0 + B0
      const char* pa = buf + OFF[0] + wr * 64 * 128;
      const char* pb = buf + OFF[1] + wc * 32 * 128;
#pragma unroll
      for (int ni = 0; ni < 2; ni++) {
        b0[ni][0] = rd(pb + ni * 16 * 128 + ro0);
        b0[ni][1] = rd(pb + ni * 16 * 128 + ro1);
      }
#pragma unroll
      for (int mi = 0; mi < 4; mi++) {
        a[mi][0] = rd(pa + mi * 16 * 128 + ro0);
        a[mi][1] = rd(pa + mi * 16 * 128 + ro1);
      }
      issue(P, std::integral_constant<int, 2>{}, st);
      retire(P, st);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_q(b0, 0, 0);
      asm volatile("s_barrier" ::: "memory");
    }
    {  // s1: B1
      const char* pb = buf + OFF[2] + wc * 32 * 128;
#pragma unroll
      for (int ni = 0; ni < 2; ni++) {
        b1[ni][0] = rd(pb + ni * 16 * 128 + ro0);
        b1[ni][1] = rd(pb + ni * 16 * 128 + ro1);
      }
      issue(P + 1, std::integral_constant<int, 3>{}, st);
      retire(P + 1, st);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_q(b1, 0, 1);
      asm volatile("s_barrier" ::: "memory");
    }
    {  // s2: A1
      const char* pa = buf + OFF[3] + wr * 64 * 128;
#pragma unroll
      for (int mi = 0; mi < 4; mi++) {
        a[mi][0] = rd(pa + mi * 16 * 128 + ro0);
        a[mi][1] = rd(pa + mi * 16 * 128 + ro1);
      }
      issue(P + 2, std::integral_constant<int, 0>{}, st);
      retire(P + 2, st);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_q(b1, 1, 1);
      asm volatile("s_barrier" ::: "memory");
    }
    {  // s3: registers only
      issue(P + 3, std::integral_constant<int, 1>{}, st);
      retire(P + 3, st);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_q(b0, 1, 0);
      asm volatile("s_barrier" ::: "memory");
    }
  };
  int u = 0;
  for (; u + 2 < nk; u++) ktile(u, std::true_type{});
  for (; u < nk; u++) ktile(u, std::false_type{});
  if (!(wave >> 2)) asm volatile("s_barrier" ::: "memory");  // both groups at the same barrier count: the ring is idle
  const EpiRes er{rD, rsrc(E ? E : D, E ? g.d_bytes : 0u), rsrc(bnb.x ? bnb.x : D, bnb.x ? g.d_bytes : 0u),
                  rsrc(bnb.y ? bnb.y : D, bnb.y ? g.d_bytes : 0u)};
  conv_epilogue<TM, TN, KFA_CONV_PP_NHALF, EPI>(g, acc, smem + wave * (256 * (TM / KFA_CONV_PP_NHALF) * TN) * 2, false,
                                                lane, m0 + wr * 128, n0 + wc * 64, PQ, rPQ, rQ, lin_d, E, stats, bnb,
                                                er);
}

// zero-fill D rows of the output pixel mapping that the GEMM does not cover
__global__ void zero_bf16(bf16_t* __restrict__ p, long n8) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x)
    reinterpret_cast<uint4*>(p)[i] = make_uint4(0, 0, 0, 0);
}

// W[Cout][R][S][Cin] -> Wt[Cin][Rs][Ss][Cout] over the tap subset r = r0 + dr*i, s = s0 + ds*j
__global__ void weight_transpose(const bf16_t* __restrict__ W, bf16_t* __restrict__ Wt, int Cout, int R, int S,
                                 int Cin, int r0, int dr, int Rs, int s0, int ds, int Ss) {
  __shared__ bf16_t tile[32][33];
  const int tap = blockIdx.z;
  const int ri = tap / Ss, si = tap - ri * Ss;
  const int r = r0 + dr * ri, s = s0 + ds * si;
  const int co0 = blockIdx.y * 32, ci0 = blockIdx.x * 32;
  for (int y = threadIdx.y; y < 32; y += blockDim.y) {
    const int co = co0 + y, ci = ci0 + threadIdx.x;
    tile[y][threadIdx.x] = (co < Cout && ci < Cin) ? W[(((long)co * R + r) * S + s) * Cin + ci] : (bf16_t)0;
  }
  __syncthreads();
  for (int y = threadIdx.y; y < 32; y += blockDim.y) {
    const int ci = ci0 + y, co = co0 + threadIdx.x;
    if (ci < Cin && co < Cout) Wt[(((long)ci * Rs + ri) * Ss + si) * Cout + co] = tile[threadIdx.x][y];
  }
}

// Every dgrad weight transpose of a training step in ONE launch (the per-call
// transposes were 61 launches / 0.35 ms per ResNet-50 step): block b finds its
// descriptor by the prefix table, then runs weight_transpose's 32x32 tile.
struct TDesc {
  const bf16_t* W;
  bf16_t* Wt;
  int Cout, R, S, Cin, r0, dr, Rs, s0, ds, Ss, gx, gy;
};

// 64 x 64 tiles, 256 threads: rows of 8 input channels (16 B) in, rows of 8 output
// channels (16 B) out, the tile staged in LDS with a 2-element row pad (the column
// reads of the write-out then spread over the banks).  The 32 x 32 / 2-byte form this
// replaces moved 1.4 TB/s (BERT-base: 238 us per step for 85 M elements); partial
// tiles and channel counts that are not multiples of 8 take the element-wise path.
__global__ __launch_bounds__(256) void weight_transpose_multi(const TDesc* __restrict__ descs,
                                                              const int* __restrict__ first, int n) {
  constexpr int T = 64, P = T + 2;
  __shared__ bf16_t tile[T * P];
  __shared__ int which;
  if (threadIdx.x == 0) {
    int lo = 0, hi = n - 1;  // last descriptor whose first block <= blockIdx.x
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (first[mid] <= (int)blockIdx.x) lo = mid; else hi = mid - 1;
    }
    which = lo;
  }
  __syncthreads();
  const TDesc d = descs[which];
  int b = (int)blockIdx.x - first[which];
  const int bx = b % d.gx;
  b /= d.gx;
  const int by = b % d.gy, tap = b / d.gy;
  const int ri = tap / d.Ss, si = tap - ri * d.Ss;
  const int r = d.r0 + d.dr * ri, s = d.s0 + d.ds * si;
  const int co0 = by * T, ci0 = bx * T;
  const long ws = (long)d.R * d.S * d.Cin;        // W stride between output channels
  const long ts = (long)d.Rs * d.Ss * d.Cout;     // Wt stride between input channels
  const bf16_t* src = d.W + ((long)r * d.S + s) * d.Cin;
  bf16_t* dst = d.Wt + ((long)ri * d.Ss + si) * d.Cout;
  const bool vec = (d.Cin % 8 == 0) && (d.Cout % 8 == 0) && co0 + T <= d.Cout && ci0 + T <= d.Cin &&
                   ((uintptr_t)d.W % 16 == 0) && ((uintptr_t)d.Wt % 16 == 0);
  const int t = threadIdx.x;
  if (vec) {
#pragma unroll
    for (int k = 0; k < 2; k++) {  // 64 rows x 8 chunks of 8 channels
      const int q = t + k * 256, row = q >> 3, ch = (q & 7) * 8;
      const uint4 v = *reinterpret_cast<const uint4*>(src + (co0 + row) * ws + ci0 + ch);
      uint32_t* tp = reinterpret_cast<uint32_t*>(tile + row * P + ch);  // 4-B aligned: P and ch even
      tp[0] = v.x; tp[1] = v.y; tp[2] = v.z; tp[3] = v.w;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int q = t + k * 256, ci = q >> 3, co = (q & 7) * 8;
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; e++)
        w[e] = (uint32_t)tile[(co + 2 * e) * P + ci] | ((uint32_t)tile[(co + 2 * e + 1) * P + ci] << 16);
      *reinterpret_cast<uint4*>(dst + (ci0 + ci) * ts + co0 + co) = make_uint4(w[0], w[1], w[2], w[3]);
    }
    return;
  }
  for (int q = t; q < T * T; q += 256) {
    const int row = q / T, ci = q % T;
    tile[row * P + ci] = (co0 + row < d.Cout && ci0 + ci < d.Cin) ? src[(co0 + row) * ws + ci0 + ci] : (bf16_t)0;
  }
  __syncthreads();
  for (int q = t; q < T * T; q += 256) {
    const int ci = q / T, co = q % T;
    if (ci0 + ci < d.Cin && co0 + co < d.Cout) dst[(ci0 + ci) * ts + co0 + co] = tile[co * P + ci];
  }
}

}  // namespace

// descs: n x 14 ints-worth descriptors (TDesc, host-packed; gx / gy = 64-wide tile counts
// over Cin / Cout), first: n block offsets, total blocks
KFA_API int kfa_tdesc_bytes() { return (int)sizeof(TDesc); }

KFA_API int kfa_weight_transpose_multi(const void* descs, const int* first, int n, int total_blocks, hipStream_t st) {
  if (n <= 0 || total_blocks <= 0) return 0;
  hipLaunchKernelGGL(weight_transpose_multi, dim3(total_blocks), dim3(256), 0, st,
                     reinterpret_cast<const TDesc*>(descs), first, n);
  return kfa_status();
}

static const bf16_t* zero_page() {
  static bf16_t* z = nullptr;
  if (!z) {
    if (hipMalloc(&z, 256) != hipSuccess) return nullptr;
    (void)hipMemset(z, 0, 256);
    (void)hipDeviceSynchronize();
  }
  return z;
}

// smallest compiled epilogue configuration covering `need` (see conv_igemm_kernel's EPI)
static unsigned pick_epi(unsigned need) {
  static const unsigned have[] = {0u, kEpiStats, kEpiE, kEpiE | kEpiEmb, kEpiStats | kEpiBnBwd,
                                  kEpiE | kEpiStats | kEpiBnBwd, kEpiE | kEpiEmb | kEpiStats | kEpiBnBwd};
  for (unsigned h : have)
    if ((need & ~h) == 0) return h;
  return kEpiAll;
}

template <int WM, int WN, int TM, int TN>
static void launch_igemm(unsigned epi, dim3 grid, dim3 block, int lds, hipStream_t st, const bf16_t* T, const bf16_t* B,
                         bf16_t* D, const bf16_t* E, float* stats, const BnBwd& bnb, const Geo& g) {
#define KFA_IG(EP)                                                                                                   \
  case EP:                                                                                                           \
    if (lds > 65536) {                                                                                               \
      static bool attr = false;                                                                                      \
      if (!attr) {                                                                                                   \
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_igemm_kernel<WM, WN, TM, TN, EP>),             \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds);                                  \
        attr = true;                                                                                                 \
      }                                                                                                              \
    }                                                                                                                \
    hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, TM, TN, EP>), grid, block, lds, st, T, B, D, E, zero_page(), stats, \
                       bnb, g);                                                                                      \
    break;
  switch (pick_epi(epi)) {
    KFA_IG(0u)
    KFA_IG(kEpiStats)
    KFA_IG(kEpiE)
    KFA_IG(kEpiE | kEpiEmb)
    KFA_IG(kEpiStats | kEpiBnBwd)
    KFA_IG(kEpiE | kEpiStats | kEpiBnBwd)
    KFA_IG(kEpiE | kEpiEmb | kEpiStats | kEpiBnBwd)
    default:
      KFA_IG(kEpiAll)
  }
#undef KFA_IG
}

// PRO launches (forward convs reading a BatchNorm's raw input): EPI 0 or stats only
template <int WM, int WN, int TM, int TN>
static void launch_igemm_pro(unsigned epi, dim3 grid, dim3 block, int lds, hipStream_t st, const bf16_t* T,
                             const bf16_t* B, bf16_t* D, float* stats, const Geo& g, const Pro& pro) {
  const BnBwd bnb{nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr};
#define KFA_IGP(EP)                                                                                                   \
  {                                                                                                                   \
    static bool attr = false;                                                                                         \
    if (!attr && lds > 65536) {                                                                                       \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_igemm_kernel<WM, WN, TM, TN, EP, true>),          \
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds);                                     \
      attr = true;                                                                                                    \
    }                                                                                                                 \
    hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, TM, TN, EP, true>), grid, block, lds, st, T, B, D, nullptr,          \
                       zero_page(), stats, bnb, g, pro);                                                              \
  }
  if (epi & kEpiStats) KFA_IGP(kEpiStats) else KFA_IGP(0u)
#undef KFA_IGP
}

template <unsigned EP>
static void launch_pp1(int wr, dim3 grid, hipStream_t st, const bf16_t* T, const bf16_t* B, bf16_t* D,
                       const bf16_t* E, float* stats, const BnBwd& bnb, const Geo& g) {
  if (wr == 4) hipLaunchKernelGGL((conv_pp_kernel<EP, 4>), grid, dim3(512), 0, st, T, B, D, E, stats, bnb, g);
  else hipLaunchKernelGGL((conv_pp_kernel<EP, 2>), grid, dim3(512), 0, st, T, B, D, E, stats, bnb, g);
}

static void launch_pp(int wr, unsigned epi, dim3 grid, hipStream_t st, const bf16_t* T, const bf16_t* B,
                      bf16_t* D, const bf16_t* E, float* stats, const BnBwd& bnb, const Geo& g) {
  switch (pick_epi(epi)) {
    case 0u: launch_pp1<0u>(wr, grid, st, T, B, D, E, stats, bnb, g); break;
    case kEpiStats: launch_pp1<kEpiStats>(wr, grid, st, T, B, D, E, stats, bnb, g); break;
    case kEpiE: launch_pp1<kEpiE>(wr, grid, st, T, B, D, E, stats, bnb, g); break;
    case kEpiE | kEpiEmb: launch_pp1<kEpiE | kEpiEmb>(wr, grid, st, T, B, D, E, stats, bnb, g); break;
    case kEpiStats | kEpiBnBwd: launch_pp1<kEpiStats | kEpiBnBwd>(wr, grid, st, T, B, D, E, stats, bnb, g); break;
    case kEpiE | kEpiStats | kEpiBnBwd:
      launch_pp1<kEpiE | kEpiStats | kEpiBnBwd>(wr, grid, st, T, B, D, E, stats, bnb, g);
      break;
    case kEpiE | kEpiEmb | kEpiStats | kEpiBnBwd:
      launch_pp1<kEpiE | kEpiEmb | kEpiStats | kEpiBnBwd>(wr, grid, st, T, B, D, E, stats, bnb, g);
      break;
    default: launch_pp1<kEpiAll>(wr, grid, st, T, B, D, E, stats, bnb, g); break;
  }
}

// variant: 0 = 128x128 tile, 1 = 128x64 tile (N <= 64), 2 = 256x256 tile (8 waves), 3 = 256x64 (N <= 64),
// 4 = 256x256 ping-pong (conv_pp_kernel: C % 64 == 0, K > 0; one block per tile),
// 6 = 512x128 ping-pong (conv_pp_kernel<.., 4>: the 128-channel layers, same conditions)
KFA_API int kfa_conv_igemm(const bf16_t* T, const bf16_t* B, bf16_t* D, const bf16_t* E, int Nb, int H, int W, int C,
                           int P, int Q, int R, int S, int sa, int ra, int oa, int ob, int N, int OH, int OW, int os,
                           int oph, int opw, int ldd, int variant, float* stats, const bf16_t* bn_x,
                           const bf16_t* bn_y, const float* bn_mean, int bn_relu, const float* bn_ss,
                           const uint8_t* bn_mb, const uint8_t* add_mb, hipStream_t st) {
  const BnBwd bnb{bn_x, bn_y, bn_ss, bn_mb, bn_mean, bn_relu, E ? add_mb : nullptr};
  if (bn_x && bn_relu && !bn_y && !bn_ss && !bn_mb) return -3;
  if ((bn_mb || (E && add_mb)) && ldd != N) return -4;  // the bit masks index [M][N] rows
  // C < 64: a BK slice spans S*C/64 whole taps of one filter row — one contiguous run of the
  // input row when the gather is stride 1 / pad 0 along w (the space-to-depth stem, stem.hip)
  const bool multi_tap = C % 8 == 0 && C < BK && BK % C == 0 && (S * C) % BK == 0 && sa == 1 && ra == 1 &&
                         oa == 0 && ob == 0;
  if ((C % BK != 0 && !multi_tap) || N % 8 != 0 || ldd % 8 != 0) return -1;
  Geo g{Nb, H, W, C, P, Q, R, S, sa, ra, oa, ob, Nb * P * Q, N, R * S * C, OH, OW, os, oph, opw, ldd, 0, 0, 0};
  if (g.K == 0) g.R = g.S = 1;  // keep index math defined; nk == 0 -> zero/addend-only epilogue
  const long tb = (long)Nb * H * W * C * 2, bb = (long)N * R * S * C * 2, db = (long)Nb * OH * OW * ldd * 2;
  if (tb >= (long)kOOB || bb >= (long)kOOB || db >= (long)kOOB) return -2;  // 32-bit buffer offsets
  g.t_bytes = (unsigned)tb;
  g.b_bytes = (unsigned)bb;
  g.d_bytes = (unsigned)db;
  if (g.M <= 0) return 0;
  int cus = 256;
  {
    static int cached = 0;
    if (!cached) {
      int dev = 0;
      hipGetDevice(&dev);
      hipDeviceGetAttribute(&cached, hipDeviceAttributeMultiprocessorCount, dev);
      if (cached <= 0) cached = 256;
    }
    cus = cached;
  }
  // persistent grid: 2 resident blocks per CU (64 KB LDS, <=256 VGPR/2 waves).
  // KFA_CONV_OVERSUB=k caps the grid at k x that (0: one block per tile), so the
  // dispatcher, not the tile ranges, balances the work when other kernels (RCCL)
  // hold part of the CUs.
  static int oversub = -1;
  if (oversub < 0) {
    const char* e = getenv("KFA_CONV_OVERSUB");
    oversub = e ? atoi(e) : 1;
    if (oversub < 0) oversub = 1;
  }
  const long slots = oversub == 0 ? (1L << 30) : 2L * cus * oversub;
  auto pgrid = [&](long tiles) { return (int)(tiles < slots ? tiles : slots); };
  const unsigned epi = (E ? kEpiE : 0u) | (stats ? kEpiStats : 0u) | (bn_x ? kEpiBnBwd : 0u) |
                       ((E && add_mb) ? kEpiEmb : 0u) | ((bn_x && bn_y && bn_relu) ? kEpiYMask : 0u);
  if (variant == 4 && C % BK == 0 && g.K > 0) {  // ping-pong 256 x 256 (grid = tiles, one block per CU resident)
    launch_pp(2, epi, dim3((unsigned)((long)kfa_ceil_div(g.M, 256) * kfa_ceil_div(N, 256))), st, T, B, D, E, stats,
              bnb, g);
  } else if (variant == 6 && C % BK == 0 && g.K > 0) {  // ping-pong 512 x 128
    launch_pp(4, epi, dim3((unsigned)((long)kfa_ceil_div(g.M, 512) * kfa_ceil_div(N, 128))), st, T, B, D, E, stats,
              bnb, g);
  } else if (variant == 3) {  // 256 x 64 tile (Cout <= 64): 4 waves of 64x64, 80 KB LDS -> 2 blocks / CU
    const int grid = pgrid((long)kfa_ceil_div(g.M, 256) * kfa_ceil_div(N, 64));
    launch_igemm<4, 1, 4, 4>(epi, dim3(grid), dim3(256), 2 * (256 + 64) * BK * 2, st, T, B, D, E, stats, bnb, g);
  } else if (variant == 1) {  // 128 x 64 tile (Cout <= 64): 4 waves of 32x64
    const long tiles = (long)kfa_ceil_div(g.M, 128) * kfa_ceil_div(N, 64);
    const int grid = (int)(tiles < 3L * cus ? tiles : 3L * cus);  // 48 KB LDS: up to 3 blocks / CU
    launch_igemm<4, 1, 2, 4>(epi, dim3(grid), dim3(256), 2 * (128 + 64) * BK * 2, st, T, B, D, E, stats, bnb, g);
  } else if (variant == 2) {  // 256 x 256 tile: 2x4 waves of 128x64, one block per CU (128 KiB LDS)
    const long tiles = (long)kfa_ceil_div(g.M, 256) * kfa_ceil_div(N, 256);
    const int grid = (int)(tiles < cus ? tiles : cus);
    launch_igemm<2, 4, 8, 4>(epi, dim3(grid), dim3(512), 2 * (256 + 256) * BK * 2, st, T, B, D, E, stats, bnb, g);
  } else {  // 128 x 128 tile: 2x2 waves of 64x64
    const int grid = pgrid((long)kfa_ceil_div(g.M, 128) * kfa_ceil_div(N, 128));
    launch_igemm<2, 2, 4, 4>(epi, dim3(grid), dim3(256), 2 * (128 + 128) * BK * 2, st, T, B, D, E, stats, bnb, g);
  }
  return kfa_status();
}

// Forward conv of relu(x * scale + shift) (a training BatchNorm + ReLU folded into
// the A operand, see Pro): T = the BN's raw input x [Nb][H][W][C], ss = its
// [scale | shift], y (optional) receives the normalised activation — only for
// stride 1 with P == H, Q == W (the centre taps then cover every pixel).  D is
// [Nb][P][Q][N]; stats as kfa_conv_igemm.
KFA_API int kfa_conv_igemm_bnpro(const bf16_t* T, const bf16_t* B, bf16_t* D, const float* ss, bf16_t* y, int Nb,
                                 int H, int W, int C, int P, int Q, int R, int S, int stride, int pad, int N,
                                 int variant, float* stats, hipStream_t st) {
  if (!ss || C % BK != 0 || N % 8 != 0 || C > 2048) return -1;
  if (y && !(stride == 1 && P == H && Q == W && 2 * pad == R - 1 && 2 * pad == S - 1)) return -5;
  Geo g{Nb, H, W, C, P, Q, R, S, stride, 1, -pad, -pad, Nb * P * Q, N, R * S * C, P, Q, 1, 0, 0, N, 0, 0, 0};
  const long tb = (long)Nb * H * W * C * 2, bb = (long)N * R * S * C * 2, db = (long)Nb * P * Q * N * 2;
  if (tb >= (long)kOOB || bb >= (long)kOOB || db >= (long)kOOB) return -2;
  g.t_bytes = (unsigned)tb;
  g.b_bytes = (unsigned)bb;
  g.d_bytes = (unsigned)db;
  if (g.M <= 0) return 0;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const Pro pro{ss, y};
  const unsigned epi = stats ? kEpiStats : 0u;
  const int tab = 8 * C;  // the [scale | shift] table behind the operand ring
  auto cap = [&](long tiles, long slots) { return (int)(tiles < slots ? tiles : slots); };
  if (variant == 3) {
    const int grid = cap((long)kfa_ceil_div(g.M, 256) * kfa_ceil_div(N, 64), 2L * cus);
    launch_igemm_pro<4, 1, 4, 4>(epi, dim3(grid), dim3(256), 2 * (256 + 64) * BK * 2 + tab, st, T, B, D, stats, g, pro);
  } else if (variant == 1) {
    const int grid = cap((long)kfa_ceil_div(g.M, 128) * kfa_ceil_div(N, 64), 3L * cus);
    launch_igemm_pro<4, 1, 2, 4>(epi, dim3(grid), dim3(256), 2 * (128 + 64) * BK * 2 + tab, st, T, B, D, stats, g, pro);
  } else if (variant == 2) {
    const int grid = cap((long)kfa_ceil_div(g.M, 256) * kfa_ceil_div(N, 256), cus);
    launch_igemm_pro<2, 4, 8, 4>(epi, dim3(grid), dim3(512), 2 * (256 + 256) * BK * 2 + tab, st, T, B, D, stats, g, pro);
  } else {
    const int grid = cap((long)kfa_ceil_div(g.M, 128) * kfa_ceil_div(N, 128), 2L * cus);
    launch_igemm_pro<2, 2, 4, 4>(epi, dim3(grid), dim3(256), 2 * (128 + 128) * BK * 2 + tab, st, T, B, D, stats, g, pro);
  }
  return kfa_status();
}

KFA_API int kfa_zero_bf16(bf16_t* p, long n, hipStream_t st) {
  if (n % 8) return -1;
  long n8 = n / 8;
  long b = (n8 + 255) / 256;
  hipLaunchKernelGGL(zero_bf16, dim3(b < 4096 ? (b < 1 ? 1 : b) : 4096), dim3(256), 0, st, p, n8);
  return kfa_status();
}

KFA_API int kfa_weight_transpose(const bf16_t* W, bf16_t* Wt, int Cout, int R, int S, int Cin, int r0, int dr, int Rs,
                                 int s0, int ds, int Ss, hipStream_t st) {
  dim3 grid(kfa_ceil_div(Cin, 32), kfa_ceil_div(Cout, 32), Rs * Ss);
  hipLaunchKernelGGL(weight_transpose, grid, dim3(32, 8), 0, st, W, Wt, Cout, R, S, Cin, r0, dr, Rs, s0, ds, Ss);
  return kfa_status();
}
