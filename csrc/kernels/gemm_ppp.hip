// Persistent ping-pong GEMM with the C write overlapped with the next tile's
// main loop — SURVEY §2.6 K1 (dense GEMM + epilogue), the BERT / W&D / ResNet-FC
// projections, forward and dgrad:
//
//   C[m][n] = epilogue( Σ_k A[m][k] · B[n][k] )      A [M][lda], B [N][ldb]: K-contiguous
//
// Main loop = gemm_pp_kernel's (gemm.hip): 256 x 256 tiles, 512 threads as two
// wave groups one s_barrier apart (on every SIMD one wave's 16 MFMAs run under
// the other wave's LDS reads + LDS-DMA issue), 64-deep k-tiles in four 16 KB
// pieces, `buffer_load ... lds` with 32-bit row offsets, 8 DMAs per lane in
// flight across the barriers, XOR-swizzled 128-B LDS rows.
//
// What is new is the ORDER of work around the tile boundary.  The kernel is
// persistent (one 512-thread block per CU, XCD-aware tile ranges) and the
// k-tile sequence of ALL of a block's tiles is one continuous pipeline: the
// pieces of tile i+1's first k-tiles are issued while tile i's last MFMAs run.
// Tile i's epilogue is not a separate stage: its 128 x 64 wave tile is four
// 64 x 32 quadrants, and the ping-pong k-tile visits them in a fixed order
// (s0: (0,0), s1: (0,1), s2: (1,1), s3: (1,0)).  In the FIRST k-tile of tile
// i+1, phase s writes quadrant s of tile i (bf16, straight from the
// accumulator registers) and zeroes it just before the phase's MFMAs start
// accumulating tile i+1 into those registers.  So the 128 KB C write of a tile
// is spread over four phases and issued while the partner wave group
// multiplies — no LDS staging (which would need vmcnt(0) with LDS-DMA in
// flight: hipcc drains every outstanding DMA before a C++ LDS store), no extra
// registers, no idle MFMA pipe while C drains.
//
// Stores: per 16-row block a lane holds 4 consecutive columns of two 16-column
// halves; one v_permlane16_swap per dword pair gives every lane 8 consecutive
// columns (lanes of row fq hold columns {0, 16, 8, 24}[fq] .. +7 of the
// quadrant), so each store is 16 B per lane, 64 contiguous bytes per row.
//
// vmcnt: stores and LDS-DMA share the in-order counter.  The wait of phase P
// retires the piece issued 4 phases earlier, so it leaves in flight the pieces
// of phases P-3..P (2 DMAs each) AND the stores of those phases:
//   vmcnt(2 * pieces + S * store-phases among P-3..P)
// — a store has ~1 k-tile of MFMA work (four phases) to drain before any wait
// depends on it.  Steady k-tiles away from a tile boundary use the fixed
// vmcnt(8); the boundary k-tiles and the pipeline tail take the runtime count.
#include "common.h"

#include <utility>

namespace {

constexpr int BK = 64;
constexpr int PIECE = 128 * BK * 2;  // bytes per LDS piece (128 rows x 64 k)
constexpr unsigned kOOB = 0x80000000u;

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) float floatx2_t;

// two floats -> packed bf16x2 (v_cvt_pk_bf16_f32: round to nearest even, NaN kept)
__device__ __forceinline__ unsigned cvt2(float lo, float hi) {
  const floatx2_t f = {lo, hi};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f, bf16x2_t));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

__device__ __forceinline__ void store16(__amdgpu_buffer_rsrc_t r, unsigned off, uint4 v) {
  using V = decltype(__builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0));
  __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<V*>(&v), r, off, 0, 0);
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (even, 0..62)
__device__ __forceinline__ void vm_wait_rt(int n) {
  switch (n) {
#define KFA_VMW(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    KFA_VMW(0) KFA_VMW(2) KFA_VMW(4) KFA_VMW(6) KFA_VMW(8) KFA_VMW(10) KFA_VMW(12) KFA_VMW(14)
    KFA_VMW(16) KFA_VMW(18) KFA_VMW(20) KFA_VMW(22) KFA_VMW(24) KFA_VMW(26) KFA_VMW(28) KFA_VMW(30)
    KFA_VMW(32) KFA_VMW(34) KFA_VMW(36) KFA_VMW(38) KFA_VMW(40) KFA_VMW(42) KFA_VMW(44) KFA_VMW(46)
    KFA_VMW(48) KFA_VMW(50) KFA_VMW(52) KFA_VMW(54) KFA_VMW(56) KFA_VMW(58) KFA_VMW(60) KFA_VMW(62)
#undef KFA_VMW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

struct PppArgs {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;
  int M, N, K, lda, ldb, ldc;
  unsigned c_bytes;
  // split remainder (split > 1): the tiles past the last full round of the grid
  // are cut into `split` k-ranges run by `split` blocks; every part leaves its fp32
  // partial accumulators in `ws` and draws a ticket from `flags[unit]`, the last
  // arriver adds the others and writes C (flags self-cleaning: it resets the counter)
  float* ws;
  int* flags;
  int split;
  // experiment (kfa_gemm_ppp_set_stagger): blocks of odd logical index start this
  // many s_memrealtime ticks (10 ns) late, so half the CUs cross their tile
  // boundaries (and issue their C bursts) half a tile after the other half
  int stagger;
  // activation epilogue (gemm_ppp_kernel<256, ..., ACT>): ACT 1: C = z = A·Bᵀ + bias (the
  // pre-activation the backward needs), Y = gelu(z); ACT 2: C = relu(A·Bᵀ + bias);
  // bias fp32 [N], N <= 8192
  bf16_t* Y;
  const float* bias;
  // GELU-backward epilogue (gemm_ppw_kernel<NT, DACT = true>): C = (A·Bᵀ) * gelu'(Zin + bias)
  // with Zin the forward pre-activation (layout of C); column sums of C go to cpart
  // ([ceil(M / 64)][N] fp32, one row per 64-row quadrant band, each entry written once)
  const bf16_t* Zin;
  float* cpart;
  // grouped-raster height in 256-row tiles (experiment knob kfa_gemm_ppp_set_gm; 0 = 4)
  int gm;
};

__device__ __forceinline__ void ppp_stagger(int ticks, int lc) {
  if (ticks > 0 && (lc & 1)) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)ticks) __builtin_amdgcn_s_sleep(4);
  }
}

constexpr int kStoresPerPhase = 4;  // one 16-B store per 16-row block of a 64 x 32 quadrant

// BN: tile width in N, 256 or 192.  A wave's 128 x WN tile (WN = BN / 4) is a
// 32-column half (nh = 0: two 16-column MFMA blocks) and a NB1-block half
// (nh = 1: two blocks at BN = 256, one at BN = 192).  BN = 192 serves N = 768
// (BERT-base's hidden size): 4 tiles per 256-row band, so M = 32768 is 512
// tiles = exactly two per CU where 256-wide tiles leave 1.5 (384 tiles, half
// the CUs idle for the second round).  Piece 2 (the nh = 1 B rows) is then 64
// rows = one DMA per lane, so a k-tile issues D = 6 + NB1 DMAs.
// NOST: timing probe — every C store dropped (the values kept live).
// SMODE: bit 0 = non-temporal C stores; bit 1 = row pairs (quadrants (0,0)+(0,1)
// in phase 0, (1,1)+(1,0) in phase 2: each 128-B row segment written in one phase)
// P3 (BN = 192 only): THREE phases per k-tile of 16 MFMAs each — s0: A0 + B0 ->
// rows 0-63 x the two 16-column blocks of the wave's first 32 columns; s1: A1 ->
// rows 64-127 x the same blocks (B0 fragments kept); s2: B1 -> both row halves x
// the third block (A0 and A1 fragments kept).  The four-phase order gives a
// 48-column wave tile 16 / 8 / 8 / 16 MFMAs per phase, and the short phases
// expose the partner group's LDS reads.  Issue: s0 A1(u+1), s1 B1(u+1), s2 A0 and
// B0 (u+2) — each piece DMA'd 3 phases (one k-tile) before its read phase and
// only into a buffer whose previous piece was read >= 2 phases earlier; every
// phase retires the DMAs of three phases ago: steady vmcnt(D = 7).
// ACT (BN = 256, SMODE = 0, no split): the bias + activation epilogue, the bias staged
// once in the 32 KB of LDS the 128 KB ring leaves free.  ACT 1 (GELU): each quadrant
// store writes z = acc + bias to C and gelu(z) to Y (8 stores per phase instead of 4,
// counted in the retire waits) — the BERT FFN-up forward needs no bias / GELU pass.
// ACT 2 (ReLU): C = relu(acc + bias) only, the plain 4 stores per phase — the ReLU
// backward reads its mask from the output (y > 0 exactly where acc + bias > 0), so no
// pre-activation is kept (the W&D MLP layers: no bias / ReLU pass, no z write).
template <int BN = 256, bool NOST = false, int SMODE = 0, bool P3 = false, int ACT = 0>
__global__ __launch_bounds__(512, 1) void gemm_ppp_kernel(PppArgs g) {
  static_assert(BN == 256 || BN == 192, "tile width");
  static_assert(!ACT || (BN == 256 && SMODE == 0 && !P3 && !NOST), "activation epilogue: plain 256-wide schedule");
  static_assert(!P3 || BN == 192, "three-phase k-tiles are the 192-wide schedule");
  static_assert(BN == 256 || !(SMODE & 2), "row pairs need two-block halves");
  constexpr int NB1 = BN == 256 ? 2 : 1;  // 16-column MFMA blocks in a wave's nh = 1 half
  constexpr int WN = BN / 4;              // wave tile width
  constexpr int TM = 8, TN = 2 + NB1;
  constexpr int D = 6 + NB1;              // DMAs per k-tile
  __shared__ __attribute__((aligned(16))) char smem[2 * 4 * PIECE];  // 128 KB: two k-tiles of four pieces
  __shared__ __attribute__((aligned(16))) float sbias[ACT ? 8192 : 1];  // ACT: the bias vector (32 KB)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  // T1: blocks that share an XCD (blockIdx % 8) get consecutive logical indices,
  // so the tiles an XCD runs at one time are neighbours in the grouped raster
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, x8 = bid & 7;
  const int lc = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (bid >> 3);
  ppp_stagger(g.stagger, lc);
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + 255) / 256, ntiles = ntm * ntn;
  const int nk = (g.K + BK - 1) / BK;  // K % 8 == 0; a partial last k-tile reads zeros past K
  // data-parallel tiles of this block (lc, lc + nwg, ...), then at most one split unit
  const int ns = g.split;
  const int ndp = ns > 1 ? ntiles / nwg : (lc < ntiles ? (ntiles - 1 - lc) / nwg + 1 : 0);
  const int unit = lc / ns, part = lc - unit * ns;
  const bool has_split = ns > 1 && lc < (ntiles - ndp * nwg) * ns;
  const int my_tiles = ndp + (has_split ? 1 : 0);
  const int skb = part * nk / ns, skl = (part + 1) * nk / ns - skb;  // the split unit's k-range
  const int J = ndp * nk + (has_split ? skl : 0);  // k-tiles this block runs, all tiles back to back
  if (J == 0) return;
  const int GM = g.gm > 0 ? g.gm : 4;
  auto tile_mn = [&](int i, int& m0, int& n0) __attribute__((always_inline)) {
    const int wg = i < ndp ? lc + i * nwg : ndp * nwg + unit;
    const int grp = wg / (GM * ntn), gm0 = grp * GM, gmn = min(GM, ntm - gm0), rem = wg - grp * GM * ntn;
    m0 = (gm0 + rem % gmn) * 256;
    n0 = (rem / gmn) * BN;
  };

  const __amdgpu_buffer_rsrc_t rA = rsrc(g.A, (unsigned)(((long)(g.M - 1) * g.lda + g.K) * 2));
  const __amdgpu_buffer_rsrc_t rB = rsrc(g.B, (unsigned)(((long)(g.N - 1) * g.ldb + g.K) * 2));
  const __amdgpu_buffer_rsrc_t rC = rsrc(g.C, g.c_bytes);
  const __amdgpu_buffer_rsrc_t rY = rsrc(ACT == 1 ? g.Y : g.C, ACT == 1 ? g.c_bytes : 0u);
  if constexpr (ACT != 0) {  // before any DMA is in flight: a plain load + LDS store + barrier
    for (int i = tid; i < 8192; i += 512) sbias[i] = i < g.N ? g.bias[i] : 0.f;
    __syncthreads();
  }
  // DMA plan: instruction j of wave w fills piece rows j*64 + w*8 + lane/8,
  // physical chunk lane&7 <- logical chunk (lane&7) ^ ((row >> 1) & 7)
  const int prow = wave * 8 + (lane >> 3);
  const int lcx = (lane & 7) ^ ((prow >> 1) & 7);
  int voff[4][2];
  // piece p of tile (m0, n0): A pieces 0 (rows h=0) / 3 (h=1), B pieces 1 (h=0) / 2 (h=1)
  auto set_voff = [&](int p, int m0, int n0) __attribute__((always_inline)) {
    const int h = (p == 2 || p == 3) ? 1 : 0;
#pragma unroll
    for (int j = 0; j < 2; j++) {
      if (p == 0 || p == 3) {
        const int m = m0 + j * 128 + h * 64 + prow;
        voff[p][j] = m < g.M ? (m * g.lda + lcx * 8) * 2 : (int)kOOB;
      } else if (p == 1 || j < NB1) {
        // piece row r -> wave column group r / rows-per-group, column h * 32 + r % rows-per-group
        const int r = j * 64 + prow, rg = h ? 16 * NB1 : 32;
        const int n = n0 + (r / rg) * WN + h * 32 + (r % rg);
        voff[p][j] = n < g.N ? (n * g.ldb + lcx * 8) * 2 : (int)kOOB;
      } else {
        voff[p][j] = (int)kOOB;
      }
    }
  };
  // Issue side, advanced ONCE per k-tile outside the phases (the phases only
  // issue): pieces 2, 3 of k-tile u fetch k-tile u+1 ("X"), pieces 0, 1 fetch
  // u+2 ("Y"); each side keeps its k index, its local tile and that tile's
  // offsets (voff[2..3] / voff[0..1]).
  // Each side also keeps its tile's k-range (base, length): the whole K for a
  // data-parallel tile, [skb, skb + skl) for the split unit.
  int xkt = 0, xti = 0, ykt = 0, yti = 0;
  int xkb = ndp > 0 ? 0 : skb, xkl = ndp > 0 ? nk : skl, ykb = xkb, ykl = xkl;
  {
    int m0, n0;
    tile_mn(0, m0, n0);
#pragma unroll
    for (int p = 0; p < 4; p++) set_voff(p, m0, n0);
  }
  auto advance = [&](bool X) __attribute__((always_inline)) {  // next k-tile of side X / Y
    int& kt = X ? xkt : ykt;
    int& ti = X ? xti : yti;
    if (++kt == (X ? xkl : ykl)) {
      kt = 0;
      if (++ti < my_tiles) {
        int m0, n0;
        tile_mn(ti, m0, n0);
        set_voff(X ? 2 : 0, m0, n0);
        set_voff(X ? 3 : 1, m0, n0);
        (X ? xkb : ykb) = ti < ndp ? 0 : skb;
        (X ? xkl : ykl) = ti < ndp ? nk : skl;
      }
    }
  };
  // Every phase issues exactly two DMAs: past the block's last k-tile the row
  // offsets are out of range (the buffer range check reads zeros, no memory
  // traffic), so the vmcnt counts never change shape at the pipeline tail.
  auto issue = [&](auto pc, int gk) __attribute__((always_inline)) {  // gk: k-tile fetched
    constexpr int p = decltype(pc)::value;
    constexpr bool X = (p == 2 || p == 3);
    char* dst = smem + (gk & 1) * (4 * PIECE) + p * PIECE + wave * 8 * 128;
    const __amdgpu_buffer_rsrc_t r = (p == 0 || p == 3) ? rA : rB;
    const int kt = X ? xkt + xkb : ykt + ykb;
    const int soff = kt * BK * 2;
    // K % 64 != 0: the last k-tile's chunks past K read zero (both operands)
    const bool live = gk < J && kt * BK + lcx * 8 < g.K;
    dma16(r, dst, live ? voff[p][0] : (int)kOOB, soff);
    if constexpr (p != 2 || NB1 == 2) dma16(r, dst + 64 * 128, live ? voff[p][1] : (int)kOOB, soff);
  };

  const int fr = lane & 15, fq = lane >> 4;
  const int ro0 = fr * 128 + ((fq ^ (fr >> 1)) << 4), ro1 = fr * 128 + (((4 + fq) ^ (fr >> 1)) << 4);
  floatx4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; i++)
#pragma unroll
    for (int j = 0; j < TM; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  short8 a[4][2], b0[2][2], b1[NB1][2];
  short8 a1r[P3 ? 4 : 1][2];  // P3: A1 fragments, live beside A0's for the s2 MFMAs

  // quadrant (mh, nh) of this wave's tile at (m0, n0) -> bf16 C, then zeroed for the next tile
  const int cb = ((fq & 1) << 4) | ((fq >> 1) << 3);
  auto store_q = [&](int mh, int nh, int m0, int n0) __attribute__((always_inline)) {
    if (NB1 == 1 && nh == 1) {  // one 16-column block: 4 consecutive columns (8 B) per lane
      const int n = n0 + wc * WN + 32 + fq * 4;
      const bool nok = n < g.N;
#pragma unroll
      for (int mi = 0; mi < 4; mi++) {
        floatx4& x = acc[2][mh * 4 + mi];
        const unsigned x0 = cvt2(x[0], x[1]), x1 = cvt2(x[2], x[3]);
        const int m = m0 + wr * 128 + mh * 64 + mi * 16 + fr;
        const unsigned off = (m < g.M && nok) ? ((unsigned)m * (unsigned)g.ldc + (unsigned)n) * 2u : kOOB;
        if constexpr (NOST) asm volatile("" :: "v"(x0), "v"(x1), "v"(off));
        else {
          using V2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(rC, 0, 0, 0));
          uint2 v = make_uint2(x0, x1);
          __builtin_amdgcn_raw_buffer_store_b64(*reinterpret_cast<V2*>(&v), rC, off, 0, (SMODE & 1) ? 2 : 0);
        }
        x = floatx4{0.f, 0.f, 0.f, 0.f};
      }
      return;
    }
    const int n = n0 + wc * WN + nh * 32 + cb;
    const bool nok = n < g.N;
    if constexpr (ACT == 2) {  // C = relu(acc + bias): the plain quadrant store of the activated value
      const int nq = n0 + wc * WN + nh * 32 + fq * 4;
      const float4 bx = *reinterpret_cast<const float4*>(sbias + nq);
      const float4 by = *reinterpret_cast<const float4*>(sbias + nq + 16);
#pragma unroll
      for (int mi = 0; mi < 4; mi++) {
        floatx4& x = acc[nh * 2][mh * 4 + mi];
        floatx4& y = acc[nh * 2 + 1][mh * 4 + mi];
        const unsigned x0 = cvt2(fmaxf(x[0] + bx.x, 0.f), fmaxf(x[1] + bx.y, 0.f));
        const unsigned x1 = cvt2(fmaxf(x[2] + bx.z, 0.f), fmaxf(x[3] + bx.w, 0.f));
        const unsigned y0 = cvt2(fmaxf(y[0] + by.x, 0.f), fmaxf(y[1] + by.y, 0.f));
        const unsigned y1 = cvt2(fmaxf(y[2] + by.z, 0.f), fmaxf(y[3] + by.w, 0.f));
        const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
        const int m = m0 + wr * 128 + mh * 64 + mi * 16 + fr;
        const unsigned off = (m < g.M && nok) ? ((unsigned)m * (unsigned)g.ldc + (unsigned)n) * 2u : kOOB;
        store16(rC, off, make_uint4(s0[0], s1[0], s0[1], s1[1]));
        x = floatx4{0.f, 0.f, 0.f, 0.f};
        y = floatx4{0.f, 0.f, 0.f, 0.f};
      }
      return;
    }
    if constexpr (ACT == 1) {
      // before the swap, x holds columns 4fq..4fq+3 of the quadrant's first 16-column
      // block, y the same of the second: their bias, then z = acc + bias -> C, gelu(z) -> Y
      const int nq = n0 + wc * WN + nh * 32 + fq * 4;
      const float4 bx = *reinterpret_cast<const float4*>(sbias + nq);
      const float4 by = *reinterpret_cast<const float4*>(sbias + nq + 16);
#pragma unroll
      for (int mi = 0; mi < 4; mi++) {
        floatx4& x = acc[nh * 2][mh * 4 + mi];
        floatx4& y = acc[nh * 2 + 1][mh * 4 + mi];
        const float zx0 = x[0] + bx.x, zx1 = x[1] + bx.y, zx2 = x[2] + bx.z, zx3 = x[3] + bx.w;
        const float zy0 = y[0] + by.x, zy1 = y[1] + by.y, zy2 = y[2] + by.z, zy3 = y[3] + by.w;
        const int m = m0 + wr * 128 + mh * 64 + mi * 16 + fr;
        const unsigned off = (m < g.M && nok) ? ((unsigned)m * (unsigned)g.ldc + (unsigned)n) * 2u : kOOB;
        const unsigned px0 = cvt2(zx0, zx1), px1 = cvt2(zx2, zx3), py0 = cvt2(zy0, zy1), py1 = cvt2(zy2, zy3);
        {
          const auto s0 = __builtin_amdgcn_permlane16_swap(px0, py0, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(px1, py1, false, false);
          store16(rC, off, make_uint4(s0[0], s1[0], s0[1], s1[1]));
        }
        {
          // GELU of the bf16-rounded z (exactly the value the backward's gelu'(z) reads)
          auto lo = [](unsigned w) { return __uint_as_float(w << 16); };
          auto hi = [](unsigned w) { return __uint_as_float(w & 0xffff0000u); };
          const auto s0 = __builtin_amdgcn_permlane16_swap(cvt2(gelu_f(lo(px0)), gelu_f(hi(px0))),
                                                            cvt2(gelu_f(lo(py0)), gelu_f(hi(py0))), false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(cvt2(gelu_f(lo(px1)), gelu_f(hi(px1))),
                                                            cvt2(gelu_f(lo(py1)), gelu_f(hi(py1))), false, false);
          store16(rY, off, make_uint4(s0[0], s1[0], s0[1], s1[1]));
        }
        x = floatx4{0.f, 0.f, 0.f, 0.f};
        y = floatx4{0.f, 0.f, 0.f, 0.f};
      }
      return;
    }
#pragma unroll
    for (int mi = 0; mi < 4; mi++) {
      floatx4& x = acc[nh * 2][mh * 4 + mi];
      floatx4& y = acc[nh * 2 + 1][mh * 4 + mi];
      unsigned x0 = cvt2(x[0], x[1]), x1 = cvt2(x[2], x[3]);
      unsigned y0 = cvt2(y[0], y[1]), y1 = cvt2(y[2], y[3]);
      const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
      const int m = m0 + wr * 128 + mh * 64 + mi * 16 + fr;
      const unsigned off = (m < g.M && nok) ? ((unsigned)m * (unsigned)g.ldc + (unsigned)n) * 2u : kOOB;
      if constexpr (NOST) asm volatile("" :: "v"(s0[0]), "v"(s1[0]), "v"(s0[1]), "v"(s1[1]), "v"(off));
      else if constexpr (SMODE & 1) {
        using V = decltype(__builtin_amdgcn_raw_buffer_load_b128(rC, 0, 0, 0));
        uint4 v = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<V*>(&v), rC, off, 0, 2);
      } else store16(rC, off, make_uint4(s0[0], s1[0], s0[1], s1[1]));
      x = floatx4{0.f, 0.f, 0.f, 0.f};
      y = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  };

  auto mfma_q = [&](auto& bb, int mh, int nh) __attribute__((always_inline)) {
    constexpr int NI = sizeof(bb) / sizeof(bb[0]);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ks++)
#pragma unroll
      for (int ni = 0; ni < NI; ni++)
#pragma unroll
        for (int mi = 0; mi < 4; mi++)
          acc[nh * 2 + ni][mh * 4 + mi] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[ni][ks], a[mi][ks], acc[nh * 2 + ni][mh * 4 + mi], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto rd = [&](const char* p) -> short8 { return *reinterpret_cast<const short8*>(p); };

  // prologue: pieces of phases -6..-1 (A0 B0 B1 A1 of k-tile 0, A0 B0 of k-tile 1);
  // P3 needs A1 before B1 (its s1 reads A1, s2 reads B1)
  issue(std::integral_constant<int, 0>{}, 0);
  issue(std::integral_constant<int, 1>{}, 0);
  advance(false);
  if constexpr (P3) {
    issue(std::integral_constant<int, 3>{}, 0);
    issue(std::integral_constant<int, 2>{}, 0);
  } else {
    issue(std::integral_constant<int, 2>{}, 0);
    issue(std::integral_constant<int, 3>{}, 0);
  }
  advance(true);
  issue(std::integral_constant<int, 0>{}, 1);
  issue(std::integral_constant<int, 1>{}, 1);
  advance(false);
  vm_wait<D>();
  asm volatile("s_barrier" ::: "memory");
  if (wr) asm volatile("s_barrier" ::: "memory");  // group 1 runs one barrier behind

  int cm0, cn0, pm0 = 0, pn0 = 0;  // compute-side tile and the previous one (whose C is being written)
  tile_mn(0, cm0, cn0);
  int ckt = 0;  // k-tile index within the compute-side tile

  // One k-tile = four phases, branch-free: MODE bit 0 = this k-tile writes the
  // previous tile's C (4 stores per phase), bit 1 = the previous k-tile did.
  // Phase s retires the piece of four phases ago, leaving in flight 2 DMAs per
  // later phase plus the stores issued among those phases (compile-time counts).
  auto ktile = [&](int u, auto mode) __attribute__((always_inline)) {
    constexpr int MODE = decltype(mode)::value;
    constexpr bool EPI = MODE & 1, PEPI = MODE & 2;
    const char* buf = smem + (u & 1) * (4 * PIECE);
    auto retire = [&](auto sc) __attribute__((always_inline)) {
      constexpr int s = decltype(sc)::value;
      // stores per phase: 4 each (quadrant per phase) or 8, 0, 8, 0 (row pairs)
      constexpr int RP = (SMODE & 2) ? 1 : 0;
      constexpr int SPP = ACT == 1 ? 8 : 4;  // stores per quadrant phase (GELU: z and gelu(z))
      constexpr int upto = RP ? 8 * (s / 2 + 1) : SPP * (s + 1);          // phases 0..s
      constexpr int after = RP ? 8 * ((3 - s + (s % 2 == 0 ? 0 : 1)) / 2) : SPP * (3 - s);  // phases s+1..3
      constexpr int n = D + (EPI ? upto : 0) + (PEPI ? after : 0);
      vm_wait<n>();
    };
    // s0: A0 + B0 -> quadrant (0, 0)
    {
      const char* pa = buf + wr * 64 * 128;
      const char* pb = buf + PIECE + wc * 32 * 128;  // 32 rows per wave column group
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
      if constexpr (EPI) {
        store_q(0, 0, pm0, pn0);
        if constexpr (SMODE & 2) store_q(0, 1, pm0, pn0);
      }
      issue(std::integral_constant<int, 2>{}, u + 1);
      retire(std::integral_constant<int, 0>{});
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_q(b0, 0, 0);
      asm volatile("s_barrier" ::: "memory");
    }
    // s1: B1 -> quadrant (0, 1)
    {
      const char* pb = buf + 2 * PIECE + wc * (16 * NB1) * 128;
#pragma unroll
      for (int ni = 0; ni < NB1; ni++) {
        b1[ni][0] = rd(pb + ni * 16 * 128 + ro0);
        b1[ni][1] = rd(pb + ni * 16 * 128 + ro1);
      }
      if constexpr (EPI && !(SMODE & 2)) store_q(0, 1, pm0, pn0);
      issue(std::integral_constant<int, 3>{}, u + 1);
      retire(std::integral_constant<int, 1>{});
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_q(b1, 0, 1);
      asm volatile("s_barrier" ::: "memory");
    }
    // s2: A1 -> quadrant (1, 1)
    {
      const char* pa = buf + 3 * PIECE + wr * 64 * 128;
#pragma unroll
      for (int mi = 0; mi < 4; mi++) {
        a[mi][0] = rd(pa + mi * 16 * 128 + ro0);
        a[mi][1] = rd(pa + mi * 16 * 128 + ro1);
      }
      if constexpr (EPI) {
        store_q(1, 1, pm0, pn0);
        if constexpr (SMODE & 2) store_q(1, 0, pm0, pn0);
      }
      issue(std::integral_constant<int, 0>{}, u + 2);
      retire(std::integral_constant<int, 2>{});
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_q(b1, 1, 1);
      asm volatile("s_barrier" ::: "memory");
    }
    // s3: registers only -> quadrant (1, 0)
    {
      if constexpr (EPI && !(SMODE & 2)) store_q(1, 0, pm0, pn0);
      issue(std::integral_constant<int, 1>{}, u + 2);
      retire(std::integral_constant<int, 3>{});
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_q(b0, 1, 0);
      asm volatile("s_barrier" ::: "memory");
    }
    advance(true);
    advance(false);
  };

  // P3 k-tile (see the kernel comment): stores per phase 4 / 4 / 8 (the two
  // one-block halves of s2 are 4 8-B stores each)
  // MODE bit 2 (LAST): the block's final k-tile (not a split unit, >= 3 k-tiles in
  // the tile): rows 0-63 x blocks 0-1 are final after s0 and are written during s1,
  // rows 64-127 x blocks 0-1 during s2 — only block 2 is left for after the loop
  // (the last tile's C write was the one nothing overlapped)
  auto ktile3 = [&](int u, auto mode) __attribute__((always_inline)) {
    constexpr int MODE = decltype(mode)::value;
    constexpr bool EPI = MODE & 1, PEPI = MODE & 2, LAST = MODE & 4;
    static_assert(!(LAST && (EPI || PEPI)), "the last k-tile carries no tile-boundary stores");
    const char* buf = smem + (u & 1) * (4 * PIECE);
    auto retire = [&](auto sc) __attribute__((always_inline)) {
      constexpr int s = decltype(sc)::value;
      constexpr int st[3] = {4, 4, 8};
      constexpr int upto = st[0] + (s >= 1 ? st[1] : 0) + (s >= 2 ? st[2] : 0);
      constexpr int after = (s < 1 ? st[1] : 0) + (s < 2 ? st[2] : 0);
      constexpr int last = s == 0 ? 0 : (s == 1 ? 4 : 8);
      vm_wait<D + (EPI ? upto : 0) + (PEPI ? after : 0) + (LAST ? last : 0)>();
    };
    auto mfma_blocks = [&](auto& bb, auto& aa, int mh, int nb0, auto nbc) __attribute__((always_inline)) {
      constexpr int NBC = decltype(nbc)::value;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ks++)
#pragma unroll
        for (int ni = 0; ni < NBC; ni++)
#pragma unroll
          for (int mi = 0; mi < 4; mi++)
            acc[nb0 + ni][mh * 4 + mi] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[ni][ks], aa[mi][ks], acc[nb0 + ni][mh * 4 + mi], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    {  // s0: A0 + B0 -> rows 0-63 x blocks 0, 1
      const char* pa = buf + wr * 64 * 128;
      const char* pb = buf + PIECE + wc * 32 * 128;
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
      if constexpr (EPI) store_q(0, 0, pm0, pn0);
      issue(std::integral_constant<int, 3>{}, u + 1);
      retire(std::integral_constant<int, 0>{});
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_blocks(b0, a, 0, 0, std::integral_constant<int, 2>{});
      asm volatile("s_barrier" ::: "memory");
    }
    {  // s1: A1 -> rows 64-127 x blocks 0, 1
      const char* pa = buf + 3 * PIECE + wr * 64 * 128;
#pragma unroll
      for (int mi = 0; mi < 4; mi++) {
        a1r[mi][0] = rd(pa + mi * 16 * 128 + ro0);
        a1r[mi][1] = rd(pa + mi * 16 * 128 + ro1);
      }
      if constexpr (EPI) store_q(1, 0, pm0, pn0);
      if constexpr (LAST) store_q(0, 0, cm0, cn0);  // final since s0
      issue(std::integral_constant<int, 2>{}, u + 1);
      retire(std::integral_constant<int, 1>{});
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_blocks(b0, a1r, 1, 0, std::integral_constant<int, 2>{});
      asm volatile("s_barrier" ::: "memory");
    }
    {  // s2: B1 -> both row halves x block 2
      const char* pb = buf + 2 * PIECE + wc * 16 * 128;
      b1[0][0] = rd(pb + ro0);
      b1[0][1] = rd(pb + ro1);
      if constexpr (EPI) {
        store_q(0, 1, pm0, pn0);
        store_q(1, 1, pm0, pn0);
      }
      if constexpr (LAST) store_q(1, 0, cm0, cn0);  // final since s1
      issue(std::integral_constant<int, 0>{}, u + 2);
      issue(std::integral_constant<int, 1>{}, u + 2);
      retire(std::integral_constant<int, 2>{});
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_blocks(b1, a, 0, 2, std::integral_constant<int, 1>{});
      mfma_blocks(b1, a1r, 1, 2, std::integral_constant<int, 1>{});
      asm volatile("s_barrier" ::: "memory");
    }
    advance(true);
    advance(false);
  };

  // tile by tile: the first k-tile of every tile after the first writes the
  // previous tile's C, the second still has those stores in its count window
  int u = 0;
  for (int t = 0; t < my_tiles; t++) {
    int k = 0;
    const int kl = t < ndp ? nk : skl;
    if (t > 0) {
      pm0 = cm0;
      pn0 = cn0;
      tile_mn(t, cm0, cn0);
      if constexpr (P3) {
        ktile3(u++, std::integral_constant<int, 1>{});
        ktile3(u++, std::integral_constant<int, 2>{});
      } else {
        ktile(u++, std::integral_constant<int, 1>{});
        ktile(u++, std::integral_constant<int, 2>{});
      }
      k = 2;
    }
    if constexpr (P3) {
      const bool last_early = t == my_tiles - 1 && !has_split && kl >= 3;
      for (; k < kl - (last_early ? 1 : 0); k++) ktile3(u++, std::integral_constant<int, 0>{});
      if (last_early) ktile3(u++, std::integral_constant<int, 4>{});
    } else
      for (; k < kl; k++) ktile(u++, std::integral_constant<int, 0>{});
  }
  if (!wr) asm volatile("s_barrier" ::: "memory");  // both groups at the same barrier count
  if (has_split) {
    // Last-arriver combine (no block ever waits for another, so the kernel
    // finishes whatever share of the CUs it gets — RCCL kernels, a side stream,
    // another process): every part publishes its fp32 partial slot
    // [TN * TM floatx4][512 threads] (coalesced 16 B per lane, the reader has the
    // same register layout), releases it at agent scope and draws a ticket; the
    // part that draws ns - 1 acquires, adds the other ns - 1 slots and writes C.
    constexpr int NR = TN * TM;
    floatx4* slots = reinterpret_cast<floatx4*>(g.ws) + (long)unit * ns * NR * 512;
    int* flag = g.flags + unit;
    {
      floatx4* dst = slots + (long)part * NR * 512 + tid;
#pragma unroll
      for (int i = 0; i < TN; i++)
#pragma unroll
        for (int j = 0; j < TM; j++) dst[(i * TM + j) * 512] = acc[i][j];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's slot stores (and the tail DMAs) done
    __syncthreads();
    int* last = reinterpret_cast<int*>(smem);  // the one LDS array: no DMA in flight after the vmcnt(0) above
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // keep: the fence's own wait can be dropped
      const int t = __hip_atomic_fetch_add(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int is_last = t == ns - 1;
      if (is_last) {
        __hip_atomic_store(flag, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // self-cleaning
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *last = is_last;
    }
    __syncthreads();
    if (!*last) return;
    // sum the slots in part order (its own slot re-read too), so C does not depend on
    // which part arrived last: bit-identical results run to run
#pragma unroll
    for (int i = 0; i < TN; i++)
#pragma unroll
      for (int j = 0; j < TM; j++) acc[i][j] = __builtin_nontemporal_load(slots + tid + (i * TM + j) * 512);
    for (int q = 1; q < ns; q++) {
      const floatx4* src = slots + (long)q * NR * 512 + tid;
#pragma unroll
      for (int i = 0; i < TN; i++)
#pragma unroll
        for (int j = 0; j < TM; j++) acc[i][j] += __builtin_nontemporal_load(src + (i * TM + j) * 512);
    }
  }
  // the last tile's C (P3 with an early-stored last k-tile: only block 2 is left)
  const bool stored_early = P3 && !has_split && (my_tiles - 1 < ndp ? nk : skl) >= 3;
  if (!stored_early) store_q(0, 0, cm0, cn0);
  store_q(0, 1, cm0, cn0);
  store_q(1, 1, cm0, cn0);
  if (!stored_early) store_q(1, 0, cm0, cn0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's zero-fill DMAs land before the LDS is released
}

// ---------------------------------------------------------------------------
// gemm_ppw_kernel: the same persistent ping-pong pipeline (256 x 256 tiles, four
// phases per 64-deep k-tile, the previous tile's C written during the next tile's
// first k-tile) with the roles of the two wave groups SPECIALISED so that no C
// store ever sits in the in-order vmcnt window of an LDS-DMA retire:
//
// * group 0 (waves 0-3) issues EVERY LDS-DMA piece (4 DMAs per 16 KB piece per
//   wave) and waits only on those (fixed vmcnt(16): the pieces of the last four
//   phases).  At a tile boundary it hands its C quadrant to group 1 through a
//   32 KB LDS hand-off area (two 16 KB halves by phase parity; inline-asm
//   ds_write_b128, so hipcc adds no vmcnt(0) for the DMAs in flight) instead of
//   storing it;
// * group 1 (waves 4-7) issues no DMA and never waits on vmcnt: at a boundary
//   phase it stores its own quadrant from its accumulators AND its partner's
//   from the hand-off area (inline-asm ds_read_b128 + counted lgkmcnt).
//
// gemm_ppp_kernel's stores share the counter with the DMAs, so when all CUs cross
// a tile boundary together (equal work per CU) the 32 MB C burst stalls every
// DMA retire behind it (profiles/r3_gemm_ppp.txt); here the burst drains from
// group 1's counter while group 0's pipeline keeps running.  LDS: 128 KB ring +
// 32 KB hand-off = the CU's whole 160 KB.  No split remainder (data-parallel tiles).
// Diagnostic build only (KFA_PW_STAMP=1: three segments per phase, 2: five): per-
// segment s_memtime cycle sums of gemm_ppw_kernel's k-loop for blocks 0..255, waves 0
// (DMA group) and 4 (store group), read back by kfa_pw_stamps (tools/ppw_stamps.py).
// The stamp's lgkmcnt(0) drains LDS reads in flight: read shares, not run times.
#ifndef KFA_PW_STAMP
#define KFA_PW_STAMP 0
#endif
#if KFA_PW_STAMP
constexpr int kPwSeg = 24;  // [phase 0..3][segment 0..4], prologue, epilogue, k-tiles, spare
__device__ unsigned g_pw_stamps[256 * 2 * kPwSeg];
__device__ __forceinline__ unsigned long long pw_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define PW_ST(i)                            \
  do {                                      \
    const unsigned long long t_ = pw_now(); \
    psum[i] += (unsigned)(t_ - plast_t);    \
    plast_t = t_;                           \
  } while (0)
#else
#define PW_ST(i) \
  do {           \
  } while (0)
#endif

constexpr int HANDOFF = 16384;  // bytes per hand-off half: 4 waves x 64 rows x 32 cols x bf16

// DACT: the GELU-backward epilogue (the BERT FFN-down data gradient dz = (df2 · W2) *
// gelu'(z1 + b1) and the FFN-up bias gradient's column sums): group 1 loads the
// quadrant's z (and the bias) one phase ahead of its store phase (its counter holds no
// DMA), multiplies, stores dz and writes the quadrant band's column sums to cpart.
// FACT 2 (bias + ReLU forward epilogue, the W&D MLP layers): group 1 loads the bias of
// the quadrant's 8 columns (the same for its own and its partner's quadrant) and stores
// relu(c + bias) from the bf16 product — the library + bias/ReLU-pass rounding — so the
// ReLU layers run on this schedule instead of gemm_ppp_kernel<..., ACT = 2>, whose C
// stores share the DMA counter (W&D layer 1: 256.6 vs 215.9 us plain, tools/bench_wd_k1680.py).
template <bool NT, bool DACT = false, int FACT = 0>
__global__ __launch_bounds__(512, 1) void gemm_ppw_kernel(PppArgs g) {
  static_assert(FACT == 0 || (FACT == 2 && !DACT), "forward epilogue: bias + ReLU, not with DACT");
  constexpr int BN = 256, WN = 64, TM = 8, TN = 4, NB1 = 2;
  constexpr int DW = 4;  // DMAs per piece per group-0 wave
  __shared__ __attribute__((aligned(16))) char smem[2 * 4 * PIECE + 2 * HANDOFF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const bool loader = wr == 0;  // group 0: DMA; group 1: stores
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, x8 = bid & 7;
  const int lc = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (bid >> 3);
  ppp_stagger(g.stagger, lc);
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + 255) / 256, ntiles = ntm * ntn;
  const int nk = (g.K + BK - 1) / BK;  // K % 8 == 0; a partial last k-tile reads zeros past K
  const int my_tiles = lc < ntiles ? (ntiles - 1 - lc) / nwg + 1 : 0;
  const int J = my_tiles * nk;
  if (J == 0) return;
#if KFA_PW_STAMP
  unsigned psum[kPwSeg] = {};
  unsigned long long plast_t = pw_now();
#endif
  const int GM = g.gm > 0 ? g.gm : 4;
  auto tile_mn = [&](int i, int& m0, int& n0) __attribute__((always_inline)) {
    const int wg = lc + i * nwg;
    const int grp = wg / (GM * ntn), gm0 = grp * GM, gmn = min(GM, ntm - gm0), rem = wg - grp * GM * ntn;
    m0 = (gm0 + rem % gmn) * 256;
    n0 = (rem / gmn) * BN;
  };
  const __amdgpu_buffer_rsrc_t rA = rsrc(g.A, (unsigned)(((long)(g.M - 1) * g.lda + g.K) * 2));
  const __amdgpu_buffer_rsrc_t rB = rsrc(g.B, (unsigned)(((long)(g.N - 1) * g.ldb + g.K) * 2));
  const __amdgpu_buffer_rsrc_t rC = rsrc(g.C, g.c_bytes);
  const __amdgpu_buffer_rsrc_t rZ = rsrc(DACT ? g.Zin : g.C, DACT ? g.c_bytes : 0u);
  // DMA plan (group 0): instruction j of wave w fills piece rows j*32 + w*8 + lane/8
  const int prow = wc * 8 + (lane >> 3);
  const int lcx = (lane & 7) ^ ((prow >> 1) & 7);
  int voff[4][DW];
  auto set_voff = [&](int p, int m0, int n0) __attribute__((always_inline)) {
    const int h = (p == 2 || p == 3) ? 1 : 0;
#pragma unroll
    for (int j = 0; j < DW; j++) {
      const int r = j * 32 + prow;  // piece row
      if (p == 0 || p == 3) {
        const int m = m0 + (r >> 6) * 128 + h * 64 + (r & 63);
        voff[p][j] = m < g.M ? (m * g.lda + lcx * 8) * 2 : (int)kOOB;
      } else {
        const int n = n0 + (r >> 5) * WN + h * 32 + (r & 31);
        voff[p][j] = n < g.N ? (n * g.ldb + lcx * 8) * 2 : (int)kOOB;
      }
    }
  };
  int xkt = 0, xti = 0, ykt = 0, yti = 0;
  {
    int m0, n0;
    tile_mn(0, m0, n0);
#pragma unroll
    for (int p = 0; p < 4; p++) set_voff(p, m0, n0);
  }
  auto advance = [&](bool X) __attribute__((always_inline)) {
    int& kt = X ? xkt : ykt;
    int& ti = X ? xti : yti;
    if (++kt == nk) {
      kt = 0;
      if (++ti < my_tiles) {
        int m0, n0;
        tile_mn(ti, m0, n0);
        set_voff(X ? 2 : 0, m0, n0);
        set_voff(X ? 3 : 1, m0, n0);
      }
    }
  };
  auto issue = [&](auto pc, int gk) __attribute__((always_inline)) {
    constexpr int p = decltype(pc)::value;
    constexpr bool X = (p == 2 || p == 3);
    if (!loader) return;
    char* dst = smem + (gk & 1) * (4 * PIECE) + p * PIECE + wc * 8 * 128;
    const __amdgpu_buffer_rsrc_t r = (p == 0 || p == 3) ? rA : rB;
    const int kt = X ? xkt : ykt;
    const int soff = kt * BK * 2;
    const bool live = gk < J && kt * BK + lcx * 8 < g.K;  // K tail: chunks past K read zero
#pragma unroll
    for (int j = 0; j < DW; j++) dma16(r, dst + j * 32 * 128, live ? voff[p][j] : (int)kOOB, soff);
  };
  const int fr = lane & 15, fq = lane >> 4;
  const int ro0 = fr * 128 + ((fq ^ (fr >> 1)) << 4), ro1 = fr * 128 + (((4 + fq) ^ (fr >> 1)) << 4);
  floatx4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; i++)
#pragma unroll
    for (int j = 0; j < TM; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  short8 a[4][2], b0[2][2], b1[NB1][2];
  const int cb = ((fq & 1) << 4) | ((fq >> 1) << 3);
  // C of quadrant (mh, nh) of this wave's tile at (m0, n0) as 4 x 16 B per lane (one per 16-row block)
  auto pack_q = [&](int mh, int nh, uint4 (&v)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int mi = 0; mi < 4; mi++) {
      floatx4& x = acc[nh * 2][mh * 4 + mi];
      floatx4& y = acc[nh * 2 + 1][mh * 4 + mi];
      const unsigned x0 = cvt2(x[0], x[1]), x1 = cvt2(x[2], x[3]);
      const unsigned y0 = cvt2(y[0], y[1]), y1 = cvt2(y[2], y[3]);
      const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
      v[mi] = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      x = floatx4{0.f, 0.f, 0.f, 0.f};
      y = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  };
  // byte offset of row block mi of quadrant (mh, nh) of wave-row group grp (kOOB past M / N)
  auto q_off = [&](int grp, int mh, int nh, int m0, int n0, int mi) __attribute__((always_inline)) {
    const int n = n0 + wc * WN + nh * 32 + cb;
    const int m = m0 + grp * 128 + mh * 64 + mi * 16 + fr;
    return (m < g.M && n < g.N) ? ((unsigned)m * (unsigned)g.ldc + (unsigned)n) * 2u : kOOB;
  };
  // DACT operands of a quadrant: zq[slot] its pre-activation rows, bq the bias of its 8 columns
  uint4 zq[1][4];
  float bq[8];
  auto zload = [&](int slot, int grp, int mh, int nh, int m0, int n0) __attribute__((always_inline)) {
    if constexpr (DACT) {
#pragma unroll
      for (int mi = 0; mi < 4; mi++) {
        auto v = __builtin_amdgcn_raw_buffer_load_b128(rZ, q_off(grp, mh, nh, m0, n0, mi), 0, 0);
        zq[slot][mi] = *reinterpret_cast<uint4*>(&v);
      }
    }
  };
  auto bload = [&](int nh, int n0) __attribute__((always_inline)) {
    if constexpr (DACT || FACT) {
      const int n = n0 + wc * WN + nh * 32 + cb;
      if (g.bias && n < g.N) {
        const float4 x = *reinterpret_cast<const float4*>(g.bias + n), y = *reinterpret_cast<const float4*>(g.bias + n + 4);
        bq[0] = x.x; bq[1] = x.y; bq[2] = x.z; bq[3] = x.w; bq[4] = y.x; bq[5] = y.y; bq[6] = y.z; bq[7] = y.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++) bq[j] = 0.f;
      }
    }
  };
  // quadrant stores of wave-row group `grp` (a group-1 wave stores its partner's with grp = 0)
  auto store_v = [&](int grp, int mh, int nh, int m0, int n0, const uint4 (&v)[4], int slot = 0)
      __attribute__((always_inline)) {
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mi = 0; mi < 4; mi++) {
      const unsigned off = q_off(grp, mh, nh, m0, n0, mi);
      using V = decltype(__builtin_amdgcn_raw_buffer_load_b128(rC, 0, 0, 0));
      uint4 w = v[mi];
      if constexpr (DACT) {  // dz = c * gelu'(z + b) from the bf16 product, as bias_act_bwd evaluates it
        float c[8], z[8];
        unpack8(w, c);
        unpack8(zq[slot][mi], z);
#pragma unroll
        for (int j = 0; j < 8; j++) {
          c[j] *= gelu_grad(z[j] + bq[j]);
          cs[j] += c[j];
        }
        w = pack8(c);
      }
      if constexpr (FACT == 2) {  // y = relu(c + b)
        float c[8];
        unpack8(w, c);
#pragma unroll
        for (int j = 0; j < 8; j++) c[j] = fmaxf(c[j] + bq[j], 0.f);
        w = pack8(c);
      }
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<V*>(&w), rC, off, 0, NT ? 2 : 0);
    }
    if constexpr (DACT) {
      // the 16 lanes of a column chunk (fr) hold 16 rows each x 4 row blocks: band total
#pragma unroll
      for (int o = 1; o < 16; o <<= 1)
#pragma unroll
        for (int j = 0; j < 8; j++) cs[j] += __shfl_xor(cs[j], o, 64);
      const int n = n0 + wc * WN + nh * 32 + cb, mb = m0 + grp * 128 + mh * 64;
      if (g.cpart && fr == 0 && n < g.N && mb < g.M) {
        float* dst = g.cpart + (long)(mb >> 6) * g.N + n;
        *reinterpret_cast<float4*>(dst) = make_float4(cs[0], cs[1], cs[2], cs[3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
      }
    }
  };
  // hand-off area of phase parity `hp`: [wave column wc][mi][lane] 16-B slots (each wave its own 4 KB)
  auto ho_addr = [&](int hp, int mi) __attribute__((always_inline)) {
    return (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(smem + 2 * 4 * PIECE + hp * HANDOFF) +
           (unsigned)((wc * 4 + mi) * 1024 + lane * 16);
  };
  // boundary phase s of the next tile's first k-tile: quadrant q of the previous tile (pm0, pn0)
  auto epi = [&](int mh, int nh, int hp, int pm0, int pn0) __attribute__((always_inline)) {
    uint4 v[4];
    pack_q(mh, nh, v);
    typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
    if (loader) {
#pragma unroll
      for (int mi = 0; mi < 4; mi++) {
        const u32x4 w = {v[mi].x, v[mi].y, v[mi].z, v[mi].w};
        asm volatile("ds_write_b128 %0, %1" ::"v"(ho_addr(hp, mi)), "v"(w) : "memory");
      }
    } else {
      if constexpr (DACT) {
        // own quadrant: its z + the bias (group 1's counter holds no DMA: plain waits), then the
        // partner's z into the same registers and its hand-off — one operand set live at a time
        zload(0, 1, mh, nh, pm0, pn0);
        bload(nh, pn0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        store_v(1, mh, nh, pm0, pn0, v);
        zload(0, 0, mh, nh, pm0, pn0);
        u32x4 pw[4];
#pragma unroll
        for (int mi = 0; mi < 4; mi++) asm volatile("ds_read_b128 %0, %1" : "=v"(pw[mi]) : "v"(ho_addr(hp, mi)) : "memory");
        asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" : "+v"(pw[0]), "+v"(pw[1]), "+v"(pw[2]), "+v"(pw[3]) :: "memory");
        __builtin_amdgcn_sched_barrier(0);
        uint4 pv[4];
#pragma unroll
        for (int mi = 0; mi < 4; mi++) pv[mi] = make_uint4(pw[mi][0], pw[mi][1], pw[mi][2], pw[mi][3]);
        store_v(0, mh, nh, pm0, pn0, pv);
        return;
      }
      if constexpr (FACT) {  // the quadrant columns' bias (group 1's counter holds no DMA: a plain wait)
        bload(nh, pn0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      u32x4 pw[4];
#pragma unroll
      for (int mi = 0; mi < 4; mi++) asm volatile("ds_read_b128 %0, %1" : "=v"(pw[mi]) : "v"(ho_addr(hp, mi)) : "memory");
      store_v(1, mh, nh, pm0, pn0, v);  // own quadrant first: its registers are ready
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pw[0]), "+v"(pw[1]), "+v"(pw[2]), "+v"(pw[3]) :: "memory");
      __builtin_amdgcn_sched_barrier(0);
      uint4 pv[4];
#pragma unroll
      for (int mi = 0; mi < 4; mi++) pv[mi] = make_uint4(pw[mi][0], pw[mi][1], pw[mi][2], pw[mi][3]);
      store_v(0, mh, nh, pm0, pn0, pv);
    }
  };
  auto mfma_q = [&](auto& bb, int mh, int nh) __attribute__((always_inline)) {
    constexpr int NI = sizeof(bb) / sizeof(bb[0]);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ks++)
#pragma unroll
      for (int ni = 0; ni < NI; ni++)
#pragma unroll
        for (int mi = 0; mi < 4; mi++)
          acc[nh * 2 + ni][mh * 4 + mi] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[ni][ks], a[mi][ks], acc[nh * 2 + ni][mh * 4 + mi], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto rd = [&](const char* p) -> short8 { return *reinterpret_cast<const short8*>(p); };

  issue(std::integral_constant<int, 0>{}, 0);
  issue(std::integral_constant<int, 1>{}, 0);
  advance(false);
  issue(std::integral_constant<int, 2>{}, 0);
  issue(std::integral_constant<int, 3>{}, 0);
  advance(true);
  issue(std::integral_constant<int, 0>{}, 1);
  issue(std::integral_constant<int, 1>{}, 1);
  advance(false);
  if (loader) vm_wait<4 * DW>();
  asm volatile("s_barrier" ::: "memory");
  if (wr) asm volatile("s_barrier" ::: "memory");
  // B0 of k-tile u is read at the end of k-tile u - 1 (after its last MFMAs, which were
  // the last use of b0) instead of with A0 in phase 0: the 12-read phase ran ~800
  // cycles against ~450 for the others (tools/ppw_stamps.py).  Not in the DACT variant
  // (register-bound: b0 live across the boundary phase spills)
  auto rd_b0 = [&](int u) __attribute__((always_inline)) {
    const char* pb = smem + (u & 1) * (4 * PIECE) + PIECE + wc * 32 * 128;
#pragma unroll
    for (int ni = 0; ni < 2; ni++) {
      b0[ni][0] = *reinterpret_cast<const short8*>(pb + ni * 16 * 128 + ro0);
      b0[ni][1] = *reinterpret_cast<const short8*>(pb + ni * 16 * 128 + ro1);
    }
  };
  if constexpr (!DACT) rd_b0(0);
  PW_ST(20);

  int cm0, cn0, pm0 = 0, pn0 = 0;
  tile_mn(0, cm0, cn0);
  // retire: group 0 leaves the pieces of the last four phases in flight; with a
  // hand-off written this phase it also drains its LDS writes before the barrier
  auto retire = [&](bool ho) __attribute__((always_inline)) {
    if (loader) {
      vm_wait<4 * DW>();
      if (ho) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  };
  auto ktile = [&](int u, auto mode, bool pre = false) __attribute__((always_inline)) {
    constexpr bool EPI = decltype(mode)::value;
    if (KFA_PW_STAMP == 3) PW_ST(19);  // k-tile entry: the previous k-tile's tail (advance, loop branch)
    const char* buf = smem + (u & 1) * (4 * PIECE);
    {  // s0: A0 (B0 was read at the end of the previous k-tile; DACT: here) -> quadrant (0, 0)
      const char* pa = buf + wr * 64 * 128;
      if constexpr (DACT) rd_b0(u);
#pragma unroll
      for (int mi = 0; mi < 4; mi++) {
        a[mi][0] = rd(pa + mi * 16 * 128 + ro0);
        a[mi][1] = rd(pa + mi * 16 * 128 + ro1);
      }
      if constexpr (EPI) epi(0, 0, 0, pm0, pn0);
      issue(std::integral_constant<int, 2>{}, u + 1);
      if (KFA_PW_STAMP == 2) PW_ST(3);
      retire(EPI);
      if (KFA_PW_STAMP == 2) PW_ST(4);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      PW_ST(0);
      mfma_q(b0, 0, 0);
      PW_ST(1);
      asm volatile("s_barrier" ::: "memory");
      PW_ST(2);
    }
    {  // s1: B1 -> quadrant (0, 1)
      const char* pb = buf + 2 * PIECE + wc * 32 * 128;
#pragma unroll
      for (int ni = 0; ni < NB1; ni++) {
        b1[ni][0] = rd(pb + ni * 16 * 128 + ro0);
        b1[ni][1] = rd(pb + ni * 16 * 128 + ro1);
      }
      if constexpr (EPI) epi(0, 1, 1, pm0, pn0);
      issue(std::integral_constant<int, 3>{}, u + 1);
      if (KFA_PW_STAMP == 2) PW_ST(8);
      retire(EPI);
      if (KFA_PW_STAMP == 2) PW_ST(9);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      PW_ST(5);
      mfma_q(b1, 0, 1);
      PW_ST(6);
      asm volatile("s_barrier" ::: "memory");
      PW_ST(7);
    }
    {  // s2: A1 -> quadrant (1, 1)
      const char* pa = buf + 3 * PIECE + wr * 64 * 128;
#pragma unroll
      for (int mi = 0; mi < 4; mi++) {
        a[mi][0] = rd(pa + mi * 16 * 128 + ro0);
        a[mi][1] = rd(pa + mi * 16 * 128 + ro1);
      }
      if constexpr (EPI) epi(1, 1, 0, pm0, pn0);
      issue(std::integral_constant<int, 0>{}, u + 2);
      if (KFA_PW_STAMP == 2) PW_ST(13);
      retire(EPI);
      if (KFA_PW_STAMP == 2) PW_ST(14);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      PW_ST(10);
      mfma_q(b1, 1, 1);
      PW_ST(11);
      asm volatile("s_barrier" ::: "memory");
      PW_ST(12);
    }
    {  // s3: registers only -> quadrant (1, 0)
      if constexpr (EPI) epi(1, 0, 1, pm0, pn0);
      (void)pre;
      issue(std::integral_constant<int, 1>{}, u + 2);
      if (KFA_PW_STAMP == 2) PW_ST(18);
      retire(EPI);
      if (KFA_PW_STAMP == 2) PW_ST(19);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      PW_ST(15);
      mfma_q(b0, 1, 0);
      PW_ST(16);
      if constexpr (!DACT) rd_b0(u + 1);  // the next k-tile's B0 (retired by this phase's vmcnt, published by its first barrier)
      asm volatile("s_barrier" ::: "memory");
      PW_ST(17);
    }
    advance(true);
    advance(false);
  };

  int u = 0;
  for (int t = 0; t < my_tiles; t++) {
    int k = 0;
    if (t > 0) {
      pm0 = cm0;
      pn0 = cn0;
      tile_mn(t, cm0, cn0);
      ktile(u++, std::true_type{});
      k = 1;
    }
    for (; k < nk; k++) ktile(u++, std::false_type{}, DACT && k == nk - 1 && t + 1 < my_tiles);
  }
  if (!wr) asm volatile("s_barrier" ::: "memory");  // both groups at the same barrier count
  // the last tile: every wave stores its own quadrants (group 0's DMAs are all issued)
  {
    uint4 v[4];
    auto tail = [&](int mh, int nh) __attribute__((always_inline)) {
      if constexpr (DACT) {
        zload(0, wr, mh, nh, cm0, cn0);
        bload(nh, cn0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if constexpr (FACT) {
        bload(nh, cn0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      pack_q(mh, nh, v);
      store_v(wr, mh, nh, cm0, cn0, v);
    };
    tail(0, 0);
    tail(0, 1);
    tail(1, 1);
    tail(1, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's zero-fill DMAs land before the LDS is released
#if KFA_PW_STAMP
  PW_ST(21);
  psum[22] = (unsigned)J;
  if (lane == 0 && bid < 256 && (wave & 3) == 0) {
#pragma unroll
    for (int i = 0; i < kPwSeg; i++) g_pw_stamps[(bid * 2 + wr) * kPwSeg + i] = psum[i];
  }
#endif
}

// ---------------------------------------------------------------------------
// gemm_ppw3_kernel: 256 x 192 tiles (N = 768: BERT-base's hidden size — at
// M = 32768 that is 512 tiles, exactly two per CU, where 256-wide tiles leave 1.5)
// on the wave-specialised persistent pipeline of gemm_ppw_kernel, with the
// THREE-phase k-tile of gemm_ppp_kernel<192, ..., P3> (16 MFMAs per phase instead
// of a 48-column wave tile's 16 / 8 / 8 / 16):
//
//   s0: A0 -> rows 0-63 x blocks 0, 1      (B0 read at the end of the previous k-tile)
//   s1: A1 -> rows 64-127 x blocks 0, 1    (B0 fragments kept)
//   s2: B1 -> rows 0-127 x block 2         (A0, A1 fragments kept); then B0 of k-tile u+1
//
// Group 0 (waves 0-3) issues every LDS-DMA: s0 A1(u+1) [4 per wave], s1 B1(u+1) [2:
// piece 2 is the 64 rows of the wave column groups' third blocks], s2 A0 + B0 (u+2)
// [8] — each piece DMA'd three phases before its read phase, into a buffer whose
// previous piece was read >= 2 phases earlier; every phase leaves exactly the last
// three phases' DMAs in flight: fixed vmcnt(14).  Group 1 (waves 4-7) issues no
// DMA and stores all C: its own quadrants from registers, group 0's from the 32 KB
// hand-off area (two 16 KB halves by phase parity, inline-asm ds ops so hipcc adds
// no vmcnt(0) behind the DMAs in flight).
//
// Stores, per tile: rows 0-127 x blocks 0-1 are final after s0 / s1 of the tile's
// LAST k-tile and are written in s1 / s2 of that k-tile; block 2 (final after s2)
// in s2 of the next tile's first k-tile.  Only the block's final tile's block 2 —
// a third of one tile — is written after the loop, where nothing overlaps it.
template <bool NT>
__global__ __launch_bounds__(512, 1) void gemm_ppw3_kernel(PppArgs g) {
  constexpr int BN = 192, WN = 48, TM = 8, TN = 3;
  constexpr int DW = 4;   // DMAs per full 16 KB piece per group-0 wave
  constexpr int VMW = 14; // group-0 DMAs of three phases: A1 4 + B1 2 + A0/B0 8
  __shared__ __attribute__((aligned(16))) char smem[2 * 4 * PIECE + 2 * HANDOFF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const bool loader = wr == 0;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, x8 = bid & 7;
  const int lc = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (bid >> 3);
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + 255) / 256, ntiles = ntm * ntn;
  const int nk = (g.K + BK - 1) / BK;
  const int my_tiles = lc < ntiles ? (ntiles - 1 - lc) / nwg + 1 : 0;
  const int J = my_tiles * nk;
  if (J == 0) return;
  const int GM = g.gm > 0 ? g.gm : 4;
  auto tile_mn = [&](int i, int& m0, int& n0) __attribute__((always_inline)) {
    const int wg = lc + i * nwg;
    const int grp = wg / (GM * ntn), gm0 = grp * GM, gmn = min(GM, ntm - gm0), rem = wg - grp * GM * ntn;
    m0 = (gm0 + rem % gmn) * 256;
    n0 = (rem / gmn) * BN;
  };
  const __amdgpu_buffer_rsrc_t rA = rsrc(g.A, (unsigned)(((long)(g.M - 1) * g.lda + g.K) * 2));
  const __amdgpu_buffer_rsrc_t rB = rsrc(g.B, (unsigned)(((long)(g.N - 1) * g.ldb + g.K) * 2));
  const __amdgpu_buffer_rsrc_t rC = rsrc(g.C, g.c_bytes);
  const int prow = wc * 8 + (lane >> 3);
  const int lcx = (lane & 7) ^ ((prow >> 1) & 7);
  int voff[4][DW];  // piece 2 uses entries 0-1 only (the compiler drops the rest)
  // pieces: 0 = A rows {0-63, 128-191}, 3 = A rows {64-127, 192-255}, 1 = the first 32
  // columns of each wave column group (128 rows), 2 = their third 16-column block (64 rows)
  auto set_voff = [&](int p, int m0, int n0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < DW; j++) {
      const int r = j * 32 + prow;
      if (p == 0 || p == 3) {
        const int m = m0 + (r >> 6) * 128 + (p == 3 ? 64 : 0) + (r & 63);
        voff[p][j] = m < g.M ? (m * g.lda + lcx * 8) * 2 : (int)kOOB;
      } else if (p == 1) {
        const int n = n0 + (r >> 5) * WN + (r & 31);
        voff[p][j] = n < g.N ? (n * g.ldb + lcx * 8) * 2 : (int)kOOB;
      } else if (j < 2) {
        const int n = n0 + (r >> 4) * WN + 32 + (r & 15);
        voff[p][j] = n < g.N ? (n * g.ldb + lcx * 8) * 2 : (int)kOOB;
      }
    }
  };
  // issue side: pieces 3, 2 fetch k-tile u + 1 ("X"), pieces 0, 1 fetch u + 2 ("Y")
  int xkt = 0, xti = 0, ykt = 0, yti = 0;
  {
    int m0, n0;
    tile_mn(0, m0, n0);
#pragma unroll
    for (int p = 0; p < 4; p++) set_voff(p, m0, n0);
  }
  auto advance = [&](bool X) __attribute__((always_inline)) {
    int& kt = X ? xkt : ykt;
    int& ti = X ? xti : yti;
    if (++kt == nk) {
      kt = 0;
      if (++ti < my_tiles) {
        int m0, n0;
        tile_mn(ti, m0, n0);
        set_voff(X ? 2 : 0, m0, n0);
        set_voff(X ? 3 : 1, m0, n0);
      }
    }
  };
  auto issue = [&](auto pc, int gk) __attribute__((always_inline)) {
    constexpr int p = decltype(pc)::value;
    constexpr bool X = (p == 2 || p == 3);
    constexpr int nd = p == 2 ? 2 : DW;
    if (!loader) return;
    char* dst = smem + (gk & 1) * (4 * PIECE) + p * PIECE + wc * 8 * 128;
    const __amdgpu_buffer_rsrc_t r = (p == 0 || p == 3) ? rA : rB;
    const int kt = X ? xkt : ykt;
    const int soff = kt * BK * 2;
    const bool live = gk < J && kt * BK + lcx * 8 < g.K;
#pragma unroll
    for (int j = 0; j < nd; j++) dma16(r, dst + j * 32 * 128, live ? voff[p][j] : (int)kOOB, soff);
  };
  const int fr = lane & 15, fq = lane >> 4;
  const int ro0 = fr * 128 + ((fq ^ (fr >> 1)) << 4), ro1 = fr * 128 + (((4 + fq) ^ (fr >> 1)) << 4);
  floatx4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; i++)
#pragma unroll
    for (int j = 0; j < TM; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  short8 a0[4][2], a1[4][2], b0[2][2], b1[2];
  const int cb = ((fq & 1) << 4) | ((fq >> 1) << 3);
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  // hand-off slot k (0..3) of phase parity hp: [wave column][k][lane] 16 B
  auto ho_addr = [&](int hp, int k) __attribute__((always_inline)) {
    return (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(smem + 2 * 4 * PIECE + hp * HANDOFF) +
           (unsigned)((wc * 4 + k) * 1024 + lane * 16);
  };
  // row half mh x blocks 0-1 of this wave's tile: 4 x 16 B per lane (8 consecutive columns
  // per 16-row block after v_permlane16_swap), accumulators zeroed
  auto pack01 = [&](int mh, uint4 (&v)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int mi = 0; mi < 4; mi++) {
      floatx4& x = acc[0][mh * 4 + mi];
      floatx4& y = acc[1][mh * 4 + mi];
      const unsigned x0 = cvt2(x[0], x[1]), x1 = cvt2(x[2], x[3]);
      const unsigned y0 = cvt2(y[0], y[1]), y1 = cvt2(y[2], y[3]);
      const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
      v[mi] = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      x = floatx4{0.f, 0.f, 0.f, 0.f};
      y = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  };
  // block 2 (both row halves): 8 row blocks x 4 consecutive columns = 8 x 8 B per lane,
  // two row blocks per 16-B slot
  auto pack2b = [&](uint4 (&v)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      floatx4& x = acc[2][2 * k];
      floatx4& y = acc[2][2 * k + 1];
      v[k] = make_uint4(cvt2(x[0], x[1]), cvt2(x[2], x[3]), cvt2(y[0], y[1]), cvt2(y[2], y[3]));
      x = floatx4{0.f, 0.f, 0.f, 0.f};
      y = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  };
  using V4 = decltype(__builtin_amdgcn_raw_buffer_load_b128(rC, 0, 0, 0));
  using V2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(rC, 0, 0, 0));
  auto store01 = [&](int grp, int mh, int m0, int n0, const uint4 (&v)[4]) __attribute__((always_inline)) {
    const int n = n0 + wc * WN + cb;
#pragma unroll
    for (int mi = 0; mi < 4; mi++) {
      const int m = m0 + grp * 128 + mh * 64 + mi * 16 + fr;
      const unsigned off = (m < g.M && n < g.N) ? ((unsigned)m * (unsigned)g.ldc + (unsigned)n) * 2u : kOOB;
      uint4 w = v[mi];
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<V4*>(&w), rC, off, 0, NT ? 2 : 0);
    }
  };
  auto store2b = [&](int grp, int m0, int n0, const uint4 (&v)[4]) __attribute__((always_inline)) {
    const int n = n0 + wc * WN + 32 + fq * 4;
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int m = m0 + grp * 128 + (2 * k + h) * 16 + fr;
        const unsigned off = (m < g.M && n < g.N) ? ((unsigned)m * (unsigned)g.ldc + (unsigned)n) * 2u : kOOB;
        uint2 w = h ? make_uint2(v[k].z, v[k].w) : make_uint2(v[k].x, v[k].y);
        __builtin_amdgcn_raw_buffer_store_b64(*reinterpret_cast<V2*>(&w), rC, off, 0, NT ? 2 : 0);
      }
  };
  // a store phase: group 0 hands its part to group 1 through the hand-off half hp;
  // group 1 stores its own part from registers, then group 0's from LDS.
  // what: 0 / 1 = row half 0 / 1 x blocks 0-1, 2 = block 2
  auto epi = [&](int what, int hp, int m0, int n0) __attribute__((always_inline)) {
    uint4 v[4];
    if (what == 2) pack2b(v);
    else pack01(what, v);
    if (loader) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const u32x4 w = {v[k].x, v[k].y, v[k].z, v[k].w};
        asm volatile("ds_write_b128 %0, %1" ::"v"(ho_addr(hp, k)), "v"(w) : "memory");
      }
    } else {
      // own part first (its registers are ready and then free), then the partner's
      if (what == 2) store2b(1, m0, n0, v);
      else store01(1, what, m0, n0, v);
      u32x4 pw[4];
#pragma unroll
      for (int k = 0; k < 4; k++) asm volatile("ds_read_b128 %0, %1" : "=v"(pw[k]) : "v"(ho_addr(hp, k)) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pw[0]), "+v"(pw[1]), "+v"(pw[2]), "+v"(pw[3]) :: "memory");
      __builtin_amdgcn_sched_barrier(0);
      uint4 pv[4];
#pragma unroll
      for (int k = 0; k < 4; k++) pv[k] = make_uint4(pw[k][0], pw[k][1], pw[k][2], pw[k][3]);
      if (what == 2) store2b(0, m0, n0, pv);
      else store01(0, what, m0, n0, pv);
    }
  };
  auto mfma_blocks = [&](auto& bb, auto& aa, int mh, int nb0, auto nbc) __attribute__((always_inline)) {
    constexpr int NBC = decltype(nbc)::value;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ks++)
#pragma unroll
      for (int ni = 0; ni < NBC; ni++)
#pragma unroll
        for (int mi = 0; mi < 4; mi++) {
          short8 bv;
          if constexpr (NBC == 1) bv = bb[ks];
          else bv = bb[ni][ks];
          acc[nb0 + ni][mh * 4 + mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv, aa[mi][ks], acc[nb0 + ni][mh * 4 + mi], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
  };
  auto rd = [&](const char* p) -> short8 { return *reinterpret_cast<const short8*>(p); };
  auto rd_b0 = [&](int u) __attribute__((always_inline)) {
    const char* pb = smem + (u & 1) * (4 * PIECE) + PIECE + wc * 32 * 128;
#pragma unroll
    for (int ni = 0; ni < 2; ni++) {
      b0[ni][0] = rd(pb + ni * 16 * 128 + ro0);
      b0[ni][1] = rd(pb + ni * 16 * 128 + ro1);
    }
  };

  // prologue: A0 B0 (k-tile 0), A1 (0), B1 (0), A0 B0 (1) — the steady state's
  // "three phases in flight" picture right before s0 of k-tile 0
  issue(std::integral_constant<int, 0>{}, 0);
  issue(std::integral_constant<int, 1>{}, 0);
  advance(false);
  issue(std::integral_constant<int, 3>{}, 0);
  issue(std::integral_constant<int, 2>{}, 0);
  advance(true);
  issue(std::integral_constant<int, 0>{}, 1);
  issue(std::integral_constant<int, 1>{}, 1);
  advance(false);
  if (loader) vm_wait<VMW>();
  asm volatile("s_barrier" ::: "memory");
  if (wr) asm volatile("s_barrier" ::: "memory");
  rd_b0(0);

  int cm0, cn0, pm0 = 0, pn0 = 0;
  tile_mn(0, cm0, cn0);
  auto retire = [&](bool ho) __attribute__((always_inline)) {
    if (loader) {
      vm_wait<VMW>();
      if (ho) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  };
  // MODE bit 0 (EPI): the tile's first k-tile (not the block's first tile) writes the
  // previous tile's block 2 in s2; bit 1 (LAST): the tile's last k-tile writes its own
  // rows 0-127 x blocks 0-1 in s1 / s2
  auto ktile = [&](int u, auto mode) __attribute__((always_inline)) {
    constexpr int MODE = decltype(mode)::value;
    constexpr bool EPI = MODE & 1, LAST = MODE & 2;
    const char* buf = smem + (u & 1) * (4 * PIECE);
    {  // s0: A0 -> rows 0-63 x blocks 0, 1
      const char* pa = buf + wr * 64 * 128;
#pragma unroll
      for (int mi = 0; mi < 4; mi++) {
        a0[mi][0] = rd(pa + mi * 16 * 128 + ro0);
        a0[mi][1] = rd(pa + mi * 16 * 128 + ro1);
      }
      issue(std::integral_constant<int, 3>{}, u + 1);
      retire(false);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_blocks(b0, a0, 0, 0, std::integral_constant<int, 2>{});
      asm volatile("s_barrier" ::: "memory");
    }
    {  // s1: A1 -> rows 64-127 x blocks 0, 1
      const char* pa = buf + 3 * PIECE + wr * 64 * 128;
#pragma unroll
      for (int mi = 0; mi < 4; mi++) {
        a1[mi][0] = rd(pa + mi * 16 * 128 + ro0);
        a1[mi][1] = rd(pa + mi * 16 * 128 + ro1);
      }
      if constexpr (LAST) epi(0, 1, cm0, cn0);  // rows 0-63 x blocks 0-1: final since s0
      issue(std::integral_constant<int, 2>{}, u + 1);
      retire(LAST);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_blocks(b0, a1, 1, 0, std::integral_constant<int, 2>{});
      asm volatile("s_barrier" ::: "memory");
    }
    {  // s2: B1 -> both row halves x block 2; then the next k-tile's B0
      const char* pb = buf + 2 * PIECE + wc * 16 * 128;
      b1[0] = rd(pb + ro0);
      b1[1] = rd(pb + ro1);
      if constexpr (EPI) epi(2, 0, pm0, pn0);   // the previous tile's block 2
      if constexpr (LAST) epi(1, 0, cm0, cn0);  // rows 64-127 x blocks 0-1: final since s1
      issue(std::integral_constant<int, 0>{}, u + 2);
      issue(std::integral_constant<int, 1>{}, u + 2);
      retire(EPI || LAST);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_blocks(b1, a0, 0, 2, std::integral_constant<int, 1>{});
      mfma_blocks(b1, a1, 1, 2, std::integral_constant<int, 1>{});
      rd_b0(u + 1);  // retired by this phase's vmcnt, published by its first barrier
      asm volatile("s_barrier" ::: "memory");
    }
    advance(true);
    advance(false);
  };
  static_assert(HANDOFF >= 4 * 4 * 1024, "hand-off half: 4 waves x 4 slots x 64 lanes x 16 B");

  int u = 0;
  for (int t = 0; t < my_tiles; t++) {
    if (t > 0) {
      pm0 = cm0;
      pn0 = cn0;
      tile_mn(t, cm0, cn0);
    }
    // nk >= 2 (K >= 128): the first and the last k-tile of a tile are different k-tiles
    if (t > 0) ktile(u++, std::integral_constant<int, 1>{});
    else ktile(u++, std::integral_constant<int, 0>{});
    for (int k = 1; k < nk - 1; k++) ktile(u++, std::integral_constant<int, 0>{});
    ktile(u++, std::integral_constant<int, 2>{});
  }
  if (!wr) asm volatile("s_barrier" ::: "memory");  // both groups at the same barrier count
  {  // the block's last tile: block 2, every wave its own (group 0's DMAs are all issued)
    uint4 v[4];
    pack2b(v);
    store2b(wr, cm0, cn0, v);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's zero-fill DMAs land before the LDS is released
}

// out[c] (+)= sum over rows of part[r][c] (the DACT epilogue's column-sum bands):
// block = 64 columns x 4 row lanes, grid = ceil(N / 64); fixed summation order.
__global__ __launch_bounds__(256) void colpart_reduce(const float* __restrict__ part, int R, int N,
                                                      float* __restrict__ out, int accumulate) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6;
  float s = 0.f;
  if (c < N)
    for (int r = rl; r < R; r += 4) s += part[(long)r * N + c];
  red[rl][threadIdx.x & 63] = s;
  __syncthreads();
  if (rl == 0 && c < N) {
    const float t = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
    out[c] = accumulate ? out[c] + t : t;
  }
}

#if KFA_PW_STAMP
KFA_API int kfa_pw_stamps(unsigned* out, int n) {
  if (n > 256 * 2 * kPwSeg) n = 256 * 2 * kPwSeg;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pw_stamps), (size_t)n * sizeof(unsigned), 0, hipMemcpyDeviceToHost);
}
#endif

int ppp_cus() {
  static int c = 0;
  if (!c) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    if (c <= 0) c = 256;
  }
  return c;
}

}  // namespace

// C = A · Bᵀ (bf16 out) on the persistent ping-pong kernel.  K % 8 == 0 (a
// partial last 64-deep k-tile reads zeros past K, e.g. the W&D MLP's K = 1680),
// N % 8 == 0, every extent within 31-bit buffer offsets; grid = min(tiles, CUs)
// (or `blocks` if > 0).  bn: tile width 256 or 192 (0 = pick: 192 when N is a
// multiple of 192 and 256-wide tiles would leave a partial last round).
// Returns 0, -1 on unsupported operands.
KFA_API int kfa_gemm_ppp_pick_bn(int M, int N);

// Split factor for the tiles past the last full round of a `cus`-block grid:
// r leftover tiles each cut into s = min(cus / r, nk / 2, 8) k-ranges when that
// is >= 2 (every block then runs the same number of k-tiles, +-1 range); 1 = no split.
static int ppp_split(long tiles, long cus, int nk) {
  const long r = tiles % cus;
  if (r == 0 || 2 * r > cus) return 1;
  long s = cus / r;
  if (s > nk / 2) s = nk / 2;
  if (s > 8) s = 8;
  return s >= 2 ? (int)s : 1;
}

// Workspace bytes kfa_gemm_ppp needs for this problem (0: no split): the
// self-cleaning unit counters (zero-initialised once), then the fp32 partial slots.
KFA_API long kfa_gemm_ppp_ws_bytes(int M, int N, int K, int bn, int blocks) {
  if (bn == 0) bn = kfa_gemm_ppp_pick_bn(M, N);
  const long tiles = (long)((M + 255) / 256) * ((N + bn - 1) / bn);
  const long cus = blocks > 0 ? blocks : ppp_cus();
  if (tiles <= 0 || K % 8) return 0;
  const int s = ppp_split(tiles, cus, (K + BK - 1) / BK);
  if (s == 1) return 0;
  const long r = tiles % cus;
  return 4096 + r * s * 256L * bn * 4;  // every part publishes (the last arriver is not known in advance)
}

KFA_API int kfa_gemm_ppp_pick_bn(int M, int N) {
  const long cus = ppp_cus();
  if (N % 192) return 256;
  const long t256 = (long)((M + 255) / 256) * ((N + 255) / 256), t192 = (long)((M + 255) / 256) * (N / 192);
  // rounds of the persistent grid, in 256-wide tile units of work
  const double r256 = (double)((t256 + cus - 1) / cus), r192 = 0.75 * (double)((t192 + cus - 1) / cus);
  return r192 < r256 ? 192 : 256;
}

static int g_stagger = 0;
// experiment knob (tools/bench_ppp.py): odd blocks start `ticks` x 10 ns late; 0 = off
KFA_API int kfa_gemm_ppp_set_stagger(int ticks) {
  g_stagger = ticks < 0 ? 0 : ticks;
  return 0;
}

static int g_gm = 0;
// experiment knob (tools/bench_wd_k1680.py): tile-raster group height (256-row tiles); 0 = 4
KFA_API int kfa_gemm_ppp_set_gm(int gm) {
  g_gm = gm < 0 ? 0 : gm;
  return 0;
}

static inline PppArgs with_gm(PppArgs a) {
  a.gm = g_gm;
  return a;
}

// Z = A · Bᵀ + bias (bf16, the pre-activation), Y = gelu(Z) on the persistent kernel with
// the bias + GELU epilogue (256-wide tiles, no split): K % 8 == 0, K >= 128, N % 8 == 0,
// N <= 8192; Z and Y share ldc.  Returns 0, -1 on unsupported operands.
KFA_API int kfa_gemm_ppp_gelu(const bf16_t* A, const bf16_t* B, bf16_t* Z, bf16_t* Y, const float* bias, int M, int N,
                              int K, int lda, int ldb, int ldc, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (K < 2 * BK || K % 8 || N % 8 || N > 8192 || lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K || ldc < N ||
      !bias || !Y)
    return -1;
  const long cb = (long)M * ldc * 2;
  if (cb >= (long)kOOB || (long)M * lda * 2 >= (long)kOOB || (long)N * ldb * 2 >= (long)kOOB) return -2;
  const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
  const long cus = ppp_cus();
  const int grid = (int)(tiles < cus ? tiles : cus);
  const PppArgs g{A, B, Z, M, N, K, lda, ldb, ldc, (unsigned)cb, nullptr, nullptr, 1, g_stagger, Y, bias};
  hipLaunchKernelGGL((gemm_ppp_kernel<256, false, 0, false, 1>), dim3(grid), dim3(512), 0, st, with_gm(g));
  return kfa_status();
}

// Y = relu(A · Bᵀ + bias) (bf16) on the persistent kernel with the bias + ReLU epilogue
// (256-wide tiles, no split; the pre-activation is not written): same operand rules as
// kfa_gemm_ppp_gelu.  Returns 0, -1 on unsupported operands.
KFA_API int kfa_gemm_ppp_relu(const bf16_t* A, const bf16_t* B, bf16_t* Y, const float* bias, int M, int N, int K,
                              int lda, int ldb, int ldc, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (K < 2 * BK || K % 8 || N % 8 || N > 8192 || lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K || ldc < N ||
      !bias || !Y)
    return -1;
  const long cb = (long)M * ldc * 2;
  if (cb >= (long)kOOB || (long)M * lda * 2 >= (long)kOOB || (long)N * ldb * 2 >= (long)kOOB) return -2;
  const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
  const long cus = ppp_cus();
  const int grid = (int)(tiles < cus ? tiles : cus);
  const PppArgs g{A, B, Y, M, N, K, lda, ldb, ldc, (unsigned)cb, nullptr, nullptr, 1, g_stagger, nullptr, bias};
  hipLaunchKernelGGL((gemm_ppp_kernel<256, false, 0, false, 2>), dim3(grid), dim3(512), 0, st, with_gm(g));
  return kfa_status();
}

// Y = relu(A · Bᵀ + bias) (bf16) on the wave-specialised persistent kernel (gemm_ppw_kernel
// <NT, false, 2>: the bias added to the bf16 product by the store waves); nt: non-temporal
// stores.  Same operand rules as kfa_gemm_ppp_relu.  Returns 0, -1 on unsupported operands.
KFA_API int kfa_gemm_ppw_relu(const bf16_t* A, const bf16_t* B, bf16_t* Y, const float* bias, int M, int N, int K,
                              int lda, int ldb, int ldc, int nt, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (K < 2 * BK || K % 8 || N % 8 || lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K || ldc < N || !bias ||
      !Y)
    return -1;
  const long cb = (long)M * ldc * 2;
  if (cb >= (long)kOOB || (long)M * lda * 2 >= (long)kOOB || (long)N * ldb * 2 >= (long)kOOB) return -2;
  const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
  const long cus = ppp_cus();
  const int grid = (int)(tiles < cus ? tiles : cus);
  const PppArgs g{A, B, Y, M, N, K, lda, ldb, ldc, (unsigned)cb, nullptr, nullptr, 1, g_stagger, nullptr, bias};
  if (nt) hipLaunchKernelGGL((gemm_ppw_kernel<true, false, 2>), dim3(grid), dim3(512), 0, st, with_gm(g));
  else hipLaunchKernelGGL((gemm_ppw_kernel<false, false, 2>), dim3(grid), dim3(512), 0, st, with_gm(g));
  return kfa_status();
}

// dz = (A · Bᵀ) * gelu'(Zin + bias) (bf16; bias fp32 [N] or null) on the wave-specialised
// persistent kernel with the GELU-backward epilogue; dbias (fp32 [N], nullable) (+)= the
// column sums of dz (via cpart: kfa_gemm_ppw_dact_part_floats(M, N) floats of scratch).
// K % 8 == 0, K >= 128, N % 8 == 0; Zin shares C's ldc.  Returns 0, -1 on unsupported operands.
KFA_API long kfa_gemm_ppw_dact_part_floats(int M, int N) { return (long)((M + 63) / 64) * N; }

KFA_API int kfa_gemm_ppw_dact(const bf16_t* A, const bf16_t* B, bf16_t* C, const bf16_t* Zin, const float* bias,
                              float* cpart, float* dbias, int accumulate, int M, int N, int K, int lda, int ldb,
                              int ldc, int nt, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (K < 2 * BK || K % 8 || N % 8 || lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K || ldc < N || !Zin ||
      (dbias && !cpart))
    return -1;
  const long cb = (long)M * ldc * 2;
  if (cb >= (long)kOOB || (long)M * lda * 2 >= (long)kOOB || (long)N * ldb * 2 >= (long)kOOB) return -2;
  const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
  const long cus = ppp_cus();
  PppArgs g{A, B, C, M, N, K, lda, ldb, ldc, (unsigned)cb, nullptr, nullptr, 1, g_stagger, nullptr, bias};
  g.Zin = Zin;
  g.cpart = dbias ? cpart : nullptr;
  const int grid = (int)(tiles < cus ? tiles : cus);
  if (nt) hipLaunchKernelGGL((gemm_ppw_kernel<true, true>), dim3(grid), dim3(512), 0, st, with_gm(g));
  else hipLaunchKernelGGL((gemm_ppw_kernel<false, true>), dim3(grid), dim3(512), 0, st, with_gm(g));
  if (dbias)
    hipLaunchKernelGGL(colpart_reduce, dim3((N + 63) / 64), dim3(256), 0, st, cpart, (M + 63) / 64, N, dbias,
                       accumulate);
  return kfa_status();
}

KFA_API int kfa_gemm_ppp(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, int lda, int ldb, int ldc,
                         int blocks, int probe, int bn, void* ws, long ws_bytes, int nosplit, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  // K >= 128: two k-tiles per tile at least (a tile's first two k-tiles carry its predecessor's stores)
  if (K < 2 * BK || K % 8 || N % 8 || lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K || ldc < N) return -1;
  const long cb = (long)M * ldc * 2;
  if (cb >= (long)kOOB || (long)M * lda * 2 >= (long)kOOB || (long)N * ldb * 2 >= (long)kOOB) return -2;
  if (bn == 0) bn = kfa_gemm_ppp_pick_bn(M, N);
  if (bn != 256 && bn != 192) return -1;
  const long tiles = (long)((M + 255) / 256) * ((N + bn - 1) / bn);
  const long cus = blocks > 0 ? blocks : ppp_cus();
  int split = nosplit ? 1 : ppp_split(tiles, cus, (K + BK - 1) / BK);
  if (split > 1 && (ws == nullptr || ws_bytes < kfa_gemm_ppp_ws_bytes(M, N, K, bn, blocks))) return -3;
  // a split grid is the whole `cus` blocks (the split units fill the last round)
  const int grid = split > 1 ? (int)cus : (int)(tiles < cus ? tiles : cus);
  const PppArgs g{A, B, C, M, N, K, lda, ldb, ldc, (unsigned)cb, ws ? reinterpret_cast<float*>((char*)ws + 4096) : nullptr,
                  reinterpret_cast<int*>(ws), split, g_stagger};
  const dim3 gd(grid), bd(512);
  if (probe == 11 || probe == 12) {  // wave-specialised stores, 256 x 192 three-phase tiles (gemm_ppw3_kernel)
    const long t3 = (long)((M + 255) / 256) * ((N + 191) / 192);
    const int gw = (int)(t3 < cus ? t3 : cus);
    const PppArgs gp{A, B, C, M, N, K, lda, ldb, ldc, (unsigned)cb, nullptr, nullptr, 1, g_stagger};
    if (probe == 11) hipLaunchKernelGGL((gemm_ppw3_kernel<false>), dim3(gw), dim3(512), 0, st, with_gm(gp));
    else hipLaunchKernelGGL((gemm_ppw3_kernel<true>), dim3(gw), dim3(512), 0, st, with_gm(gp));
    return kfa_status();
  }
  if (probe == 9 || probe == 10) {  // wave-specialised stores (gemm_ppw_kernel): 256-wide, data-parallel tiles only
    const int gw = (int)(tiles < cus ? tiles : cus);
    const PppArgs gp{A, B, C, M, N, K, lda, ldb, ldc, (unsigned)cb, nullptr, nullptr, 1, g_stagger};
    if (probe == 9) hipLaunchKernelGGL((gemm_ppw_kernel<false>), dim3(gw), dim3(512), 0, st, with_gm(gp));
    else hipLaunchKernelGGL((gemm_ppw_kernel<true>), dim3(gw), dim3(512), 0, st, with_gm(gp));
    return kfa_status();
  }
  if (bn == 192) {  // three-phase k-tiles (P3); probe 7 / 8: the four-phase schedule (with / without stores)
    if (probe == 1 || probe == 6) hipLaunchKernelGGL((gemm_ppp_kernel<192, true, 0, true>), gd, bd, 0, st, with_gm(g));
    else if (probe == 7) hipLaunchKernelGGL((gemm_ppp_kernel<192, false>), gd, bd, 0, st, with_gm(g));
    else if (probe == 8) hipLaunchKernelGGL((gemm_ppp_kernel<192, true>), gd, bd, 0, st, with_gm(g));
    else if (probe == 2) hipLaunchKernelGGL((gemm_ppp_kernel<192, false, 1>), gd, bd, 0, st, with_gm(g));
    else hipLaunchKernelGGL((gemm_ppp_kernel<192, false, 0, true>), gd, bd, 0, st, with_gm(g));
    return kfa_status();
  }
  if (probe == 1)  // timing probe: no C stores
    hipLaunchKernelGGL((gemm_ppp_kernel<256, true>), gd, bd, 0, st, with_gm(g));
  else if (probe == 2)  // store-policy experiments: nt / row pairs / both
    hipLaunchKernelGGL((gemm_ppp_kernel<256, false, 1>), gd, bd, 0, st, with_gm(g));
  else if (probe == 3)
    hipLaunchKernelGGL((gemm_ppp_kernel<256, false, 2>), gd, bd, 0, st, with_gm(g));
  else if (probe == 4)
    hipLaunchKernelGGL((gemm_ppp_kernel<256, false, 3>), gd, bd, 0, st, with_gm(g));
  else
    hipLaunchKernelGGL((gemm_ppp_kernel<256, false>), gd, bd, 0, st, with_gm(g));
  return kfa_status();
}
