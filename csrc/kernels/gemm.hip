// Dense GEMM with fused epilogues on MFMA (bf16 in, fp32 accumulate) — SURVEY
// §2.6 K1 "GEMM + bias (+ReLU/GELU) epilogue": the BERT encoder projections
// (forward and dgrad), the MLM transform / pooler and the Wide&Deep MLP.
//
//   C[m][n] = epilogue( Σ_k A[m][k] · B[n][k] )    A [M][lda], B [N][ldb]: K-contiguous
//
//   forward  y  = act(x·Wᵀ + b) : A = x,  B = W   ([out][in], as stored)
//   dgrad    dx = dy·W          : A = dy, B = Wᵀ  (transposed once per backward)
//
// Epilogue, fused into the tile write-out:
//   v = acc + bias[n]                (fp32, before any rounding)
//   v += E[m][n]                     (residual-gradient join)
//   Z[m][n] = v                      (pre-activation, kept for the backward)
//   v = act(v);  v *= act'(Zin[m][n]) (forward activation / backward of one)
//   C[m][n] = v;  dbias[n] += Σ_m v  (fp32 column sums: one atomic per column per wave tile)
//
// CDNA4 tiling (cdna_hip_programming.md §5): 512 threads = 8 waves, block tile
// 256 x BN (BN = 256: 2x4 waves of 128x64; BN = 128: 4x2 waves of 64x64),
// v_mfma_f32_16x16x32_bf16, K advances 32 per LDS slot.  Operands move
// HBM/L2 -> LDS by LDS-DMA (global_load_lds, 16 B per lane) into a 4-slot
// ring: k-step t+3 is issued while t is multiplied, ONE raw s_barrier per
// k-step, and the counted vmcnt in front of it keeps the two younger k-steps
// in flight (never vmcnt(0) in the main loop — "Pipelining across barriers").
// Slot rows are 64 B; 16-B chunk c of row r is stored at c ^ ((r >> 2) & 2),
// applied on the per-lane SOURCE address (rule 21): with MI355X's ds_read_b128
// lane groups ({0-3,12-15,20-27}, ...) every 16x16x32 operand read is
// conflict-free.  Blocks sharing an XCD take consecutive tiles of one A
// row-panel (T1, bijective remap).  Each wave stages its tile through LDS so
// the write-out is 16 B per lane, 8 rows x 128 B per wave instruction.
#include "common.h"

#include <utility>

namespace {

// Compile-time loop: f(std::integral_constant<int, 0>) ... f(<N-1>) — keeps
// register-array indices constant where `#pragma unroll` is not honoured
// (a runtime index sends the whole accumulator array to scratch, rule 20).
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int GK = 32;     // k per ring slot (one MFMA k-step)
constexpr int NSLOT = 4;   // ring depth: prefetch distance NSLOT - 1
constexpr unsigned kOOB = 0x80000000u;

enum Act { kNone = 0, kGelu = 1, kTanh = 2, kRelu = 3 };

__device__ __forceinline__ float act_fwd(float z, int act) {
  switch (act) {
    case kGelu: return gelu_f(z);
    case kTanh: return tanhf(z);
    case kRelu: return fmaxf(z, 0.f);
    default: return z;
  }
}

__device__ __forceinline__ float act_bwd(float z, int act) {
  switch (act) {
    case kGelu: return gelu_grad(z);
    case kTanh: {
      const float t = tanhf(z);
      return 1.f - t * t;
    }
    case kRelu: return z > 0.f ? 1.f : 0.f;
    default: return 1.f;
  }
}

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;
  const bf16_t* E;     // addend [M][ldc] or null
  const float* bias;   // [N] or null
  bf16_t* Z;           // pre-activation out [M][ldc] or null
  const bf16_t* Zin;   // activation-derivative input [M][ldc] or null
  float* dbias;        // column sums [N] (atomic) or null
  float* dpart;        // with dbias: per-wave-row-block partial column sums [ceil(M / rows)][N] (plain stores)
  int M, N, K, lda, ldb, ldc, act, dact;
  unsigned c_bytes;    // extent of C / E / Z / Zin
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return *reinterpret_cast<uint4*>(&v);
}
// aux: cache policy (2 = non-temporal: streamed past the caches)
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, unsigned off, uint4 v, int aux = 0) {
  using V = decltype(__builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0));
  if (aux == 2) __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<V*>(&v), r, off, 0, 2);
  else __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<V*>(&v), r, off, 0, 0);
}

// 16 B per lane HBM/L2 -> LDS.  A plain device function: the builtin named
// directly inside the templated kernel's lambda stops clang's host pass from
// emitting the kernel's launch stub.
__device__ __forceinline__ void lds_dma16(const bf16_t* src, bf16_t* dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// 16 B per lane buffer -> LDS DMA (buffer_load_dwordx4 ... lds), soff wave-uniform
__device__ __forceinline__ void pp_dma(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else static_assert(N < 0, "vm_wait: add the literal");
}

// k-step t+1 landed for this wave; `ahead` younger k-steps (0..2) may stay in flight
template <int GL>
__device__ __forceinline__ void ring_wait(int ahead) {
  if (ahead >= 2) vm_wait<2 * GL>();
  else if (ahead == 1) vm_wait<GL>();
  else vm_wait<0>();
}

// acc[ni][mi][r] += bias[nw + 16 ni + 4 fq + r] from wave-uniform SCALAR loads
// (constant address space -> s_load) of the wave's 64 bias values: no VGPR-
// destination global load, so hipcc does not drain vmcnt(0) (and with it the
// LDS-DMA pieces in flight) before the bias is used.
template <int TM, int TN>
__device__ __forceinline__ void add_bias_scalar(const GemmArgs& g, floatx4 (&acc)[TN][TM], int nw, int fq) {
  const int nb = __builtin_amdgcn_readfirstlane(nw);
  typedef __attribute__((address_space(4))) const float cfloat;
  cfloat* cbias = reinterpret_cast<cfloat*>(reinterpret_cast<uintptr_t>(g.bias));
#pragma unroll
  for (int ni = 0; ni < TN; ni++) {
    float b4[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      // column nb + 16 ni + 4 q' + r for this lane's q' = fq: select among the 4 uniform quads
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int col = nb + ni * 16 + q * 4 + r;
        v[r] = col < g.N ? cbias[col] : 0.f;
      }
      if (q == 0) { b4[0] = v[0]; b4[1] = v[1]; b4[2] = v[2]; b4[3] = v[3]; }
      else if (fq == q) { b4[0] = v[0]; b4[1] = v[1]; b4[2] = v[2]; b4[3] = v[3]; }
    }
#pragma unroll
    for (int mi = 0; mi < TM; mi++) {
      acc[ni][mi][0] += b4[0];
      acc[ni][mi][1] += b4[1];
      acc[ni][mi][2] += b4[2];
      acc[ni][mi][3] += b4[3];
    }
  }
}

// Write-out of one wave tile (acc[ni][mi][r] = C(m = mw + 16mi + fr, n = nw + 16ni + 4fq + r)):
// bias, addend, pre-activation, activation (forward or backward), dbias column
// sums, staged through the wave's private LDS area `stage` (16TM rows x 32TN
// bytes) so every store is 16 B per lane, 8 rows x 128 B per wave instruction.
// NTST: non-temporal C / Z stores.
template <int TM, int TN, int PTM = TM, bool NTST = false>
__device__ __forceinline__ void tile_epilogue(const GemmArgs& g, floatx4 (&acc)[TN][TM], char* stage, int lane, int mw,
                                              int nw) {
  const int fr = lane & 15, fq = lane >> 4;
  // ROWS: the wave tile's rows; staged PTM m-tiles (16 PTM rows) per pass
  constexpr int ROWS = 16 * TM, RB = 32 * TN, IT = 16 * PTM / 8;  // rows, bytes per staged row, row groups per lane per pass
  static_assert(TM % PTM == 0, "whole passes");
  if (g.bias) {
#pragma unroll
    for (int ni = 0; ni < TN; ni++) {
      const int n = nw + ni * 16 + fq * 4;
      const float4 bb = n < g.N ? *reinterpret_cast<const float4*>(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int mi = 0; mi < TM; mi++) {
        acc[ni][mi][0] += bb.x;
        acc[ni][mi][1] += bb.y;
        acc[ni][mi][2] += bb.z;
        acc[ni][mi][3] += bb.w;
      }
    }
  }
  const int c = lane & 7;
  const int n = nw + c * 8;
  const bool nok = n < g.N;
  const __amdgpu_buffer_rsrc_t rC = rsrc(g.C, g.c_bytes);
  const __amdgpu_buffer_rsrc_t rE = rsrc(g.E ? g.E : g.C, g.E ? g.c_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rZ = rsrc(g.Z ? g.Z : g.C, g.Z ? g.c_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rZi = rsrc(g.Zin ? g.Zin : g.C, g.Zin ? g.c_bytes : 0u);
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  static_for<TM / PTM>([&](auto pc) {
    constexpr int pass = decltype(pc)::value;
    if (pass) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave read back its previous pass
#pragma unroll
    for (int mj = 0; mj < PTM; mj++)
#pragma unroll
      for (int ni = 0; ni < TN; ni++) {
        const int mi = pass * PTM + mj;
        const int row = mj * 16 + fr, col = ni * 16 + fq * 4;
        char* dst = stage + row * RB + (((col >> 3) ^ (row & 7)) << 4) + (col & 7) * 2;
        const uint2 v = make_uint2(pack2(acc[ni][mi][0], acc[ni][mi][1]), pack2(acc[ni][mi][2], acc[ni][mi][3]));
        *reinterpret_cast<uint2*>(dst) = v;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave reads back only its own stage
#pragma unroll 4
  for (int it = 0; it < IT; it++) {
    const int r = it * 8 + (lane >> 3);
    const int m = mw + pass * 16 * PTM + r;
    const unsigned off = (m < g.M && nok) ? ((unsigned)m * (unsigned)g.ldc + (unsigned)n) * 2u : kOOB;
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(stage + r * RB + ((c ^ (r & 7)) << 4)), f);
    if (g.E) {
      float h[8];
      unpack8(bload(rE, off), h);
#pragma unroll
      for (int j = 0; j < 8; j++) f[j] += h[j];
    }
    if (g.Z) bstore(rZ, off, pack8(f), NTST ? 2 : 0);
    if (g.act) {
#pragma unroll
      for (int j = 0; j < 8; j++) f[j] = act_fwd(f[j], g.act);
    }
    if (g.Zin) {
      float z[8];
      unpack8(bload(rZi, off), z);
#pragma unroll
      for (int j = 0; j < 8; j++) f[j] *= act_bwd(z[j], g.dact);
    }
    const uint4 o = pack8(f);
    bstore(rC, off, o, NTST ? 2 : 0);
    if (g.dbias && off != kOOB) {
      float q[8];
      unpack8(o, q);  // the bf16-rounded values the next layer sees
#pragma unroll
      for (int j = 0; j < 8; j++) cs[j] += q[j];
    }
  }
  });
  if (g.dbias) {
#pragma unroll
    for (int o = 8; o < 64; o <<= 1)
#pragma unroll
      for (int j = 0; j < 8; j++) cs[j] += __shfl_xor(cs[j], o, 64);
    if (lane < 8 && nok) {
      if (g.dpart) {  // M / ROWS partials per column, summed by gemm_dbias_reduce: no L2-serialised atomics
        float* pp = g.dpart + (long)(mw / ROWS) * g.N + n;
        *reinterpret_cast<float4*>(pp) = make_float4(cs[0], cs[1], cs[2], cs[3]);
        *reinterpret_cast<float4*>(pp + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++) atomicAdd(g.dbias + n + j, cs[j]);
      }
    }
  }
}

template <int BN, int NS = NSLOT, int NW = 8>
__global__ __launch_bounds__(NW * 64, 8 / NW) void gemm_nt_kernel(GemmArgs g, const bf16_t* __restrict__ zp) {
  constexpr int BM = 256;
  constexpr int WN = BN / 64, WM = NW / WN;          // waves along N / M
  constexpr int TM = BM / WM / 16, TN = 4;           // wave tile: 16*TM rows x 64 columns
  constexpr int A_SLOT = BM * GK, B_SLOT = BN * GK;  // elements per ring slot
  constexpr int GA = BM / (16 * NW), GB = BN / (16 * NW);  // LDS-DMA instructions per wave per k-step (16 rows each)
  constexpr int GL = GA + GB;
  __shared__ __attribute__((aligned(16))) bf16_t smem[NS * (A_SLOT + B_SLOT)];
  bf16_t* As = smem;
  bf16_t* Bs = smem + NS * A_SLOT;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS-DMA bases in SGPRs
  const int wm = wave % WM, wn = wave / WM;
  // T1: blocks that share an XCD (blockIdx % 8) take consecutive tiles (bijective remap)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, x8 = bid & 7;
  const int wg = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (bid >> 3);
  // Grouped raster: consecutive tiles walk GM row-panels column-major, so the
  // ~32 tiles an XCD runs at once form a GM x (32/GM) block whose A and B
  // panels fit its 4 MB L2 together (row-major order would stream all of B
  // past every A panel).
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + BM - 1) / BM;
  constexpr int GM = 4;
  const int grp = wg / (GM * ntn), gm0 = grp * GM, gmn = min(GM, ntm - gm0), rem = wg - grp * GM * ntn;
  const int m0 = (gm0 + rem % gmn) * BM, n0 = (rem / gmn) * BN;

  // LDS-DMA plan: instruction i of wave w fills rows (w*G + i)*16 + lane/4, physical
  // chunk lane&3, from logical chunk (lane&3) ^ swz(row), swz(row) = (row >> 2) & 2
  const int lrow = lane >> 2, lch = (lane & 3) ^ ((lane >> 4) & 2);
  // sources as 32-bit buffer offsets, k-step in the scalar offset; rows past M / N
  // (and chunks past K) get an offset past the buffer: read as 0 by the range check
  const __amdgpu_buffer_rsrc_t rA = rsrc(g.A, (unsigned)(((long)(g.M - 1) * g.lda + g.K) * 2));
  const __amdgpu_buffer_rsrc_t rB = rsrc(g.B, (unsigned)(((long)(g.N - 1) * g.ldb + g.K) * 2));
  int a_vo[GA], b_vo[GB];
#pragma unroll
  for (int i = 0; i < GA; i++) {
    const int m = m0 + (wave * GA + i) * 16 + lrow;
    a_vo[i] = m < g.M ? (m * g.lda + lch * 8) * 2 : (int)kOOB;
  }
#pragma unroll
  for (int i = 0; i < GB; i++) {
    const int n = n0 + (wave * GB + i) * 16 + lrow;
    b_vo[i] = n < g.N ? (n * g.ldb + lch * 8) * 2 : (int)kOOB;
  }
  auto issue = [&](int kt) {
    const int slot = kt % NS, k0 = kt * GK;
    const bool kin = k0 + lch * 8 < g.K;  // K tail (K % 8 == 0): chunks past K read as 0
#pragma unroll
    for (int i = 0; i < GA; i++)
      pp_dma(rA, reinterpret_cast<char*>(As + slot * A_SLOT + (wave * GA + i) * 16 * GK), kin ? a_vo[i] : (int)kOOB,
             k0 * 2);
#pragma unroll
    for (int i = 0; i < GB; i++)
      pp_dma(rB, reinterpret_cast<char*>(Bs + slot * B_SLOT + (wave * GB + i) * 16 * GK), kin ? b_vo[i] : (int)kOOB,
             k0 * 2);
  };

  // this lane's 16-B operand piece of a 16-row tile: row fr, logical chunk fq
  const int fr = lane & 15, fq = lane >> 4;
  const int loff = fr * GK + ((fq ^ ((fr >> 2) & 2)) << 3);
  floatx4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; i++)
#pragma unroll
    for (int j = 0; j < TM; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K + GK - 1) / GK;
  // NS-slot ring: k-step t+NS-1 is issued while t multiplies (slot of t-1:
  // every wave passed the barrier after reading it); the barrier closing t
  // waits for t+1 with min(NS-2, ...) younger k-steps left in flight.
  for (int i = 0; i < NS - 1; i++)
    if (i < nk) issue(i);
  ring_wait<GL>(min(NS - 2, nk - 1));
  asm volatile("s_barrier" ::: "memory");
  for (int t = 0; t < nk; t++) {
    if (t + NS - 1 < nk) issue(t + NS - 1);
    const bf16_t* At = As + (t % NS) * A_SLOT + wm * TM * 16 * GK + loff;
    const bf16_t* Bt = Bs + (t % NS) * B_SLOT + wn * TN * 16 * GK + loff;
    short8 af[TM], bq[TN];
#pragma unroll
    for (int i = 0; i < TN; i++) bq[i] = *reinterpret_cast<const short8*>(Bt + i * 16 * GK);
#pragma unroll
    for (int i = 0; i < TM; i++) af[i] = *reinterpret_cast<const short8*>(At + i * 16 * GK);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ni = 0; ni < TN; ni++)
#pragma unroll
      for (int mi = 0; mi < TM; mi++)
        acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[ni], af[mi], acc[ni][mi], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    ring_wait<GL>((t + NS - 1 < nk ? t + NS - 1 : nk - 1) - (t + 1));
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

  // ---- epilogue: acc[ni][mi][r] = C(m = m0 + wm*16TM + 16mi + fr, n = n0 + wn*64 + 16ni + 4fq + r)
  // ring is idle: every wave passed the last barrier
  tile_epilogue<TM, TN>(g, acc, reinterpret_cast<char*>(smem) + wave * (16 * TM) * (32 * TN), lane, m0 + wm * 16 * TM,
                        n0 + wn * 64);
}

// ---------------------------------------------------------------------------
// Persistent variant: one 512-thread block per CU sweeps a contiguous range of
// tiles (XCD-aware, grouped raster) and the 4-slot LDS-DMA ring runs straight
// across tile boundaries — the next tile's first three k-steps land while the
// current tile's last MFMAs and its epilogue run, so the per-tile ring fill is
// paid once per block, not once per tile (the fixed cost that held the
// per-tile kernel at ~27 % MFMA busy on K = 768, docs/kernels.md).
// The epilogue stages each wave's rows through a PRIVATE 4 KB LDS area (32
// rows x 128 B per pass), so it needs no workgroup barrier and never touches
// the ring.  Its stores are fire-and-forget: the counted vmcnt before each
// k-step's barrier leaves them (and the younger k-steps) in flight —
//   N(s) = GL * (k-steps issued after s+1) + XS * (epilogues issued after s+1)
// with XS = the epilogue's C-store instructions.  Other epilogue VMEM ops
// (addend / pre-activation / derivative loads and stores, dbias atomics) only
// make N an under-count of the younger operations: safe, merely slower.
// Bias values are read with wave-uniform scalar loads (lgkmcnt, not vmcnt).
template <int BN>
__global__ __launch_bounds__(512) void gemm_pt_kernel(GemmArgs g, const bf16_t* __restrict__ zp) {
  constexpr int BM = 256;
  constexpr int WN = BN / 64, WM = 8 / WN;
  constexpr int TM = BM / WM / 16, TN = 4;
  constexpr int A_SLOT = BM * GK, B_SLOT = BN * GK;
  constexpr int GA = BM / 128, GB = BN / 128;
  constexpr int GL = GA + GB;
  constexpr int PASSES = TM / 2;            // 32 staged rows per pass
  constexpr int XS = PASSES * 4;            // C-store instructions per epilogue (4 per pass per lane)
  constexpr int STG = 32 * 128;             // bytes of private staging per wave
  __shared__ __attribute__((aligned(16))) bf16_t smem[NSLOT * (A_SLOT + B_SLOT) + 8 * STG / 2];
  bf16_t* As = smem;
  bf16_t* Bs = smem + NSLOT * A_SLOT;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS-DMA bases in SGPRs
  const int wm = wave % WM, wn = wave / WM;
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + BM - 1) / BM;
  const int ntiles = ntm * ntn;
  // blocks that share an XCD (b % 8) sweep one contiguous range of the tile order
  const int nwg = gridDim.x;
  const int G8 = nwg < 8 ? nwg : 8;
  const int xcd = blockIdx.x % G8, slot = blockIdx.x / G8;
  const int nslot = (nwg - xcd + G8 - 1) / G8;
  const int t_lo = (int)((long)ntiles * xcd / G8), t_hi = (int)((long)ntiles * (xcd + 1) / G8);
  const int my_tiles = t_hi - t_lo > slot ? (t_hi - t_lo - slot + nslot - 1) / nslot : 0;
  constexpr int GM = 4;
  auto tile_mn = [&](int i, int& m0, int& n0) __attribute__((always_inline)) {
    const int wg = t_lo + slot + i * nslot;
    const int grp = wg / (GM * ntn), gm0 = grp * GM, gmn = min(GM, ntm - gm0), rem = wg - grp * GM * ntn;
    m0 = (gm0 + rem % gmn) * BM;
    n0 = (rem / gmn) * BN;
  };

  const int lrow = lane >> 2, lch = (lane & 3) ^ ((lane >> 4) & 2);
  const bf16_t* a_src[GA];
  const bf16_t* b_src[GB];
  int src_tile = -1;
  const int nk = (g.K + GK - 1) / GK;
  const int total = my_tiles * nk;
  auto issue = [&](int s) __attribute__((always_inline)) {
    const int ti = s / nk, kt = s - ti * nk;
    if (ti != src_tile) {
      int m0, n0;
      tile_mn(ti, m0, n0);
#pragma unroll
      for (int i = 0; i < GA; i++) {
        const int m = m0 + (wave * GA + i) * 16 + lrow;
        a_src[i] = m < g.M ? g.A + (long)m * g.lda + lch * 8 : nullptr;
      }
#pragma unroll
      for (int i = 0; i < GB; i++) {
        const int n = n0 + (wave * GB + i) * 16 + lrow;
        b_src[i] = n < g.N ? g.B + (long)n * g.ldb + lch * 8 : nullptr;
      }
      src_tile = ti;
    }
    const int sl = s & (NSLOT - 1), k0 = kt * GK;
    const bool kin = k0 + lch * 8 < g.K;
#pragma unroll
    for (int i = 0; i < GA; i++)
      lds_dma16((a_src[i] && kin) ? a_src[i] + k0 : zp, As + sl * A_SLOT + (wave * GA + i) * 16 * GK);
#pragma unroll
    for (int i = 0; i < GB; i++)
      lds_dma16((b_src[i] && kin) ? b_src[i] + k0 : zp, Bs + sl * B_SLOT + (wave * GB + i) * 16 * GK);
  };

  const int fr = lane & 15, fq = lane >> 4;
  const int loff = fr * GK + ((fq ^ ((fr >> 2) & 2)) << 3);
  floatx4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; i++)
#pragma unroll
    for (int j = 0; j < TM; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  char* stage = reinterpret_cast<char*>(smem + NSLOT * (A_SLOT + B_SLOT)) + wave * STG;
  const int wn_u = __builtin_amdgcn_readfirstlane(wn), wm_u = __builtin_amdgcn_readfirstlane(wm);
  const __amdgpu_buffer_rsrc_t rC = rsrc(g.C, g.c_bytes);
  const __amdgpu_buffer_rsrc_t rE = rsrc(g.E ? g.E : g.C, g.E ? g.c_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rZ = rsrc(g.Z ? g.Z : g.C, g.Z ? g.c_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rZi = rsrc(g.Zin ? g.Zin : g.C, g.Zin ? g.c_bytes : 0u);

  auto epilogue = [&](int ti) __attribute__((always_inline)) {
    int m0, n0;
    tile_mn(ti, m0, n0);
    const int nw = n0 + wn_u * 64;
    if (g.bias) add_bias_scalar<TM, TN>(g, acc, nw, fq);
    const int c = lane & 7;
    const int n = nw + c * 8;
    const bool nok = n < g.N;
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    static_for<PASSES>([&](auto psc) {
      constexpr int ps = decltype(psc)::value;
#pragma unroll
      for (int mj = 0; mj < 2; mj++)
#pragma unroll
        for (int ni = 0; ni < TN; ni++) {
          const int mi = ps * 2 + mj;
          const int row = mj * 16 + fr, col = ni * 16 + fq * 4;
          *reinterpret_cast<uint2*>(stage + row * 128 + (((col >> 3) ^ (row & 7)) << 4) + (col & 7) * 2) =
              make_uint2(pack2(acc[ni][mi][0], acc[ni][mi][1]), pack2(acc[ni][mi][2], acc[ni][mi][3]));
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave reads back only its own stage
      uint4 v[4];
#pragma unroll
      for (int it = 0; it < 4; it++) {
        const int r = it * 8 + (lane >> 3);
        v[it] = *reinterpret_cast<const uint4*>(stage + r * 128 + ((c ^ (r & 7)) << 4));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // next pass overwrites the stage
#pragma unroll
      for (int it = 0; it < 4; it++) {
        const int r = it * 8 + (lane >> 3);
        const int m = m0 + wm_u * (16 * TM) + ps * 32 + r;
        const unsigned off = (m < g.M && nok) ? ((unsigned)m * (unsigned)g.ldc + (unsigned)n) * 2u : kOOB;
        float f[8];
        unpack8(v[it], f);
        if (g.E) {
          float h[8];
          unpack8(bload(rE, off), h);
#pragma unroll
          for (int j = 0; j < 8; j++) f[j] += h[j];
        }
        if (g.Z) bstore(rZ, off, pack8(f));
        if (g.act) {
#pragma unroll
          for (int j = 0; j < 8; j++) f[j] = act_fwd(f[j], g.act);
        }
        if (g.Zin) {
          float z[8];
          unpack8(bload(rZi, off), z);
#pragma unroll
          for (int j = 0; j < 8; j++) f[j] *= act_bwd(z[j], g.dact);
        }
        const uint4 o = pack8(f);
        bstore(rC, off, o);
        if (g.dbias && off != kOOB) {
          float q[8];
          unpack8(o, q);
#pragma unroll
          for (int j = 0; j < 8; j++) cs[j] += q[j];
        }
      }
    });
    if (g.dbias) {
#pragma unroll
      for (int o = 8; o < 64; o <<= 1)
#pragma unroll
        for (int j = 0; j < 8; j++) cs[j] += __shfl_xor(cs[j], o, 64);
      if (lane < 8 && nok)
#pragma unroll
        for (int j = 0; j < 8; j++) atomicAdd(g.dbias + n + j, cs[j]);
    }
#pragma unroll
    for (int i = 0; i < TN; i++)
#pragma unroll
      for (int j = 0; j < TM; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  };

  if (total == 0) return;
  issue(0);
  if (total > 1) issue(1);
  if (total > 2) issue(2);
  ring_wait<GL>(total > 2 ? 2 : total - 1);
  asm volatile("s_barrier" ::: "memory");
  for (int s = 0; s < total; s++) {
    if (s + 3 < total) issue(s + 3);  // slot (s+3)&3 = (s-1)&3: every wave passed the barrier after reading it
    const int kt = s % nk;
    const bf16_t* At = As + (s & (NSLOT - 1)) * A_SLOT + wm * TM * 16 * GK + loff;
    const bf16_t* Bt = Bs + (s & (NSLOT - 1)) * B_SLOT + wn * TN * 16 * GK + loff;
    short8 af[TM], bq[TN];
#pragma unroll
    for (int i = 0; i < TN; i++) bq[i] = *reinterpret_cast<const short8*>(Bt + i * 16 * GK);
#pragma unroll
    for (int i = 0; i < TM; i++) af[i] = *reinterpret_cast<const short8*>(At + i * 16 * GK);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ni = 0; ni < TN; ni++)
#pragma unroll
      for (int mi = 0; mi < TM; mi++)
        acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[ni], af[mi], acc[ni][mi], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (kt == nk - 1) epilogue(s / nk);
    if (s + 1 < total) {
      // ops issued after k-step s+1: younger k-steps, plus the stores of epilogues run at
      // iterations s-2..s (each issued after that iteration's k-step issue)
      const int steps = min(s + 3, total - 1) - (s + 1);
      int eps = 0;
#pragma unroll
      for (int e = 0; e < 3; e++) {
        const int ei = s - e;
        if (ei >= 0 && ei % nk == nk - 1) eps++;
      }
      const int nwait = GL * steps + XS * eps;
      switch (nwait) {
#define KFA_VMW(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
        KFA_VMW(0) KFA_VMW(1) KFA_VMW(2) KFA_VMW(3) KFA_VMW(4) KFA_VMW(5) KFA_VMW(6) KFA_VMW(7)
        KFA_VMW(8) KFA_VMW(9) KFA_VMW(10) KFA_VMW(11) KFA_VMW(12) KFA_VMW(13) KFA_VMW(14) KFA_VMW(15)
        KFA_VMW(16) KFA_VMW(17) KFA_VMW(18) KFA_VMW(19) KFA_VMW(20) KFA_VMW(21) KFA_VMW(22) KFA_VMW(23)
        KFA_VMW(24) KFA_VMW(25) KFA_VMW(26) KFA_VMW(27) KFA_VMW(28) KFA_VMW(29) KFA_VMW(30) KFA_VMW(31)
        KFA_VMW(32) KFA_VMW(33) KFA_VMW(34) KFA_VMW(35) KFA_VMW(36) KFA_VMW(37) KFA_VMW(38) KFA_VMW(39)
        KFA_VMW(40) KFA_VMW(41) KFA_VMW(42) KFA_VMW(43) KFA_VMW(44) KFA_VMW(45) KFA_VMW(46) KFA_VMW(47)
        KFA_VMW(48) KFA_VMW(49) KFA_VMW(50) KFA_VMW(51) KFA_VMW(52) KFA_VMW(53) KFA_VMW(54) KFA_VMW(55)
        KFA_VMW(56) KFA_VMW(57) KFA_VMW(58) KFA_VMW(59) KFA_VMW(60) KFA_VMW(61) KFA_VMW(62)
#undef KFA_VMW
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
}


// ---------------------------------------------------------------------------
// Ping-pong 256x256 kernel (cdna_hip_programming.md §5, "The 256² 8-phase
// template"): 512 threads = two wave GROUPS (waves 0-3 own output rows
// 0-127, waves 4-7 rows 128-255; wave w owns the 128 x 64 tile at
// (w >> 2, w & 3)), one block per CU, BK = 64, two LDS buffers of 64 KB.
// Each k-tile is split into four 16 KB PIECES (128 rows x 64 k), ordered by
// when the waves first need them:
//   piece 0 "A0": A rows {0-63, 128-191}   (each group's first 64 rows)
//   piece 1 "B0": B rows {64c + 0..31}      (each wave's first 32 columns)
//   piece 2 "B1": B rows {64c + 32..63}
//   piece 3 "A1": A rows {64-127, 192-255}
// and the k-tile runs in four PHASES of 16 MFMAs per wave (one 64 x 32
// quadrant of the wave tile, K = 64):
//   s0: read A0 (8 x ds_read_b128) + B0 (4) -> rows 0-63  x cols 0-31
//   s1: read B1 (4)                         -> rows 0-63  x cols 32-63
//   s2: read A1 (8)                         -> rows 64-127 x cols 32-63
//   s3: (registers only)                    -> rows 64-127 x cols 0-31
// Phase = { ds_reads + one piece's LDS-DMA (2 buffer_load ... lds per lane)
// ; counted vmcnt ; s_barrier ; lgkmcnt(0) ; 16 MFMAs ; s_barrier }.  Group 1
// runs ONE barrier behind group 0 (an extra s_barrier before its first phase),
// so on every SIMD (one wave of each group) one wave's MFMAs overlap the other
// wave's LDS reads and DMA issue — the MFMA pipe never waits for the reads.
// Hazards (P = global phase 4u + s; a piece read in phase Q is free for a DMA
// from phase Q + 2; a DMA retired by the vmcnt of phase W is readable from
// phase W + 1):
//   phase 4u+0 issues B1(u+1), 4u+1 A1(u+1), 4u+2 A0(u+2), 4u+3 B0(u+2)
// — the piece of phase P belongs to k-tile (P + 6) >> 2 — and the vmcnt of
// phase P retires the piece of phase P - 4: four pieces (8 DMAs/lane, ~2000
// cycles) stay in flight across the barriers, never vmcnt(0) in steady state.
// Operand rows go through 32-bit buffer offsets (rows past M / N read as 0 by
// the buffer range check); the k-tile advances in the scalar offset.  LDS
// image: 128-B rows, 16-B chunk c of row r stored at c ^ ((r >> 1) & 7) via the
// per-lane SOURCE address (rule 21): conflict-free for the 16x16x32 fragment
// reads (ds_read_b128 lane groups, MI355X_MICROARCH.md §LDS).
constexpr int PP_BK = 64;
constexpr int PP_PIECE = 128 * PP_BK * 2;  // bytes per piece


template <int N>
__device__ __forceinline__ void pp_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
}
// retire every DMA except the pieces issued in the `younger` (0..4) most recent phases
__device__ __forceinline__ void pp_retire(int younger) {
  if (younger >= 4) pp_vmcnt<8>();
  else if (younger == 3) pp_vmcnt<6>();
  else if (younger == 2) pp_vmcnt<4>();
  else if (younger == 1) pp_vmcnt<2>();
  else pp_vmcnt<0>();
}

template <bool PROBE_NO_EPI = false, bool NTST = false>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(GemmArgs g) {
  constexpr int TM = 8, TN = 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * 4 * PP_PIECE];  // 128 KB
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  // T1 XCD remap + grouped raster (as gemm_nt_kernel)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, x8 = bid & 7;
  const int wg = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (bid >> 3);
  const int ntn = (g.N + 255) / 256, ntm = (g.M + 255) / 256;
  constexpr int GM = 4;
  const int grp = wg / (GM * ntn), gm0 = grp * GM, gmn = min(GM, ntm - gm0), rem = wg - grp * GM * ntn;
  const int m0 = (gm0 + rem % gmn) * 256, n0 = (rem / gmn) * 256;

  const __amdgpu_buffer_rsrc_t rA = rsrc(g.A, (unsigned)(((long)(g.M - 1) * g.lda + g.K) * 2));
  const __amdgpu_buffer_rsrc_t rB = rsrc(g.B, (unsigned)(((long)(g.N - 1) * g.ldb + g.K) * 2));
  // DMA plan: instruction j of wave w fills piece rows j*64 + w*8 + lane/8,
  // physical chunk lane&7 <- logical chunk (lane&7) ^ ((row >> 1) & 7)
  const int prow = wave * 8 + (lane >> 3);
  const int lc = (lane & 7) ^ ((prow >> 1) & 7);
  int voff[4][2];
#pragma unroll
  for (int j = 0; j < 2; j++) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int m = m0 + j * 128 + h * 64 + prow;
      voff[h ? 3 : 0][j] = m < g.M ? (m * g.lda + lc * 8) * 2 : (int)kOOB;
      const int n = n0 + (2 * j + (prow >> 5)) * 64 + h * 32 + (prow & 31);
      voff[h ? 2 : 1][j] = n < g.N ? (n * g.ldb + lc * 8) * 2 : (int)kOOB;
    }
  }
  const int nk = g.K / PP_BK;
  const int plast = 4 * nk - 7;  // last phase that issues a piece
  // STEADY (compile-time): the phase is known to issue its piece (k-tile < nk)
  // and to retire with vmcnt(8) — no runtime count in the main loop.
  auto issue = [&](int P, auto pc, auto steady) __attribute__((always_inline)) {
    constexpr int p = decltype(pc)::value;
    const int kt = (P + 6) >> 2;
    if (decltype(steady)::value || kt < nk) {
      char* dst = smem + (kt & 1) * (4 * PP_PIECE) + p * PP_PIECE + wave * 8 * 128;
      const __amdgpu_buffer_rsrc_t r = (p == 0 || p == 3) ? rA : rB;
      pp_dma(r, dst, voff[p][0], kt * PP_BK * 2);
      pp_dma(r, dst + 64 * 128, voff[p][1], kt * PP_BK * 2);
    }
  };
  auto retire = [&](int P, auto steady) __attribute__((always_inline)) {
    if constexpr (decltype(steady)::value) {
      pp_vmcnt<8>();
    } else {
      const int younger = min(P, plast) - (P - 3) + 1;
      pp_retire(younger < 0 ? 0 : younger);
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
  if (wr) asm volatile("s_barrier" ::: "memory");  // group 1 runs one barrier behind

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
    const char* buf = smem + (u & 1) * (4 * PP_PIECE);
    const int P = 4 * u;
    // s0: A0 + B0
    {
      const char* pa = buf + wr * 64 * 128;
      const char* pb = buf + PP_PIECE + wc * 32 * 128;
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
    // s1: B1
    {
      const char* pb = buf + 2 * PP_PIECE + wc * 32 * 128;
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
    // s2: A1
    {
      const char* pa = buf + 3 * PP_PIECE + wr * 64 * 128;
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
    // s3: registers only
    {
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
  if (!wr) asm volatile("s_barrier" ::: "memory");  // both groups at the same barrier count: the ring is idle
  if (PROBE_NO_EPI && g.M >= 0) return;  // timing probe (tools/bench_gemm.py): main loop only
  tile_epilogue<TM, TN, TM, NTST>(g, acc, smem + wave * (16 * TM) * (32 * TN), lane, m0 + wr * 128, n0 + wc * 64);
}


}  // namespace

namespace {
// dbias[n] += Σ_p part[p][n]: blockIdx.y takes every RS-th partial row of 256
// columns (8 independent loads in flight per thread), then one atomic per
// column per row split — RS adds per address instead of P.
constexpr int kDbRS = 16;
__global__ __launch_bounds__(256) void gemm_dbias_reduce(const float* __restrict__ part, float* __restrict__ dbias,
                                                        int P, int N) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int p = blockIdx.y;
  for (; p + 7 * kDbRS < P; p += 8 * kDbRS)
#pragma unroll
    for (int j = 0; j < 8; j++) a[j] += part[(long)(p + j * kDbRS) * N + n];
  for (; p < P; p += kDbRS) a[0] += part[(long)p * N + n];
  atomicAdd(dbias + n, ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7])));
}
}  // namespace

static const bf16_t* gemm_zero_page() {
  static bf16_t* z = nullptr;
  if (!z) {
    if (hipMalloc(&z, 256) != hipSuccess) return nullptr;
    (void)hipMemset(z, 0, 256);
    (void)hipDeviceSynchronize();
  }
  return z;
}

static int gemm_cus() {
  static int c = 0;
  if (!c) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    if (c <= 0) c = 256;
  }
  return c;
}

// Tile width for an M x N output: whole waves of tiles over the CUs, a 256x128
// tile costing ~0.55 of a 256x256 one (lower arithmetic intensity).
KFA_API int kfa_gemm_pick_bn(int M, int N) {
  const long tm = (M + 255) / 256;
  const long cus = gemm_cus();
  const long w256 = (tm * ((N + 255) / 256) + cus - 1) / cus;
  const long w128 = (tm * ((N + 127) / 128) + cus - 1) / cus;
  return (N <= 128 || 0.55 * (double)w128 < (double)w256) ? 128 : 256;
}

// C = epilogue(A · Bᵀ); see the file comment.  bn: 0 = auto, 128 or 256;
// persistent: the tile-sweeping kernel (K >= 64), else one block per tile.
// Rows per dbias partial (one wave's M extent) of the kernel kfa_gemm_nt picks; 0 =
// the kernel keeps per-column atomics (persistent variant).
static int gemm_part_rows(int M, int N, int bn, int persistent) {
  if (bn == 0) bn = kfa_gemm_pick_bn(M, N);
  if (persistent == 1) return 0;
  if (persistent == 3) return 64;             // <128, 3, 8>: 4 x 2 waves of 64 x 64
  if (persistent == 4) return 128;            // <128, 3, 4>: 2 x 2 waves of 128 x 64
  if (persistent == 5 || persistent == 6) return 128;  // ping-pong 256 x 256: 2 x 4 waves of 128 x 64
  return bn == 256 ? 128 : 64;                // <256>: 2 x 4 waves of 128 x 64; <128>: 4 x 2 of 64 x 64
}

// Floats of the dbias partial workspace kfa_gemm_nt needs (0: none).
KFA_API long kfa_gemm_dpart_floats(int M, int N, int bn, int persistent) {
  const int r = gemm_part_rows(M, N, bn, persistent);
  return r ? (long)((M + r - 1) / r) * N : 0;
}

// C = epilogue(A · Bᵀ); see the file comment.  bn: 0 = auto, 128 or 256;
// persistent: 0 = one block per tile, 1 = the tile-sweeping kernel (K >= 64),
// 3 / 4 = 256 x 128 tiles on a 3-slot ring, two blocks per CU (8 / 4 waves).
// dbias with dpart (kfa_gemm_dpart_floats floats): per-wave partial column sums
// + one reduce launch instead of M / rows atomics per column.
KFA_API int kfa_gemm_nt(const bf16_t* A, const bf16_t* B, bf16_t* C, const bf16_t* E, const float* bias, bf16_t* Z,
                        const bf16_t* Zin, float* dbias, float* dpart, int M, int N, int K, int lda, int ldb, int ldc,
                        int act, int dact, int bn, int persistent, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || K % 8 || N % 8 || lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K || ldc < N) return -1;
  if (act < 0 || act > 3 || dact < 0 || dact > 3) return -1;
  if (persistent == 1 && K < 2 * GK) persistent = 0;
  // ping-pong kernel: K in whole 64-deep k-tiles, operand extents within 31-bit buffer offsets
  if ((persistent == 5 || persistent == 6 || persistent == 7) && (K % PP_BK || (long)M * lda * 2 >= (long)kOOB || (long)N * ldb * 2 >= (long)kOOB)) persistent = 4;  // same dbias partial rows (128)
  const long cb = (long)M * ldc * 2;
  if (cb >= (long)kOOB) return -2;  // 32-bit buffer offsets in the epilogue
  if ((long)M * lda * 2 >= (long)kOOB || (long)N * ldb * 2 >= (long)kOOB) return -2;  // ... and the operand DMA
  const int prow = gemm_part_rows(M, N, bn, persistent);
  if (bn == 0) bn = kfa_gemm_pick_bn(M, N);
  if (persistent == 3 || persistent == 4) bn = 128;
  if (persistent == 5 || persistent == 6 || persistent == 7) bn = 256;
  const long tiles = (long)((M + 255) / 256) * ((N + bn - 1) / bn);
  if (tiles >= (1L << 31)) return -2;
  if (!dbias || !prow) dpart = nullptr;
  const GemmArgs g{A, B, C, E, bias, Z, Zin, dbias, dpart, M, N, K, lda, ldb, ldc, act, dact, (unsigned)cb};
  if (persistent == 1) {
    const long cus = gemm_cus();
    const int grid = (int)(tiles < cus ? tiles : cus);
    if (bn == 256)
      hipLaunchKernelGGL((gemm_pt_kernel<256>), dim3(grid), dim3(512), 0, st, g, gemm_zero_page());
    else if (bn == 128)
      hipLaunchKernelGGL((gemm_pt_kernel<128>), dim3(grid), dim3(512), 0, st, g, gemm_zero_page());
    else
      return -1;
  } else if (persistent == 7) {  // probe: ping-pong main loop without the epilogue (C untouched)
    hipLaunchKernelGGL((gemm_pp_kernel<true, false>), dim3((unsigned)tiles), dim3(512), 0, st, g);
  } else if (persistent == 6) {  // ping-pong with non-temporal C / Z stores
    hipLaunchKernelGGL((gemm_pp_kernel<false, true>), dim3((unsigned)tiles), dim3(512), 0, st, g);
  } else if (persistent == 5) {
    hipLaunchKernelGGL((gemm_pp_kernel<false, false>), dim3((unsigned)tiles), dim3(512), 0, st, g);
  } else if (persistent == 4) {
    hipLaunchKernelGGL((gemm_nt_kernel<128, 3, 4>), dim3((unsigned)tiles), dim3(256), 0, st, g, gemm_zero_page());
  } else if (persistent == 3) {
    hipLaunchKernelGGL((gemm_nt_kernel<128, 3>), dim3((unsigned)tiles), dim3(512), 0, st, g, gemm_zero_page());
  } else if (bn == 256) {
    hipLaunchKernelGGL((gemm_nt_kernel<256>), dim3((unsigned)tiles), dim3(512), 0, st, g, gemm_zero_page());
  } else if (bn == 128) {
    hipLaunchKernelGGL((gemm_nt_kernel<128>), dim3((unsigned)tiles), dim3(512), 0, st, g, gemm_zero_page());
  } else {
    return -1;
  }
  if (dpart)
    hipLaunchKernelGGL(gemm_dbias_reduce, dim3((N + 255) / 256, kDbRS), dim3(256), 0, st, dpart, dbias,
                       (M + prow - 1) / prow, N);
  return kfa_status();
}
