// Weight gradient of NHWC convolution / dense layers on MFMA (bf16 in, fp32
// accumulate) — SURVEY §2.6 K7 (conv wgrad) and K1 (dW = dYᵀ·X).
//
//   dW[co][n] = Σ_k dY[k][co] · X̂[k][n],   n = (r, s, ci),  k = (img, p, q)
//   X̂[k][(r,s,ci)] = X[img][p*st - pad + r][q*st - pad + s][ci]   (0 outside)
//
// The reduction runs over output PIXELS, which are the slow (row) dimension of
// both operands: dY and X are stored channel-contiguous, so a k-slice of either
// operand arrives as [k][channel] rows.  MFMA wants each lane's 8 k-values of
// one row/column, i.e. the transpose — CDNA4's ds_read_b64_tr_b16 (T10) does
// it in the LDS read: tiles are DMA'd (global_load_lds, 16 B/lane) lane-linear
// into [k][128]-element images with the conflict-free XOR swizzle
//   off(row, chunk) = 256*row + 16*(chunk ^ (((row&3)<<2) | ((row>>2)&3)))
// applied on the per-lane SOURCE address, and each MFMA operand is two
// transposed 8-byte reads.
//
// Blocks: 256 threads, 128x128 (2x2 waves), 64x128 (Co <= 64) or 128x64 (N <= 64)
// tiles, BK = 64 pixels,
// double-buffered (<= 64 KiB LDS, 2 blocks/CU).  Split-K over pixels when the
// weight has too few tiles to fill the chip: each block
// writes an fp32 partial tile; a second kernel sums the partials and adds them
// (converted) straight into the flat gradient buffer (bf16 or fp32).
#include <cstdlib>
#include <utility>

#include "common.h"

namespace {

constexpr int BKW = 64;

struct WGeo {
  int H, W, Ci, P, Q, Co, R, S, st, pad;
  int N;        // R*S*Ci
  int K;        // Nb*P*Q  (pixels)
  int kchunk;   // pixels per split (multiple of BKW)
  unsigned x_bytes;  // extent of X (buffer range)
};

__device__ __forceinline__ int fdiv(int x, int d, float rcp) {
  int q = (int)((float)x * rcp);
  const int r = x - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

constexpr unsigned kOOB = 0x80000000u;  // a buffer offset past every extent: the load returns 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wrsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// 16 B per lane buffer -> LDS DMA; a plain device function (the builtin inside the
// templated kernel's lambda stops clang's host pass from emitting launch stubs)
#ifndef KFA_WG_PART_ST_NT
#define KFA_WG_PART_ST_NT 0  // A/B: split-K partial stores non-temporal
#endif
#ifndef KFA_WG_DY_AUX
#define KFA_WG_DY_AUX 0
#endif
#ifndef KFA_WG_X_AUX
#define KFA_WG_X_AUX 0
#endif
template <int AUX = 0>
__device__ __forceinline__ void buf_dma16(__amdgpu_buffer_rsrc_t r, bf16_t* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, AUX);
}

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

// [k][WIDTH] bf16 LDS images (WIDTH = 128 or 64 elements = 256 / 128-B rows),
// 16-B chunks XOR-swizzled so both the lane-linear DMA fill and the
// ds_read_b64_tr_b16 operand reads are conflict-free:
//   256-B rows: chunk ^ (((row&3)<<2) | ((row>>2)&3))           (16 chunks)
//   128-B rows: chunk ^ 2*(((row>>1)&1) | (((row>>3)&1)<<1))     (8 chunks; keeps 32-B pairs)
template <int WIDTH>
__device__ __forceinline__ int img_swz(int row) {
  if constexpr (WIDTH == 128) return ((row & 3) << 2) | ((row >> 2) & 3);
  else return 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
}
template <int WIDTH>
__device__ __forceinline__ int img_off(int row, int col) {  // byte offset of element (row, col)
  return WIDTH * 2 * row + 16 * ((col >> 3) ^ img_swz<WIDTH>(row)) + 2 * (col & 7);
}

// MFMA operand (8 consecutive k of one column) via two transposed reads:
// rows kb + 8g + q and kb + 8g + 4 + q, columns cb + 4p (T10 lane map).
template <int WIDTH>
__device__ __forceinline__ short8 tr_operand(const bf16_t* tile, int kb, int cb, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int col = cb + 4 * p;
  const int r0 = kb + 8 * g + q;
  const char* base = reinterpret_cast<const char*>(tile);
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + img_off<WIDTH>(r0, col)));
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + img_off<WIDTH>(r0 + 4, col)));
  return short8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// The same transposed read as inline asm, for the hand-counted ping-pong kernel:
// hipcc puts an s_waitcnt vmcnt(0) in front of every compiler-visible
// ds_read_b64_tr_b16 that follows an LDS-DMA into the same array (it cannot tell
// the pieces apart), draining the whole DMA pipeline once per phase; the asm form
// is ordered by the kernel's own counted vmcnt + s_barrier + lgkmcnt(0) instead.
// OFF: the read's constant byte offset (piece and k-half), folded into the instruction.
template <int OFF>
__device__ __forceinline__ v4i16 ds_tr16(unsigned addr) {
  v4i16 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}

// tr_operand through ds_tr16: k-half KS's row offset (32 rows; the swizzle repeats
// every 16) as the immediate
template <int WIDTH, int KS>
__device__ __forceinline__ short8 tr_operand_asm(const bf16_t* tile, int cb, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int col = cb + 4 * p, r0 = 8 * g + q;
  const unsigned b = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const bf16_t*)tile;
  const v4i16 a = ds_tr16<KS * 32 * WIDTH * 2>(b + (unsigned)img_off<WIDTH>(r0, col));
  const v4i16 c = ds_tr16<KS * 32 * WIDTH * 2>(b + (unsigned)img_off<WIDTH>(r0 + 4, col));
  return short8{a[0], a[1], a[2], a[3], c[0], c[1], c[2], c[3]};
}

// WM x WN waves, each TM x TN MFMA 16x16 tiles: block tile BM = 16*WM*TM output
// channels x BN = 16*WN*TN (r,s,ci) columns.  OUT_PART: fp32 split-K partials;
// otherwise the epilogue accumulates straight into the (bf16/fp32) gradient.
template <int WM, int WN, int TM, int TN>
__global__ __launch_bounds__(64 * WM * WN, 2) void wgrad_kernel(const bf16_t* __restrict__ dY, const bf16_t* __restrict__ X,
                                                                float* __restrict__ part, void* __restrict__ grad,
                                                                int grad_f32, int accumulate, const bf16_t* __restrict__ Z,
                                                                WGeo g) {
  constexpr int NW = WM * WN;
  constexpr int BM = 16 * WM * TM, BN = 16 * WN * TN;
  // a 256-wide tile is held as two 128-wide sub-images (the swizzles are for 64 / 128)
  constexpr int WA = BM > 128 ? 128 : BM, WB = BN > 128 ? 128 : BN;  // sub-image widths
  constexpr int A_RPI = 1024 / (WA * 2), B_RPI = 1024 / (WB * 2);    // sub-image rows per 1-KiB wave instruction
  constexpr int A_IPS = BKW / A_RPI, B_IPS = BKW / B_RPI;            // instructions per sub-image per k-step
  constexpr int A_IPW = (BM / WA) * A_IPS / NW, B_IPW = (BN / WB) * B_IPS / NW;  // instructions per wave per k-step
  constexpr int A_CPR = WA / 8, B_CPR = WB / 8;                      // 16-B chunks per sub-image row
  static_assert(A_IPW * NW == (BM / WA) * A_IPS && B_IPW * NW == (BN / WB) * B_IPS, "wgrad staging split");
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* As = smem;                    // [2][BM / WA][BKW][WA]
  bf16_t* Bs = smem + 2 * BKW * BM;     // [2][BN / WB][BKW][WB]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS-DMA bases in SGPRs
  const int wm = wave % WM, wn = wave / WM;
  const int ntn = (g.N + BN - 1) / BN;
  // XCD-aware order (T1, bijective remap): the hardware deals block ids round-
  // robin over the 8 XCDs; renumber so the blocks an XCD runs together are the
  // weight tiles of ONE pixel split — they re-read the same dY rows and
  // overlapping X windows (one per tap), which then hit that XCD's L2 instead
  // of HBM (a 3x3 layer's 5-9 tiles otherwise read each split from HBM 5-9x).
  const int nwg = gridDim.x * gridDim.y, bid = blockIdx.x + blockIdx.y * gridDim.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, x8 = bid & 7;
  const int ord = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (bid >> 3);
  const int tile = ord % gridDim.x, split = ord / gridDim.x;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int kb = split * g.kchunk;
  const int ke = min(g.K, kb + g.kchunk);
  if (kb >= ke) return;
  const int nsteps = (ke - kb + BKW - 1) / BKW;

  // staging plan: instruction j fills sub-image j / IPS, rows (j % IPS)*RPI + lane / CPR,
  // physical chunk lane % CPR (logical chunk ^ swizzle applied on the source address)
  int a_m[A_IPW], a_row[A_IPW], a_lds[A_IPW];
  bool a_ok[A_IPW];
#pragma unroll
  for (int i = 0; i < A_IPW; i++) {
    const int j = wave * A_IPW + i, si = j / A_IPS, jj = j % A_IPS;
    const int row = jj * A_RPI + lane / A_CPR;
    const int ch = (lane % A_CPR) ^ img_swz<WA>(row);
    a_row[i] = row;
    a_m[i] = m0 + si * WA + ch * 8;
    a_ok[i] = a_m[i] < g.Co;
    a_lds[i] = si * BKW * WA + jj * A_RPI * WA;
  }
  int b_ci[B_IPW], b_r[B_IPW], b_s[B_IPW], b_row[B_IPW], b_lds[B_IPW];
  bool b_ok[B_IPW];
#pragma unroll
  for (int i = 0; i < B_IPW; i++) {
    const int j = wave * B_IPW + i, si = j / B_IPS, jj = j % B_IPS;
    const int row = jj * B_RPI + lane / B_CPR;
    const int ch = (lane % B_CPR) ^ img_swz<WB>(row);
    const int n = n0 + si * WB + ch * 8;
    b_row[i] = row;
    b_ok[i] = n < g.N;
    b_lds[i] = si * BKW * WB + jj * B_RPI * WB;
    const int tap = b_ok[i] ? n / g.Ci : 0;
    b_ci[i] = n - tap * g.Ci;
    b_r[i] = tap / g.S;
    b_s[i] = tap - b_r[i] * g.S;
  }
  const int PQ = g.P * g.Q;
  const float rPQ = 1.f / (float)PQ, rQ = 1.f / (float)g.Q;
  const bool lin_b = g.R == 1 && g.S == 1 && g.st == 1 && g.pad == 0;  // X row k is pixel k
  const __amdgpu_buffer_rsrc_t rA = wrsrc(dY, (unsigned)g.K * (unsigned)g.Co * 2u);
  const __amdgpu_buffer_rsrc_t rX = wrsrc(X, g.x_bytes);
  int a_vo[A_IPW], b_vo[B_IPW];
#pragma unroll
  for (int i = 0; i < A_IPW; i++) a_vo[i] = a_ok[i] ? (a_row[i] * g.Co + a_m[i]) * 2 : (int)kOOB;
#pragma unroll
  for (int i = 0; i < B_IPW; i++) b_vo[i] = b_ok[i] ? (b_row[i] * g.Ci + b_ci[i]) * 2 : (int)kOOB;
  // gathered X rows: each B instruction's pixel k = kb + step*BKW + b_row advances by
  // BKW per k-step, so its (image, p, q) is carried incrementally (a few adds and
  // compares per step) instead of two divisions per instruction per k-step
  // (not in the 8-wave variant: it is at the VGPR limit, and the three carried
  // digits per instruction turned into scratch spills there: -4 % ResNet-50)
  constexpr bool INC = NW < 8;
  constexpr int NI = INC ? B_IPW : 1;
  int b_img[NI], b_p[NI], b_q[NI];
  const int dq = BKW % g.Q, dp = (BKW / g.Q) % g.P, dimg = BKW / PQ;  // BKW pixels in (img, p, q) digits
#pragma unroll
  for (int i = 0; i < (INC ? B_IPW : 0); i++) {
    const int k = kb + b_row[i];
    const int img = fdiv(k, PQ, rPQ), rem = k - img * PQ;
    b_img[i] = img;
    b_p[i] = fdiv(rem, g.Q, rQ);
    b_q[i] = rem - b_p[i] * g.Q;
  }

  // DMA sources as 32-bit buffer offsets (buffer_load ... lds): dY rows and
  // pointwise X rows are fixed per lane with the k-step in the SCALAR offset
  // (splits are whole k-steps, so only the tensor's end is partial: the range
  // check reads it as 0); gathered X rows compute their offset per step.
  auto issue = [&](int step, int buf) {
    const int k0 = kb + step * BKW;
#pragma unroll
    for (int i = 0; i < A_IPW; i++) buf_dma16<KFA_WG_DY_AUX>(rA, As + buf * BKW * BM + a_lds[i], a_vo[i], k0 * g.Co * 2);
    if (lin_b) {
#pragma unroll
      for (int i = 0; i < B_IPW; i++) buf_dma16<KFA_WG_X_AUX>(rX, Bs + buf * BKW * BN + b_lds[i], b_vo[i], k0 * g.Ci * 2);
      return;
    }
#pragma unroll
    for (int i = 0; i < B_IPW; i++) {
      const int k = k0 + b_row[i];
      int vo = (int)kOOB;
      if (k < ke && b_ok[i]) {
        int img, p, q;
        if constexpr (INC) {
          img = b_img[i];
          p = b_p[i];
          q = b_q[i];
        } else {
          img = fdiv(k, PQ, rPQ);
          const int rem = k - img * PQ;
          p = fdiv(rem, g.Q, rQ);
          q = rem - p * g.Q;
        }
        const int h = p * g.st - g.pad + b_r[i], w = q * g.st - g.pad + b_s[i];
        if ((unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W)
          vo = ((((img * g.H + h) * g.W) + w) * g.Ci + b_ci[i]) * 2;
      }
      buf_dma16<KFA_WG_X_AUX>(rX, Bs + buf * BKW * BN + b_lds[i], vo, 0);
      if constexpr (INC) {  // advance this row's pixel by BKW (issue() runs once per step, in order)
        int q = b_q[i] + dq, p = b_p[i] + dp, img = b_img[i] + dimg;
        if (q >= g.Q) { q -= g.Q; p++; }
        if (p >= g.P) { p -= g.P; img++; }
        b_q[i] = q;
        b_p[i] = p;
        b_img[i] = img;
      }
    }
  };

  floatx4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; a++)
#pragma unroll
    for (int b = 0; b < TM; b++) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  issue(0, 0);
  for (int st = 0; st < nsteps; st++) {
    const int buf = st & 1;
    if (st + 1 < nsteps) {
      issue(st + 1, buf ^ 1);
      if constexpr (A_IPW + B_IPW == 10) asm volatile("s_waitcnt vmcnt(10)\n\ts_barrier" ::: "memory");
      else if constexpr (A_IPW + B_IPW == 8) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
      else if constexpr (A_IPW + B_IPW == 6) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
      else if constexpr (A_IPW + B_IPW == 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const bf16_t* At = As + buf * BKW * BM;
    const bf16_t* Bt = Bs + buf * BKW * BN;
    // Operand reads as inline asm (tr_operand_asm): hipcc waited vmcnt(0) in front of
    // the builtin reads — for the NEXT step's DMAs issued just above — so no step's
    // loads overlapped its own MFMAs.  The waits are explicit: both k-halves' reads,
    // a counted wait for k-half 0's, its MFMAs (k-half 1's reads still landing), a
    // wait, k-half 1's MFMAs; the 8-wave variant (at the VGPR limit) reads, waits and
    // multiplies one k-half at a time.
    constexpr bool PIPE = NW < 8;
    short8 af[2][TM], bf[2][TN];
    auto rd_ks = [&](auto kc) __attribute__((always_inline)) {
      constexpr int ks = decltype(kc)::value;
#pragma unroll
      for (int i = 0; i < TM; i++) {
        const int c = wm * TM * 16 + i * 16;  // within one sub-image (TM * 16 <= 128, aligned)
        af[ks][i] = tr_operand_asm<WA, ks>(At + (c / WA) * BKW * WA, c % WA, lane);
      }
#pragma unroll
      for (int i = 0; i < TN; i++) {
        const int c = wn * TN * 16 + i * 16;
        bf[ks][i] = tr_operand_asm<WB, ks>(Bt + (c / WB) * BKW * WB, c % WB, lane);
      }
    };
    auto mfma_ks = [&](int ks) __attribute__((always_inline)) {
#pragma unroll
      for (int ni = 0; ni < TN; ni++)
#pragma unroll
        for (int mi = 0; mi < TM; mi++)
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ks][ni], af[ks][mi], acc[ni][mi], 0, 0, 0);
    };
    rd_ks(std::integral_constant<int, 0>{});
    if constexpr (PIPE) {
      // both k-halves' reads in flight; k-half 0's retired = at most RH younger ones
      // outstanding (the 4-bit counter caps the count at 15: a read more is waited for)
      constexpr int RH = 2 * (TM + TN) < 15 ? 2 * (TM + TN) : 15;
      rd_ks(std::integral_constant<int, 1>{});
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(RH) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      mfma_ks(0);
      __builtin_amdgcn_sched_barrier(0);
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mfma_ks(0);
      __builtin_amdgcn_sched_barrier(0);
      rd_ks(std::integral_constant<int, 1>{});
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mfma_ks(1);
    __builtin_amdgcn_sched_barrier(0);
    lds_barrier();
  }
  // lane holds D[n = .. + (lane>>4)*4 + i][m = .. + (lane&15)]: 4 consecutive n per store
#pragma unroll
  for (int ni = 0; ni < TN; ni++) {
    const int n = n0 + wn * TN * 16 + ni * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int mi = 0; mi < TM; mi++) {
      const int m = m0 + wm * TM * 16 + mi * 16 + (lane & 15);
      if (m >= g.Co || n >= g.N) continue;
      floatx4 v = acc[ni][mi];
      const long e = (long)m * g.N + n;
      if (part) {
#if KFA_WG_PART_ST_NT
        __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(part + (long)split * g.Co * g.N + e));
#else
        *reinterpret_cast<floatx4*>(part + (long)split * g.Co * g.N + e) = v;
#endif
      } else if (grad_f32) {
        floatx4* gp = reinterpret_cast<floatx4*>(reinterpret_cast<float*>(grad) + e);
        *gp = accumulate ? *gp + v : v;
      } else {
        uint2* gp = reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(grad) + e);
        if (accumulate) {
          const uint2 o = *gp;
          v[0] += bf2f(o.x & 0xffff); v[1] += bf2f(o.x >> 16); v[2] += bf2f(o.y & 0xffff); v[3] += bf2f(o.y >> 16);
        }
        *gp = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Ping-pong 256x256 weight gradient for POINTWISE layers (dense dW = dYᵀ·X, 1x1
// stride-1 convs: X row k is pixel k).  The main loop of wgrad_kernel<2,4,8,4>
// runs its 8 waves in lockstep (every wave reads its fragments, then every wave
// multiplies: the MFMA pipe idles during the reads, ~840 TFLOP/s on the BERT
// wgrads).  Here the schedule is gemm_pp_kernel's (gemm.hip): two wave groups
// one s_barrier apart, so on every SIMD one wave's MFMAs run under the other's
// LDS reads and DMA issue; 64-deep k-tiles in four 16 KB pieces ordered by first
// use; 8 LDS-DMA per lane in flight across the barriers.  What changes is the
// operand layout: both operands arrive k-major ([k][channel] rows), so a piece is
// a [64 k][128 channel] image (256-B rows, the img_swz<128> chunk swizzle applied
// on the source address) and each MFMA operand is two ds_read_b64_tr_b16.
//   piece 0 "A0": dY columns m0 + {0-63, 128-191}    (each wave group's first 64 rows)
//   piece 1 "B0": X columns  n0 + 64c + {0..31}      (each wave's first 32 columns)
//   piece 2 "B1": X columns  n0 + 64c + {32..63}
//   piece 3 "A1": dY columns m0 + {64-127, 192-255}
// One block per (tile, pixel split), as wgrad_kernel; fp32 partials or a direct
// (accumulating) write into the gradient.
constexpr int WP_BK = 64;
constexpr int WP_PIECE = WP_BK * 128 * 2;  // 64 k-rows x 128 channels, bytes

template <int N>
__device__ __forceinline__ void wp_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
}
__device__ __forceinline__ void wp_retire(int younger) {  // all but the pieces of the `younger` newest phases
  if (younger >= 4) wp_vmcnt<8>();
  else if (younger == 3) wp_vmcnt<6>();
  else if (younger == 2) wp_vmcnt<4>();
  else if (younger == 1) wp_vmcnt<2>();
  else wp_vmcnt<0>();
}

// Diagnostic build only (KFA_WP_STAMP=1: three segments per phase, 2: five):
// per-segment s_memtime cycle sums of the k-loop of blocks 0..255, waves 0 and 4
// (one per wave group), read back by kfa_wp_stamps (tools/wgrad_stamps.py).  The
// stamp's lgkmcnt(0) drains LDS reads in flight, so read shares, not run times.
#ifndef KFA_WP_STAMP
#define KFA_WP_STAMP 0
#endif
#if KFA_WP_STAMP
constexpr int kWpSeg = 24;  // [phase 0..3][segment 0..4], prologue, epilogue, k-tiles, spare
__device__ unsigned g_wp_stamps[256 * 2 * kWpSeg];
__device__ __forceinline__ unsigned long long wp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define WP_ST(i)                          \
  do {                                    \
    const unsigned long long t_ = wp_now(); \
    wsum[i] += (unsigned)(t_ - wlast);    \
    wlast = t_;                           \
  } while (0)
#else
#define WP_ST(i) \
  do {           \
  } while (0)
#endif

// GATHER: X is the implicit im2col of an NHWC activation (3x3 / strided / padded
// convs): an X column n is a fixed (r, s, ci) per lane and piece, its row a pixel k
// whose (image, p, q) each lane carries per DMA row across k-tiles (the B0 / B1
// pieces of one k-tile are issued back to back, then the rows advance 64 pixels);
// taps outside the image and pixels past K read 0 through the buffer range check.
template <bool GATHER>
__global__ __launch_bounds__(512, 1) void wgrad_pp_kernel(const bf16_t* __restrict__ dY, const bf16_t* __restrict__ X,
                                                          float* __restrict__ part, void* __restrict__ grad,
                                                          int grad_f32, int accumulate, WGeo g) {
  constexpr int TM = 8, TN = 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * 4 * WP_PIECE];  // 128 KB
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int ntn = (g.N + 255) / 256;
  const int nwg = gridDim.x * gridDim.y, bid = blockIdx.x + blockIdx.y * gridDim.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, x8 = bid & 7;
  const int ord = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (bid >> 3);
  const int tile = ord % gridDim.x, split = ord / gridDim.x;
  const int m0 = (tile / ntn) * 256, n0 = (tile % ntn) * 256;
  const int kb = split * g.kchunk;
  const int ke = min(g.K, kb + g.kchunk);
  if (kb >= ke) return;
  const int nk = (ke - kb + WP_BK - 1) / WP_BK;
#if KFA_WP_STAMP
  unsigned wsum[kWpSeg] = {};
  unsigned long long wlast = wp_now();
#endif

  const __amdgpu_buffer_rsrc_t rA = wrsrc(dY, (unsigned)g.K * (unsigned)g.Co * 2u);
  const __amdgpu_buffer_rsrc_t rB = wrsrc(X, GATHER ? g.x_bytes : (unsigned)g.K * (unsigned)g.Ci * 2u);
  // DMA plan: instruction j (0, 1) of wave w fills piece rows 4 (2w + j) + lane / 16,
  // physical chunk lane & 15 <- logical chunk (lane & 15) ^ img_swz<128>(row)
  int voff[4][2];
  // GATHER (Ci % 64 == 0, host-checked: a 64-channel group never straddles taps, so the
  // B0 / B1 columns of a lane share (r, s) and differ by 32 channels):
  int gx_rs[2], gx_ci[2];            // [j] tap (r - pad) << 16 | (s - pad) & 0xffff, channel of the lane's B0 column
  int gk_img[2], gk_p[2], gk_q[2];   // [j] pixel of the lane's X row in the next k-tile
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const int row = 4 * (2 * wave + j) + (lane >> 4);
    const int c = ((lane & 15) ^ img_swz<128>(row)) * 8;  // piece column of this lane's 8 channels
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int m = m0 + h * 64 + (c < 64 ? c : 128 + c - 64);
      voff[h ? 3 : 0][j] = m < g.Co ? (row * g.Co + m) * 2 : (int)kOOB;
      const int n = n0 + (c >> 5) * 64 + h * 32 + (c & 31);
      voff[h ? 2 : 1][j] = n < g.N ? (row * g.Ci + n) * 2 : (int)kOOB;
      if (GATHER && h == 0) {
        const int tap = n / g.Ci, r = tap / g.S, sx = tap - r * g.S;
        gx_ci[j] = n - tap * g.Ci;
        // past the last tap: r - pad = 0x4000, never in range (H < 2^14 host-checked)
        gx_rs[j] = (int)((unsigned)(n < g.N ? r - g.pad : 0x4000) << 16) | ((sx - g.pad) & 0xffff);
      }
    }
    if constexpr (GATHER) {
      const int PQ = g.P * g.Q;
      const int k = kb + row;
      const int img = fdiv(k, PQ, 1.f / (float)PQ), rem = k - img * PQ;
      gk_img[j] = img;
      gk_p[j] = fdiv(rem, g.Q, 1.f / (float)g.Q);
      gk_q[j] = rem - gk_p[j] * g.Q;
    }
  }
  const int nimg = g.K / (g.P * g.Q);  // pixels past K belong to image nimg and beyond
  const int dq = WP_BK % g.Q, dp = (WP_BK / g.Q) % g.P, dimg = WP_BK / (g.P * g.Q);  // 64 pixels in digits
  const int plast = 4 * nk - 7;  // last phase that issues a piece
  auto issue = [&](int P, auto pc, auto steady) __attribute__((always_inline)) {
    constexpr int p = decltype(pc)::value;
    const int kt = (P + 6) >> 2;
    if (decltype(steady)::value || kt < nk) {
      char* dst = smem + (kt & 1) * (4 * WP_PIECE) + p * WP_PIECE + wave * 2 * 1024;
      constexpr bool isA = p == 0 || p == 3;
      if constexpr (GATHER && !isA) {
        constexpr int h = p == 2;
#pragma unroll
        for (int j = 0; j < 2; j++) {
          const int hh = gk_p[j] * g.st + (gx_rs[j] >> 16), ww = gk_q[j] * g.st + (int)(short)(gx_rs[j] & 0xffff);
          const bool ok = gk_img[j] < nimg && (unsigned)hh < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
          const int vo = ok ? (((gk_img[j] * g.H + hh) * g.W + ww) * g.Ci + gx_ci[j] + h * 32) * 2 : (int)kOOB;
          buf_dma16<0>(rB, reinterpret_cast<bf16_t*>(dst + j * 1024), vo, 0);
          if constexpr (h == 1) {  // B1 closes this k-tile's X rows: advance them 64 pixels
            int q = gk_q[j] + dq, pp = gk_p[j] + dp, img = gk_img[j] + dimg;
            if (q >= g.Q) { q -= g.Q; pp++; }
            if (pp >= g.P) { pp -= g.P; img++; }
            gk_q[j] = q;
            gk_p[j] = pp;
            gk_img[j] = img;
          }
        }
      } else {
        const int soff = (kb + kt * WP_BK) * (isA ? g.Co : g.Ci) * 2;
        buf_dma16<0>(isA ? rA : rB, reinterpret_cast<bf16_t*>(dst), voff[p][0], soff);
        buf_dma16<0>(isA ? rA : rB, reinterpret_cast<bf16_t*>(dst + 1024), voff[p][1], soff);
      }
    }
  };
  auto retire = [&](int P, auto steady) __attribute__((always_inline)) {
    if constexpr (decltype(steady)::value) {
      wp_vmcnt<8>();
    } else {
      const int younger = min(P, plast) - (P - 3) + 1;
      wp_retire(younger < 0 ? 0 : younger);
    }
  };

  floatx4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; i++)
#pragma unroll
    for (int j = 0; j < TM; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // Operand registers: ah = A rows 32-63 of the wave's current 64-row half (MFMA rows
  // mi 2-3), b0 = B0, and two slots sx / sy that alternate, k-tile by k-tile, between
  // A rows 0-31 (mi 0-1) and B1.  The next k-tile's A0 rows 0-31 go into the slot B1
  // vacates after phase 2, in phase 3 (whose reads were empty), so the four phases
  // read 16 / 8 / 16 / 8 operands instead of 24 / 8 / 16 / 0: the 24-read phase ran
  // 600+ cycles against the partner group's ~300 of MFMAs (tools/wgrad_stamps.py).
  // A0 (piece 0) of k-tile u + 1 was DMA'd at phase 4u - 2, five phases before that
  // read (retired by phase 4u + 2's vmcnt, published by its barrier) — the same
  // distance as every other piece.
  // (BAL; the gathered variant keeps the 24 / 8 / 16 / 0 order: with its per-lane pixel
  // state the next image's addresses spill)
  constexpr bool BAL = !GATHER;
  short8 ah[2][2], b0[2][2], sx[2][2], sy[2][2];
  // operand (8 consecutive k of column cb + 4 (lane & 3)) of piece PC, k-half KS of the
  // k-tile image at `buf`: tr_operand<128>'s two reads with the piece / k-half offsets
  // as immediates (a k-half is 32 rows: the swizzle repeats every 16)
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg = lane >> 4;
  auto rd = [&](const char* buf, auto pc, int cb, auto kc) __attribute__((always_inline)) -> short8 {
    constexpr int OFF = decltype(pc)::value * WP_PIECE + decltype(kc)::value * 32 * 256;
    const unsigned b = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)buf;
    const int col = cb + 4 * tp, r0 = 8 * tg + tq;
    const v4i16 x = ds_tr16<OFF>(b + (unsigned)img_off<128>(r0, col));
    const v4i16 y = ds_tr16<OFF>(b + (unsigned)img_off<128>(r0 + 4, col));
    return short8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  // A rows 16 h .. 16 h + 31 of the wave's 64-row half (piece PC) into `dst`; B columns
  // (piece PC) of the wave into `dst`
  auto rd_a = [&](short8 (&dst)[2][2], const char* buf, auto pc, int h) __attribute__((always_inline)) {
#pragma unroll
    for (int mi = 0; mi < 2; mi++) {
      dst[mi][0] = rd(buf, pc, wr * 64 + (h + mi) * 16, I0{});
      dst[mi][1] = rd(buf, pc, wr * 64 + (h + mi) * 16, I1{});
    }
  };
  auto rd_b = [&](short8 (&dst)[2][2], const char* buf, auto pc) __attribute__((always_inline)) {
#pragma unroll
    for (int ni = 0; ni < 2; ni++) {
      dst[ni][0] = rd(buf, pc, wc * 32 + ni * 16, I0{});
      dst[ni][1] = rd(buf, pc, wc * 32 + ni * 16, I1{});
    }
  };

  issue(-6, std::integral_constant<int, 0>{}, std::false_type{});
  issue(-5, std::integral_constant<int, 1>{}, std::false_type{});
  issue(-4, std::integral_constant<int, 2>{}, std::false_type{});
  issue(-3, std::integral_constant<int, 3>{}, std::false_type{});
  issue(-2, std::integral_constant<int, 0>{}, std::false_type{});
  issue(-1, std::integral_constant<int, 1>{}, std::false_type{});
  retire(-1, std::false_type{});
  asm volatile("s_barrier" ::: "memory");
  if (wr) asm volatile("s_barrier" ::: "memory");  // group 1 runs one barrier behind
  if constexpr (BAL) rd_a(sx, smem, I0{}, 0);  // k-tile 0's A0 rows 0-31 (retired and published above)
  WP_ST(20);

  // quadrant (mh, nh) of the wave tile: A rows mi 0-1 from `alo`, 2-3 from ah
  auto mfma_q = [&](short8 (&alo)[2][2], short8 (&bb)[2][2], int mh, int nh) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ks++)
#pragma unroll
      for (int ni = 0; ni < 2; ni++)
#pragma unroll
        for (int mi = 0; mi < 4; mi++)
          acc[nh * 2 + ni][mh * 4 + mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              bb[ni][ks], mi < 2 ? alo[mi][ks] : ah[mi - 2][ks], acc[nh * 2 + ni][mh * 4 + mi], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // k-tile u; sp holds its A0 rows 0-31 on entry, sq is free (and holds the next
  // k-tile's A0 rows 0-31 on exit)
  auto ktile = [&](int u, auto st, short8 (&sp)[2][2], short8 (&sq)[2][2]) __attribute__((always_inline)) {
    const char* buf = smem + (u & 1) * (4 * WP_PIECE);
    const int P = 4 * u;
    {  // s0: A0 rows 32-63 (piece 0) + B0 (piece 1)
      if constexpr (!BAL) rd_a(sp, buf, I0{}, 0);
      rd_a(ah, buf, I0{}, 2);
      rd_b(b0, buf, I1{});
      issue(P, I2{}, st);
      if (KFA_WP_STAMP >= 2) WP_ST(3);
      retire(P, st);
      if (KFA_WP_STAMP >= 2) WP_ST(4);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);  // the MFMAs read the asm reads' registers: keep them behind the wait
      WP_ST(0);
      mfma_q(sp, b0, 0, 0);
      WP_ST(1);
      asm volatile("s_barrier" ::: "memory");
      WP_ST(2);
    }
    {  // s1: B1 (piece 2) into the free slot
      rd_b(sq, buf, I2{});
      issue(P + 1, I3{}, st);
      if (KFA_WP_STAMP >= 2) WP_ST(8);
      retire(P + 1, st);
      if (KFA_WP_STAMP >= 2) WP_ST(9);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      WP_ST(5);
      mfma_q(sp, sq, 0, 1);
      WP_ST(6);
      asm volatile("s_barrier" ::: "memory");
      WP_ST(7);
    }
    {  // s2: A1 (piece 3): rows 0-31 into sp (A0's are done), 32-63 into ah
      rd_a(sp, buf, I3{}, 0);
      rd_a(ah, buf, I3{}, 2);
      issue(P + 2, I0{}, st);
      if (KFA_WP_STAMP >= 2) WP_ST(13);
      retire(P + 2, st);
      if (KFA_WP_STAMP >= 2) WP_ST(14);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      WP_ST(10);
      mfma_q(sp, sq, 1, 1);
      WP_ST(11);
      asm volatile("s_barrier" ::: "memory");
      WP_ST(12);
    }
    {  // s3: the next k-tile's A0 rows 0-31 into sq (B1 is done)
      if constexpr (BAL)
        if (decltype(st)::value || u + 1 < nk) rd_a(sq, smem + ((u + 1) & 1) * (4 * WP_PIECE), I0{}, 0);
      issue(P + 3, I1{}, st);
      if (KFA_WP_STAMP >= 2) WP_ST(18);
      retire(P + 3, st);
      if (KFA_WP_STAMP >= 2) WP_ST(19);
      asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      WP_ST(15);
      mfma_q(sp, b0, 1, 0);
      WP_ST(16);
      asm volatile("s_barrier" ::: "memory");
      WP_ST(17);
    }
  };
  int u = 0;
  if constexpr (BAL) {
    for (; u + 3 < nk; u += 2) {  // steady (u + 2 < nk) pairs: the slots swap roles every k-tile
      ktile(u, std::true_type{}, sx, sy);
      ktile(u + 1, std::true_type{}, sy, sx);
    }
    // the last 1-3 k-tiles (u even here)
    if (u < nk) ktile(u, std::false_type{}, sx, sy);
    if (u + 1 < nk) ktile(u + 1, std::false_type{}, sy, sx);
    if (u + 2 < nk) ktile(u + 2, std::false_type{}, sx, sy);
  } else {
    for (; u + 2 < nk; u++) ktile(u, std::true_type{}, sx, sy);
    for (; u < nk; u++) ktile(u, std::false_type{}, sx, sy);
  }
  if (!wr) asm volatile("s_barrier" ::: "memory");  // both groups at the same barrier count

  // acc[ni][mi] = D[m = m0 + 128 wr + 16 mi + fr][n = n0 + 64 wc + 16 ni + 4 fq + r]
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int ni = 0; ni < TN; ni++) {
    const int n = n0 + wc * 64 + ni * 16 + fq * 4;
#pragma unroll
    for (int mi = 0; mi < TM; mi++) {
      const int m = m0 + wr * 128 + mi * 16 + fr;
      if (m >= g.Co || n >= g.N) continue;
      floatx4 v = acc[ni][mi];
      const long e = (long)m * g.N + n;
      if (part) {
        *reinterpret_cast<floatx4*>(part + (long)split * g.Co * g.N + e) = v;
      } else if (grad_f32) {
        floatx4* gp = reinterpret_cast<floatx4*>(reinterpret_cast<float*>(grad) + e);
        *gp = accumulate ? *gp + v : v;
      } else {
        uint2* gp = reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(grad) + e);
        if (accumulate) {
          const uint2 o = *gp;
          v[0] += bf2f(o.x & 0xffff); v[1] += bf2f(o.x >> 16); v[2] += bf2f(o.y & 0xffff); v[3] += bf2f(o.y >> 16);
        }
        *gp = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
    }
  }
#if KFA_WP_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial tile's stores drained
  WP_ST(21);
  wsum[22] = (unsigned)nk;
  if (lane == 0 && bid < 256 && (wave & 3) == 0) {
#pragma unroll
    for (int i = 0; i < kWpSeg; i++) g_wp_stamps[(bid * 2 + wr) * kWpSeg + i] = wsum[i];
  }
#endif
}

#if KFA_WP_STAMP
KFA_API int kfa_wp_stamps(unsigned* out, int n) {
  if (n > 256 * 2 * kWpSeg) n = 256 * 2 * kWpSeg;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wp_stamps), (size_t)n * sizeof(unsigned), 0, hipMemcpyDeviceToHost);
}
#endif

// grad[i] (+)= sum_s part[s][i].  Block = 64 element-lanes (4 elements each)
// x 4 split-lanes; each thread keeps 8 independent loads in flight (the split
// count reaches hundreds for the early, pixel-heavy layers), then an LDS
// reduce over the split-lanes.
#ifndef KFA_WG_PART_NT
#define KFA_WG_PART_NT 1  // +0.15 % ResNet-50 (docs/kernels.md)
#endif
__device__ __forceinline__ floatx4 ldpart(const float* p) {  // split-K partials: read exactly once
#if KFA_WG_PART_NT
  return __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(p));
#else
  return *reinterpret_cast<const floatx4*>(p);
#endif
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int splits, long total,
                                                           void* __restrict__ grad, int grad_f32, int accumulate) {
  __shared__ floatx4 red[4][64];
  const int el = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const long i = (long)blockIdx.x * 64 + el;  // float4 index
  // the gradient being accumulated into is read up front (lanes that write it), so its
  // round trip overlaps the partial loads instead of following the block reduction
  floatx4 g0 = floatx4{0.f, 0.f, 0.f, 0.f};
  uint2 gb = make_uint2(0u, 0u);
  if (accumulate && sl == 0 && i < total / 4) {
    if (grad_f32) g0 = reinterpret_cast<const floatx4*>(grad)[i];
    else gb = reinterpret_cast<const uint2*>(grad)[i];
  }
  floatx4 s = floatx4{0.f, 0.f, 0.f, 0.f};
  if (i < total / 4) {
    int k = sl;
    for (; k + 28 < splits; k += 32) {
      floatx4 v[8];
#pragma unroll
      for (int u = 0; u < 8; u++) v[u] = ldpart(part + (long)(k + 4 * u) * total + i * 4);
#pragma unroll
      for (int u = 0; u < 8; u++) s += v[u];
    }
    for (; k < splits; k += 4) s += ldpart(part + (long)k * total + i * 4);
  }
  red[sl][el] = s;
  __syncthreads();
  if (sl != 0 || i >= total / 4) return;
  s = red[0][el] + red[1][el] + red[2][el] + red[3][el];
  if (grad_f32) {
    reinterpret_cast<floatx4*>(grad)[i] = accumulate ? g0 + s : s;
  } else {
    if (accumulate) {
      s[0] += bf2f(gb.x & 0xffff); s[1] += bf2f(gb.x >> 16); s[2] += bf2f(gb.y & 0xffff); s[3] += bf2f(gb.y >> 16);
    }
    reinterpret_cast<uint2*>(grad)[i] = make_uint2(pack2(s[0], s[1]), pack2(s[2], s[3]));
  }
}

const bf16_t* zero_page() {
  static bf16_t* z = nullptr;
  if (!z) {
    if (hipMalloc(&z, 256) != hipSuccess) return nullptr;
    (void)hipMemset(z, 0, 256);
    (void)hipDeviceSynchronize();
  }
  return z;
}

int num_cus() {
  static int cached = 0;
  if (!cached) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cached, hipDeviceAttributeMultiprocessorCount, dev);
    if (cached <= 0) cached = 256;
  }
  return cached;
}

// 64x256 tiles for the Co = 64 weights (stem, 256->64 1x1s): KFA_WGRAD_WIDE64=0 keeps 64x128
bool wide64() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("KFA_WGRAD_WIDE64");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

// KFA_WGRAD_WIDE64_ANY=1: 64x256 tiles for every Co <= 64 weight with N >= 512 (the
// 3x3 64-channel convs, N = 576: the last tile is a quarter full) instead of 64x128
// with 64x32 wave tiles, which read 1.5 LDS operands per MFMA
bool wide64_any() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("KFA_WGRAD_WIDE64_ANY");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  return v == 1;
}

// KFA_WGRAD_PP=0: pointwise 256x256 weight gradients on the lockstep wgrad_kernel
// instead of the ping-pong wgrad_pp_kernel
static int wgrad_pp_mode() {  // 0 off, 1 size rule (default), 2 every pointwise weight (experiments)
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("KFA_WGRAD_PP");
    v = e ? atoi(e) : 1;
  }
  return v;
}
bool wgrad_pp_on() { return wgrad_pp_mode() != 0; }

struct WPlan {
  int variant;   // 0: 128x128, 1: 64x128 (Co <= 64), 2: 128x64 (N <= 64), 3: 64x64 (both), 4: 256x256 (8 waves),
                 // 5: 64x256 (Co <= 64, N % 256 == 0: 64x64 wave tiles instead of 64x32)
  int BM, BN, tiles, splits, kchunk, threads, blocks_per_cu;
};

// KFA_WGRAD_PP_GATHER=0: gathered (3x3 / strided) big weights stay on the lockstep
// 8-wave wgrad_kernel instead of wgrad_pp_kernel<true>
static bool wgrad_pp_gather() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("KFA_WGRAD_PP_GATHER");
    v = e ? atoi(e) : 1;
  }
  return v != 0;
}

// pointwise weights the ping-pong kernel takes (edge tiles masked, so any Co / N);
// gathered ones (wgrad_pp_kernel<true>) where the lockstep kernel would take 256x256 tiles
static bool pp_shape(long K, int Co, int N, bool pointwise, int Ci = 0, int H = 0, int W = 0) {
  if (!wgrad_pp_on()) return false;
  if (!pointwise) return wgrad_pp_gather() && Ci % 64 == 0 && Co % 256 == 0 && N % 256 == 0 && K >= 8192 && H < 16384 && W < 16384;
  // per-shape table (tools/bench_wgrad_pp.py, 1x MI355X): wins from 256 x 256 channels up (BERT dW -4..-9 %,
  // ResNet-50 1x1s at 50176 / 200704 pixels -2..-5 %); the 128-channel ResNet shapes lose 10-24 %
  // a short reduction takes the ping-pong kernel too when its 256 x 256 tiles alone fill the
  // chip (no split-K): the BERT MLM decoder, 5120 x 30528 x 768, 320.6 -> 286.8 us
  const long tiles = (long)((Co + 255) / 256) * ((N + 255) / 256);
  return wgrad_pp_mode() == 2 ? (Co >= 128 && N >= 128)
                              : (Co >= 256 && N >= 256 && (K >= 8192 || tiles >= num_cus()));
}

WPlan plan(long K, int Co, int N, bool pointwise = false) {
  WPlan p;
  // 256x256 (8 waves of 128x64, one block per CU): half the operand bytes per
  // MFMA of the 128x128 tile — for the long reductions of big weights
  if ((Co % 256 == 0 && N % 256 == 0 && K >= 8192) || pp_shape(K, Co, N, pointwise)) p.variant = 4;
  else if (Co <= 64 && wide64() && (N % 256 == 0 || (N >= 512 && wide64_any()))) p.variant = 5;
  else p.variant = Co <= 64 ? (N <= 64 ? 3 : 1) : (N <= 64 ? 2 : 0);
  p.BM = p.variant == 4 ? 256 : ((p.variant == 1 || p.variant == 3 || p.variant == 5) ? 64 : 128);
  p.BN = (p.variant == 4 || p.variant == 5) ? 256 : ((p.variant == 2 || p.variant == 3) ? 64 : 128);
  p.threads = p.variant == 4 ? 512 : 256;
  p.blocks_per_cu = p.variant == 4 ? 1 : 2;
  p.tiles = ((Co + p.BM - 1) / p.BM) * ((N + p.BN - 1) / p.BN);
  // one wave of blocks, each >= 4 k-steps; big-weight layers run
  // without split-K and accumulate in the epilogue (no partial round trip)
  const long steps = (K + BKW - 1) / BKW;
  long splits = ((long)p.blocks_per_cu * num_cus()) / p.tiles;
  splits = splits < 1 ? 1 : splits;
  // each split >= min_steps k-steps (KFA_WGRAD_MIN_STEPS, default 4): more steps per
  // split = fewer fp32 partial slabs to write and reduce, at the cost of idle CUs
  static int min_steps = -1;
  if (min_steps < 0) {
    const char* e = getenv("KFA_WGRAD_MIN_STEPS");
    min_steps = e ? atoi(e) : 4;
    if (min_steps < 1) min_steps = 4;
  }
  const long max_splits = steps / min_steps > 0 ? steps / min_steps : 1;
  if (splits > max_splits) splits = max_splits;
  const long per = (steps + splits - 1) / splits;
  p.kchunk = (int)(per * BKW);
  p.splits = (int)((steps + per - 1) / per);
  return p;
}

}  // namespace

KFA_API long kfa_wgrad_part_floats(int Nb, int P, int Q, int Co, int R, int S, int Ci) {
  // (the pointwise test cannot see stride / pad here: the plan may over-size, never under-size)
  const WPlan p0 = plan((long)Nb * P * Q, Co, R * S * Ci), p1 = plan((long)Nb * P * Q, Co, R * S * Ci, R == 1 && S == 1);
  const WPlan& p = p0.splits >= p1.splits ? p0 : p1;
  return p.splits > 1 ? (long)p.splits * Co * R * S * Ci : 0;
}

// dW (+)= conv weight gradient, written into `grad` ([Co][R][S][Ci], bf16 or fp32).
KFA_API int kfa_conv_wgrad(const bf16_t* dY, const bf16_t* X, void* grad, int grad_f32, int accumulate, float* part,
                           int Nb, int H, int W, int Ci, int P, int Q, int Co, int R, int S, int st, int pad,
                           hipStream_t s) {
  if (Ci % 8 || Co % 8) return -1;
  const long K = (long)Nb * P * Q;
  if (K >= (1L << 24)) return -2;  // fp32-reciprocal pixel division is exact below 2^24
  // 32-bit buffer offsets (dY rows, X pixels; the scalar k offset included)
  if (K * Co * 2 >= (long)kOOB || (long)Nb * H * W * Ci * 2 >= (long)kOOB) return -2;
  WGeo g{H, W, Ci, P, Q, Co, R, S, st, pad, R * S * Ci, (int)K, 0, (unsigned)((long)Nb * H * W * Ci * 2)};
  const bool pointwise = R == 1 && S == 1 && st == 1 && pad == 0;
  const WPlan p = plan(K, Co, g.N, pointwise);
  g.kchunk = p.kchunk;
  const size_t lds = (size_t)2 * BKW * (p.BM + p.BN) * sizeof(bf16_t);
  float* pp = p.splits > 1 ? part : nullptr;
  if (p.splits > 1 && !part) return -3;
  dim3 grid(p.tiles, p.splits);
  if (p.variant == 0)
    hipLaunchKernelGGL((wgrad_kernel<2, 2, 4, 4>), grid, dim3(256), lds, s, dY, X, pp, grad, grad_f32, accumulate,
                       zero_page(), g);
  else if (p.variant == 1)
    hipLaunchKernelGGL((wgrad_kernel<1, 4, 4, 2>), grid, dim3(256), lds, s, dY, X, pp, grad, grad_f32, accumulate,
                       zero_page(), g);
  else if (p.variant == 2)
    hipLaunchKernelGGL((wgrad_kernel<4, 1, 2, 4>), grid, dim3(256), lds, s, dY, X, pp, grad, grad_f32, accumulate,
                       zero_page(), g);
  else if (p.variant == 3)
    hipLaunchKernelGGL((wgrad_kernel<2, 2, 2, 2>), grid, dim3(256), lds, s, dY, X, pp, grad, grad_f32, accumulate,
                       zero_page(), g);
  else if (p.variant == 5) {
    static bool attr = false;  // 80 KiB of dynamic LDS (2 blocks / CU)
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_kernel<1, 4, 4, 4>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr = true;
    }
    hipLaunchKernelGGL((wgrad_kernel<1, 4, 4, 4>), grid, dim3(256), lds, s, dY, X, pp, grad, grad_f32, accumulate,
                       zero_page(), g);
  }
  else if (pp_shape(K, Co, g.N, pointwise, Ci, H, W)) {
    // pointwise, long reduction, big weight: ping-pong 256x256 (BERT-base dW: 2304x768 142 -> 129 us,
    // 3072x768 176 -> 168; the ResNet 1x1 shapes measured equal or slower: tools/bench_wgrad_pp.py)
    if (pointwise)
      hipLaunchKernelGGL(wgrad_pp_kernel<false>, grid, dim3(512), 0, s, dY, X, pp, grad, grad_f32, accumulate, g);
    else
      hipLaunchKernelGGL(wgrad_pp_kernel<true>, grid, dim3(512), 0, s, dY, X, pp, grad, grad_f32, accumulate, g);
  }
  else {
    static bool attr = false;  // 128 KiB of dynamic LDS
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_kernel<2, 4, 8, 4>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr = true;
    }
    hipLaunchKernelGGL((wgrad_kernel<2, 4, 8, 4>), grid, dim3(512), lds, s, dY, X, pp, grad, grad_f32, accumulate,
                       zero_page(), g);
  }
  if (p.splits > 1) {
    const long total = (long)Co * g.N;
    const long blocks = (total / 4 + 63) / 64;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, part, p.splits, total, grad,
                       grad_f32, accumulate);
  }
  return kfa_status();
}
