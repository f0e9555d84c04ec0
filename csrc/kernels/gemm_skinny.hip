// Skinny-M GEMM with split-K and an in-kernel last-arriver reduction — SURVEY
// §2.6 K1 for the small-batch dense layers (ResNet-50's FC [256 x 2048] x
// [2048 x 1000] forward and data gradient; reference xw_plus_b of
// mnist_replica.py:164-167 at the head of the network):
//
//   C[m][n] = bf16( Σ_k A[m][k] · B[n][k]  (+ bias[n]) )     A [M][lda], B [N][ldb]
//
// (Larger M runs as several 256-row bands, blockIdx.z: the same non-persistent
// 256 x 64 tiles then serve the mid-size GEMMs whose 256 x 256 tiles would leave
// most CUs idle — BERT's MLM transform 5120 x 768 x 768 has 60 of those, 240 of
// these.)
// With one 256-row band there are only ceil(N / 64) output tiles (16 for the
// FC), far too few blocks for 256 CUs, and each tile's reduction (K = 2048) is
// short.  So every tile's K is cut into S slices (S x tiles ~ the CU count):
// block (tile, slice) multiplies its 256 x 64 tile over K / S, publishes the fp32
// partial in register layout (coalesced 16 B per lane) and draws a ticket; the
// slice that draws S - 1 sums the S partials in slice order (bit-identical
// results whatever the arrival order), adds the bias and writes the bf16 tile.
// No block ever waits for another (forward progress under any co-residency).
//
// Block = 4 waves; wave w owns rows 64w .. 64w+63 x the tile's 64 columns
// (4 x 4 MFMA 16x16x32 bf16 blocks, operands swapped so each lane's 4 accumulator
// registers are 4 consecutive COLUMNS of one row: 8-byte stores).  Operands are
// DMA'd into LDS (`buffer_load ... lds`, 16 B per lane, XOR-swizzled on the
// source address), double-buffered, one barrier pair per 64-deep k-step; rows
// past M and k past K read as zero through the buffer range check.
#include "common.h"

namespace {

constexpr int BK = 64;
constexpr int BM = 256, BN = 64;
constexpr unsigned kOOB = 0x80000000u;

struct SkArgs {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;
  const float* bias;  // [N] fp32 or null
  int M, N, K, lda, ldb, ldc, S, kchunk;  // kchunk: k per slice (multiple of BK)
  unsigned a_bytes, b_bytes, c_bytes;
  float* ws;   // [tiles][S][16 floatx4][256 threads]
  int* cnt;    // [tiles] tickets, zero on entry and on exit
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// element offset of (row, 16-B chunk) in a [rows][BK] LDS image, chunk XOR-swizzled
__device__ __forceinline__ int swz(int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3); }

__global__ __launch_bounds__(256, 2) void gemm_skinny_kernel(SkArgs g) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * (BM + BN) * BK];  // 80 KB: two k-steps of A and B
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int slice = blockIdx.y, band = blockIdx.z;
  const int tile = band * gridDim.x + blockIdx.x;  // partial-slot / ticket index
  const int n0 = blockIdx.x * BN, m0 = band * BM;
  const int kb = slice * g.kchunk;
  const int klen = min(g.kchunk, g.K - kb);
  const int nk = klen > 0 ? (klen + BK - 1) / BK : 0;
  const __amdgpu_buffer_rsrc_t rA = rsrc(g.A, g.a_bytes), rB = rsrc(g.B, g.b_bytes);

  // DMA plan: wave-instruction i of wave w fills image rows 8 (4i + w) .. +7 (A: i < 8, B: i < 2);
  // lane -> row (lane >> 3), physical chunk (lane & 7) <- logical chunk (lane & 7) ^ ((row >> 1) & 7)
  const int lr = lane >> 3;
  int a_off[8], b_off[2], a_ck[8], b_ck[2];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int row = 8 * (4 * i + wave) + lr;
    const int ck = (lane & 7) ^ ((row >> 1) & 7);
    a_ck[i] = ck * 8;
    a_off[i] = m0 + row < g.M ? ((m0 + row) * g.lda + kb + ck * 8) * 2 : (int)kOOB;
  }
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const int row = 8 * (4 * i + wave) + lr, n = n0 + row;
    const int ck = (lane & 7) ^ ((row >> 1) & 7);
    b_ck[i] = ck * 8;
    b_off[i] = n < g.N ? (n * g.ldb + kb + ck * 8) * 2 : (int)kOOB;
  }
  auto issue = [&](int t, int buf) __attribute__((always_inline)) {
    const int k = t * BK;  // within the slice
    char* As = reinterpret_cast<char*>(smem + buf * (BM + BN) * BK);
    char* Bs = As + BM * BK * 2;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const bool ok = k + a_ck[i] < klen;  // k tail past the slice (and K) reads zero
      dma16(rA, As + 8 * (4 * i + wave) * BK * 2, ok ? a_off[i] : (int)kOOB, k * 2);
    }
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const bool ok = k + b_ck[i] < klen;
      dma16(rB, Bs + 8 * (4 * i + wave) * BK * 2, ok ? b_off[i] : (int)kOOB, k * 2);
    }
  };

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  if (nk > 0) issue(0, 0);
  for (int t = 0; t < nk; t++) {
    const int buf = t & 1;
    if (t + 1 < nk) {
      issue(t + 1, buf ^ 1);
      asm volatile("s_waitcnt vmcnt(10)\n\ts_barrier" ::: "memory");  // step t landed, t+1 in flight
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const bf16_t* Ab = smem + buf * (BM + BN) * BK;
    const bf16_t* Bb = Ab + BM * BK;
#pragma unroll
    for (int ks = 0; ks < 2; ks++) {
      short8 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; i++) af[i] = *reinterpret_cast<const short8*>(Ab + swz(wave * 64 + i * 16 + fr, ks * 4 + fq));
#pragma unroll
      for (int i = 0; i < 4; i++) bf[i] = *reinterpret_cast<const short8*>(Bb + swz(i * 16 + fr, ks * 4 + fq));
#pragma unroll
      for (int ni = 0; ni < 4; ni++)
#pragma unroll
        for (int mi = 0; mi < 4; mi++)
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ni], af[mi], acc[ni][mi], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // buf free for step t+2's DMA
  }

  // acc[ni][mi][r] = C(m = 64 wave + 16 mi + fr, n = n0 + 16 ni + 4 fq + r)
  if (g.S > 1) {
    floatx4* slots = reinterpret_cast<floatx4*>(g.ws) + (long)tile * g.S * 16 * 256;
    floatx4* dst = slots + (long)slice * 16 * 256 + tid;
#pragma unroll
    for (int ni = 0; ni < 4; ni++)
#pragma unroll
      for (int mi = 0; mi < 4; mi++) dst[(ni * 4 + mi) * 256] = acc[ni][mi];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* last = reinterpret_cast<int*>(smem);  // every DMA has landed: the LDS is free
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int tk = __hip_atomic_fetch_add(g.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int is_last = tk == g.S - 1;
      if (is_last) {
        __hip_atomic_store(g.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *last = is_last;
    }
    __syncthreads();
    if (!*last) return;
    // slot order, 8 slots' loads in flight per step
#pragma unroll
    for (int ni = 0; ni < 4; ni++)
#pragma unroll
      for (int mi = 0; mi < 4; mi++) acc[ni][mi] = __builtin_nontemporal_load(slots + tid + (ni * 4 + mi) * 256);
    for (int s = 1; s < g.S; s++) {
      const floatx4* src = slots + (long)s * 16 * 256 + tid;
#pragma unroll
      for (int ni = 0; ni < 4; ni++)
#pragma unroll
        for (int mi = 0; mi < 4; mi++) acc[ni][mi] += __builtin_nontemporal_load(src + (ni * 4 + mi) * 256);
    }
  }
  const __amdgpu_buffer_rsrc_t rC = rsrc(g.C, g.c_bytes);
#pragma unroll
  for (int ni = 0; ni < 4; ni++) {
    const int n = n0 + ni * 16 + fq * 4;
    const bool nok = n < g.N;  // N % 4 == 0: a lane's 4 columns are all in or all out
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g.bias && nok) b = *reinterpret_cast<const float4*>(g.bias + n);
#pragma unroll
    for (int mi = 0; mi < 4; mi++) {
      const int m = m0 + wave * 64 + mi * 16 + fr;
      const floatx4 v = acc[ni][mi];
      uint2 o = make_uint2(pack2(v[0] + b.x, v[1] + b.y), pack2(v[2] + b.z, v[3] + b.w));
      const unsigned off = (m < g.M && nok) ? ((unsigned)m * (unsigned)g.ldc + (unsigned)n) * 2u : kOOB;
      using V2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(rC, 0, 0, 0));
      __builtin_amdgcn_raw_buffer_store_b64(*reinterpret_cast<V2*>(&o), rC, off, 0, 0);
    }
  }
}

int sk_cus() {
  static int c = 0;
  if (!c) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    if (c <= 0) c = 256;
  }
  return c;
}

// slices per tile: about one block per CU in total, each slice >= 2 k-steps
// (tiles = 256 x 64 output tiles over every 256-row band)
void sk_plan(int M, int N, int K, int want_splits, int& tiles, int& S, int& kchunk) {
  tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int nks = (K + BK - 1) / BK;
  S = want_splits > 0 ? want_splits : sk_cus() / tiles;
  if (S > nks / 2) S = nks / 2;
  if (S < 1) S = 1;
  const int per = (nks + S - 1) / S;
  kchunk = per * BK;
  S = (nks + per - 1) / per;
}

}  // namespace

// workspace bytes of kfa_gemm_skinny (counters, then the partial slots); 0: no split
KFA_API long kfa_gemm_skinny_ws_bytes(int M, int N, int K, int splits) {
  int tiles, S, kc;
  sk_plan(M, N, K, splits, tiles, S, kc);
  if (S <= 1) return 0;
  return 4096 + (long)tiles * S * 16 * 256 * 16;
}

// C = A · Bᵀ (+ bias); K % 8 == 0 (16-B DMA pieces), N % 4 == 0, strides % 8 == 0.
// ws: kfa_gemm_skinny_ws_bytes bytes whose first 4096 are zero (the kernel leaves them zero).
// splits: 0 = pick.  Returns 0, -1 on unsupported operands, -3 on a missing workspace.
KFA_API int kfa_gemm_skinny(const bf16_t* A, const bf16_t* B, bf16_t* C, const float* bias, int M, int N, int K,
                            int lda, int ldb, int ldc, int splits, void* ws, long ws_bytes, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || K % 8 || N % 4 || lda % 8 || ldb % 8 || ldc % 4 || lda < K || ldb < K || ldc < N) return -1;
  const long ab = ((long)(M - 1) * lda + K) * 2, bb = ((long)(N - 1) * ldb + K) * 2, cb = (long)M * ldc * 2;
  if (ab >= (long)kOOB || bb >= (long)kOOB || cb >= (long)kOOB) return -2;
  int tiles, S, kc;
  sk_plan(M, N, K, splits, tiles, S, kc);
  if ((long)tiles * S * 16 * 256 * 16 + 4096 > (1L << 40)) return -1;
  if (S > 1 && (ws == nullptr || ws_bytes < kfa_gemm_skinny_ws_bytes(M, N, K, splits) || tiles > 1024)) return -3;
  const SkArgs g{A, B, C, bias, M, N, K, lda, ldb, ldc, S, kc, (unsigned)ab, (unsigned)bb, (unsigned)cb,
                 S > 1 ? reinterpret_cast<float*>((char*)ws + 4096) : nullptr, S > 1 ? reinterpret_cast<int*>(ws) : nullptr};
  const int bands = (M + BM - 1) / BM;
  hipLaunchKernelGGL(gemm_skinny_kernel, dim3(tiles / bands, S, bands), dim3(256), 0, st, g);
  return kfa_status();
}
