// BatchNorm (+ residual add) (+ ReLU) for NHWC bf16 activations, fp32 params.
// SURVEY §2.6 K8 (ResNet-50: 53 BN layers).  x is viewed as [M = N*H*W, C].
//
// Forward (train):  stats_partial -> finalize -> apply     (3 launches)
//   apply: y = act(x*scale[c] + shift[c] (+ res))
// Backward:         bwd_partial   -> bwd_finalize -> bwd_apply
//   dz  = dy * (y > 0)            (ReLU mask taken from the saved OUTPUT y)
//   dx  = a[c]*dz + b[c]*x + k[c] (BN backward folded into 3 per-channel coefs)
//   dres = dz                      (residual branch gradient, same pass)
//
// Memory-bound: every pass streams rows with 16-B/lane loads; each thread owns
// a fixed group of 8 channels so per-channel coefficients live in registers.
// Row sums use a per-channel pivot (x[0][c]) to avoid E[x^2]-E[x]^2
// cancellation; cross-block partials are combined in fp64.
#include <cstdlib>

#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int kSlots = 64;  // atomic accumulation slots (see combine2)

struct Geom {
  int tpr;     // threads per row (each owns 8 channels per channel-group step)
  int rpi;     // rows per block iteration
  int gx;      // row blocks
  long chunk;  // rows per block (multiple of rpi)
};

Geom geom(long M, int C, int max_blocks) {
  Geom g;
  int cv = C / 8;
  g.tpr = cv < NT ? cv : NT;
  g.rpi = NT / g.tpr;
  long want = (M + (long)g.rpi * 8 - 1) / ((long)g.rpi * 8);
  long gx = want < max_blocks ? want : max_blocks;
  if (gx < 1) gx = 1;
  long chunk = (M + gx - 1) / gx;
  chunk = (chunk + g.rpi - 1) / g.rpi * g.rpi;
  g.chunk = chunk;
  g.gx = (int)((M + chunk - 1) / chunk);
  return g;
}

// Activation-sized inputs are read once per pass: non-temporal loads keep them from
// displacing the tensors the next kernels re-read from L2 / the Infinity Cache
// (ResNet-50 +1.9 %, docs/kernels.md).  Outputs stay write-back (the next conv
// reads them right away: non-temporal stores there measured -1..-2.5 %).
#ifndef KFA_BN_LD_NT
#define KFA_BN_LD_NT 1
#endif
__device__ __forceinline__ uint4 ld16(const bf16_t* p) {
#if KFA_BN_LD_NT
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v[0], v[1], v[2], v[3]);
#else
  return *reinterpret_cast<const uint4*>(p);
#endif
}
#ifndef KFA_BN_NT
#define KFA_BN_NT 0
#endif
// rows per thread whose loads are issued together in the apply passes
#ifndef KFA_BN_ROWS
#define KFA_BN_ROWS 2
#endif
constexpr int kRows = KFA_BN_ROWS;

// Block reduction of the per-thread channel sums (two accumulators x 8 channels per
// thread): each thread writes two 16-B rows per accumulator, [accumulator][channel
// half][thread][4] (lane-contiguous: conflict-free ds_write_b128; the earlier
// [thread][8] rows put 8 lanes on every bank), regions 16 dwords past a multiple of 32
// so the column reads (ds_read_b32: bank = dword mod 32 per 32-lane half) of the two
// halves land on disjoint banks.
constexpr int kRedStride = NT * 4 + 16;
constexpr int kRedFloats = 4 * kRedStride;
__device__ __forceinline__ void red_put(float* sh, int t, const float s1[8], const float s2[8]) {
  *reinterpret_cast<float4*>(sh + 0 * kRedStride + t * 4) = make_float4(s1[0], s1[1], s1[2], s1[3]);
  *reinterpret_cast<float4*>(sh + 1 * kRedStride + t * 4) = make_float4(s1[4], s1[5], s1[6], s1[7]);
  *reinterpret_cast<float4*>(sh + 2 * kRedStride + t * 4) = make_float4(s2[0], s2[1], s2[2], s2[3]);
  *reinterpret_cast<float4*>(sh + 3 * kRedStride + t * 4) = make_float4(s2[4], s2[5], s2[6], s2[7]);
}
// value j (channel j of its 8) of accumulator a written by thread tt
__device__ __forceinline__ float red_get(const float* sh, int a, int tt, int j) {
  return sh[(a * 2 + (j >> 2)) * kRedStride + tt * 4 + (j & 3)];
}
// activation-sized outputs (y, dx, dres)
__device__ __forceinline__ void st16(bf16_t* p, uint4 v) {
#if KFA_BN_NT
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(*reinterpret_cast<u32x4*>(&v), reinterpret_cast<u32x4*>(p));
#else
  *reinterpret_cast<uint4*>(p) = v;
#endif
}

// ------------------------------------------------------------------ forward stats
// block sums -> slot accumulators [kSlots][2][C] (shifted sum, shifted sum of squares)
__global__ __launch_bounds__(NT) void bn_stats_partial(const bf16_t* __restrict__ x, float* __restrict__ part,
                                                        long M, int C, long chunk, int tpr, int rpi) {
  __shared__ __attribute__((aligned(16))) float sh[kRedFloats];
  const int t = threadIdx.x;
  const int cg = t % tpr, r0 = t / tpr;
  const bool active = r0 < rpi;
  const int cv = C / 8;
  const long rb = (long)blockIdx.x * chunk;
  const long re = rb + chunk < M ? rb + chunk : M;
  for (int g0 = 0; g0 < cv; g0 += tpr) {
    const int c0 = (g0 + cg) * 8;
    float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (active && g0 + cg < cv) {
      float K[8];
      unpack8(ld16(x + c0), K);
      long r = rb + r0;
      for (; r + 3L * rpi < re; r += 4L * rpi) {
        uint4 v0 = ld16(x + r * C + c0), v1 = ld16(x + (r + rpi) * C + c0);
        uint4 v2 = ld16(x + (r + 2L * rpi) * C + c0), v3 = ld16(x + (r + 3L * rpi) * C + c0);
        float f[8];
        unpack8(v0, f);
#pragma unroll
        for (int j = 0; j < 8; j++) { float d = f[j] - K[j]; s1[j] += d; s2[j] += d * d; }
        unpack8(v1, f);
#pragma unroll
        for (int j = 0; j < 8; j++) { float d = f[j] - K[j]; s1[j] += d; s2[j] += d * d; }
        unpack8(v2, f);
#pragma unroll
        for (int j = 0; j < 8; j++) { float d = f[j] - K[j]; s1[j] += d; s2[j] += d * d; }
        unpack8(v3, f);
#pragma unroll
        for (int j = 0; j < 8; j++) { float d = f[j] - K[j]; s1[j] += d; s2[j] += d * d; }
      }
      for (; r < re; r += rpi) {
        float f[8];
        unpack8(ld16(x + r * C + c0), f);
#pragma unroll
        for (int j = 0; j < 8; j++) { float d = f[j] - K[j]; s1[j] += d; s2[j] += d * d; }
      }
    }
    if (active) {
      red_put(sh, r0 * tpr + cg, s1, s2);
    }
    __syncthreads();
    const int width = tpr * 8;
    for (int idx = t; idx < 2 * width; idx += NT) {
      const int a = idx / width, c = idx % width;
      if (g0 * 8 + c < C) {
        float acc = 0.f;
        for (int rr = 0; rr < rpi; rr++) acc += red_get(sh, a, rr * tpr + (c >> 3), c & 7);
        __hip_atomic_fetch_add(&part[((long)(blockIdx.x % kSlots) * 2 + a) * C + g0 * 8 + c], acc,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
  }
}

// Cross-block combine: partial kernels atomically add their block sums into
// kSlots slot rows ([kSlots][2][C], slot = block % kSlots, so each address
// sees gx/kSlots adds); finalize sums the slots in fp64 and ZEROES them again,
// leaving the workspace clean for the next BN layer on the stream.
// Finalize blocks are 64 channels x kGroups slot groups (1024 threads): each
// thread read-and-zeroes kSlots / kGroups slot pairs, all in flight at once,
// and the groups are summed through LDS in a fixed order (deterministic).  One
// 64-thread block per 64 channels walking all 64 slots serially was latency
// bound (128 dependent-batch device-scope atomics: ~6.6 us per finalize).
constexpr int kGroups = 16;
static_assert(kSlots % kGroups == 0, "slot groups");

__device__ __forceinline__ bool combine2(float* __restrict__ part, int C, int c, double& a, double& b) {
  __shared__ double ra[kGroups][64], rb[kGroups][64];
  const int lx = threadIdx.x, ly = threadIdx.y;
  float va[kSlots / kGroups], vb[kSlots / kGroups];
#pragma unroll
  for (int i = 0; i < kSlots / kGroups; i++) {
    va[i] = vb[i] = 0.f;
    if (c < C) {
      float* pa = part + ((long)(ly + kGroups * i) * 2) * C + c;
      // read-and-zero at the coherence point: the adds came from other XCDs'
      // workgroups, so plain loads could hit a stale line of THIS XCD's L2
      va[i] = __hip_atomic_exchange(pa, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      vb[i] = __hip_atomic_exchange(pa + C, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  double sa = 0.0, sb = 0.0;
#pragma unroll
  for (int i = 0; i < kSlots / kGroups; i++) {
    sa += (double)va[i];
    sb += (double)vb[i];
  }
  ra[ly][lx] = sa;
  rb[ly][lx] = sb;
  __syncthreads();
  if (ly != 0 || c >= C) return false;
  a = 0.0;
  b = 0.0;
#pragma unroll
  for (int j = 0; j < kGroups; j++) {
    a += ra[j][lx];
    b += rb[j][lx];
  }
  return true;
}

__global__ __launch_bounds__(64 * kGroups) void bn_finalize(const bf16_t* __restrict__ x, float* __restrict__ part, int gx, long M, int C,
                            const float* __restrict__ gamma, const float* __restrict__ beta,
                            float* __restrict__ rmean, float* __restrict__ rvar, float* __restrict__ save_mean,
                            float* __restrict__ save_invstd, float* __restrict__ scale, float* __restrict__ shift,
                            float eps, float momentum) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  // the per-channel operands are loaded BEFORE the slot exchanges, so their latency
  // overlaps the atomics' round trip instead of following it
  const bool own = threadIdx.y == 0 && c < C;
  float g = 1.f, bt = 0.f, rm0 = 0.f, rv0 = 0.f, kx = 0.f;
  if (own) {
    if (gamma) g = gamma[c];
    if (beta) bt = beta[c];
    if (rmean) { rm0 = rmean[c]; rv0 = rvar[c]; }
    if (x) kx = bf2f(x[c]);
  }
  double a, b;
  if (!combine2(part, C, c, a, b)) return;
  const double K = x ? (double)kx : 0.0;  // x == nullptr: un-shifted sums (fused in the conv epilogue)
  const double m1 = a / (double)M;
  double var = b / (double)M - m1 * m1;
  if (var < 0.0) var = 0.0;
  const double mean = K + m1;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  save_mean[c] = (float)mean;
  save_invstd[c] = invstd;
  scale[c] = g * invstd;
  shift[c] = bt - (float)mean * g * invstd;
  if (rmean) {
    const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
    rmean[c] = (1.f - momentum) * rm0 + momentum * (float)mean;
    rvar[c] = (1.f - momentum) * rv0 + momentum * (float)unbiased;
  }
}

__global__ void bn_finalize_eval(const float* __restrict__ gamma, const float* __restrict__ beta,
                                 const float* __restrict__ rmean, const float* __restrict__ rvar, int C, float eps,
                                 float* __restrict__ scale, float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = rsqrtf(rvar[c] + eps);
  const float g = gamma ? gamma[c] : 1.f;
  scale[c] = g * inv;
  shift[c] = (beta ? beta[c] : 0.f) - rmean[c] * g * inv;
}

// ------------------------------------------------------------------ forward apply
// ReLU bit mask of the output (MB): bit j of byte (row*C + c0)/8 is y[c0+j] > 0
// (the bf16 value the backward would have read) — for BN+residual+ReLU, whose
// mask cannot be recomputed from x alone; the backward then reads 1/8 B instead
// of the 2-B output per element.
__device__ __forceinline__ unsigned pos_bits(const uint4 v) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
  unsigned m = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const unsigned lo = w[i] & 0xffffu, hi = w[i] >> 16;
    m |= (lo != 0u && !(lo & 0x8000u)) ? (1u << (2 * i)) : 0u;
    m |= (hi != 0u && !(hi & 0x8000u)) ? (1u << (2 * i + 1)) : 0u;
  }
  return m;
}

// RAFF: the residual is itself a BatchNorm's RAW input r, normalised here with
// that BN's [scale | shift] (rss, 2C floats): z = x*sc + sh + (r*rsc + rsh) —
// a ResNet downsample block's two BNs in one pass (the downsample BN's output
// is never written or re-read).
template <bool RELU, bool RES, bool MB, bool RAFF = false>
__global__ __launch_bounds__(NT) void bn_apply(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                               bf16_t* __restrict__ y, uint8_t* __restrict__ mb,
                                               const float* __restrict__ scale, const float* __restrict__ shift,
                                               long M, int C, long chunk, int tpr, int rpi,
                                               const float* __restrict__ rss = nullptr) {
  const int t = threadIdx.x;
  const int cg = t % tpr, r0 = t / tpr;
  if (r0 >= rpi) return;
  const int cv = C / 8;
  const long rb = (long)blockIdx.x * chunk;
  const long re = rb + chunk < M ? rb + chunk : M;
  for (int g = cg; g < cv; g += tpr) {
    const int c0 = g * 8;
    float sc[8], sf[8], rsc[8], rsf[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      sc[j] = scale[c0 + j];
      sf[j] = shift[c0 + j];
      rsc[j] = RAFF ? rss[c0 + j] : 1.f;
      rsf[j] = RAFF ? rss[C + c0 + j] : 0.f;
    }
    auto one = [&](const uint4 v, const uint4 q4, long o) {
      float f[8], q[8];
      unpack8(v, f);
      if (RES) unpack8(q4, q);
#pragma unroll
      for (int j = 0; j < 8; j++) {
        float z = fmaf(f[j], sc[j], sf[j]);
        if (RES) z += RAFF ? fmaf(q[j], rsc[j], rsf[j]) : q[j];
        f[j] = RELU ? fmaxf(z, 0.f) : z;
      }
      const uint4 out = pack8(f);
      st16(y + o, out);
      if (MB) mb[o >> 3] = (uint8_t)pos_bits(out);
    };
    long r = rb + r0;
    for (; r + (kRows - 1L) * rpi < re; r += (long)kRows * rpi) {  // kRows rows' loads in flight
      uint4 v[kRows], q[kRows];
#pragma unroll
      for (int i = 0; i < kRows; i++) {
        const long o = (r + (long)i * rpi) * C + c0;
        v[i] = ld16(x + o);
        q[i] = RES ? ld16(res + o) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < kRows; i++) one(v[i], q[i], (r + (long)i * rpi) * C + c0);
    }
    for (; r < re; r += rpi) {
      const long o = r * C + c0;
      one(ld16(x + o), RES ? ld16(res + o) : make_uint4(0, 0, 0, 0), o);
    }
  }
}

// The apply passes keep no per-block partials, so their grid need not follow the
// statistics passes' (max_row_blocks caps C >= 1024 at 512-1024 blocks: 2-4 per
// CU, too few loads in flight to stream at HBM rate).  KFA_BN_APPLY_BLOCKS=0
// restores the shared geometry.  Cap 16384 (round 5; was 4096): ResNet-50 13,107-13,130
// vs 13,020-13,028 img/s on one box (tools/gpu_r5_bnblocks.sh), flat from 16384 up.
static Geom apply_geom(long M, int C) {
  static int cap = -1;
  if (cap < 0) {
    const char* e = getenv("KFA_BN_APPLY_BLOCKS");
    cap = e ? atoi(e) : 16384;
    if (cap < 0) cap = 16384;
  }
  int shared = (1 << 20) / C;  // == max_row_blocks(C)
  shared = shared > 2048 ? 2048 : (shared < 64 ? 64 : shared);
  return geom(M, C, cap > 0 ? cap : shared);
}

static void launch_apply(int relu, const bf16_t* res, uint8_t* mb, dim3 grid, hipStream_t s, const bf16_t* x,
                         bf16_t* y, const float* scale, const float* shift, long M, int C, long chunk, int tpr,
                         int rpi, const float* rss = nullptr) {
  {
    const Geom ga = apply_geom(M, C);
    grid = dim3(ga.gx);
    chunk = ga.chunk;
    tpr = ga.tpr;
    rpi = ga.rpi;
  }
  if (rss && relu && res && mb)
    hipLaunchKernelGGL((bn_apply<true, true, true, true>), grid, dim3(NT), 0, s, x, res, y, mb, scale, shift, M, C,
                       chunk, tpr, rpi, rss);
  else if (rss && relu && res)
    hipLaunchKernelGGL((bn_apply<true, true, false, true>), grid, dim3(NT), 0, s, x, res, y, mb, scale, shift, M, C,
                       chunk, tpr, rpi, rss);
  else if (rss && res)
    hipLaunchKernelGGL((bn_apply<false, true, false, true>), grid, dim3(NT), 0, s, x, res, y, mb, scale, shift, M, C,
                       chunk, tpr, rpi, rss);
  else if (relu && res && mb)
    hipLaunchKernelGGL((bn_apply<true, true, true>), grid, dim3(NT), 0, s, x, res, y, mb, scale, shift, M, C, chunk,
                       tpr, rpi);
  else if (relu && res)
    hipLaunchKernelGGL((bn_apply<true, true, false>), grid, dim3(NT), 0, s, x, res, y, mb, scale, shift, M, C, chunk,
                       tpr, rpi);
  else if (relu)
    hipLaunchKernelGGL((bn_apply<true, false, false>), grid, dim3(NT), 0, s, x, res, y, mb, scale, shift, M, C, chunk,
                       tpr, rpi);
  else if (res)
    hipLaunchKernelGGL((bn_apply<false, true, false>), grid, dim3(NT), 0, s, x, res, y, mb, scale, shift, M, C, chunk,
                       tpr, rpi);
  else
    hipLaunchKernelGGL((bn_apply<false, false, false>), grid, dim3(NT), 0, s, x, res, y, mb, scale, shift, M, C,
                       chunk, tpr, rpi);
}

// ------------------------------------------------------------------ backward
// ReLU mask of the backward.  MASK 0: none; 1: from the forward output y
// (y > 0); 2: recomputed from the forward input x and the layer's saved
// scale / shift (relu(fma(x, sc, sh)) > 0 exactly as bn_apply evaluated it), so
// the bn1 / bn2 backward of a bottleneck never reads y — 2 of its 8 bytes per
// element (ResNet: 33 BN backward passes per step).
// MASK 3: from the forward's output bit mask (BN + residual + ReLU, see bn_apply).
template <int MASK>
__device__ __forceinline__ void masked_dy(const uint4 dv, const uint4 yv, const float xf[8], const float sc[8],
                                          const float sf[8], unsigned bits, float dz[8]) {
  unpack8(dv, dz);
  if (MASK == 3) {
#pragma unroll
    for (int j = 0; j < 8; j++) dz[j] = ((bits >> j) & 1u) ? dz[j] : 0.f;
  } else if (MASK == 1) {
    float yy[8];
    unpack8(yv, yy);
#pragma unroll
    for (int j = 0; j < 8; j++) dz[j] = yy[j] > 0.f ? dz[j] : 0.f;
  } else if (MASK == 2) {
#pragma unroll
    for (int j = 0; j < 8; j++) dz[j] = fmaf(xf[j], sc[j], sf[j]) > 0.f ? dz[j] : 0.f;
  }
}

template <int MASK>
__device__ __forceinline__ void load_ss(const float* __restrict__ ss, int C, int c0, float sc[8], float sf[8]) {
#pragma unroll
  for (int j = 0; j < 8; j++) {
    sc[j] = MASK == 2 ? ss[c0 + j] : 0.f;
    sf[j] = MASK == 2 ? ss[C + c0 + j] : 0.f;
  }
}

// block sums -> slot accumulators [kSlots][2][C]: sum(dz), sum(dz*(x-mean))
template <int MASK>
__global__ __launch_bounds__(NT) void bn_bwd_partial(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                     const bf16_t* __restrict__ y, const uint8_t* __restrict__ mb,
                                                     const float* __restrict__ ss,
                                                     const float* __restrict__ mean, float* __restrict__ part, long M,
                                                     int C, long chunk, int tpr, int rpi) {
  __shared__ __attribute__((aligned(16))) float sh[kRedFloats];
  const int t = threadIdx.x;
  const int cg = t % tpr, r0 = t / tpr;
  const bool active = r0 < rpi;
  const int cv = C / 8;
  const long rb = (long)blockIdx.x * chunk;
  const long re = rb + chunk < M ? rb + chunk : M;
  for (int g0 = 0; g0 < cv; g0 += tpr) {
    const int c0 = (g0 + cg) * 8;
    float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (active && g0 + cg < cv) {
      float mu[8], sc[8], sf[8];
#pragma unroll
      for (int j = 0; j < 8; j++) mu[j] = mean[c0 + j];
      load_ss<MASK>(ss, C, c0, sc, sf);
      long r = rb + r0;
      for (; r + rpi < re; r += 2L * rpi) {
        const long o0 = r * C + c0, o1 = (r + rpi) * C + c0;
        uint4 d0 = ld16(dy + o0), d1 = ld16(dy + o1);
        uint4 x0 = ld16(x + o0), x1 = ld16(x + o1);
        uint4 y0 = make_uint4(0, 0, 0, 0), y1 = y0;
        if (MASK == 1) { y0 = ld16(y + o0); y1 = ld16(y + o1); }
        unsigned b0 = 0, b1 = 0;
        if (MASK == 3) { b0 = mb[o0 >> 3]; b1 = mb[o1 >> 3]; }
        float dz[8], xf[8];
        unpack8(x0, xf);
        masked_dy<MASK>(d0, y0, xf, sc, sf, b0, dz);
#pragma unroll
        for (int j = 0; j < 8; j++) { s1[j] += dz[j]; s2[j] += dz[j] * (xf[j] - mu[j]); }
        unpack8(x1, xf);
        masked_dy<MASK>(d1, y1, xf, sc, sf, b1, dz);
#pragma unroll
        for (int j = 0; j < 8; j++) { s1[j] += dz[j]; s2[j] += dz[j] * (xf[j] - mu[j]); }
      }
      for (; r < re; r += rpi) {
        const long o = r * C + c0;
        uint4 yv = make_uint4(0, 0, 0, 0);
        if (MASK == 1) yv = ld16(y + o);
        const unsigned bits = MASK == 3 ? (unsigned)mb[o >> 3] : 0u;
        float dz[8], xf[8];
        unpack8(ld16(x + o), xf);
        masked_dy<MASK>(ld16(dy + o), yv, xf, sc, sf, bits, dz);
#pragma unroll
        for (int j = 0; j < 8; j++) { s1[j] += dz[j]; s2[j] += dz[j] * (xf[j] - mu[j]); }
      }
    }
    if (active) {
      red_put(sh, r0 * tpr + cg, s1, s2);
    }
    __syncthreads();
    const int width = tpr * 8;
    for (int idx = t; idx < 2 * width; idx += NT) {
      const int a = idx / width, c = idx % width;
      if (g0 * 8 + c < C) {
        float acc = 0.f;
        for (int rr = 0; rr < rpi; rr++) acc += red_get(sh, a, rr * tpr + (c >> 3), c & 7);
        __hip_atomic_fetch_add(&part[((long)(blockIdx.x % kSlots) * 2 + a) * C + g0 * 8 + c], acc,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
  }
}

// coef layout: [3][C] = a, b, k   ;  dx = a*dz + b*x + k
__global__ __launch_bounds__(64 * kGroups) void bn_bwd_finalize(float* __restrict__ part, int gx, long M, int C, const float* __restrict__ gamma,
                                const float* __restrict__ mean, const float* __restrict__ invstd,
                                float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ coef,
                                int accumulate) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  const bool own = threadIdx.y == 0 && c < C;  // operands ahead of the slot exchanges (see bn_finalize)
  float inv = 0.f, g = 1.f, mu = 0.f, dg0 = 0.f, db0 = 0.f;
  if (own) {
    inv = invstd[c];
    if (gamma) g = gamma[c];
    mu = mean[c];
    if (accumulate && dgamma) dg0 = dgamma[c];
    if (accumulate && dbeta) db0 = dbeta[c];
  }
  double sdy, sdx;
  if (!combine2(part, C, c, sdy, sdx)) return;
  const float dg = (float)sdx * inv;  // sum(dz * xhat)
  // accumulate: the outputs are views into the flat gradient bucket (+=)
  if (dgamma) dgamma[c] = accumulate ? dg0 + dg : dg;
  if (dbeta) dbeta[c] = accumulate ? db0 + (float)sdy : (float)sdy;
  const float a = g * inv;
  const float b = -g * inv * inv * inv * (float)(sdx / (double)M);
  const float k = -a * (float)(sdy / (double)M) - b * mu;
  coef[c] = a;
  coef[C + c] = b;
  coef[2 * C + c] = k;
}

template <int MASK, bool DRES>
__global__ __launch_bounds__(NT) void bn_bwd_apply(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                   const bf16_t* __restrict__ y, const uint8_t* __restrict__ mb,
                                                   const float* __restrict__ ss,
                                                   const float* __restrict__ coef, bf16_t* __restrict__ dx,
                                                   bf16_t* __restrict__ dres, long M, int C, long chunk, int tpr,
                                                   int rpi) {
  const int t = threadIdx.x;
  const int cg = t % tpr, r0 = t / tpr;
  if (r0 >= rpi) return;
  const int cv = C / 8;
  const long rb = (long)blockIdx.x * chunk;
  const long re = rb + chunk < M ? rb + chunk : M;
  for (int g = cg; g < cv; g += tpr) {
    const int c0 = g * 8;
    float ca[8], cb[8], ck[8], sc[8], sf[8];
#pragma unroll
    for (int j = 0; j < 8; j++) { ca[j] = coef[c0 + j]; cb[j] = coef[C + c0 + j]; ck[j] = coef[2 * C + c0 + j]; }
    load_ss<MASK>(ss, C, c0, sc, sf);
    auto one = [&](long o, const uint4 dv, const uint4 xv, const uint4 yv, unsigned bits) {
      float dz[8], xf[8], out[8];
      unpack8(xv, xf);
      masked_dy<MASK>(dv, yv, xf, sc, sf, bits, dz);
#pragma unroll
      for (int j = 0; j < 8; j++) out[j] = fmaf(ca[j], dz[j], fmaf(cb[j], xf[j], ck[j]));
      st16(dx + o, pack8(out));
      if (DRES) st16(dres + o, pack8(dz));
    };
    // kRows rows per iteration with every load issued before any row is computed, as
    // bn_apply: kRows times the bytes in flight per thread
    long r = rb + r0;
    for (; r + (kRows - 1L) * rpi < re; r += (long)kRows * rpi) {
      uint4 yv[kRows], dv[kRows], xv[kRows];
      unsigned bits[kRows];
#pragma unroll
      for (int i = 0; i < kRows; i++) {
        const long o = (r + (long)i * rpi) * C + c0;
        yv[i] = MASK == 1 ? ld16(y + o) : make_uint4(0, 0, 0, 0);
        bits[i] = MASK == 3 ? (unsigned)mb[o >> 3] : 0u;
        dv[i] = ld16(dy + o);
        xv[i] = ld16(x + o);
      }
#pragma unroll
      for (int i = 0; i < kRows; i++) one((r + (long)i * rpi) * C + c0, dv[i], xv[i], yv[i], bits[i]);
    }
    for (; r < re; r += rpi) {
      const long o = r * C + c0;
      uint4 yv = make_uint4(0, 0, 0, 0);
      if (MASK == 1) yv = ld16(y + o);
      one(o, ld16(dy + o), ld16(x + o), yv, MASK == 3 ? (unsigned)mb[o >> 3] : 0u);
    }
  }
}

// bn_bwd_apply for a BN whose residual input r is another BatchNorm's RAW input
// (the bn_apply RAFF forward): instead of writing the residual-branch gradient
// dres = dz, accumulate THAT BN's backward statistics sum(dz), sum(dz*(r - rmean))
// into its slot workspace (rslots); its own backward then re-derives dz from dy
// and the ReLU mask (kfa_bn_bwd_prestats, mask mode 3).  Same channel-group
// loop and LDS block reduction as bn_bwd_partial.
template <int MASK>
__global__ __launch_bounds__(NT) void bn_bwd_apply_rstats(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                          const bf16_t* __restrict__ y, const uint8_t* __restrict__ mb,
                                                          const float* __restrict__ ss, const float* __restrict__ coef,
                                                          bf16_t* __restrict__ dx, const bf16_t* __restrict__ r,
                                                          const float* __restrict__ rmean, float* __restrict__ rslots,
                                                          long M, int C, long chunk, int tpr, int rpi) {
  __shared__ __attribute__((aligned(16))) float sh[kRedFloats];
  const int t = threadIdx.x;
  const int cg = t % tpr, r0 = t / tpr;
  const bool active = r0 < rpi;
  const int cv = C / 8;
  const long rb = (long)blockIdx.x * chunk;
  const long re = rb + chunk < M ? rb + chunk : M;
  for (int g0 = 0; g0 < cv; g0 += tpr) {
    const int c0 = (g0 + cg) * 8;
    float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (active && g0 + cg < cv) {
      float ca[8], cb[8], ck[8], sc[8], sf[8], mu[8];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        ca[j] = coef[c0 + j];
        cb[j] = coef[C + c0 + j];
        ck[j] = coef[2 * C + c0 + j];
        mu[j] = rmean[c0 + j];
      }
      load_ss<MASK>(ss, C, c0, sc, sf);
      auto one = [&](long o, const uint4 dv, const uint4 xv, const uint4 rv, const uint4 yv, unsigned bits) {
        float dz[8], xf[8], rf[8], out[8];
        unpack8(xv, xf);
        unpack8(rv, rf);
        masked_dy<MASK>(dv, yv, xf, sc, sf, bits, dz);
#pragma unroll
        for (int j = 0; j < 8; j++) {
          out[j] = fmaf(ca[j], dz[j], fmaf(cb[j], xf[j], ck[j]));
          s1[j] += dz[j];
          s2[j] += dz[j] * (rf[j] - mu[j]);
        }
        st16(dx + o, pack8(out));
      };
      long row = rb + r0;
      for (; row + rpi < re; row += 2L * rpi) {  // two rows in flight (see bn_bwd_apply)
        const long o0 = row * C + c0, o1 = (row + rpi) * C + c0;
        uint4 y0 = make_uint4(0, 0, 0, 0), y1 = y0;
        if (MASK == 1) { y0 = ld16(y + o0); y1 = ld16(y + o1); }
        const unsigned b0 = MASK == 3 ? (unsigned)mb[o0 >> 3] : 0u, b1 = MASK == 3 ? (unsigned)mb[o1 >> 3] : 0u;
        const uint4 d0 = ld16(dy + o0), d1 = ld16(dy + o1), x0 = ld16(x + o0), x1 = ld16(x + o1);
        const uint4 q0 = ld16(r + o0), q1 = ld16(r + o1);
        one(o0, d0, x0, q0, y0, b0);
        one(o1, d1, x1, q1, y1, b1);
      }
      for (; row < re; row += rpi) {
        const long o = row * C + c0;
        uint4 yv = make_uint4(0, 0, 0, 0);
        if (MASK == 1) yv = ld16(y + o);
        one(o, ld16(dy + o), ld16(x + o), ld16(r + o), yv, MASK == 3 ? (unsigned)mb[o >> 3] : 0u);
      }
    }
    if (active) {
      red_put(sh, r0 * tpr + cg, s1, s2);
    }
    __syncthreads();
    const int width = tpr * 8;
    for (int idx = t; idx < 2 * width; idx += NT) {
      const int a = idx / width, c = idx % width;
      if (g0 * 8 + c < C) {
        float acc = 0.f;
        for (int rr = 0; rr < rpi; rr++) acc += red_get(sh, a, rr * tpr + (c >> 3), c & 7);
        __hip_atomic_fetch_add(&rslots[((long)(blockIdx.x % kSlots) * 2 + a) * C + g0 * 8 + c], acc,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
  }
}

}  // namespace

// ====================================================================== C ABI
// cap row blocks so each partial array stays <= 1M floats (finalize reads it all)
static int max_row_blocks(int C) {
  int m = (1 << 20) / C;
  return m > 2048 ? 2048 : (m < 64 ? 64 : m);
}

// Two workspaces: `slots` (kfa_bn_slot_floats, ZERO-initialised once, kept
// clean by every finalize) and `coef` (kfa_bn_coef_floats, scratch).  They
// must not alias: the slot region's layout depends on C.
KFA_API long kfa_bn_slot_floats(int C) { return 2L * kSlots * C; }
KFA_API long kfa_bn_coef_floats(int C) { return 3L * C; }

static bool bn_shape_ok(long M, int C) { return M > 0 && C >= 8 && (C % 8) == 0; }

KFA_API int kfa_bn_fwd_train(const bf16_t* x, const bf16_t* res, bf16_t* y, const float* gamma, const float* beta,
                             float* rmean, float* rvar, float* save_mean, float* save_invstd, float* slots,
                             float* coefws, long M, int C, float eps, float momentum, int relu, uint8_t* mb,
                             hipStream_t s) {
  if (!bn_shape_ok(M, C)) return -1;
  Geom g = geom(M, C, max_row_blocks(C));
  float* part = slots;
  float* scale = coefws;
  float* shift = scale + C;
  hipLaunchKernelGGL(bn_stats_partial, dim3(g.gx), dim3(NT), 0, s, x, part, M, C, g.chunk, g.tpr, g.rpi);
  hipLaunchKernelGGL(bn_finalize, dim3(kfa_ceil_div(C, 64)), dim3(64, kGroups), 0, s, x, part, g.gx, M, C, gamma, beta, rmean,
                     rvar, save_mean, save_invstd, scale, shift, eps, momentum);
  launch_apply(relu, res, mb, dim3(g.gx), s, x, y, scale, shift, M, C, g.chunk, g.tpr, g.rpi);
  return kfa_status();
}

// Statistics pass alone (shifted sums into `slots`); used by the conv forward
// tuner (ops/conv.py) to price "vendor conv + separate BN statistics pass"
// against the fused-statistics implicit GEMM.  The caller cleans `slots`.
KFA_API int kfa_bn_stats_partial(const bf16_t* x, float* slots, long M, int C, hipStream_t s) {
  if (!bn_shape_ok(M, C)) return -1;
  Geom g = geom(M, C, max_row_blocks(C));
  hipLaunchKernelGGL(bn_stats_partial, dim3(g.gx), dim3(NT), 0, s, x, slots, M, C, g.chunk, g.tpr, g.rpi);
  return kfa_status();
}

// Training forward whose statistics were already accumulated into `slots`
// (un-shifted sum / sum of squares) by the producing convolution's epilogue
// (kfa_conv_igemm with a stats pointer): finalize + apply only — the stats
// pass over the conv output is gone.
KFA_API int kfa_bn_fwd_train_prestats(const bf16_t* x, const bf16_t* res, bf16_t* y, const float* gamma,
                                      const float* beta, float* rmean, float* rvar, float* save_mean,
                                      float* save_invstd, float* slots, float* coefws, long M, int C, float eps,
                                      float momentum, int relu, uint8_t* mb, hipStream_t s) {
  if (!bn_shape_ok(M, C)) return -1;
  Geom g = geom(M, C, max_row_blocks(C));
  float* scale = coefws;
  float* shift = scale + C;
  hipLaunchKernelGGL(bn_finalize, dim3(kfa_ceil_div(C, 64)), dim3(64, kGroups), 0, s, nullptr, slots, g.gx, M, C, gamma, beta,
                     rmean, rvar, save_mean, save_invstd, scale, shift, eps, momentum);
  launch_apply(relu, res, mb, dim3(g.gx), s, x, y, scale, shift, M, C, g.chunk, g.tpr, g.rpi);
  return kfa_status();
}

// y = act(x * scale + shift) with a given [scale | shift] (2C floats): the apply pass of a
// training BatchNorm whose finalize already ran (kfa_bn_finalize) and whose consumer could
// not take the normalisation into its own operand load (ops/batchnorm.py, lazy outputs).
KFA_API int kfa_bn_apply_ss(const bf16_t* x, bf16_t* y, const float* ss, long M, int C, int relu, hipStream_t s) {
  if (!bn_shape_ok(M, C) || !ss) return -1;
  Geom g = geom(M, C, max_row_blocks(C));
  launch_apply(relu, nullptr, nullptr, dim3(g.gx), s, x, y, ss, ss + C, M, C, g.chunk, g.tpr, g.rpi);
  return kfa_status();
}

KFA_API int kfa_bn_fwd_eval(const bf16_t* x, const bf16_t* res, bf16_t* y, const float* gamma, const float* beta,
                            const float* rmean, const float* rvar, float* ws, long M, int C, float eps, int relu,
                            hipStream_t s) {
  if (!bn_shape_ok(M, C)) return -1;
  Geom g = geom(M, C, max_row_blocks(C));
  float* scale = ws;
  float* shift = ws + C;
  hipLaunchKernelGGL(bn_finalize_eval, dim3(kfa_ceil_div(C, 256)), dim3(256), 0, s, gamma, beta, rmean, rvar, C, eps,
                     scale, shift);
  launch_apply(relu, res, nullptr, dim3(g.gx), s, x, y, scale, shift, M, C, g.chunk, g.tpr, g.rpi);
  return kfa_status();
}

template <int MASK>
static void launch_bwd_apply(const Geom&, const bf16_t* dy, const bf16_t* x, const bf16_t* y, const uint8_t* mb,
                             const float* ss, const float* coef, bf16_t* dx, bf16_t* dres, long M, int C,
                             hipStream_t s) {
  const Geom g = apply_geom(M, C);
  if (dres)
    hipLaunchKernelGGL((bn_bwd_apply<MASK, true>), dim3(g.gx), dim3(NT), 0, s, dy, x, y, mb, ss, coef, dx, dres, M, C,
                       g.chunk, g.tpr, g.rpi);
  else
    hipLaunchKernelGGL((bn_bwd_apply<MASK, false>), dim3(g.gx), dim3(NT), 0, s, dy, x, y, mb, ss, coef, dx, dres, M,
                       C, g.chunk, g.tpr, g.rpi);
}

// ReLU mask source when relu != 0, first present of: y (the forward OUTPUT), mb
// (the forward's output bit mask), ss (the forward's [scale | shift], 2C floats,
// only valid for a forward without residual).
static int mask_mode(int relu, const bf16_t* y, const uint8_t* mb, const float* ss) {
  if (!relu) return 0;
  if (y) return 1;
  if (mb) return 3;
  return ss ? 2 : -1;
}

static void launch_bwd_apply_any(int mm, const Geom& g, const bf16_t* dy, const bf16_t* x, const bf16_t* y,
                                 const uint8_t* mb, const float* ss, const float* coef, bf16_t* dx, bf16_t* dres,
                                 long M, int C, hipStream_t s) {
  if (mm == 3) launch_bwd_apply<3>(g, dy, x, y, mb, ss, coef, dx, dres, M, C, s);
  else if (mm == 2) launch_bwd_apply<2>(g, dy, x, y, mb, ss, coef, dx, dres, M, C, s);
  else if (mm == 1) launch_bwd_apply<1>(g, dy, x, y, mb, ss, coef, dx, dres, M, C, s);
  else launch_bwd_apply<0>(g, dy, x, y, mb, ss, coef, dx, dres, M, C, s);
}

// Backward whose partial sums (sum(dz), sum(dz*(x-mean))) were accumulated into
// `slots` by the dgrad epilogue that produced dy (kfa_conv_igemm with bn_x):
// finalize + apply only.
KFA_API int kfa_bn_bwd_prestats(const bf16_t* dy, const bf16_t* x, const bf16_t* y, const float* gamma,
                                const float* save_mean, const float* save_invstd, bf16_t* dx, bf16_t* dres,
                                float* dgamma, float* dbeta, float* slots, float* coefws, long M, int C, int relu,
                                int accumulate, const float* ss, const uint8_t* mb, hipStream_t s) {
  if (!bn_shape_ok(M, C)) return -1;
  const int mm = mask_mode(relu, y, mb, ss);
  if (mm < 0) return -2;
  Geom g = geom(M, C, max_row_blocks(C));
  float* coef = coefws;
  hipLaunchKernelGGL(bn_bwd_finalize, dim3(kfa_ceil_div(C, 64)), dim3(64, kGroups), 0, s, slots, g.gx, M, C, gamma,
                     save_mean, save_invstd, dgamma, dbeta, coef, accumulate);
  launch_bwd_apply_any(mm, g, dy, x, y, mb, ss, coef, dx, dres, M, C, s);
  return kfa_status();
}

KFA_API int kfa_bn_bwd(const bf16_t* dy, const bf16_t* x, const bf16_t* y, const float* gamma, const float* save_mean,
                       const float* save_invstd, bf16_t* dx, bf16_t* dres, float* dgamma, float* dbeta, float* slots,
                       float* coefws, long M, int C, int relu, int accumulate, const float* ss, const uint8_t* mb,
                       hipStream_t s) {
  if (!bn_shape_ok(M, C)) return -1;
  const int mm = mask_mode(relu, y, mb, ss);
  if (mm < 0) return -2;
  Geom g = geom(M, C, max_row_blocks(C));
  float* part = slots;
  float* coef = coefws;
  if (mm == 3)
    hipLaunchKernelGGL(bn_bwd_partial<3>, dim3(g.gx), dim3(NT), 0, s, dy, x, y, mb, ss, save_mean, part, M, C,
                       g.chunk, g.tpr, g.rpi);
  else if (mm == 2)
    hipLaunchKernelGGL(bn_bwd_partial<2>, dim3(g.gx), dim3(NT), 0, s, dy, x, y, mb, ss, save_mean, part, M, C,
                       g.chunk, g.tpr, g.rpi);
  else if (mm == 1)
    hipLaunchKernelGGL(bn_bwd_partial<1>, dim3(g.gx), dim3(NT), 0, s, dy, x, y, mb, ss, save_mean, part, M, C,
                       g.chunk, g.tpr, g.rpi);
  else
    hipLaunchKernelGGL(bn_bwd_partial<0>, dim3(g.gx), dim3(NT), 0, s, dy, x, y, mb, ss, save_mean, part, M, C,
                       g.chunk, g.tpr, g.rpi);
  hipLaunchKernelGGL(bn_bwd_finalize, dim3(kfa_ceil_div(C, 64)), dim3(64, kGroups), 0, s, part, g.gx, M, C, gamma,
                     save_mean, save_invstd, dgamma, dbeta, coef, accumulate);
  launch_bwd_apply_any(mm, g, dy, x, y, mb, ss, coef, dx, dres, M, C, s);
  return kfa_status();
}

// ---------------------------------------------------------------- downsample-block pair
// A ResNet downsample block ends in relu(bn3(x) + bn_ds(r)): r (the downsample
// conv's output) is normalised inside bn3's apply pass (bn_apply RAFF) instead
// of by a pass of its own, and bn_ds's backward statistics are gathered by
// bn3's backward apply pass instead of a partial pass over a written dres.

// Forward finalize alone (bn_ds): scale / shift into ss = [scale | shift] (2C),
// batch mean / invstd, running statistics.  prestats = 0: the statistics pass
// over x runs first (else the producing conv's epilogue accumulated them).
KFA_API int kfa_bn_finalize(const bf16_t* x, float* slots, long M, int C, const float* gamma, const float* beta,
                            float* rmean, float* rvar, float* save_mean, float* save_invstd, float* ss, float eps,
                            float momentum, int prestats, hipStream_t s) {
  if (!bn_shape_ok(M, C)) return -1;
  Geom g = geom(M, C, max_row_blocks(C));
  if (!prestats)
    hipLaunchKernelGGL(bn_stats_partial, dim3(g.gx), dim3(NT), 0, s, x, slots, M, C, g.chunk, g.tpr, g.rpi);
  hipLaunchKernelGGL(bn_finalize, dim3(kfa_ceil_div(C, 64)), dim3(64, kGroups), 0, s, prestats ? nullptr : x, slots,
                     g.gx, M, C, gamma, beta, rmean, rvar, save_mean, save_invstd, ss, ss + C, eps, momentum);
  return kfa_status();
}

// bn3 forward with the residual r normalised by rss (bn_ds's [scale | shift]).
KFA_API int kfa_bn_fwd_train_dual(const bf16_t* x, const bf16_t* r, bf16_t* y, const float* gamma, const float* beta,
                                  float* rmean, float* rvar, float* save_mean, float* save_invstd, float* slots,
                                  float* ss, long M, int C, float eps, float momentum, int relu, uint8_t* mb,
                                  const float* rss, int prestats, hipStream_t s) {
  if (!bn_shape_ok(M, C) || !r || !rss) return -1;
  if (kfa_bn_finalize(x, slots, M, C, gamma, beta, rmean, rvar, save_mean, save_invstd, ss, eps, momentum, prestats,
                      s))
    return -1;
  Geom g = geom(M, C, max_row_blocks(C));
  launch_apply(relu, r, mb, dim3(g.gx), s, x, y, ss, ss + C, M, C, g.chunk, g.tpr, g.rpi, rss);
  return kfa_status();
}

// bn3 backward (statistics from `slots`, accumulated by the consuming dgrad
// epilogue when prestats, else by its own partial pass) whose apply pass also
// accumulates bn_ds's backward statistics into rslots (see bn_bwd_apply_rstats);
// no residual gradient is written.
KFA_API int kfa_bn_bwd_rstats(const bf16_t* dy, const bf16_t* x, const bf16_t* y, const float* gamma,
                              const float* save_mean, const float* save_invstd, bf16_t* dx, float* dgamma,
                              float* dbeta, float* slots, float* coefws, long M, int C, int relu, int accumulate,
                              const float* ss, const uint8_t* mb, const bf16_t* r, const float* rmean, float* rslots,
                              int prestats, hipStream_t s) {
  if (!bn_shape_ok(M, C) || !r || !rmean || !rslots) return -1;
  const int mm = mask_mode(relu, y, mb, ss);
  if (mm < 0 || mm == 2) return -2;  // a mask recomputed from x alone is wrong with a residual
  Geom g = geom(M, C, max_row_blocks(C));
  if (!prestats) {
    if (mm == 3)
      hipLaunchKernelGGL(bn_bwd_partial<3>, dim3(g.gx), dim3(NT), 0, s, dy, x, y, mb, ss, save_mean, slots, M, C,
                         g.chunk, g.tpr, g.rpi);
    else if (mm == 1)
      hipLaunchKernelGGL(bn_bwd_partial<1>, dim3(g.gx), dim3(NT), 0, s, dy, x, y, mb, ss, save_mean, slots, M, C,
                         g.chunk, g.tpr, g.rpi);
    else if (mm == 0)
      hipLaunchKernelGGL(bn_bwd_partial<0>, dim3(g.gx), dim3(NT), 0, s, dy, x, y, mb, ss, save_mean, slots, M, C,
                         g.chunk, g.tpr, g.rpi);
    else
      return -2;  // mask from x is invalid with a residual
  }
  hipLaunchKernelGGL(bn_bwd_finalize, dim3(kfa_ceil_div(C, 64)), dim3(64, kGroups), 0, s, slots, g.gx, M, C, gamma,
                     save_mean, save_invstd, dgamma, dbeta, coefws, accumulate);
  if (mm == 3)
    hipLaunchKernelGGL(bn_bwd_apply_rstats<3>, dim3(g.gx), dim3(NT), 0, s, dy, x, y, mb, ss, coefws, dx, r, rmean,
                       rslots, M, C, g.chunk, g.tpr, g.rpi);
  else if (mm == 1)
    hipLaunchKernelGGL(bn_bwd_apply_rstats<1>, dim3(g.gx), dim3(NT), 0, s, dy, x, y, mb, ss, coefws, dx, r, rmean,
                       rslots, M, C, g.chunk, g.tpr, g.rpi);
  else
    hipLaunchKernelGGL(bn_bwd_apply_rstats<0>, dim3(g.gx), dim3(NT), 0, s, dy, x, y, mb, ss, coefws, dx, r, rmean,
                       rslots, M, C, g.chunk, g.tpr, g.rpi);
  return kfa_status();
}
