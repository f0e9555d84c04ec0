// Max pooling (ResNet stem 3x3/s2/p1) for NHWC bf16, forward + backward
// (SURVEY §2.6 K9).  Forward stores the 0..k*k-1 window position of each max
// as uint8; backward is a GATHER over the <= ceil(k/s)^2 windows that cover an
// input pixel, so it needs no atomics and no zero-fill pass.
// Each thread handles 8 channels (16-B vectors).
#include <cstdlib>

#include "common.h"

namespace {

// Index math in 32 bits (the launchers require < 2^31 16-B vectors): 64-bit
// div/mod by runtime divisors were the bulk of the instruction stream, leaving
// the stem pool at ~2 TB/s.  One vector per thread, no grid-stride loop.
template <typename IT>
__global__ __launch_bounds__(256) void maxpool_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                   uint8_t* __restrict__ idx, int N, int H, int W, int C, int Ho,
                                                   int Wo, int k, int s, int p) {
  const IT cv = C / 8;
  const IT total = (IT)N * Ho * Wo * cv;
  for (IT v = (IT)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += (IT)gridDim.x * blockDim.x) {
    const int cg = (int)(v % cv);
    IT t = v / cv;
    const int ow = (int)(t % (IT)Wo);
    t /= (IT)Wo;
    const int oh = (int)(t % (IT)Ho);
    const int n = (int)(t / (IT)Ho);
    float best[8];
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; j++) { best[j] = -INFINITY; bi[j] = 0; }
    for (int kh = 0; kh < k; kh++) {
      const int ih = oh * s - p + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < k; kw++) {
        const int iw = ow * s - p + kw;
        if (iw < 0 || iw >= W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(x + (((long)n * H + ih) * W + iw) * C + cg * 8), f);
        const int pos = kh * k + kw;
#pragma unroll
        for (int j = 0; j < 8; j++)
          if (f[j] > best[j] || (f[j] != f[j] && best[j] == best[j])) { best[j] = f[j]; bi[j] = pos; }
      }
    }
    const long o = (((long)n * Ho + oh) * Wo + ow) * C + cg * 8;
    *reinterpret_cast<uint4*>(y + o) = pack8(best);
    if (idx) {
      uint2 packed;
      packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
      packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
      *reinterpret_cast<uint2*>(idx + o) = packed;
    }
  }
}

template <typename IT>
__global__ __launch_bounds__(256) void maxpool_bwd(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                   bf16_t* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                   int Wo, int k, int s, int p) {
  const IT cv = C / 8;
  const IT total = (IT)N * H * W * cv;
  for (IT v = (IT)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += (IT)gridDim.x * blockDim.x) {
    const int cg = (int)(v % cv);
    IT t = v / cv;
    const int iw = (int)(t % (IT)W);
    t /= (IT)W;
    const int ih = (int)(t % (IT)H);
    const int n = (int)(t / (IT)H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // windows oh with oh*s - p <= ih <= oh*s - p + k - 1
    const int oh0 = max(0, (ih + p - k + s) / s), oh1 = min(Ho - 1, (ih + p) / s);
    const int ow0 = max(0, (iw + p - k + s) / s), ow1 = min(Wo - 1, (iw + p) / s);
    for (int oh = oh0; oh <= oh1; oh++) {
      const int kh = ih - (oh * s - p);
      if (kh < 0 || kh >= k) continue;
      for (int ow = ow0; ow <= ow1; ow++) {
        const int kw = iw - (ow * s - p);
        if (kw < 0 || kw >= k) continue;
        const int pos = kh * k + kw;
        const long o = (((long)n * Ho + oh) * Wo + ow) * C + cg * 8;
        const uint2 pk = *reinterpret_cast<const uint2*>(idx + o);
        float g[8];
        unpack8(*reinterpret_cast<const uint4*>(dy + o), g);
        const uint32_t w[2] = {pk.x, pk.y};
#pragma unroll
        for (int j = 0; j < 8; j++)
          if ((int)((w[j >> 2] >> ((j & 3) * 8)) & 0xff) == pos) acc[j] += g[j];
      }
    }
    *reinterpret_cast<uint4*>(dx + (((long)n * H + ih) * W + iw) * C + cg * 8) = pack8(acc);
  }
}

// 3x3 / stride 2 (the ResNet stem): every window load issued before any is
// used — the generic loops' bounds `continue`s serialised the 9 (fwd) / 4 (bwd)
// loads of a thread, leaving the pool latency-bound at 2-3 TB/s.  Out-of-range
// taps load a clamped (valid) address and are masked afterwards.
// BN: x is the PRE-BatchNorm tensor; every window element is first mapped to
// relu(fma(x, scale[c], shift[c])) (ss = [scale | shift]) in fp32 and the max is
// rounded to bf16 once: rounding is monotone, so the output equals the max of the
// bf16 values the BN + ReLU apply pass would have written (only the argmax among
// taps that round to the same bf16 value can differ), and fmaxf(., 0) already maps
// NaN to 0, so the NaN-propagating compare is dropped — 5 VALU ops per element and
// tap instead of 11 (the stem pool is VALU-bound).  The stem's BN output is never
// materialised (its backward recomputes the mask from x).
template <bool BN>
__global__ __launch_bounds__(256) void maxpool3s2_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                      uint8_t* __restrict__ idx, int N, int H, int W, int C, int Ho,
                                                      int Wo, int p, const float* __restrict__ ss) {
  const unsigned cv = C / 8;
  const unsigned total = (unsigned)N * Ho * Wo * cv;
  const unsigned v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= total) return;
  const int cg = (int)(v % cv);
  unsigned t = v / cv;
  const int ow = (int)(t % (unsigned)Wo);
  t /= (unsigned)Wo;
  const int oh = (int)(t % (unsigned)Ho);
  const int n = (int)(t / (unsigned)Ho);
  const bf16_t* xb = x + (long)n * H * W * C + cg * 8;
  uint4 in[9];
  bool ok[9];
#pragma unroll
  for (int kh = 0; kh < 3; kh++)
#pragma unroll
    for (int kw = 0; kw < 3; kw++) {
      const int ih = oh * 2 - p + kh, iw = ow * 2 - p + kw;
      ok[kh * 3 + kw] = ih >= 0 && ih < H && iw >= 0 && iw < W;
      const int ch = min(max(ih, 0), H - 1), cw = min(max(iw, 0), W - 1);
      in[kh * 3 + kw] = *reinterpret_cast<const uint4*>(xb + ((long)ch * W + cw) * C);
    }
  float best[8], sc[8], sf[8];
  int bi[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    best[j] = -INFINITY;
    bi[j] = 0;
    sc[j] = BN ? ss[cg * 8 + j] : 1.f;
    sf[j] = BN ? ss[C + cg * 8 + j] : 0.f;
  }
#pragma unroll
  for (int pos = 0; pos < 9; pos++) {
    if (!ok[pos]) continue;
    float f[8];
    unpack8(in[pos], f);
    if (BN) {
#pragma unroll
      for (int j = 0; j < 8; j++) f[j] = fmaxf(fmaf(f[j], sc[j], sf[j]), 0.f);
    }
#pragma unroll
    for (int j = 0; j < 8; j++)
      if (f[j] > best[j] || (!BN && f[j] != f[j] && best[j] == best[j])) { best[j] = f[j]; bi[j] = pos; }
  }
  const long o = (long)v * 8;  // output NHWC offset == vector index * 8
  *reinterpret_cast<uint4*>(y + o) = pack8(best);
  if (idx) {
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
    *reinterpret_cast<uint2*>(idx + o) = packed;
  }
}

// Same op, two horizontally adjacent outputs (ow, ow + 1) per thread: their
// windows share a column, so 15 loads (each BN-mapped once) serve 2 outputs
// instead of 18 — and each thread keeps 15 loads in flight (the one-output form
// is latency-bound: 9 loads, then wait).  Wo odd: the last pair's second output is masked.
template <bool BN>
__global__ __launch_bounds__(256) void maxpool3s2_fwd2(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                       uint8_t* __restrict__ idx, int N, int H, int W, int C, int Ho,
                                                       int Wo, int p, const float* __restrict__ ss) {
  const unsigned cv = C / 8;
  const unsigned wp = (unsigned)(Wo + 1) / 2;
  const unsigned total = (unsigned)N * Ho * wp * cv;
  const unsigned v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= total) return;
  const int cg = (int)(v % cv);
  unsigned t = v / cv;
  const int ow0 = (int)(t % wp) * 2;
  t /= wp;
  const int oh = (int)(t % (unsigned)Ho);
  const int n = (int)(t / (unsigned)Ho);
  const bf16_t* xb = x + (long)n * H * W * C + cg * 8;
  uint4 in[15];
  bool ok[15];
#pragma unroll
  for (int kh = 0; kh < 3; kh++)
#pragma unroll
    for (int kw = 0; kw < 5; kw++) {
      const int ih = oh * 2 - p + kh, iw = ow0 * 2 - p + kw;
      ok[kh * 5 + kw] = ih >= 0 && ih < H && iw >= 0 && iw < W;
      const int ch = min(max(ih, 0), H - 1), cw = min(max(iw, 0), W - 1);
      in[kh * 5 + kw] = *reinterpret_cast<const uint4*>(xb + ((long)ch * W + cw) * C);
    }
  float sc[8], sf[8], best0[8], best1[8];
  int bi0[8], bi1[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    sc[j] = BN ? ss[cg * 8 + j] : 1.f;
    sf[j] = BN ? ss[C + cg * 8 + j] : 0.f;
    best0[j] = best1[j] = -INFINITY;
    bi0[j] = bi1[j] = 0;
  }
#pragma unroll
  for (int kh = 0; kh < 3; kh++)
#pragma unroll
    for (int kw = 0; kw < 5; kw++) {
      const int q = kh * 5 + kw;
      if (!ok[q]) continue;
      float f[8];
      unpack8(in[q], f);
      if (BN) {
#pragma unroll
        for (int j = 0; j < 8; j++) f[j] = fmaxf(fmaf(f[j], sc[j], sf[j]), 0.f);
      }
      if (kw < 3) {  // output ow0: window columns 0..2, tap index kh * 3 + kw
#pragma unroll
        for (int j = 0; j < 8; j++)
          if (f[j] > best0[j] || (!BN && f[j] != f[j] && best0[j] == best0[j])) { best0[j] = f[j]; bi0[j] = kh * 3 + kw; }
      }
      if (kw >= 2) {  // output ow0 + 1: window columns 2..4
#pragma unroll
        for (int j = 0; j < 8; j++)
          if (f[j] > best1[j] || (!BN && f[j] != f[j] && best1[j] == best1[j])) { best1[j] = f[j]; bi1[j] = kh * 3 + kw - 2; }
      }
    }
  const long o0 = ((((long)n * Ho + oh) * Wo) + ow0) * C + cg * 8;
  *reinterpret_cast<uint4*>(y + o0) = pack8(best0);
  if (idx) {
    *reinterpret_cast<uint2*>(idx + o0) = make_uint2(bi0[0] | (bi0[1] << 8) | (bi0[2] << 16) | (bi0[3] << 24),
                                                     bi0[4] | (bi0[5] << 8) | (bi0[6] << 16) | (bi0[7] << 24));
  }
  if (ow0 + 1 < Wo) {
    const long o1 = o0 + C;
    *reinterpret_cast<uint4*>(y + o1) = pack8(best1);
    if (idx) {
      *reinterpret_cast<uint2*>(idx + o1) = make_uint2(bi1[0] | (bi1[1] << 8) | (bi1[2] << 16) | (bi1[3] << 24),
                                                       bi1[4] | (bi1[5] << 8) | (bi1[6] << 16) | (bi1[7] << 24));
    }
  }
}

__global__ __launch_bounds__(256) void maxpool3s2_bwd(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                      bf16_t* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                      int Wo, int p) {
  const unsigned cv = C / 8;
  const unsigned total = (unsigned)N * H * W * cv;
  const unsigned v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= total) return;
  const int cg = (int)(v % cv);
  unsigned t = v / cv;
  const int iw = (int)(t % (unsigned)W);
  t /= (unsigned)W;
  const int ih = (int)(t % (unsigned)H);
  const int n = (int)(t / (unsigned)H);
  // covering windows: oh in {oh1 - 1, oh1} with oh1 = (ih + p) / 2 (k = 3, s = 2)
  const int oh1 = (ih + p) >> 1, ow1 = (iw + p) >> 1;
  uint4 g[4];
  uint2 pk[4];
  bool ok[4];
  int pos[4];
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++) {
      const int oh = oh1 - a, ow = ow1 - b;
      const int kh = ih - (oh * 2 - p), kw = iw - (ow * 2 - p);
      const int w = a * 2 + b;
      ok[w] = oh >= 0 && oh < Ho && ow >= 0 && ow < Wo && kh < 3 && kw < 3;
      pos[w] = kh * 3 + kw;
      const long o = (((long)n * Ho + min(max(oh, 0), Ho - 1)) * Wo + min(max(ow, 0), Wo - 1)) * C + cg * 8;
      g[w] = *reinterpret_cast<const uint4*>(dy + o);
      pk[w] = *reinterpret_cast<const uint2*>(idx + o);
    }
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int w = 0; w < 4; w++) {
    if (!ok[w]) continue;
    float f[8];
    unpack8(g[w], f);
    const uint32_t q[2] = {pk[w].x, pk[w].y};
#pragma unroll
    for (int j = 0; j < 8; j++)
      if ((int)((q[j >> 2] >> ((j & 3) * 8)) & 0xff) == pos[w]) acc[j] += f[j];
  }
  *reinterpret_cast<uint4*>(dx + (long)v * 8) = pack8(acc);
}

// Same gradient, one thread per 2 x 2 block of input pixels x 8 channels: input rows
// 2t-p, 2t-p+1 are covered by exactly the windows t-1, t (columns likewise), so the
// block's four outputs share ONE set of 4 window loads (dy + argmax bytes) instead
// of 4 each — a quarter of the gathers and index math of maxpool3s2_bwd.
// STATS (C == 64 only): the pool gradient feeds a BatchNorm + ReLU backward (the
// ResNet stem): also accumulate that BN's backward statistics sum(dz) and
// sum(dz * (x - mean)), dz = the written (bf16) gradient where relu(fma(x, scale,
// shift)) > 0, into the BN slots ([64 slots][2][C], slot = block % 64) — the
// statistics pass over the 4x-pooled-size gradient and x is then skipped
// (kfa_bn_bwd_prestats).  Lanes with the same 8-channel group (lane % 8) reduce
// by butterfly; lane L then adds channel 8 (L % 8) + L / 8: one 64-lane atomic
// per statistic per wave.
struct PoolBnStats {
  const bf16_t* x;
  const float* ss;    // the BN forward's [scale | shift]
  const float* mean;
  float* slots;
};

template <bool STATS>
__global__ __launch_bounds__(256) void maxpool3s2_bwd4(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                       bf16_t* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                       int Wo, int p, int T, int U, PoolBnStats bs) {
  const unsigned cv = C / 8;
  const unsigned total = (unsigned)N * T * U * cv;
  const unsigned v = blockIdx.x * blockDim.x + threadIdx.x;
  if (!STATS && v >= total) return;
  const bool live = v < total;  // STATS: every lane takes part in the butterfly
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mu[8], sc[8], sf[8];
  const int cg = (int)(v % cv);
  if (STATS)
#pragma unroll
    for (int j = 0; j < 8; j++) {
      mu[j] = bs.mean[cg * 8 + j];
      sc[j] = bs.ss[cg * 8 + j];
      sf[j] = bs.ss[C + cg * 8 + j];
    }
  unsigned q = v / cv;
  const int u = (int)(q % (unsigned)U);
  q /= (unsigned)U;
  const int t = (int)(q % (unsigned)T);
  const int n = live ? (int)(q / (unsigned)T) : 0;  // a STATS tail lane past the work only loads in-bounds rows
  uint4 g[4];
  uint2 pk[4];
  bool ok[4];
#pragma unroll
  for (int b = 0; b < 2; b++)    // window row t - 1 + b
#pragma unroll
    for (int e = 0; e < 2; e++) {  // window column u - 1 + e
      const int oh = t - 1 + b, ow = u - 1 + e, w = b * 2 + e;
      ok[w] = live && oh >= 0 && oh < Ho && ow >= 0 && ow < Wo;
      const long o = (((long)n * Ho + min(max(oh, 0), Ho - 1)) * Wo + min(max(ow, 0), Wo - 1)) * C + cg * 8;
      g[w] = *reinterpret_cast<const uint4*>(dy + o);
      pk[w] = *reinterpret_cast<const uint2*>(idx + o);
    }
#pragma unroll
  for (int a = 0; a < 2; a++)      // input row 2t - p + a
#pragma unroll
    for (int c = 0; c < 2; c++) {  // input column 2u - p + c
      const int ih = 2 * t - p + a, iw = 2 * u - p + c;
      if (!live || ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int b = 0; b < 2; b++)
#pragma unroll
        for (int e = 0; e < 2; e++) {
          const int kh = a + 2 - 2 * b, kw = c + 2 - 2 * e;  // tap of (ih, iw) in window (t-1+b, u-1+e)
          const int w = b * 2 + e;
          if (kh > 2 || kw > 2 || !ok[w]) continue;
          const int pos = kh * 3 + kw;
          float f[8];
          unpack8(g[w], f);
          const uint32_t qq[2] = {pk[w].x, pk[w].y};
#pragma unroll
          for (int j = 0; j < 8; j++)
            if ((int)((qq[j >> 2] >> ((j & 3) * 8)) & 0xff) == pos) acc[j] += f[j];
        }
      const long o = (((long)n * H + ih) * W + iw) * C + cg * 8;
      const uint4 packed = pack8(acc);
      *reinterpret_cast<uint4*>(dx + o) = packed;
      if (STATS) {
        float dz[8], xf[8];
        unpack8(packed, dz);  // the bf16 values the BN backward apply will read
        unpack8(*reinterpret_cast<const uint4*>(bs.x + o), xf);
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const float d = fmaf(xf[j], sc[j], sf[j]) > 0.f ? dz[j] : 0.f;
          s1[j] += d;
          s2[j] += d * (xf[j] - mu[j]);
        }
      }
    }
  if (STATS) {
#pragma unroll
    for (int o = 8; o < 64; o <<= 1)
#pragma unroll
      for (int j = 0; j < 8; j++) { s1[j] += __shfl_xor(s1[j], o, 64); s2[j] += __shfl_xor(s2[j], o, 64); }
    const int lane = threadIdx.x & 63, jj = lane >> 3;
    float a1 = s1[0], a2 = s2[0];
#pragma unroll
    for (int j = 1; j < 8; j++) {
      a1 = jj == j ? s1[j] : a1;
      a2 = jj == j ? s2[j] : a2;
    }
    const int ch = (lane & 7) * 8 + jj;
    float* slot = bs.slots + (long)(blockIdx.x % 64) * 2 * C;
    __hip_atomic_fetch_add(slot + ch, a1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(slot + C + ch, a2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// KFA_POOL_BWD4=0: one thread per input pixel (maxpool3s2_bwd) instead of per 2 x 2 block
bool pool_bwd4() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("KFA_POOL_BWD4");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

int grid_for(long work) {
  long b = (work + 255) / 256;
  return (int)(b < (1L << 20) ? (b < 1 ? 1 : b) : (1L << 20));
}

// two outputs per thread (maxpool3s2_fwd2); KFA_POOL_PAIRS=0 keeps one
bool pool_pairs() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("KFA_POOL_PAIRS");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

}  // namespace

KFA_API int kfa_maxpool_fwd(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo,
                            int k, int s, int p, hipStream_t st) {
  if (C % 8 || k > 15) return -1;
  const long work = (long)N * Ho * Wo * (C / 8);
  if (k == 3 && s == 2 && p <= 1 && work < (1L << 31) && (long)N * H * W * C < (1L << 40) && pool_pairs())
    hipLaunchKernelGGL(maxpool3s2_fwd2<false>, dim3((unsigned)(((long)N * Ho * ((Wo + 1) / 2) * (C / 8) + 255) / 256)),
                       dim3(256), 0, st, x, y, idx, N, H, W, C, Ho, Wo, p, nullptr);
  else if (k == 3 && s == 2 && p <= 1 && work < (1L << 31) && (long)N * H * W * C < (1L << 40))
    hipLaunchKernelGGL(maxpool3s2_fwd<false>, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st, x, y, idx, N, H,
                       W, C, Ho, Wo, p, nullptr);
  else if (work < (1L << 31))
    hipLaunchKernelGGL(maxpool_fwd<unsigned>, dim3(grid_for(work)), dim3(256), 0, st, x, y, idx, N, H, W, C, Ho, Wo, k,
                       s, p);
  else
    hipLaunchKernelGGL(maxpool_fwd<long>, dim3(grid_for(work)), dim3(256), 0, st, x, y, idx, N, H, W, C, Ho, Wo, k, s,
                       p);
  return kfa_status();
}

KFA_API int kfa_maxpool_bwd(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C, int Ho,
                            int Wo, int k, int s, int p, hipStream_t st) {
  if (C % 8 || k > 15) return -1;
  const long work = (long)N * H * W * (C / 8);
  const int T = (H + p + 1) / 2, U = (W + p + 1) / 2;
  const long work4 = (long)N * T * U * (C / 8);
  if (k == 3 && s == 2 && p <= 1 && pool_bwd4() && work4 < (1L << 31))
    hipLaunchKernelGGL(maxpool3s2_bwd4<false>, dim3((unsigned)((work4 + 255) / 256)), dim3(256), 0, st, dy, idx, dx, N,
                       H, W, C, Ho, Wo, p, T, U, PoolBnStats{nullptr, nullptr, nullptr, nullptr});
  else if (k == 3 && s == 2 && p <= 1 && work < (1L << 31))
    hipLaunchKernelGGL(maxpool3s2_bwd, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st, dy, idx, dx, N, H, W, C,
                       Ho, Wo, p);
  else if (work < (1L << 31))
    hipLaunchKernelGGL(maxpool_bwd<unsigned>, dim3(grid_for(work)), dim3(256), 0, st, dy, idx, dx, N, H, W, C, Ho, Wo,
                       k, s, p);
  else
    hipLaunchKernelGGL(maxpool_bwd<long>, dim3(grid_for(work)), dim3(256), 0, st, dy, idx, dx, N, H, W, C, Ho, Wo, k,
                       s, p);
  return kfa_status();
}

// 3x3/s2 max-pool gradient of maxpool(relu(bn(x))) with that BN's backward
// statistics accumulated into `slots` (see maxpool3s2_bwd4<true>); C == 64.
// Then kfa_bn_bwd_prestats finishes the BN backward.
KFA_API int kfa_maxpool_bwd_bnstats(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C,
                                    int Ho, int Wo, int p, const bf16_t* x, const float* ss, const float* mean,
                                    float* slots, hipStream_t st) {
  const int T = (H + p + 1) / 2, U = (W + p + 1) / 2;
  const long work4 = (long)N * T * U * (C / 8);
  if (C != 64 || p > 1 || work4 >= (1L << 31) || !x || !ss || !mean || !slots) return -1;
  hipLaunchKernelGGL(maxpool3s2_bwd4<true>, dim3((unsigned)((work4 + 255) / 256)), dim3(256), 0, st, dy, idx, dx, N, H,
                     W, C, Ho, Wo, p, T, U, PoolBnStats{x, ss, mean, slots});
  return kfa_status();
}

// Stem BatchNorm + ReLU + 3x3/s2 max pool in one pass over the PRE-BN tensor
// (see maxpool3s2_fwd<true>); ss = the BN's [scale | shift] (kfa_bn_finalize).
KFA_API int kfa_maxpool_fwd_bn(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo,
                               int k, int s, int p, const float* ss, hipStream_t st) {
  const long work = (long)N * Ho * Wo * (C / 8);
  if (C % 8 || k != 3 || s != 2 || p > 1 || !ss || work >= (1L << 31) || (long)N * H * W * C >= (1L << 40)) return -1;
  if (pool_pairs()) {
    const long w2 = (long)N * Ho * ((Wo + 1) / 2) * (C / 8);
    hipLaunchKernelGGL(maxpool3s2_fwd2<true>, dim3((unsigned)((w2 + 255) / 256)), dim3(256), 0, st, x, y, idx, N, H,
                       W, C, Ho, Wo, p, ss);
  } else {
    hipLaunchKernelGGL(maxpool3s2_fwd<true>, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st, x, y, idx, N, H,
                       W, C, Ho, Wo, p, ss);
  }
  return kfa_status();
}

// ---------------------------------------------------------------- global average pool
// NHWC [N][HW][C] bf16 -> [N][C] bf16 (fp32 sums) and its backward
// dx[n][hw][c] = dy[n][c] / HW written straight in NHWC — the ResNet head (the
// ATen mean backward expanded, scaled, converted and re-laid-out the 51 MB
// gradient in four passes, ~0.13 ms per step).  One thread per 8 channels.
namespace {
__global__ __launch_bounds__(256) void gap_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int N, int HW,
                                                      int C) {
  const int cv = C / 8;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * cv) return;
  const int n = t / cv, c8 = t - n * cv;
  const bf16_t* p = x + (long)n * HW * C + c8 * 8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int i = 0;
  for (; i + 3 < HW; i += 4) {  // four rows in flight
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = *reinterpret_cast<const uint4*>(p + (long)(i + u) * C);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      float f[8];
      unpack8(v[u], f);
#pragma unroll
      for (int j = 0; j < 8; j++) s[j] += f[j];
    }
  }
  for (; i < HW; i++) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(p + (long)i * C), f);
#pragma unroll
    for (int j = 0; j < 8; j++) s[j] += f[j];
  }
  const float r = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < 8; j++) s[j] *= r;
  *reinterpret_cast<uint4*>(y + (long)n * C + c8 * 8) = pack8(s);
}

__global__ __launch_bounds__(256) void gap_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, int N,
                                                      int HW, int C) {
  const int cv = C / 8;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)N * HW * cv) return;
  const int c8 = (int)(t % cv);
  const long nhw = t / cv;
  const int n = (int)(nhw / HW);
  float f[8];
  unpack8(*reinterpret_cast<const uint4*>(dy + (long)n * C + c8 * 8), f);
  const float r = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < 8; j++) f[j] *= r;
  *reinterpret_cast<uint4*>(dx + t * 8) = pack8(f);
}
}  // namespace

KFA_API int kfa_gap_fwd(const bf16_t* x, bf16_t* y, int N, int HW, int C, hipStream_t st) {
  if (C % 8 || N <= 0 || HW <= 0) return -1;
  const int th = N * (C / 8);
  hipLaunchKernelGGL(gap_fwd_kernel, dim3((th + 255) / 256), dim3(256), 0, st, x, y, N, HW, C);
  return kfa_status();
}

KFA_API int kfa_gap_bwd(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8 || N <= 0 || HW <= 0) return -1;
  const long th = (long)N * HW * (C / 8);
  if (th >= (1L << 31)) return -2;
  hipLaunchKernelGGL(gap_bwd_kernel, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, st, dy, dx, N, HW, C);
  return kfa_status();
}
