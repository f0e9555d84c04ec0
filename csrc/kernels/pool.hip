// Max pooling (ResNet stem 3x3/s2/p1) for NHWC bf16, forward + backward
// (SURVEY §2.6 K9).  Forward stores the 0..k*k-1 window position of each max
// as uint8; backward is a GATHER over the <= ceil(k/s)^2 windows that cover an
// input pixel, so it needs no atomics and no zero-fill pass.
// Each thread handles 8 channels (16-B vectors).
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void maxpool_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                   uint8_t* __restrict__ idx, int N, int H, int W, int C, int Ho,
                                                   int Wo, int k, int s, int p) {
  const int cv = C / 8;
  const long total = (long)N * Ho * Wo * cv;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(v % cv);
    long t = v / cv;
    const int ow = (int)(t % Wo);
    t /= Wo;
    const int oh = (int)(t % Ho);
    const int n = (int)(t / Ho);
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

__global__ __launch_bounds__(256) void maxpool_bwd(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                   bf16_t* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                   int Wo, int k, int s, int p) {
  const int cv = C / 8;
  const long total = (long)N * H * W * cv;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(v % cv);
    long t = v / cv;
    const int iw = (int)(t % W);
    t /= W;
    const int ih = (int)(t % H);
    const int n = (int)(t / H);
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

int grid_for(long work) {
  long b = (work + 255) / 256;
  return (int)(b < 4096 ? (b < 1 ? 1 : b) : 4096);
}

}  // namespace

KFA_API int kfa_maxpool_fwd(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo,
                            int k, int s, int p, hipStream_t st) {
  if (C % 8 || k > 15) return -1;
  hipLaunchKernelGGL(maxpool_fwd, dim3(grid_for((long)N * Ho * Wo * (C / 8))), dim3(256), 0, st, x, y, idx, N, H, W,
                     C, Ho, Wo, k, s, p);
  return kfa_status();
}

KFA_API int kfa_maxpool_bwd(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C, int Ho,
                            int Wo, int k, int s, int p, hipStream_t st) {
  if (C % 8 || k > 15) return -1;
  hipLaunchKernelGGL(maxpool_bwd, dim3(grid_for((long)N * H * W * (C / 8))), dim3(256), 0, st, dy, idx, dx, N, H, W,
                     C, Ho, Wo, k, s, p);
  return kfa_status();
}
