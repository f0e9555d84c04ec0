// Wide & Deep input assembly (SURVEY §2.6 K6 around the sharded lookup):
//
//   forward:  rows [B][F][E+8] bf16 (deep features, then the wide weight, then pad)
//             dense [B][Dp] fp32 (already zero-padded to Dp % 8 == 0)
//          -> x    [B][Dp + F*E] bf16 = [bf16(dense) | rows[:, :, :E] flattened]
//             wide [B] fp32 = sum_f rows[b][f][E]
//   backward: dx [B][Dp + F*E] bf16, dwide [B] fp32
//          -> drows [B][F][E+8] bf16 = [dx[b, Dp + f*E : +E] | dwide[b] | 0 ... 0]
//
// One pass each way instead of the PyTorch slice / reshape / pad / cat / cast
// chain (and its autograd mirror: a zero-filled [B, F, E+8] gradient plus
// strided copies) — 16 % of the Wide&Deep step was that ATen glue.
// One thread per 16-byte piece of the output row; a block covers whole rows.
#include "common.h"

namespace {

// x row b, piece j (8 bf16): j < Dp/8 from dense, else from rows
__global__ __launch_bounds__(256) void wd_input_fwd(const bf16_t* __restrict__ rows, const float* __restrict__ dense,
                                                    bf16_t* __restrict__ x, float* __restrict__ wide, int B, int F,
                                                    int E, int Dp) {
  const int RW = E + 8;                   // row width in elements
  const int pcs = (Dp + F * E) / 8;       // 16-B pieces per x row
  const long total = (long)B * pcs;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += (long)gridDim.x * blockDim.x) {
    const int b = (int)(v / pcs), j = (int)(v - (long)b * pcs);
    uint4 o;
    if (j < Dp / 8) {
      const float4 a = *reinterpret_cast<const float4*>(dense + (long)b * Dp + j * 8);
      const float4 c = *reinterpret_cast<const float4*>(dense + (long)b * Dp + j * 8 + 4);
      const float f[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
      o = pack8(f);
    } else {
      const int e = (j - Dp / 8) * 8, f = e / E, k = e - f * E;
      o = *reinterpret_cast<const uint4*>(rows + ((long)b * F + f) * RW + k);
    }
    *reinterpret_cast<uint4*>(x + (long)b * (Dp + F * E) + j * 8) = o;
  }
  // wide sums: one thread per example
  for (long b = (long)blockIdx.x * blockDim.x + threadIdx.x; b < B; b += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int f = 0; f < F; f++) s += bf2f(rows[(b * F + f) * RW + E]);
    wide[b] = s;
  }
}

// drows row (b, f), piece j of E/8 + 1: deep pieces from dx, the last = [dwide, 0 x 7]
__global__ __launch_bounds__(256) void wd_input_bwd(const bf16_t* __restrict__ dx, const float* __restrict__ dwide,
                                                    bf16_t* __restrict__ drows, int B, int F, int E, int Dp) {
  const int RW = E + 8, pcs = RW / 8;
  const long total = (long)B * F * pcs;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += (long)gridDim.x * blockDim.x) {
    const long r = v / pcs;
    const int j = (int)(v - r * pcs);
    const int b = (int)(r / F), f = (int)(r - (long)b * F);
    uint4 o;
    if (j < E / 8) {
      o = *reinterpret_cast<const uint4*>(dx + (long)b * (Dp + F * E) + Dp + f * E + j * 8);
    } else {
      const float g[8] = {dwide[b], 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      o = pack8(g);
    }
    *reinterpret_cast<uint4*>(drows + r * RW + j * 8) = o;
  }
}

// ---- output head + loss (the deep tower's 1-wide projection, the wide linear
// over the dense features, sigmoid cross-entropy), forward and backward in one
// pass each (+ a deterministic reduction of per-block partials), replacing two
// GEMV-shaped hipBLASLt calls per direction and the ATen loss chain (~0.3 ms of
// the 2.4 ms W&D step on hipBLASLt / ATen, profiles/r4_wide_deep_b65536_head.md).
//   z_b    = x_b . w + out_b + wide_b + dpad_b . wd
//   loss   = mean_b [ max(z, 0) - z y + log1p(exp(-|z|)) ]
//   pmy_b  = sigmoid(z_b) - y_b  (saved for the backward)
// Backward with g_b = dloss * pmy_b / B:
//   dx_b = g_b w (bf16), dwide_b = g_b, dw = sum_b g_b x_b, dwd = sum_b g_b dpad_b, db = sum_b g_b
// One 32-lane half-wave per row (H / 8 16-B pieces over its lanes); per-block partials.
constexpr int kHeadRowsPerBlock = 8;  // half-waves of a 256-thread block
constexpr int kHeadMaxPieces = 2;     // H <= 512
constexpr int kHeadMaxDp = 64;

__global__ __launch_bounds__(256) void wd_head_fwd(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                                   const float* __restrict__ ob, const float* __restrict__ wide,
                                                   const float* __restrict__ dpad, const float* __restrict__ wd,
                                                   const float* __restrict__ y, float* __restrict__ pmy,
                                                   float* __restrict__ part, int B, int H, int Dp) {
  __shared__ float red[kHeadRowsPerBlock];
  const int hw = threadIdx.x >> 5, l = threadIdx.x & 31, npc = H / 8;
  float lsum = 0.f;
  for (long b = (long)blockIdx.x * kHeadRowsPerBlock + hw; b < B; b += (long)gridDim.x * kHeadRowsPerBlock) {
    float s = 0.f;
    for (int j = l; j < npc; j += 32) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + b * H + j * 8), f);
      const float4 w0 = *reinterpret_cast<const float4*>(w + j * 8), w1 = *reinterpret_cast<const float4*>(w + j * 8 + 4);
      s += f[0] * w0.x + f[1] * w0.y + f[2] * w0.z + f[3] * w0.w + f[4] * w1.x + f[5] * w1.y + f[6] * w1.z + f[7] * w1.w;
    }
    for (int j = l; j < Dp; j += 32) s += dpad[b * Dp + j] * wd[j];
#pragma unroll
    for (int o = 16; o; o >>= 1) s += __shfl_xor(s, o, 32);
    if (l == 0) {
      const float z = s + ob[0] + wide[b], yy = y[b];
      pmy[b] = 1.f / (1.f + expf(-z)) - yy;
      lsum += fmaxf(z, 0.f) - z * yy + log1pf(expf(-fabsf(z)));
    }
  }
  if (l == 0) red[hw] = lsum;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < kHeadRowsPerBlock; i++) t += red[i];
    part[blockIdx.x] = t;
  }
}

// loss[0] = sum(part[0..n)) / B in a fixed order (one block)
__global__ __launch_bounds__(256) void wd_head_loss(const float* __restrict__ part, int n, int B,
                                                    float* __restrict__ loss) {
  __shared__ float red[256];
  float t = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) t += part[i];
  red[threadIdx.x] = t;
  __syncthreads();
  for (int o = 128; o; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = red[0] / (float)B;
}

// part: [gridDim.x][H + Dp + 1] = per-block (dw | dwd | db)
__global__ __launch_bounds__(256) void wd_head_bwd(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                                   const float* __restrict__ dpad, const float* __restrict__ pmy,
                                                   const float* __restrict__ dloss, bf16_t* __restrict__ dx,
                                                   float* __restrict__ dwide, float* __restrict__ part, int B, int H,
                                                   int Dp) {
  extern __shared__ float sh[];  // [kHeadRowsPerBlock][H + Dp + 1]
  const int hw = threadIdx.x >> 5, l = threadIdx.x & 31, npc = H / 8, W = H + Dp + 1;
  const float gs = dloss[0] / (float)B;
  float acc[kHeadMaxPieces][8] = {}, dacc[kHeadMaxDp / 32] = {}, bacc = 0.f;
  float wr[kHeadMaxPieces][8];
#pragma unroll
  for (int q = 0; q < kHeadMaxPieces; q++) {
    const int j = l + 32 * q;
#pragma unroll
    for (int e = 0; e < 8; e++) wr[q][e] = j < npc ? w[j * 8 + e] : 0.f;
  }
  for (long b = (long)blockIdx.x * kHeadRowsPerBlock + hw; b < B; b += (long)gridDim.x * kHeadRowsPerBlock) {
    const float g = gs * pmy[b];
#pragma unroll
    for (int q = 0; q < kHeadMaxPieces; q++) {
      const int j = l + 32 * q;
      if (j < npc) {
        float f[8], o[8];
        unpack8(*reinterpret_cast<const uint4*>(x + b * H + j * 8), f);
#pragma unroll
        for (int e = 0; e < 8; e++) {
          acc[q][e] += g * f[e];
          o[e] = g * wr[q][e];
        }
        *reinterpret_cast<uint4*>(dx + b * H + j * 8) = pack8(o);
      }
    }
#pragma unroll
    for (int q = 0; q < kHeadMaxDp / 32; q++) {
      const int j = l + 32 * q;
      if (j < Dp) dacc[q] += g * dpad[b * Dp + j];
    }
    if (l == 0) {
      dwide[b] = g;
      bacc += g;
    }
  }
  float* mine = sh + hw * W;
#pragma unroll
  for (int q = 0; q < kHeadMaxPieces; q++) {
    const int j = l + 32 * q;
    if (j < npc)
#pragma unroll
      for (int e = 0; e < 8; e++) mine[j * 8 + e] = acc[q][e];
  }
#pragma unroll
  for (int q = 0; q < kHeadMaxDp / 32; q++) {
    const int j = l + 32 * q;
    if (j < Dp) mine[H + j] = dacc[q];
  }
  if (l == 0) mine[H + Dp] = bacc;
  __syncthreads();
  for (int c = threadIdx.x; c < W; c += 256) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < kHeadRowsPerBlock; i++) t += sh[i * W + c];
    part[(long)blockIdx.x * W + c] = t;
  }
}

// out[c] = sum over n blocks of part[blk][c] in a fixed order, c < W: block = 16
// columns x 16 row groups; thread (row group g, column) sums partial rows g, g+16,
// ... and the 16 group sums meet in LDS in group order (a single thread per column
// walking all n partials was 235 us: n dependent loads)
__global__ __launch_bounds__(256) void wd_head_reduce(const float* __restrict__ part, int n, int W,
                                                      float* __restrict__ out) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float t = 0.f;
  if (c < W)
    for (int i = g; i < n; i += 16) t += part[(long)i * W + c];
  red[g][cl] = t;
  __syncthreads();
  if (g == 0 && c < W) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; k++) s += red[k][cl];
    out[c] = s;
  }
}

// blocks of the head kernels: 8 rows per block-iteration, at most 256 blocks (the
// backward's partial rows: 256 x (H + Dp + 1) floats)
int head_blocks(int B) {
  const int b = (B + kHeadRowsPerBlock - 1) / kHeadRowsPerBlock;
  return b < 256 ? b : 256;
}

int blocks_for(long n) {
  const long b = (n + 255) / 256;
  return (int)(b < 8192 ? (b < 1 ? 1 : b) : 8192);
}

}  // namespace

// E % 8 == 0, Dp % 8 == 0; all pointers 16-B aligned (checked by the caller)
KFA_API int kfa_wd_input_fwd(const bf16_t* rows, const float* dense, bf16_t* x, float* wide, int B, int F, int E,
                             int Dp, hipStream_t st) {
  if (E % 8 || Dp % 8 || B <= 0) return -1;
  hipLaunchKernelGGL(wd_input_fwd, dim3(blocks_for((long)B * ((Dp + F * E) / 8))), dim3(256), 0, st, rows, dense, x,
                     wide, B, F, E, Dp);
  return kfa_status();
}

// blocks of the head kernels for B rows (the partial buffers hold this many rows)
KFA_API int kfa_wd_head_blocks(int B) { return head_blocks(B); }

// H % 8 == 0, H <= 512, Dp <= 64; x / dx 16-B aligned rows; part: head_blocks(B) floats;
// loss: one float (written); pmy: B floats (written, for the backward)
KFA_API int kfa_wd_head_fwd(const bf16_t* x, const float* w, const float* ob, const float* wide, const float* dpad,
                            const float* wd, const float* y, float* pmy, float* part, float* loss, int B, int H, int Dp,
                            hipStream_t st) {
  if (B <= 0 || H % 8 || H > 8 * 32 * kHeadMaxPieces || Dp < 0 || Dp > kHeadMaxDp) return -1;
  const int nb = head_blocks(B);
  hipLaunchKernelGGL(wd_head_fwd, dim3(nb), dim3(256), 0, st, x, w, ob, wide, dpad, wd, y, pmy, part, B, H, Dp);
  hipLaunchKernelGGL(wd_head_loss, dim3(1), dim3(256), 0, st, part, nb, B, loss);
  return kfa_status();
}

// part: head_blocks(B) * (H + Dp + 1) floats of scratch; grads: H + Dp + 1 floats (dw | dwd | db)
KFA_API int kfa_wd_head_bwd(const bf16_t* x, const float* w, const float* dpad, const float* pmy, const float* dloss,
                            bf16_t* dx, float* dwide, float* part, float* grads, int B, int H, int Dp, hipStream_t st) {
  if (B <= 0 || H % 8 || H > 8 * 32 * kHeadMaxPieces || Dp < 0 || Dp > kHeadMaxDp) return -1;
  const int nb = head_blocks(B), W = H + Dp + 1;
  hipLaunchKernelGGL(wd_head_bwd, dim3(nb), dim3(256), kHeadRowsPerBlock * W * 4, st, x, w, dpad, pmy, dloss, dx,
                     dwide, part, B, H, Dp);
  hipLaunchKernelGGL(wd_head_reduce, dim3((W + 15) / 16), dim3(256), 0, st, part, nb, W, grads);
  return kfa_status();
}

KFA_API int kfa_wd_input_bwd(const bf16_t* dx, const float* dwide, bf16_t* drows, int B, int F, int E, int Dp,
                             hipStream_t st) {
  if (E % 8 || Dp % 8 || B <= 0) return -1;
  hipLaunchKernelGGL(wd_input_bwd, dim3(blocks_for((long)B * F * ((E + 8) / 8))), dim3(256), 0, st, dx, dwide, drows,
                     B, F, E, Dp);
  return kfa_status();
}
