// Wide & Deep input assembly (SURVEY §2.6 K6 around the sharded lookup):
//
//   forward:  rows [B][F][E+8] bf16 (deep features, then the wide weight, then pad)
//             dense [B][Dn] fp32, Dn <= Dp (zero-padded here to Dp % 8 == 0 columns)
//          -> x    [B][Dp + F*E] bf16 = [bf16(dense | 0) | rows[:, :, :E] flattened]
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
                                                    int E, int Dp, int Dn) {
  const int RW = E + 8;                   // row width in elements
  const int pcs = (Dp + F * E) / 8;       // 16-B pieces per x row
  const long total = (long)B * pcs;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += (long)gridDim.x * blockDim.x) {
    const int b = (int)(v / pcs), j = (int)(v - (long)b * pcs);
    uint4 o;
    if (j < Dp / 8) {  // the raw dense row (Dn wide, any alignment), zero beyond Dn
      float f[8];
#pragma unroll
      for (int k = 0; k < 8; k++) f[k] = j * 8 + k < Dn ? dense[(long)b * Dn + j * 8 + k] : 0.f;
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

// The lookup and the assembly in one pass (world 1: every table row is local): x row b,
// piece j from the raw dense features (j < Dp/8) or straight from the fp32 table row
// gid[b*F + f] (rounded to bf16, as the lookup's bf16 output would be); wide[b] = the
// sum over f of bf16(table[gid][E]) in f order — bit-equal to kfa_embed_fwd +
// kfa_wd_input_fwd without the [B*F, E+8] bf16 rows round trip through HBM.
__global__ __launch_bounds__(256) void wd_gather_fwd(const long* __restrict__ gid, const long* __restrict__ offs,
                                                     const float* __restrict__ table,
                                                     const float* __restrict__ dense, bf16_t* __restrict__ x,
                                                     float* __restrict__ wide, int B, int F, int E, int Dp, int Dn) {
  const int RW = E + 8;
  const int pcs = (Dp + F * E) / 8;
  const long total = (long)B * pcs;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += (long)gridDim.x * blockDim.x) {
    const int b = (int)(v / pcs), j = (int)(v - (long)b * pcs);
    float f8[8];
    if (j < Dp / 8) {
#pragma unroll
      for (int k = 0; k < 8; k++) f8[k] = j * 8 + k < Dn ? dense[(long)b * Dn + j * 8 + k] : 0.f;
    } else {
      const int e = (j - Dp / 8) * 8, f = e / E, k = e - f * E;
      const float* src = table + (gid[(long)b * F + f] + (offs ? offs[f] : 0)) * RW + k;
      const float4 a = *reinterpret_cast<const float4*>(src), c = *reinterpret_cast<const float4*>(src + 4);
      f8[0] = a.x; f8[1] = a.y; f8[2] = a.z; f8[3] = a.w; f8[4] = c.x; f8[5] = c.y; f8[6] = c.z; f8[7] = c.w;
    }
    *reinterpret_cast<uint4*>(x + (long)b * (Dp + F * E) + j * 8) = pack8(f8);
  }
  for (long b = (long)blockIdx.x * blockDim.x + threadIdx.x; b < B; b += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int f = 0; f < F; f++) s += bf2f(f2bf(table[(gid[b * F + f] + (offs ? offs[f] : 0)) * RW + E]));
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

// The head's weights (w [H], wd [>= Dn]) are read in the parameters' own dtype
// (WBF: bf16, the flat-buffer compute copy; else fp32) and the labels as int64
// or fp32 (yint), the dense features raw ([B][Dn]): no cast / pad kernels before it.
template <bool WBF>
__device__ __forceinline__ void head_w8(const void* w, int j, float* o) {
  if (WBF) {
    unpack8(*reinterpret_cast<const uint4*>(static_cast<const bf16_t*>(w) + j * 8), o);
  } else {
    const float4 a = *reinterpret_cast<const float4*>(static_cast<const float*>(w) + j * 8);
    const float4 c = *reinterpret_cast<const float4*>(static_cast<const float*>(w) + j * 8 + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = c.x; o[5] = c.y; o[6] = c.z; o[7] = c.w;
  }
}

template <bool WBF>
__device__ __forceinline__ float head_w1(const void* w, int j) {
  return WBF ? bf2f(static_cast<const bf16_t*>(w)[j]) : static_cast<const float*>(w)[j];
}

template <bool WBF>
__global__ __launch_bounds__(256) void wd_head_fwd(const bf16_t* __restrict__ x, const void* __restrict__ w,
                                                   const float* __restrict__ ob, const float* __restrict__ wide,
                                                   const float* __restrict__ dense, const void* __restrict__ wd,
                                                   const void* __restrict__ y, int yint, float* __restrict__ pmy,
                                                   float* __restrict__ part, int B, int H, int Dn) {
  __shared__ float red[kHeadRowsPerBlock];
  const int hw = threadIdx.x >> 5, l = threadIdx.x & 31, npc = H / 8;
  float lsum = 0.f;
  for (long b = (long)blockIdx.x * kHeadRowsPerBlock + hw; b < B; b += (long)gridDim.x * kHeadRowsPerBlock) {
    float s = 0.f;
    for (int j = l; j < npc; j += 32) {
      float f[8], wv[8];
      unpack8(*reinterpret_cast<const uint4*>(x + b * H + j * 8), f);
      head_w8<WBF>(w, j, wv);
#pragma unroll
      for (int e = 0; e < 8; e++) s += f[e] * wv[e];
    }
    for (int j = l; j < Dn; j += 32) s += dense[b * Dn + j] * head_w1<WBF>(wd, j);
#pragma unroll
    for (int o = 16; o; o >>= 1) s += __shfl_xor(s, o, 32);
    if (l == 0) {
      const float yy = yint ? (float)static_cast<const long*>(y)[b] : static_cast<const float*>(y)[b];
      const float z = s + ob[0] + wide[b];
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

// part: [gridDim.x][H + Dn + 1] = per-block (dw | dwd | db)
template <bool WBF>
__global__ __launch_bounds__(256) void wd_head_bwd(const bf16_t* __restrict__ x, const void* __restrict__ w,
                                                   const float* __restrict__ dense, const float* __restrict__ pmy,
                                                   const float* __restrict__ dloss, bf16_t* __restrict__ dx,
                                                   float* __restrict__ dwide, float* __restrict__ part, int B, int H,
                                                   int Dn) {
  extern __shared__ float sh[];  // [kHeadRowsPerBlock][H + Dn + 1]
  const int hw = threadIdx.x >> 5, l = threadIdx.x & 31, npc = H / 8, W = H + Dn + 1;
  const float gs = dloss[0] / (float)B;
  float acc[kHeadMaxPieces][8] = {}, dacc[kHeadMaxDp / 32] = {}, bacc = 0.f;
  float wr[kHeadMaxPieces][8];
#pragma unroll
  for (int q = 0; q < kHeadMaxPieces; q++) {
    const int j = l + 32 * q;
    if (j < npc) {
      head_w8<WBF>(w, j, wr[q]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; e++) wr[q][e] = 0.f;
    }
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
      if (j < Dn) dacc[q] += g * dense[b * Dn + j];
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
    if (j < Dn) mine[H + j] = dacc[q];
  }
  if (l == 0) mine[H + Dn] = bacc;
  __syncthreads();
  for (int c = threadIdx.x; c < W; c += 256) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < kHeadRowsPerBlock; i++) t += sh[i * W + c];
    part[(long)blockIdx.x * W + c] = t;
  }
}

// Sum over n blocks of part[blk][pc] in a fixed order for output column c < H + Dp + 1
// (dw | dwd padded to Dp | db; part holds H + Dn + 1 columns, the pad columns are 0):
// block = 16 columns x 16 row groups; thread (row group g, column) sums partial rows
// g, g+16, ... and the 16 group sums meet in LDS in group order (a single thread per
// column walking all n partials was 235 us: n dependent loads).
// Direct mode (gw != nullptr): the sums are ADDED into the parameters' own gradient
// buffers — gw [H] and gwd [Dp] in the weights' dtype (WBF: bf16), gb [1] fp32 — the
// flat-buffer views the optimizer reads (parallel/flat.py direct-gradient protocol):
// no fp32 -> bf16 casts and no autograd accumulate kernels after the head.
template <bool WBF>
__global__ __launch_bounds__(256) void wd_head_reduce(const float* __restrict__ part, int n, int H, int Dn, int Dp,
                                                      float* __restrict__ out, void* __restrict__ gw,
                                                      void* __restrict__ gwd, float* __restrict__ gb) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl, Wp = H + Dn + 1, Wo = H + Dp + 1;
  const int pc = c < H + Dn ? c : (c < H + Dp ? -1 : H + Dn);  // -1: a pad column (sum 0)
  float t = 0.f;
  if (c < Wo && pc >= 0)
    for (int i = g; i < n; i += 16) t += part[(long)i * Wp + pc];
  red[g][cl] = t;
  __syncthreads();
  if (g == 0 && c < Wo) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; k++) s += red[k][cl];
    if (gw == nullptr) {
      out[c] = s;
    } else if (c == H + Dp) {
      gb[0] += s;
    } else {
      void* dst = c < H ? gw : gwd;
      const int i = c < H ? c : c - H;
      if (WBF) {
        bf16_t* p = static_cast<bf16_t*>(dst) + i;
        *p = f2bf(bf2f(*p) + s);
      } else {
        static_cast<float*>(dst)[i] += s;
      }
    }
  }
}

// blocks of the head backward: 8 rows per block-iteration, at most 512 blocks (the partial
// rows: 512 x (H + Dp + 1) floats; 256 / 512 / 1024 measured 34.79-34.97 / 35.00-35.03 /
// 35.03 M ex/s on W&D, tools/gpu_r6_wdheadb.sh)
int head_blocks(int B) {
  static int cap = -1;  // KFA_WD_HEAD_BWD_BLOCKS: A/B knob
  if (cap < 0) {
    const char* e = getenv("KFA_WD_HEAD_BWD_BLOCKS");
    cap = (e && atoi(e) > 0) ? atoi(e) : 512;
  }
  const int b = (B + kHeadRowsPerBlock - 1) / kHeadRowsPerBlock;
  return b < cap ? b : cap;
}

// the forward keeps one partial float per block: up to 2048 blocks (8 per CU), so each
// half-wave walks 4 rows at B = 65536 instead of 32 — its x rows come from HBM when the
// producing GEMM stored them non-temporally, and 256 blocks left that latency exposed
int head_fwd_blocks(int B) {
  static int cap = -1;  // KFA_WD_HEAD_FWD_BLOCKS: A/B knob (256 = the backward's grid)
  if (cap < 0) {
    const char* e = getenv("KFA_WD_HEAD_FWD_BLOCKS");
    cap = (e && atoi(e) > 0) ? atoi(e) : 2048;
  }
  const int b = (B + kHeadRowsPerBlock - 1) / kHeadRowsPerBlock;
  return b < cap ? b : cap;
}

int blocks_for(long n) {
  const long b = (n + 255) / 256;
  return (int)(b < 8192 ? (b < 1 ? 1 : b) : 8192);
}

}  // namespace

// E % 8 == 0, Dp % 8 == 0, 0 <= Dn <= Dp; rows / x 16-B aligned (checked by the caller);
// dense: [B][Dn] fp32, contiguous
KFA_API int kfa_wd_input_fwd(const bf16_t* rows, const float* dense, bf16_t* x, float* wide, int B, int F, int E,
                             int Dp, int Dn, hipStream_t st) {
  if (E % 8 || Dp % 8 || B <= 0 || Dn < 0 || Dn > Dp) return -1;
  hipLaunchKernelGGL(wd_input_fwd, dim3(blocks_for((long)B * ((Dp + F * E) / 8))), dim3(256), 0, st, rows, dense, x,
                     wide, B, F, E, Dp, Dn);
  return kfa_status();
}

// blocks of the head kernels for B rows (the partial buffers hold this many rows)
KFA_API int kfa_wd_head_blocks(int B) { return head_blocks(B); }
KFA_API int kfa_wd_head_fwd_blocks(int B) { return head_fwd_blocks(B); }

// H % 8 == 0, H <= 512, Dn <= 64; x / dx 16-B aligned rows, w 16-B aligned; wbf: w / wd
// are bf16 (else fp32); y: B labels, int64 (yint) or fp32; dense: [B][Dn] fp32; part:
// head_fwd_blocks(B) floats; loss: one float (written); pmy: B floats (written, for the backward)
KFA_API int kfa_wd_head_fwd(const bf16_t* x, const void* w, const float* ob, const float* wide, const float* dense,
                            const void* wd, const void* y, int yint, int wbf, float* pmy, float* part, float* loss,
                            int B, int H, int Dn, hipStream_t st) {
  if (B <= 0 || H % 8 || H > 8 * 32 * kHeadMaxPieces || Dn < 0 || Dn > kHeadMaxDp) return -1;
  const int nb = head_fwd_blocks(B);
  if (wbf)
    hipLaunchKernelGGL(wd_head_fwd<true>, dim3(nb), dim3(256), 0, st, x, w, ob, wide, dense, wd, y, yint, pmy, part, B,
                       H, Dn);
  else
    hipLaunchKernelGGL(wd_head_fwd<false>, dim3(nb), dim3(256), 0, st, x, w, ob, wide, dense, wd, y, yint, pmy, part,
                       B, H, Dn);
  hipLaunchKernelGGL(wd_head_loss, dim3(1), dim3(256), 0, st, part, nb, B, loss);
  return kfa_status();
}

// part: head_blocks(B) * (H + Dn + 1) floats of scratch.  Either grads: H + Dp + 1 floats
// (dw | dwd | db, written), or gw / gwd / gb: the parameters' gradient buffers (dw, dwd
// in the weights' dtype, db fp32), added to in place; Dn <= Dp
KFA_API int kfa_wd_head_bwd(const bf16_t* x, const void* w, const float* dense, const float* pmy, const float* dloss,
                            bf16_t* dx, float* dwide, float* part, float* grads, void* gw, void* gwd, float* gb,
                            int wbf, int B, int H, int Dn, int Dp, hipStream_t st) {
  if (B <= 0 || H % 8 || H > 8 * 32 * kHeadMaxPieces || Dn < 0 || Dn > Dp || Dp > kHeadMaxDp) return -1;
  if (gw ? (!gwd || !gb) : !grads) return -1;
  const int nb = head_blocks(B), W = H + Dn + 1;
  const int nblk = (H + Dp + 1 + 15) / 16;
  if (wbf) {
    hipLaunchKernelGGL(wd_head_bwd<true>, dim3(nb), dim3(256), kHeadRowsPerBlock * W * 4, st, x, w, dense, pmy, dloss,
                       dx, dwide, part, B, H, Dn);
    hipLaunchKernelGGL(wd_head_reduce<true>, dim3(nblk), dim3(256), 0, st, part, nb, H, Dn, Dp, grads, gw, gwd, gb);
  } else {
    hipLaunchKernelGGL(wd_head_bwd<false>, dim3(nb), dim3(256), kHeadRowsPerBlock * W * 4, st, x, w, dense, pmy, dloss,
                       dx, dwide, part, B, H, Dn);
    hipLaunchKernelGGL(wd_head_reduce<false>, dim3(nblk), dim3(256), 0, st, part, nb, H, Dn, Dp, grads, gw, gwd, gb);
  }
  return kfa_status();
}

// table: fp32 [rows][E + 8] (16-B aligned rows: E % 8 == 0), gid: B*F int64 rows of it
// (+ offs[f], nullable: per-feature table offsets for per-table ids); dense [B][Dn] fp32,
// Dn <= Dp, Dp % 8 == 0; x 16-B aligned
KFA_API int kfa_wd_gather_fwd(const long* gid, const long* offs, const float* table, const float* dense, bf16_t* x,
                              float* wide, int B, int F, int E, int Dp, int Dn, hipStream_t st) {
  if (E % 8 || Dp % 8 || B <= 0 || Dn < 0 || Dn > Dp) return -1;
  hipLaunchKernelGGL(wd_gather_fwd, dim3(blocks_for((long)B * ((Dp + F * E) / 8))), dim3(256), 0, st, gid, offs,
                     table, dense, x, wide, B, F, E, Dp, Dn);
  return kfa_status();
}

KFA_API int kfa_wd_input_bwd(const bf16_t* dx, const float* dwide, bf16_t* drows, int B, int F, int E, int Dp,
                             hipStream_t st) {
  if (E % 8 || Dp % 8 || B <= 0) return -1;
  hipLaunchKernelGGL(wd_input_bwd, dim3(blocks_for((long)B * F * ((E + 8) / 8))), dim3(256), 0, st, dx, dwide, drows,
                     B, F, E, Dp);
  return kfa_status();
}
