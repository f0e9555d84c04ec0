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

KFA_API int kfa_wd_input_bwd(const bf16_t* dx, const float* dwide, bf16_t* drows, int B, int F, int E, int Dp,
                             hipStream_t st) {
  if (E % 8 || Dp % 8 || B <= 0) return -1;
  hipLaunchKernelGGL(wd_input_bwd, dim3(blocks_for((long)B * F * ((E + 8) / 8))), dim3(256), 0, st, dx, dwide, drows,
                     B, F, E, Dp);
  return kfa_status();
}
