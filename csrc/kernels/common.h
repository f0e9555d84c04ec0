// Shared helpers for the CDNA4 (gfx950) kernels of kubeflow_controller_amd.
// bf16 is carried as raw uint16 bits so every kernel controls its own
// vector width (16 B per lane loads, cdna_hip_programming.md Guideline 13).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define KFA_API extern "C" __attribute__((visibility("default")))

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) short short8;   // 8 x bf16 MFMA operand
typedef __attribute__((ext_vector_type(4))) float floatx4;
typedef __attribute__((ext_vector_type(16))) float floatx16;

__device__ __forceinline__ float bf2f(uint32_t b) { return __uint_as_float(b << 16); }

// float -> bf16, round to nearest even, NaN kept quiet: gfx950's v_cvt_pk_bf16_f32
// (one VALU op per PAIR — the integer rounding sequence it replaces took ~7 per element,
// a visible share of the VALU-bound attention kernels, profiles/pmc/r4_attention.md)
typedef __attribute__((ext_vector_type(2))) __bf16 kfa_bf16x2_t;
typedef __attribute__((ext_vector_type(2))) float kfa_floatx2_t;

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  const kfa_floatx2_t f = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, kfa_bf16x2_t));
}

__device__ __forceinline__ uint32_t f2bf(float f) { return pack2(f, 0.f) & 0xffffu; }

// unpack a 16-byte vector of 8 bf16 into floats
__device__ __forceinline__ void unpack8(const uint4 v, float f[8]) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint4 pack8(const float f[8]) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// GELU for bf16-rounded outputs: erf by Abramowitz & Stegun 7.1.26 (|error| <=
// 1.5e-7, far below bf16's 2^-8 relative step) from one v_rcp + one v_exp + a
// degree-5 Horner chain, instead of the library erff (~3x the VALU work: the
// GEMM epilogue runs it on every output element).  gelu_grad shares the
// exponential between the CDF and the density:  x = z/sqrt2, E = exp(-x^2),
//   gelu(z) = z/2 (1 + erf x),   gelu'(z) = (1 + erf x)/2 + z E / sqrt(2 pi).
__device__ __forceinline__ float erf_as(float x, float& e) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.f));
  e = __expf(-a * a);
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
  return copysignf(1.f - poly * e, x);
}
__device__ __forceinline__ float gelu_f(float z) {
  float e;
  return 0.5f * z * (1.f + erf_as(z * 0.70710678118654752f, e));
}
__device__ __forceinline__ float gelu_grad(float z) {
  float e;
  const float cdf = 0.5f * (1.f + erf_as(z * 0.70710678118654752f, e));
  return fmaf(z * 0.39894228040143268f, e, cdf);
}

// Dropout counter hash: keep element i under a (well-mixed, per-launch) 64-bit
// seed iff drop_hash(seed, i) >= p * 2^32, so forward and backward regenerate
// the same mask from (seed, index) and no mask is ever stored.  The seed folds
// into the index with wave-uniform keys and each element costs one 32-bit
// integer finaliser (lowbias32: two 32-bit multiplies, ~12 VALU) — the
// splitmix64 finaliser used before took three 64-bit multiplies (~70 VALU
// slots) and made the dropout hash the largest cost of the attention, LayerNorm
// and hidden-dropout kernels (BERT-base: 100M+ hashed elements per layer).
__device__ __forceinline__ uint32_t drop_hash(uint64_t seed, uint64_t i) {
  uint32_t x = ((uint32_t)i ^ (uint32_t)seed) + (uint32_t)(seed >> 32) + __umul24((uint32_t)(i >> 32), 0x9E3779u);
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

static inline int kfa_status() { return (int)hipGetLastError(); }

static inline int kfa_ceil_div(long a, long b) { return (int)((a + b - 1) / b); }
