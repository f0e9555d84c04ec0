// Segment-reduce sparse optimizer for the row-sharded embedding tables
// (Wide&Deep PS owners; reference semantics: the PS's
// sparse apply of mnist_replica.py:184,256 on looked-up rows only).
//
// The atomic path (sparse.hip) adds every (row, D-vector) gradient into a
// table-sized fp32 scratch and then hands each element to one occurrence by an
// atomic exchange: 2 x n x D atomics per step and a 4*rows*D-byte scratch.
// Here the step's ids are SORTED instead, so all occurrences of a row sit next
// to each other and one workgroup can sum them without atomics:
//
//   1. ids -> u32 keys + positions, radix-sorted on the low ``nbits`` bits
//      (radix_sort.h: own LSD passes; the table's row count bounds the key width);
//   2. per 64-entry chunk of the sorted list: the last segment head in the chunk;
//   3. exclusive max-scan over the chunks (radix_sort.h) -> start of the segment
//      that spans each chunk's first entry;
//   4. per chunk: gather its 64 gradient rows (bf16, by position) into LDS, sum
//      each segment in fp32 (segmented wave scan) and apply Adam / SGD to that row of the master table
//      and its moments.  A segment that crosses a chunk edge (hot rows span many
//      chunks under the power-law ids) is pre-reduced in the chunk and added
//      with D atomics to the slot of the chunk it starts in;
//   5. per chunk whose last segment starts in it and crosses its end: apply the
//      slot (and zero it: the [chunks, D] slot buffer is self-cleaning).
//
// Elements whose summed gradient is exactly 0 are left untouched (lazy Adam,
// same as the atomic path and ShardedEmbedding._apply_cpu).
#include "common.h"

#include "radix_sort.h"

namespace {

constexpr int CH = 64;   // sorted entries per chunk (one wave of keys)
constexpr int MAXD = 248;  // CH x (D + 4) fp32 rows in LDS: 64 KB at most

struct OptP {
  float lr, b1, b2, eps, wd, c1, c2, gscale;
};

// Where seg_apply_kernel reads entry r's gradient row: g [n][D] bf16 (dx == nullptr), or
// (the Wide&Deep lookup, r = b * F + f) straight from the MLP input gradient dx [B][XW]
// bf16 — row r's first E columns at dx[b][Dp + f E ...] — then bf16(dwide[b]) and zeros:
// the [n][E + 8] rows kfa_wd_input_bwd would materialise, without the HBM round trip.
struct WdSrc {
  const bf16_t* dx;
  const float* dwide;
  int F, E, Dp, XW;
};

// keys = ids (+ offs[i % F]: per-feature table offsets, so a caller holding [B][F]
// per-table ids needs no separate global-row pass), pos = identity
__global__ __launch_bounds__(256) void seg_prep_kernel(const long* __restrict__ ids, const long* __restrict__ offs,
                                                       int F, unsigned* __restrict__ keys, int* __restrict__ pos, int n) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    keys[i] = (unsigned)(ids[i] + (offs ? offs[i % F] : 0));
    pos[i] = i;
  }
}

// lh[c] = sorted position of the last segment head inside chunk c, or -1
__global__ __launch_bounds__(256) void seg_heads_kernel(const unsigned* __restrict__ sk, int* __restrict__ lh, int n,
                                                        int nch) {
  const int lane = threadIdx.x & 63;
  for (int c = blockIdx.x * 4 + (threadIdx.x >> 6); c < nch; c += gridDim.x * 4) {
    const int i = c * CH + lane;
    bool head = false;
    if (i < n) head = (i == 0) || sk[i] != sk[i - 1];
    const unsigned long long mask = __ballot(head);
    if (lane == 0) lh[c] = mask ? c * CH + 63 - __clzll(mask) : -1;
  }
}

// optimizer on 4 consecutive elements of one table row (one float4 of w, m, v)
template <int OPT>
__device__ __forceinline__ void apply4(float* __restrict__ w, float* __restrict__ m, float* __restrict__ v, long e0,
                                       const float4 g4, const OptP& p) {
  const float g[4] = {g4.x, g4.y, g4.z, g4.w};
  float4* w4 = reinterpret_cast<float4*>(w + e0);
  float wr[4];
  *reinterpret_cast<float4*>(wr) = *w4;
  if (OPT == 0) {
    float4* m4 = reinterpret_cast<float4*>(m + e0);
    float4* v4 = reinterpret_cast<float4*>(v + e0);
    float mr[4], vr[4];
    *reinterpret_cast<float4*>(mr) = *m4;
    *reinterpret_cast<float4*>(vr) = *v4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (g[i] == 0.f) continue;
      const float gi = g[i] * p.gscale;
      mr[i] = p.b1 * mr[i] + (1.f - p.b1) * gi;
      vr[i] = p.b2 * vr[i] + (1.f - p.b2) * gi * gi;
      const float upd = (mr[i] * p.c1) / (sqrtf(vr[i] * p.c2) + p.eps) + p.wd * wr[i];
      wr[i] -= p.lr * upd;
    }
    *m4 = *reinterpret_cast<float4*>(mr);
    *v4 = *reinterpret_cast<float4*>(vr);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (g[i] != 0.f) wr[i] -= p.lr * g[i] * p.gscale;
  }
  *w4 = *reinterpret_cast<float4*>(wr);
}

// One chunk of CH sorted entries per workgroup.  The gradient rows are gathered
// into LDS (consecutive threads read consecutive 16-byte pieces of a row); then
// for each 8-column slice a wave holds one entry per lane and runs a segmented
// inclusive scan across its lanes (head flags from a ballot over the keys), so
// the last lane of every segment ends up with that segment's fp32 sum - hot rows
// that fill the whole chunk reduce in log2(64) shuffle steps, not 64 serial adds.
// The sums go back to LDS (over the segment's first row) and the optimizer pass
// maps consecutive threads to consecutive 16-byte pieces of one table row, so
// the w / m / v read-modify-writes stay coalesced per row.
template <int OPT>
__global__ __launch_bounds__(256) void seg_apply_kernel(const unsigned* __restrict__ sk, const int* __restrict__ pos,
                                                        const bf16_t* __restrict__ g, const int* __restrict__ segbeg,
                                                        float* __restrict__ slots, float* __restrict__ w,
                                                        float* __restrict__ m, float* __restrict__ v, int n, int D,
                                                        OptP p, WdSrc ws) {
  extern __shared__ float rows[];   // [CH][D + 4] fp32 (row padding spreads the lanes' LDS banks)
  __shared__ int sstart[CH + 1];
  __shared__ unsigned skey[CH];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int c = blockIdx.x;
  const int c0 = c * CH;
  const int cnt = min(CH, n - c0);
  const int V = D >> 3, RS = D + 4;
  for (int it = t; it < cnt * V; it += 256) {
    const int e = it / V, vv = it - e * V;
    float f[8];
    if (ws.dx == nullptr) {
      const uint4 q = *reinterpret_cast<const uint4*>(g + (long)pos[c0 + e] * D + vv * 8);
      unpack8(q, f);
    } else {
      const int r = pos[c0 + e], b = r / ws.F, fi = r - b * ws.F;
      if (vv * 8 < ws.E) {
        unpack8(*reinterpret_cast<const uint4*>(ws.dx + (long)b * ws.XW + ws.Dp + fi * ws.E + vv * 8), f);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = 0.f;
        if (vv * 8 == ws.E) f[0] = bf2f(f2bf(ws.dwide[b]));
      }
    }
    float4* dst = reinterpret_cast<float4*>(rows + e * RS + vv * 8);
    dst[0] = make_float4(f[0], f[1], f[2], f[3]);
    dst[1] = make_float4(f[4], f[5], f[6], f[7]);
  }
  // segment structure of the chunk (every wave derives it from the same 64 keys)
  const bool in = lane < cnt;
  const unsigned k = in ? sk[c0 + lane] : 0u;
  const unsigned kp = __shfl_up(k, 1);
  const bool head = in && (lane == 0 || k != kp);
  const unsigned long long mask = __ballot(head);
  const unsigned long long upto = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1ull);
  const int sbeg = 63 - __clzll(mask & upto);          // first lane of this lane's segment
  const bool tail = in && (lane == cnt - 1 || ((mask >> (lane + 1)) & 1ull));
  const int nseg = __popcll(mask);
  if (wv == 0) {
    if (head) sstart[__popcll(mask & upto) - 1] = lane;
    if (in) skey[lane] = k;
    if (lane == 0) sstart[nseg] = cnt;
  }
  __syncthreads();
  for (int vv = wv; vv < V; vv += 4) {
    float x[8];
    if (in) {
      const float4* src = reinterpret_cast<const float4*>(rows + lane * RS + vv * 8);
      *reinterpret_cast<float4*>(x) = src[0];
      *reinterpret_cast<float4*>(x + 4) = src[1];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = 0.f;
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const bool take = lane - d >= sbeg;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float y = __shfl_up(x[i], d);
        if (take) x[i] += y;
      }
    }
    if (tail && lane != sbeg) {   // segment sum over its first row (a wave only touches its own slice)
      float4* dst = reinterpret_cast<float4*>(rows + sbeg * RS + vv * 8);
      dst[0] = *reinterpret_cast<float4*>(x);
      dst[1] = *reinterpret_cast<float4*>(x + 4);
    }
  }
  __syncthreads();
  const bool cont_prev = c0 > 0 && sk[c0 - 1] == skey[0];
  const bool cont_next = c0 + cnt < n && sk[c0 + cnt] == skey[cnt - 1];
  const int Q = D >> 2;   // float4 pieces per row: consecutive threads, consecutive 16 bytes of one row
  for (int it = t; it < nseg * Q; it += 256) {
    const int s = it / Q, q = it - s * Q;
    const int b = sstart[s];
    const float4 x = *reinterpret_cast<const float4*>(rows + b * RS + q * 4);
    const bool first_cross = s == 0 && cont_prev;
    const bool last_cross = s == nseg - 1 && cont_next;
    if (!first_cross && !last_cross) {
      apply4<OPT>(w, m, v, (long)skey[b] * D + q * 4, x, p);
    } else {   // crosses a chunk edge: pre-reduced here, applied by seg_fixup_kernel
      const int start = first_cross ? segbeg[c] : c0 + b;
      float* dst = slots + (long)(start / CH) * D + q * 4;
      if (x.x != 0.f) atomicAdd(dst + 0, x.x);
      if (x.y != 0.f) atomicAdd(dst + 1, x.y);
      if (x.z != 0.f) atomicAdd(dst + 2, x.z);
      if (x.w != 0.f) atomicAdd(dst + 3, x.w);
    }
  }
}

// chunks whose last segment starts inside them and runs past their end own a slot
template <int OPT>
__global__ __launch_bounds__(256) void seg_fixup_kernel(const unsigned* __restrict__ sk, const int* __restrict__ lh,
                                                        float* __restrict__ slots, float* __restrict__ w,
                                                        float* __restrict__ m, float* __restrict__ v, int n, int nch,
                                                        int D, OptP p) {
  const int lane = threadIdx.x & 63;
  for (int c = blockIdx.x * 4 + (threadIdx.x >> 6); c < nch; c += gridDim.x * 4) {
    const int c1 = min(n, (c + 1) * CH);
    if (c1 >= n || lh[c] < 0 || sk[c1] != sk[c1 - 1]) continue;
    const long row = sk[c1 - 1];
    for (int q = lane; q < (D >> 2); q += 64) {
      float4* s4 = reinterpret_cast<float4*>(slots + (long)c * D + q * 4);
      const float4 g4 = *s4;
      *s4 = make_float4(0.f, 0.f, 0.f, 0.f);
      apply4<OPT>(w, m, v, row * D + q * 4, g4, p);
    }
  }
}

inline long align256(long x) { return (x + 255) & ~255L; }

}  // namespace

KFA_API long kfa_seg_slot_floats(long n, int D) { return ((n + CH - 1) / CH) * (long)D; }

// scratch bytes for kfa_seg_sparse_apply (the slot buffer is separate: it must stay zeroed)
KFA_API long kfa_seg_ws_bytes(long n, int nbits) {
  const long nch = (n + CH - 1) / CH;
  (void)nbits;
  return 4 * align256(n * 4) + 2 * align256(nch * 4) + kfa_radix::hist_bytes(n);
}

namespace {
struct WsLayout {
  unsigned *keys_in, *keys;
  int *pos_in, *pos, *lh, *segbeg, *hist;
};

WsLayout layout(void* ws, long n, int nbits) {
  const long nch = (n + CH - 1) / CH;
  char* p = (char*)ws;
  WsLayout L;
  L.keys_in = (unsigned*)p; p += align256(n * 4);
  L.pos_in = (int*)p;       p += align256(n * 4);
  L.keys = (unsigned*)p;    p += align256(n * 4);
  L.pos = (int*)p;          p += align256(n * 4);
  L.lh = (int*)p;           p += align256(nch * 4);
  L.segbeg = (int*)p;       p += align256(nch * 4);
  L.hist = (int*)p;
  (void)nbits;
  return L;
}

bool bad_args(long n, int nbits, long ws_bytes) {
  return n > 0x7fffffffL || nbits < 1 || nbits > 32 || ws_bytes < kfa_seg_ws_bytes(n, nbits);
}
}  // namespace

namespace {
int seg_apply_launch(const void* g, WdSrc src, long n, int D, int nbits, const void* ws, float* slots, float* w,
                     float* m, float* v, int opt, float lr, float b1, float b2, float eps, float wd, float c1, float c2,
                     float gscale, hipStream_t s) {
  const int ni = (int)n;
  const int nch = (ni + CH - 1) / CH;
  WsLayout L = layout(const_cast<void*>(ws), n, nbits);
  const OptP op{lr, b1, b2, eps, wd, c1, c2, gscale};
  const size_t lds = (size_t)CH * (D + 4) * sizeof(float);
  const int gh = min(16384, (nch + 3) / 4);
  if (opt == 0) {
    hipLaunchKernelGGL(seg_apply_kernel<0>, dim3(nch), dim3(256), lds, s, L.keys, L.pos, (const bf16_t*)g, L.segbeg,
                       slots, w, m, v, ni, D, op, src);
    hipLaunchKernelGGL(seg_fixup_kernel<0>, dim3(gh), dim3(256), 0, s, L.keys, L.lh, slots, w, m, v, ni, nch, D, op);
  } else {
    hipLaunchKernelGGL(seg_apply_kernel<1>, dim3(nch), dim3(256), lds, s, L.keys, L.pos, (const bf16_t*)g, L.segbeg,
                       slots, w, m, v, ni, D, op, src);
    hipLaunchKernelGGL(seg_fixup_kernel<1>, dim3(gh), dim3(256), 0, s, L.keys, L.lh, slots, w, m, v, ni, nch, D, op);
  }
  return kfa_status();
}
}  // namespace

// Gradient-independent half: sort the ids and find the segment structure into ws
// (it only needs the ids, so the caller may run it on a side stream as soon as the
// forward lookup has its ids, overlapped with the dense layers).
static int seg_prepare(const long* ids, const long* offs, int F, long n, int nbits, void* ws, long ws_bytes,
                       hipStream_t s);

KFA_API int kfa_seg_prepare(const long* ids, long n, int nbits, void* ws, long ws_bytes, hipStream_t s) {
  return seg_prepare(ids, nullptr, 1, n, nbits, ws, ws_bytes, s);
}

// the same for ids [n / F][F] of F tables stored back to back: row = ids[i] + offs[i % F]
KFA_API int kfa_seg_prepare_off(const long* ids, const long* offs, int F, long n, int nbits, void* ws, long ws_bytes,
                                hipStream_t s) {
  if (F <= 0 || !offs || (n > 0 && n % F)) return (int)hipErrorInvalidValue;
  return seg_prepare(ids, offs, F, n, nbits, ws, ws_bytes, s);
}

static int seg_prepare(const long* ids, const long* offs, int F, long n, int nbits, void* ws, long ws_bytes,
                       hipStream_t s) {
  if (n <= 0) return 0;
  if (bad_args(n, nbits, ws_bytes)) return (int)hipErrorInvalidValue;
  const int ni = (int)n;
  const int nch = (ni + CH - 1) / CH;
  WsLayout L = layout(ws, n, nbits);
  const int gp = min(16384, (ni + 255) / 256);
  hipLaunchKernelGGL(seg_prep_kernel, dim3(gp), dim3(256), 0, s, ids, offs, F, L.keys_in, L.pos_in, ni);
  int e = kfa_radix::sort_pairs(L.keys_in, L.pos_in, L.keys, L.pos, ni, nbits, L.hist, s);
  if (e) return e;
  const int gh = min(16384, (nch + 3) / 4);
  hipLaunchKernelGGL(seg_heads_kernel, dim3(gh), dim3(256), 0, s, L.keys, L.lh, ni, nch);
  // segbeg[c] = last segment head before entry c*CH = start of the segment holding that
  // entry whenever it is not a head itself (the only case seg_apply_kernel reads it)
  e = (int)hipMemcpyAsync(L.segbeg, L.lh, (size_t)nch * 4, hipMemcpyDeviceToDevice, s);
  if (e) return e;
  e = kfa_radix::scan_max_excl(L.segbeg, nch, -1, s);
  if (e) return e;
  return kfa_status();
}

// Gradient half, on a ws filled by kfa_seg_prepare for the same ids.
// g: bf16 [n, D] (row r = gradient of ids[r]); slots: fp32 [kfa_seg_slot_floats],
// zero on entry and on exit; opt 0 = Adam, 1 = SGD.
KFA_API int kfa_seg_apply(const void* g, long n, int D, int nbits, const void* ws, long ws_bytes, float* slots,
                          float* w, float* m, float* v, int opt, float lr, float b1, float b2, float eps, float wd,
                          float c1, float c2, float gscale, hipStream_t s) {
  if (n <= 0) return 0;
  if (bad_args(n, nbits, ws_bytes) || D % 8 != 0 || D > MAXD) return (int)hipErrorInvalidValue;
  return seg_apply_launch(g, WdSrc{nullptr, nullptr, 1, 0, 0, 0}, n, D, nbits, ws, slots, w, m, v, opt, lr, b1, b2,
                          eps, wd, c1, c2, gscale, s);
}

// kfa_seg_apply with the gradient rows read from the Wide&Deep MLP input gradient
// (see WdSrc): dx [n / F][XW] bf16 (16-B aligned rows), dwide [n / F] fp32; D == E + 8.
KFA_API int kfa_seg_apply_wd(const void* dx, const float* dwide, int F, int E, int Dp, int XW, long n, int D,
                             int nbits, const void* ws, long ws_bytes, float* slots, float* w, float* m, float* v,
                             int opt, float lr, float b1, float b2, float eps, float wd, float c1, float c2,
                             float gscale, hipStream_t s) {
  if (n <= 0) return 0;
  if (bad_args(n, nbits, ws_bytes) || D % 8 != 0 || D > MAXD || D != E + 8 || E % 8 || F <= 0 || n % F ||
      Dp % 8 || XW % 8 || Dp + F * E > XW || !dx || !dwide)
    return (int)hipErrorInvalidValue;
  return seg_apply_launch(nullptr, WdSrc{(const bf16_t*)dx, dwide, F, E, Dp, XW}, n, D, nbits, ws, slots, w, m, v, opt,
                          lr, b1, b2, eps, wd, c1, c2, gscale, s);
}

// both halves on one stream
KFA_API int kfa_seg_sparse_apply(const long* ids, const void* g, long n, int D, int nbits, void* ws, long ws_bytes,
                                 float* slots, float* w, float* m, float* v, int opt, float lr, float b1, float b2,
                                 float eps, float wd, float c1, float c2, float gscale, hipStream_t s) {
  if (n > 0 && (D % 8 != 0 || D > MAXD)) return (int)hipErrorInvalidValue;
  const int rc = kfa_seg_prepare(ids, n, nbits, ws, ws_bytes, s);
  if (rc) return rc;
  return kfa_seg_apply(g, n, D, nbits, ws, ws_bytes, slots, w, m, v, opt, lr, b1, b2, eps, wd, c1, c2, gscale, s);
}

// Test / bench entry of the pair sort alone: sorts (keys, vals) of n entries on the
// low nbits bits in place (stable); ws: kfa_radix_ws_bytes(n).
KFA_API long kfa_radix_ws_bytes(long n) { return 2 * kfa_radix::align256(n * 4) + kfa_radix::hist_bytes(n); }

KFA_API int kfa_radix_sort_pairs(unsigned* keys, int* vals, long n, int nbits, void* ws, long ws_bytes,
                                 hipStream_t s) {
  if (n <= 0) return 0;
  if (n > 0x7fffffffL || nbits < 1 || nbits > 32 || ws_bytes < kfa_radix_ws_bytes(n)) return (int)hipErrorInvalidValue;
  char* p = (char*)ws;
  unsigned* k1 = (unsigned*)p;
  int* v1 = (int*)(p + kfa_radix::align256(n * 4));
  int* hist = (int*)(p + 2 * kfa_radix::align256(n * 4));
  int e = kfa_radix::sort_pairs(keys, vals, k1, v1, (int)n, nbits, hist, s);
  if (e) return e;
  e = (int)hipMemcpyAsync(keys, k1, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
  if (!e) e = (int)hipMemcpyAsync(vals, v1, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
  return e;
}

// exclusive prefix max of a[0..n) in place from init (test entry of the chunk-head scan)
KFA_API int kfa_scan_max_excl(int* a, long n, int init, hipStream_t s) {
  return kfa_radix::scan_max_excl(a, (int)n, init, s);
}
