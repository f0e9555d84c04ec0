// LSD radix sort of (u32 key, i32 value) pairs on the low `nbits` bits of the
// key — the id sort of the segment-reduce sparse optimizer (segsparse.hip,
// SURVEY §2.6 K6), replacing hipCUB's DeviceRadixSort / DeviceScan.
//
// Each pass sorts on one digit of DB <= 9 bits (passes = ceil(nbits / 9), the
// digit width balanced over them: a 25-bit key of the 22.9 M-row W&D table is
// 3 passes of 9 / 8 / 8 bits) in three launches:
//   1. radix_hist: one block per tile of TILE = 8192 entries counts its digits
//      in LDS (ds_add) and writes hist[digit][tile] (digit-major);
//   2. scan_excl: ONE 1024-thread block turns hist into exclusive prefix sums —
//      the global output offset of (digit, tile);
//   3. radix_scatter: the tile again, in 16 rounds of 512 entries (round-major,
//      then wave, then lane = the input order, so the sort is stable); within a
//      wave the lanes holding the same digit find each other with one ballot
//      per digit bit (no LDS atomics), the wave's digit counts go through LDS,
//      and every entry's position is  offset(digit, tile) + entries of that
//      digit in earlier rounds + in earlier waves of this round + in lower lanes.
// Keys and values of a tile are loaded into registers up front (16 loads of
// each in flight per thread) and the pass ping-pongs between two buffers.
#pragma once
#include "common.h"

namespace kfa_radix {

constexpr int BLOCK = 512;             // threads per tile block (8 waves)
constexpr int ITEMS = 16;              // entries per thread
constexpr int TILE = BLOCK * ITEMS;    // 8192 entries per tile
constexpr int MAXB = 9;                // digit bits per pass at most
constexpr int NW = BLOCK / 64;

inline int passes(int nbits) { return (nbits + MAXB - 1) / MAXB; }
inline int tiles(long n) { return (int)((n + TILE - 1) / TILE); }
inline long align256(long x) { return (x + 255) & ~255L; }
// scratch: the digit histogram of one pass (the pass buffers are the caller's)
inline long hist_bytes(long n) { return align256((long)(1 << MAXB) * tiles(n) * 4); }

template <int DB>
__global__ __launch_bounds__(BLOCK) void radix_hist(const unsigned* __restrict__ keys, int n, int shift,
                                                    int* __restrict__ hist, int ntiles) {
  constexpr int BINS = 1 << DB;
  __shared__ int cnt[BINS];
  for (int d = threadIdx.x; d < BINS; d += BLOCK) cnt[d] = 0;
  __syncthreads();
  const long base = (long)blockIdx.x * TILE;
  unsigned k[ITEMS];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const long i = base + r * BLOCK + threadIdx.x;
    k[r] = i < n ? keys[i] : 0u;
  }
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const long i = base + r * BLOCK + threadIdx.x;
    if (i < n) atomicAdd(&cnt[(k[r] >> shift) & (BINS - 1)], 1);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < BINS; d += BLOCK) hist[(long)d * ntiles + blockIdx.x] = cnt[d];
}

// exclusive prefix (sum, or max when MAX) over a[0..n) in place, one 1024-thread block:
// each thread reduces a contiguous run, the run totals are scanned through LDS, then
// each run is rewritten with its exclusive prefix
template <bool MAX>
__global__ __launch_bounds__(1024) void scan_excl(int* __restrict__ a, int n, int init) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int per = (n + 1023) / 1024;
  const int b = min(n, t * per), e = min(n, b + per);
  int acc = MAX ? init : 0;
  for (int i = b; i < e; ++i) acc = MAX ? max(acc, a[i]) : acc + a[i];
  part[t] = acc;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan of the run totals
    const int y = t >= o ? part[t - o] : (MAX ? init : 0);
    __syncthreads();
    part[t] = MAX ? max(part[t], y) : part[t] + y;
    __syncthreads();
  }
  int run = t ? part[t - 1] : (MAX ? init : 0);
  for (int i = b; i < e; ++i) {
    const int x = a[i];
    a[i] = run;
    run = MAX ? max(run, x) : run + x;
  }
}

template <int DB>
__global__ __launch_bounds__(BLOCK) void radix_scatter(const unsigned* __restrict__ kin, const int* __restrict__ vin,
                                                       unsigned* __restrict__ kout, int* __restrict__ vout, int n,
                                                       int shift, const int* __restrict__ off, int ntiles) {
  constexpr int BINS = 1 << DB;
  __shared__ int run[BINS];
  __shared__ int wcnt[NW][BINS];
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  for (int d = t; d < BINS; d += BLOCK) {
    run[d] = off[(long)d * ntiles + blockIdx.x];
#pragma unroll
    for (int q = 0; q < NW; ++q) wcnt[q][d] = 0;
  }
  const long base = (long)blockIdx.x * TILE;
  unsigned k[ITEMS];
  int v[ITEMS];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const long i = base + r * BLOCK + t;
    k[r] = i < n ? kin[i] : 0u;
    v[r] = i < n ? vin[i] : 0;
  }
  __syncthreads();
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const long i = base + r * BLOCK + t;
    const bool valid = i < n;
    const int d = (int)((k[r] >> shift) & (BINS - 1));
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < DB; ++b) {
      const bool bit = (d >> b) & 1;
      const unsigned long long bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    const int rank = __popcll(peers & below);
    if (valid && rank == 0) wcnt[w][d] = __popcll(peers);
    __syncthreads();
    if (valid) {
      int pos = run[d] + rank;
      for (int q = 0; q < w; ++q) pos += wcnt[q][d];
      kout[pos] = k[r];
      vout[pos] = v[r];
    }
    __syncthreads();
    for (int dd = t; dd < BINS; dd += BLOCK) {
      int s = 0;
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        s += wcnt[q][dd];
        wcnt[q][dd] = 0;
      }
      run[dd] += s;
    }
    __syncthreads();
  }
}

template <int DB>
inline void pass(const unsigned* kin, const int* vin, unsigned* kout, int* vout, int n, int shift, int* hist,
                 hipStream_t s) {
  const int nt = tiles(n);
  hipLaunchKernelGGL(radix_hist<DB>, dim3(nt), dim3(BLOCK), 0, s, kin, n, shift, hist, nt);
  hipLaunchKernelGGL(scan_excl<false>, dim3(1), dim3(1024), 0, s, hist, (1 << DB) * nt, 0);
  hipLaunchKernelGGL(radix_scatter<DB>, dim3(nt), dim3(BLOCK), 0, s, kin, vin, kout, vout, n, shift, hist, nt);
}

// Sort (k0, v0) on bits [0, nbits) of the keys, stable.  (k1, v1) are the other
// pass buffers; the sorted pairs end in (k1, v1) (one device copy when the pass
// count is even).  hist: hist_bytes(n) of scratch.  Returns the HIP status.
inline int sort_pairs(unsigned* k0, int* v0, unsigned* k1, int* v1, int n, int nbits, int* hist, hipStream_t s) {
  if (n <= 0) return 0;
  const int np = passes(nbits);
  const int db = (nbits + np - 1) / np;
  unsigned* ks[2] = {k0, k1};
  int* vs[2] = {v0, v1};
  for (int p = 0; p < np; ++p) {
    const unsigned* ki = ks[p & 1];
    const int* vi = vs[p & 1];
    unsigned* ko = ks[(p + 1) & 1];
    int* vo = vs[(p + 1) & 1];
    const int sh = p * db;
    switch (db) {
      case 1: pass<1>(ki, vi, ko, vo, n, sh, hist, s); break;
      case 2: pass<2>(ki, vi, ko, vo, n, sh, hist, s); break;
      case 3: pass<3>(ki, vi, ko, vo, n, sh, hist, s); break;
      case 4: pass<4>(ki, vi, ko, vo, n, sh, hist, s); break;
      case 5: pass<5>(ki, vi, ko, vo, n, sh, hist, s); break;
      case 6: pass<6>(ki, vi, ko, vo, n, sh, hist, s); break;
      case 7: pass<7>(ki, vi, ko, vo, n, sh, hist, s); break;
      case 8: pass<8>(ki, vi, ko, vo, n, sh, hist, s); break;
      default: pass<9>(ki, vi, ko, vo, n, sh, hist, s); break;
    }
  }
  if (np % 2 == 0) {  // the result is back in (k0, v0)
    hipError_t e = hipMemcpyAsync(k1, k0, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(v1, v0, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return (int)e;
  }
  return (int)hipGetLastError();
}

// exclusive max-scan of a[0..n) in place, starting from `init` (one block)
inline int scan_max_excl(int* a, int n, int init, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(scan_excl<true>, dim3(1), dim3(1024), 0, s, a, n, init);
  return (int)hipGetLastError();
}

}  // namespace kfa_radix
