// LSD radix sort of (u32 key, i32 value) pairs on the low `nbits` bits of the
// key — the id sort of the segment-reduce sparse optimizer (segsparse.hip,
// SURVEY §2.6 K6), replacing hipCUB's DeviceRadixSort / DeviceScan.
//
// Each pass sorts on one digit of DB <= 9 bits (passes = ceil(nbits / 9), the
// digit width balanced over them: a 25-bit key of the 22.9 M-row W&D table is
// 3 passes of 9 / 8 / 8 bits) in three launches:
//   1. radix_hist: one block per tile of TILE = 4096 entries counts its digits
//      in LDS (one ds_add per distinct digit per wave) and writes
//      cnt[digit][tile] (digit-major);
//   2. radix_digit_scan: one block per digit turns its row of tile counts into
//      exclusive prefixes (offset of (digit, tile) among that digit's entries)
//      and writes the digit's total;
//   3. radix_scatter: the tile again.  Its entries are ranked in 8 rounds of 512
//      (round-major, then wave, then lane = input order, so the sort is stable):
//      lanes holding the same digit find each other with one ballot per digit
//      bit, wave counts go through LDS.  Each entry is first written to its
//      position in the TILE's sorted order (an LDS image), then the image is
//      streamed out in order — runs of one digit land on consecutive global
//      positions, so the stores coalesce.  The global base of a digit is the
//      exclusive scan of the digit totals, which every scatter block recomputes
//      in LDS (512 values) instead of a fourth launch.
// The pass ping-pongs between two buffers.
#pragma once
#include "common.h"

namespace kfa_radix {

constexpr int BLOCK = 512;             // threads per tile block (8 waves)
constexpr int ITEMS = 8;               // entries per thread
constexpr int TILE = BLOCK * ITEMS;    // 4096 entries per tile (two scatter blocks per CU)
constexpr int MAXB = 9;                // digit bits per pass at most
constexpr int NW = BLOCK / 64;

inline int passes(int nbits) { return (nbits + MAXB - 1) / MAXB; }
inline int tiles(long n) { return (int)((n + TILE - 1) / TILE); }
inline long align256(long x) { return (x + 255) & ~255L; }
// scratch of one pass: tile counts, their within-digit prefixes, the digit totals
inline long hist_bytes(long n) { return 2 * align256((long)(1 << MAXB) * tiles(n) * 4) + align256((1 << MAXB) * 4); }

// lanes of the wave whose entry is valid and has digit d (one ballot per digit bit)
template <int DB>
__device__ __forceinline__ unsigned long long match_digit(int d, bool valid) {
  unsigned long long peers = __ballot(valid);
#pragma unroll
  for (int b = 0; b < DB; ++b) {
    const bool bit = (d >> b) & 1;
    const unsigned long long bb = __ballot(bit);
    peers &= bit ? bb : ~bb;
  }
  return peers;
}

// Counting goes through one LDS atomic per distinct digit per wave (the lowest
// lane of each digit's peer set adds their count): the W&D ids are heavily
// skewed, and per-entry atomics on one hot bin serialise (measured 58 us per
// 1.7 M-key pass vs a few us of bandwidth).
template <int DB>
__global__ __launch_bounds__(BLOCK) void radix_hist(const unsigned* __restrict__ keys, int n, int shift,
                                                    int* __restrict__ cnt, int ntiles) {
  constexpr int BINS = 1 << DB;
  __shared__ int c[BINS];
  for (int d = threadIdx.x; d < BINS; d += BLOCK) c[d] = 0;
  __syncthreads();
  const long base = (long)blockIdx.x * TILE;
  unsigned k[ITEMS];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const long i = base + r * BLOCK + threadIdx.x;
    k[r] = i < n ? keys[i] : 0u;
  }
  const unsigned long long below = (1ull << (threadIdx.x & 63)) - 1ull;
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const long i = base + r * BLOCK + threadIdx.x;
    const int d = (int)((k[r] >> shift) & (BINS - 1));
    const unsigned long long peers = match_digit<DB>(d, i < n);
    if (i < n && __popcll(peers & below) == 0) atomicAdd(&c[d], __popcll(peers));
  }
  __syncthreads();
  for (int d = threadIdx.x; d < BINS; d += BLOCK) cnt[(long)d * ntiles + blockIdx.x] = c[d];
}

// exclusive prefix sum of x over the 256-thread block (returns it; *total = block sum)
__device__ __forceinline__ int block_excl_sum256(int x, int* red, int& total) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int v = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  if (lane == 63) red[w] = v;
  __syncthreads();
  int before = 0;
  for (int q = 0; q < w; ++q) before += red[q];
  total = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return before + v - x;
}

// one block per digit: offs[d][t] = sum_{t' < t} cnt[d][t'], tot[d] = sum_t cnt[d][t]
__global__ __launch_bounds__(256) void radix_digit_scan(const int* __restrict__ cnt, int* __restrict__ offs,
                                                        int* __restrict__ tot, int ntiles) {
  __shared__ int red[4];
  const long row = (long)blockIdx.x * ntiles;
  int carry = 0;
  for (int b0 = 0; b0 < ntiles; b0 += 256) {
    const int t = b0 + threadIdx.x;
    const int x = t < ntiles ? cnt[row + t] : 0;
    int s;
    const int e = block_excl_sum256(x, red, s);
    if (t < ntiles) offs[row + t] = carry + e;
    carry += s;
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

template <int DB>
__global__ __launch_bounds__(BLOCK) void radix_scatter(const unsigned* __restrict__ kin, const int* __restrict__ vin,
                                                       unsigned* __restrict__ kout, int* __restrict__ vout, int n,
                                                       int shift, const int* __restrict__ cnt,
                                                       const int* __restrict__ offs, const int* __restrict__ tot,
                                                       int ntiles) {
  constexpr int BINS = 1 << DB;
  __shared__ unsigned lk[TILE];
  __shared__ int lv[TILE];
  __shared__ int lbase[BINS];   // exclusive prefix of this tile's digit counts (tile-local)
  __shared__ int gbase[BINS];   // global position of the tile's first entry of each digit
  __shared__ int lstart[BINS];  // tile-local start of each digit in the sorted image
  __shared__ int wcnt[NW][BINS];
  __shared__ int wtot[2][NW];
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  // tile-local and global digit bases: block scans over the BINS digits (BINS <= BLOCK)
  {
    const int c = t < BINS ? cnt[(long)t * ntiles + blockIdx.x] : 0;
    const int g = t < BINS ? tot[t] : 0;
    int vc = c, vg = g;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int yc = __shfl_up(vc, o, 64), yg = __shfl_up(vg, o, 64);
      if (lane >= o) { vc += yc; vg += yg; }
    }
    if (lane == 63) { wtot[0][w] = vc; wtot[1][w] = vg; }
    __syncthreads();
    int bc = 0, bg = 0;
    for (int q = 0; q < w; ++q) { bc += wtot[0][q]; bg += wtot[1][q]; }
    if (t < BINS) {
      lbase[t] = lstart[t] = bc + vc - c;
      gbase[t] = bg + vg - g + offs[(long)t * ntiles + blockIdx.x];
    }
    for (int d = t; d < BINS; d += BLOCK) {
#pragma unroll
      for (int q = 0; q < NW; ++q) wcnt[q][d] = 0;
    }
  }
  const long base = (long)blockIdx.x * TILE;
  const int cnt_tile = (int)(n - base < TILE ? n - base : TILE);
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
    const unsigned long long peers = match_digit<DB>(d, valid);
    const int rank = __popcll(peers & below);
    if (valid && rank == 0) wcnt[w][d] = __popcll(peers);
    __syncthreads();
    if (valid) {
      int pos = lbase[d] + rank;
      for (int q = 0; q < w; ++q) pos += wcnt[q][d];
      lk[pos] = k[r];
      lv[pos] = v[r];
    }
    __syncthreads();
    for (int dd = t; dd < BINS; dd += BLOCK) {
      int s = 0;
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        s += wcnt[q][dd];
        wcnt[q][dd] = 0;
      }
      lbase[dd] += s;  // next round's entries of digit dd follow these
    }
    __syncthreads();
  }
  // stream the sorted tile out in order
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const int i = r * BLOCK + t;
    if (i >= cnt_tile) break;
    const unsigned kk = lk[i];
    const int d = (int)((kk >> shift) & (BINS - 1));
    const int g = gbase[d] + (i - lstart[d]);
    kout[g] = kk;
    vout[g] = lv[i];
  }
}

template <int DB>
inline void pass(const unsigned* kin, const int* vin, unsigned* kout, int* vout, int n, int shift, int* hist,
                 hipStream_t s) {
  const int nt = tiles(n);
  int* cnt = hist;
  int* offs = hist + align256((long)(1 << MAXB) * nt * 4) / 4;
  int* tot = offs + align256((long)(1 << MAXB) * nt * 4) / 4;
  hipLaunchKernelGGL(radix_hist<DB>, dim3(nt), dim3(BLOCK), 0, s, kin, n, shift, cnt, nt);
  hipLaunchKernelGGL(radix_digit_scan, dim3(1 << DB), dim3(256), 0, s, cnt, offs, tot, nt);
  hipLaunchKernelGGL(radix_scatter<DB>, dim3(nt), dim3(BLOCK), 0, s, kin, vin, kout, vout, n, shift, cnt, offs, tot,
                     nt);
}

// Sort (k0, v0) on bits [0, nbits) of the keys, stable.  (k1, v1) are the other
// pass buffers; the sorted pairs end in (k1, v1) (one device copy when the pass
// count is even).  hist: hist_bytes(n) of scratch.  Returns the HIP status.
inline int sort_pairs(unsigned* k0, int* v0, unsigned* k1, int* v1, int n, int nbits, int* hist, hipStream_t s) {
  if (n <= 0) return 0;
  const int np = passes(nbits);
  // digit widths balanced over the passes and summing to exactly nbits (25 -> 9 / 8 / 8):
  // bits at and above nbits never take part (hipCUB end_bit semantics)
  const int base = nbits / np, extra = nbits % np;
  unsigned* ks[2] = {k0, k1};
  int* vs[2] = {v0, v1};
  int sh = 0;
  for (int p = 0; p < np; ++p) {
    const unsigned* ki = ks[p & 1];
    const int* vi = vs[p & 1];
    unsigned* ko = ks[(p + 1) & 1];
    int* vo = vs[(p + 1) & 1];
    const int db = base + (p < extra ? 1 : 0);
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
    sh += db;
  }
  if (np % 2 == 0) {  // the result is back in (k0, v0)
    hipError_t e = hipMemcpyAsync(k1, k0, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(v1, v0, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return (int)e;
  }
  return (int)hipGetLastError();
}

// exclusive prefix max of a[0..n) in place from `init`: ONE 1024-thread block
// walks the array in chunks of 4096 (int4 per thread, coalesced), scanning each
// chunk through wave shuffles + LDS and carrying the running max between chunks
__global__ __launch_bounds__(1024) void scan_max_excl_kernel(int* __restrict__ a, int n, int init) {
  __shared__ int wmax[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int carry = init;
  for (int c0 = 0; c0 < n; c0 += 4096) {
    const int i0 = c0 + t * 4;
    int x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = i0 + j < n ? a[i0 + j] : init;
    const int m = max(max(x[0], x[1]), max(x[2], x[3]));
    int v = m;  // inclusive max-scan of the thread maxima over the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(v, o, 64);
      if (lane >= o) v = max(v, y);
    }
    if (lane == 63) wmax[w] = v;
    __syncthreads();
    int before = carry;
    for (int q = 0; q < w; ++q) before = max(before, wmax[q]);
    int chunk_max = carry;
    for (int q = 0; q < 16; ++q) chunk_max = max(chunk_max, wmax[q]);
    int run = max(before, __shfl_up(v, 1, 64));
    if (lane == 0) run = before;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (i0 + j < n) a[i0 + j] = run;
      run = max(run, x[j]);
    }
    carry = chunk_max;
    __syncthreads();
  }
}

// exclusive max-scan of a[0..n) in place, starting from `init` (one block)
inline int scan_max_excl(int* a, int n, int init, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(scan_max_excl_kernel, dim3(1), dim3(1024), 0, s, a, n, init);
  return (int)hipGetLastError();
}

}  // namespace kfa_radix
