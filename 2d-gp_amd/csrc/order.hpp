// order.hpp — point ordering and the index plumbing around it, on the device.
//
// The ozaki engine orders training and grid points along a Z-order curve (ozaki.hpp,
// morton_code_kernel) so that the exact zeros of K* cluster into skippable int8 GEMM slabs.
// Everything that order touches runs here, so no framework kernel sits on the hot path:
//   * a stable LSD radix sort of the 64-bit codes with their index permutation (8-bit digits;
//     equal codes keep their input order, so the permutation is deterministic);
//   * the gather of the points into that order;
//   * the padded, permuted observation vector of a fit (the reference's obs = [u; v] stacking,
//     GP_laser.py:98-99, krig.py:375-394, in the fit's point order);
//   * the LAPACK status words' first-failure encoding for an all-reduce MIN.
// The predict's scatter back to the caller's grid order is fused into predict_finalize_kernel.
#pragma once
#include "common.hpp"

namespace gp2d {

constexpr int RS_BITS = 8;
constexpr int RS_BINS = 1 << RS_BITS;
constexpr int RS_THREADS = 256;
constexpr int RS_ROUNDS = 16;                          // rounds of 256 keys per tile
constexpr int RS_TILE = RS_THREADS * RS_ROUNDS;        // keys per workgroup

// hist[d·ntiles + b] = number of keys of tile b whose digit (key >> shift) & 255 is d
__global__ __launch_bounds__(RS_THREADS) void radix_hist_kernel(const uint64_t* __restrict__ keys, int64_t n, int shift,
                                                                uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[RS_BINS];
  const int tid = threadIdx.x;
  h[tid] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int64_t e = base + r * RS_THREADS + tid;
    if (e < n) atomicAdd(&h[(keys[e] >> shift) & (RS_BINS - 1)], 1u);   // a count: order-free
  }
  __syncthreads();
  hist[(int64_t)tid * gridDim.x + blockIdx.x] = h[tid];
}

// In place: exclusive prefix sum of hist in (digit, tile) order → each tile's first output slot
// per digit.  One 1024-thread workgroup; thread t owns a contiguous run of the array.
__global__ __launch_bounds__(1024) void radix_scan_kernel(uint32_t* __restrict__ hist, int64_t count) {
  __shared__ uint32_t part[1024];
  const int tid = threadIdx.x;
  const int64_t per = (count + 1023) / 1024;
  const int64_t lo = min<int64_t>(count, tid * per), hi = min<int64_t>(count, lo + per);
  uint32_t s = 0;
  for (int64_t i = lo; i < hi; ++i) s += hist[i];
  part[tid] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {   // Hillis-Steele inclusive scan of the run sums
    const uint32_t v = tid >= o ? part[tid - o] : 0u;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  uint32_t run = tid ? part[tid - 1] : 0u;
  for (int64_t i = lo; i < hi; ++i) {
    const uint32_t c = hist[i];
    hist[i] = run;
    run += c;
  }
}

// Stable scatter of one digit pass.  A tile's keys go in index order: round r, wave w, lane l
// is element base + 256r + 64w + l.  Within a wave the lanes with the same digit find each other
// by 8 ballots (one per digit bit); an element's slot = the tile's offset for its digit + the
// digit's count in earlier rounds + in earlier waves of this round + its rank among its peers.
// vin == nullptr: the first pass, values are the element indices.
__global__ __launch_bounds__(RS_THREADS) void radix_scatter_kernel(const uint64_t* __restrict__ kin,
                                                                   const int64_t* __restrict__ vin, int64_t n,
                                                                   int shift, const uint32_t* __restrict__ offs,
                                                                   uint64_t* __restrict__ kout,
                                                                   int64_t* __restrict__ vout) {
  __shared__ uint32_t run[RS_BINS];
  __shared__ uint32_t wcnt[RS_THREADS / 64][RS_BINS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  run[tid] = offs[(int64_t)tid * gridDim.x + blockIdx.x];
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int r = 0; r < RS_ROUNDS; ++r) {
    if (base + r * RS_THREADS >= n) break;   // uniform across the workgroup
#pragma unroll
    for (int q = 0; q < RS_THREADS / 64; ++q) wcnt[q][tid] = 0;
    __syncthreads();
    const int64_t e = base + r * RS_THREADS + tid;
    const bool valid = e < n;
    uint64_t key = 0;
    int64_t val = 0;
    if (valid) {
      key = kin[e];
      val = vin ? vin[e] : e;
    }
    const int d = (int)((key >> shift) & (RS_BINS - 1));
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < RS_BITS; ++b) {
      const uint64_t bb = __ballot((d >> b) & 1);
      peers &= ((d >> b) & 1) ? bb : ~bb;
    }
    const int rank = __popcll(peers & lt);
    if (valid && rank == 0) wcnt[w][d] = (uint32_t)__popcll(peers);   // the group's lowest lane
    __syncthreads();
    if (valid) {
      uint32_t slot = run[d] + (uint32_t)rank;
      for (int q = 0; q < w; ++q) slot += wcnt[q][d];
      kout[slot] = key;
      vout[slot] = val;
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int q = 0; q < RS_THREADS / 64; ++q) add += wcnt[q][tid];
    run[tid] += add;
  }
}

// dst[j][c] = src[order[j]][c] for rows of `dim` doubles, one thread per element
__global__ __launch_bounds__(256) void gather_rows_kernel(const double* __restrict__ src, const int64_t* __restrict__ order,
                                                          int64_t n, int64_t dim, double* __restrict__ dst) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * dim) return;
  const int64_t j = t / dim, c = t - j * dim;
  dst[t] = src[order[j] * dim + c];
}

// Observation vector of a fit: out[c·npad + i] = y[c·ntr + perm[i]] for i < ntr (perm may be
// NULL: the identity), 0 in the padding — the reference's stacking [u_1..u_N, v_1..v_N]
// (GP_laser.py:98-99) in the fit's point order.
__global__ __launch_bounds__(256) void obs_pad_kernel(const double* __restrict__ y, int64_t ntr, int64_t npad, int bd,
                                                      const int64_t* __restrict__ perm, double* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)bd * npad) return;
  const int64_t c = t / npad, i = t - c * npad;
  out[t] = (i < ntr) ? y[c * ntr + (perm ? perm[i] : i)] : 0.0;
}

// 0 ↔ INT32_MAX on LAPACK status words (an involution): applied before and after an
// all-reduce MIN, it turns the reduction into "the first failing minor, or 0".
__global__ __launch_bounds__(64) void status_flip_kernel(int* __restrict__ s, int count) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= count) return;
  const int v = s[i];
  s[i] = (v == 0) ? 0x7fffffff : (v == 0x7fffffff ? 0 : v);
}

}  // namespace gp2d
