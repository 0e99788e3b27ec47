// dfact.hpp — device helpers of the distributed factor (one job's POTRF + TRTRI over several
// GPUs; host side gp2d.hip gp2d_dfact_*, gp2d/distributed.py fit_distributed).
//
// 1-D block-cyclic by 512-column super-blocks: rank s mod P owns super-column s.  Every rank
// holds the whole n×n K_y but reads and writes only its own super-columns, which end up holding
// W = L⁻¹ (right-looking TRTRI fused into the right-looking POTRF: at step s every rank applies
// the broadcast panel [D_s = L_ss⁻¹; L21] to its trailing K_y columns AND to its W columns
// J ≤ s: X[s] = D_s·R[s] (out of place, D_s = L_ss⁻¹ shipped in the panel), R[t>s] −= L[t,s]·X[s]).  The GEMMs run on gemm_f64_kernel with
// block-cyclic column tiles (GemmParams::jgrp / jstep / cyc_lower).
#pragma once
#include "common.hpp"

namespace gp2d {

constexpr int DF_SB = 512;           // super-block width: four 128-wide GEMM tiles, so every
constexpr int DF_SBT = DF_SB / 128;  // trailing update is a K = 512 product (the SYRK tile runs
                                     // 58 vs 51 TF/s at K = 512 than at K = 256)

// Column block s of A becomes the s-th block column of the identity (rows of the super-block:
// I, every other row: 0): the TRTRI's initial right-hand side R[:, s] = E_s, written once the
// owner has read its K_y panel.  One row per workgroup, one element pair per thread.
__global__ __launch_bounds__(DF_SB / 2) void dfact_reset_col_kernel(double* __restrict__ A, int64_t n, int64_t lda,
                                                                    int64_t c0) {
  const int64_t i = blockIdx.x;
  const int c = 2 * (int)threadIdx.x;
  if (i >= n) return;
  const int64_t r = i - c0;             // row within the super-block, if any
  d2 v;
  v.x = (r == c) ? 1.0 : 0.0;
  v.y = (r == c + 1) ? 1.0 : 0.0;
  *reinterpret_cast<d2*>(A + i * lda + c0 + c) = v;
}

// X[i][col] = T[i][col] for the DF_SB rows of a super-block and this rank's owned super-columns
// (the q-th at column (first + q·P)·DF_SB): the out-of-place TRTRI step's result copied back.
// One workgroup per (owned super-column, row), one element pair per thread.
__global__ __launch_bounds__(DF_SB / 2) void dfact_copy_owned_kernel(const double* __restrict__ T, int64_t ldt,
                                                                     double* __restrict__ X, int64_t ldx, int first,
                                                                     int P) {
  const int64_t col = (int64_t)(first + (int)blockIdx.x * P) * DF_SB + 2 * threadIdx.x;
  const int64_t i = blockIdx.y;
  *reinterpret_cast<d2*>(X + i * ldx + col) = *reinterpret_cast<const d2*>(T + i * ldt + col);
}

// α from the owned columns (fit_distributed): z = W·y = Σ_t W[:, t]·y[t] in super-column order,
// then α[t] = W[:, t]ᵀ·z — every piece computed from one super-column, the same for any P.  One
// launch covers `count` super-columns t = t0 + q·dt (blockIdx.y = q).
// zpart[q][i] = Σ_{k ∈ super-column t, k ≤ i} W[i][k]·y[k] (0 above the super-block): one wave per
// row, 8 columns per lane in a fixed order, a fixed shuffle reduction.
__global__ __launch_bounds__(256) void dfact_zpart_kernel(const double* __restrict__ W, int64_t n, int64_t ldw,
                                                          int t0, int dt, const double* __restrict__ y,
                                                          double* __restrict__ zpart) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t c0 = (int64_t)(t0 + (int)blockIdx.y * dt) * DF_SB;
  if (i >= n) return;
  double s = 0.0;
  if (i >= c0) {
    const double* w = W + i * ldw + c0;
#pragma unroll
    for (int u = 0; u < DF_SB / 64; ++u) {
      const int64_t k = c0 + lane + 64 * u;
      s += (k <= i) ? w[lane + 64 * u] * y[k] : 0.0;
    }
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) zpart[(int64_t)blockIdx.y * n + i] = s;
}

// part[q][seg][c] = Σ_{i ∈ [c0 + 128·seg, +128), i ≥ c0 + c} W[i][c0 + c]·z[i] (0 for segments below
// the super-block's rows): one thread per column of the super-column (reads of a row coalesced
// over the threads); the n/128 segments are summed afterwards in a fixed order.
__global__ __launch_bounds__(256) void dfact_alpha_part_kernel(const double* __restrict__ W, int64_t n, int64_t ldw,
                                                               int t0, int dt, const double* __restrict__ z,
                                                               double* __restrict__ part) {
  const int c = (int)blockIdx.x * 256 + (int)threadIdx.x;   // < DF_SB
  const int64_t seg = blockIdx.y, q = blockIdx.z;
  const int64_t c0 = (int64_t)(t0 + (int)q * dt) * DF_SB;
  const int64_t r0 = seg * 128, col = c0 + c;
  double s = 0.0;
  if (r0 + 128 > c0)
    for (int64_t i = (r0 > col ? r0 : col); i < r0 + 128; ++i) s += W[i * ldw + col] * z[i];
  part[(q * (n / 128) + seg) * DF_SB + c] = s;
}

// out[q][c] = Σ_seg part[q][seg][c] in segment order
__global__ __launch_bounds__(256) void dfact_alpha_sum_kernel(const double* __restrict__ part, int64_t nseg,
                                                              double* __restrict__ out) {
  const int c = (int)blockIdx.x * 256 + (int)threadIdx.x;
  const int64_t q = blockIdx.y;
  const double* p = part + q * nseg * DF_SB + c;
  double s = 0.0;
  for (int64_t g = 0; g < nseg; ++g) s += p[g * DF_SB];
  out[q * DF_SB + c] = s;
}

// A failed diagonal block reports its local leading-minor order in *tmp; the first failure
// of the whole factorisation is kept in *info as a global order.
__global__ void dfact_info_kernel(int* __restrict__ info, const int* __restrict__ tmp, int64_t off) {
  if (threadIdx.x == 0 && *tmp != 0 && *info == 0) *info = (int)(off + *tmp);
}

// Row-block packing of a lower-triangular n×n matrix (n a multiple of 128): row block rb keeps
// columns [0, 128·(rb+1)), stored row-major one block after the other — ≈ n²/2 doubles, the
// factor broadcast's payload (gp2d_pack_lower).  One workgroup per (512-column chunk, row block).
template <bool UNPACK>
__global__ __launch_bounds__(256) void pack_lower_kernel(double* __restrict__ W, int64_t n, int64_t ldw,
                                                         double* __restrict__ P) {
  const int64_t rb = blockIdx.y, r0 = rb * 128, c1 = r0 + 128;
  const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
  if (c >= c1) return;
  const int64_t off = 128 * 128 * (rb * (rb + 1) / 2);
#pragma unroll 4
  for (int r = 0; r < 128; ++r) {
    d2* w = reinterpret_cast<d2*>(W + (r0 + r) * ldw + c);
    d2* p = reinterpret_cast<d2*>(P + off + r * c1 + c);
    if (UNPACK) *w = *p; else *p = *w;
  }
}

}  // namespace gp2d
