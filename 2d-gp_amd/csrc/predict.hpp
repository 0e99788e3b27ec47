// predict.hpp — posterior mean / variance epilogue kernels for the predict stage.
//
// Replaces getMean (GP_scripts.py:44-46), the Kss − Ks·Ki·Ksᵀ diagonal of
// GP_laser.py:128-131 and sklearn's predict(return_std=True) (_gpr.py:436-490).
// The dominant contraction (‖L⁻¹k*‖² per column) is gemm_f64_kernel<.., EPI_COLSQ>.
#pragma once
#include "common.hpp"

namespace gp2d {

constexpr int MEAN_SEG = 128;  // rows per mean partial segment

// pm[seg][c] = Σ_{r in seg} alpha[r] · B[r][c]   (B = K(train, grid chunk), n × ncols)
__global__ __launch_bounds__(256) void mean_part_kernel(const double* __restrict__ B, int64_t ldb, int64_t ncols,
                                                        const double* __restrict__ alpha, double* __restrict__ pm) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.y * MEAN_SEG;
  if (c >= ncols) return;
  double s = 0.0;
#pragma unroll 8
  for (int r = 0; r < MEAN_SEG; ++r) s += alpha[r0 + r] * B[(r0 + r) * ldb + c];
  pm[(int64_t)blockIdx.y * ncols + c] = s;
}

// Combine partials in fixed order and scatter to the [u..., v...] outputs.  order (optional):
// grid point c0 + loc of this (reordered) chunk is the caller's point order[c0 + loc], so the
// outputs land in the caller's order (the ozaki engine predicts its grid in Morton order).
__global__ __launch_bounds__(256) void predict_finalize_kernel(
    const double* __restrict__ pm, int64_t nmseg, const double* __restrict__ P, int64_t npseg,
    int64_t ncols, int64_t cpad, int64_t cvalid, int64_t c0, int64_t m, double kss, double add,
    int clip, int compute_var, double* __restrict__ mean, double* __restrict__ var,
    const int64_t* __restrict__ order) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncols) return;
  const int64_t comp = c / cpad, loc = c - comp * cpad;
  if (loc >= cvalid) return;
  double mu = 0.0;
  // the same left-to-right sums; unrolled so that eight partials are in flight per thread
#pragma unroll 8
  for (int64_t g = 0; g < nmseg; ++g) mu += pm[g * ncols + c];
  const int64_t o = comp * m + (order ? order[c0 + loc] : c0 + loc);
  mean[o] = mu;
  if (compute_var) {
    double q = 0.0;
#pragma unroll 8
    for (int64_t g = 0; g < npseg; ++g) q += P[g * ncols + c];
    double v = kss - q + add;
    if (clip && v < 0.0) v = 0.0;
    var[o] = v;
  }
}

}  // namespace gp2d
