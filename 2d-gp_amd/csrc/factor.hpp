// factor.hpp — blocked Cholesky (POTRF), triangular inverse (TRTRI) and the
// α = K_y⁻¹y solve for the fit stage.
//
// Replaces np.linalg.inv(K) (GP_laser.py:118, GP_scripts.py:50) and the
// Cholesky + cho_solve inside GPy / sklearn (_gpr.py:349-360).
//
// POTRF, right-looking, NB = 128:
//   for each block column k:
//     potrf_diag_kernel : one workgroup factors the 128×128 diagonal block in LDS,
//                         writes L_kk and inv(L_kk) (in-place trti2 in LDS)
//     panel TRSM        : L_ik = A_ik · inv(L_kk)ᵀ   (MFMA GEMM, NT, in place)
//     trailing SYRK     : A_ij −= L_ik L_jkᵀ, lower tiles only (MFMA GEMM, NT)
// TRTRI, in place, recursive doubling over 128-blocks (log2(n/128) levels, each one
// batched pair of MFMA GEMMs):  W21 = −W22 · (L21 · W11).
#pragma once
#include "common.hpp"
#include "gemm_f64.hpp"

namespace gp2d {

constexpr int DSP = NB + 16;  // LDS row stride (doubles) of the diagonal block: ≡16 mod 32

__global__ __launch_bounds__(256) void potrf_diag_kernel(double* __restrict__ A, int64_t lda, int k0,
                                                         double* __restrict__ dinv, int* info) {
  __shared__ double S[NB * DSP];
  __shared__ double col[NB];
  const int tid = threadIdx.x;
  double* Ab = A + (int64_t)k0 * lda + k0;
  for (int idx = tid; idx < NB * NB; idx += 256) {
    const int i = idx >> 7, j = idx & (NB - 1);
    S[i * DSP + j] = (j <= i) ? Ab[(int64_t)i * lda + j] : 0.0;
  }
  __syncthreads();
  const int ty = tid >> 4, tx = tid & 15;
  bool reported = false;
  // right-looking unblocked Cholesky of the LDS-resident block
  for (int j = 0; j < NB; ++j) {
    const double d = S[j * DSP + j];
    if (!(d > 0.0) && tid == 0 && !reported) {
      reported = true;
      if (info) atomicCAS(info, 0, k0 + j + 1);
    }
    const double rd = sqrt(d);
    const double ird = 1.0 / rd;
    __syncthreads();  // everyone has read S[j][j]
    for (int i = j + 1 + tid; i < NB; i += 256) {
      const double v = S[i * DSP + j] * ird;
      S[i * DSP + j] = v;
      col[i] = v;
    }
    if (tid == 0) S[j * DSP + j] = rd;
    __syncthreads();
    for (int i = j + 1 + ty; i < NB; i += 16) {
      const double ci = col[i];
      for (int k = j + 1 + tx; k <= i; k += 16) S[i * DSP + k] -= ci * col[k];
    }
    __syncthreads();
  }
  for (int idx = tid; idx < NB * NB; idx += 256) {
    const int i = idx >> 7, j = idx & (NB - 1);
    Ab[(int64_t)i * lda + j] = (j <= i) ? S[i * DSP + j] : 0.0;
  }
  // in-place inverse (LAPACK trti2 order: columns right to left)
  for (int j = NB - 1; j >= 0; --j) {
    const double ajj = 1.0 / S[j * DSP + j];
    const int i = j + 1 + (tid >> 1), h = tid & 1;
    double t = 0.0;
    if (i < NB)
      for (int k = j + 1 + h; k <= i; k += 2) t += S[i * DSP + k] * S[k * DSP + j];
    t += __shfl_xor(t, 1);
    __syncthreads();  // all reads of column j done
    if (i < NB && h == 0) S[i * DSP + j] = -ajj * t;
    if (tid == 0) S[j * DSP + j] = ajj;
    __syncthreads();
  }
  if (dinv) {
    double* D = dinv + (int64_t)(k0 / NB) * NB * NB;
    for (int idx = tid; idx < NB * NB; idx += 256) {
      const int i = idx >> 7, j = idx & (NB - 1);
      D[idx] = (j <= i) ? S[i * DSP + j] : 0.0;
    }
  }
}

// Zero the strict upper triangle outside the diagonal blocks.
__global__ __launch_bounds__(256) void zero_upper_kernel(double* __restrict__ A, int64_t n, int64_t lda) {
  const int64_t i = blockIdx.y;
  const int64_t j = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
  const int64_t jstart = (i / NB + 1) * NB;
  if (j >= jstart && j < n) *reinterpret_cast<d2*>(A + i * lda + j) = d2{0.0, 0.0};
}

// Copy the inverted diagonal blocks into A's diagonal (TRTRI level 0).
__global__ __launch_bounds__(256) void put_diag_blocks_kernel(double* __restrict__ A, int64_t lda,
                                                              const double* __restrict__ dinv) {
  const int b = blockIdx.y;
  const int idx = blockIdx.x * 256 + threadIdx.x;  // < NB*NB
  const int i = idx >> 7, j = idx & (NB - 1);
  A[((int64_t)b * NB + i) * lda + (int64_t)b * NB + j] = dinv[(int64_t)b * NB * NB + idx];
}

// Stand-alone diagonal-block inversion (used when gp2d_trtri gets no dinv).
__global__ __launch_bounds__(256) void trti2_diag_kernel(const double* __restrict__ A, int64_t lda,
                                                         double* __restrict__ dinv) {
  __shared__ double S[NB * DSP];
  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  const double* Ab = A + (int64_t)b * NB * lda + (int64_t)b * NB;
  for (int idx = tid; idx < NB * NB; idx += 256) {
    const int i = idx >> 7, j = idx & (NB - 1);
    S[i * DSP + j] = (j <= i) ? Ab[(int64_t)i * lda + j] : 0.0;
  }
  __syncthreads();
  for (int j = NB - 1; j >= 0; --j) {
    const double ajj = 1.0 / S[j * DSP + j];
    const int i = j + 1 + (tid >> 1), h = tid & 1;
    double t = 0.0;
    if (i < NB)
      for (int k = j + 1 + h; k <= i; k += 2) t += S[i * DSP + k] * S[k * DSP + j];
    t += __shfl_xor(t, 1);
    __syncthreads();
    if (i < NB && h == 0) S[i * DSP + j] = -ajj * t;
    if (tid == 0) S[j * DSP + j] = ajj;
    __syncthreads();
  }
  double* D = dinv + (int64_t)b * NB * NB;
  for (int idx = tid; idx < NB * NB; idx += 256) {
    const int i = idx >> 7, j = idx & (NB - 1);
    D[idx] = (j <= i) ? S[i * DSP + j] : 0.0;
  }
}

// z = W y for lower-triangular W: one wave per row, lanes stride the row.
__global__ __launch_bounds__(256) void trmv_n_lower_kernel(const double* __restrict__ W, int64_t n, int64_t ldw,
                                                           const double* __restrict__ y, double* __restrict__ z) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  const double* w = W + i * ldw;
  double s = 0.0;
  for (int64_t k = lane; k <= i; k += 64) s += w[k] * y[k];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) z[i] = s;
}

// part[seg][j] = Σ_{i in seg, i >= j} W[i][j] z[i]  (segments of 128 rows).
__global__ __launch_bounds__(256) void trmv_t_lower_part_kernel(const double* __restrict__ W, int64_t n, int64_t ldw,
                                                                const double* __restrict__ z, double* __restrict__ part) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t seg = blockIdx.y;
  const int64_t i0 = seg * NB;
  double s = 0.0;
  if (j < n && i0 + NB > j) {
    for (int64_t i = (i0 > j ? i0 : j); i < i0 + NB; ++i) s += W[i * ldw + j] * z[i];
  }
  if (j < n) part[seg * n + j] = s;
}

__global__ __launch_bounds__(256) void sum_segments_kernel(const double* __restrict__ part, int64_t nseg, int64_t n,
                                                           double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  double s = 0.0;
  for (int64_t g = 0; g < nseg; ++g) s += part[g * n + j];
  out[j] = s;
}

}  // namespace gp2d
