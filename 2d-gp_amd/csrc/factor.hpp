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

constexpr int DSP = NB + 16;

#ifndef GP2D_STAMP
#define GP2D_STAMP(slot) ((void)0)  // dev builds (tools/microbench) record phase timestamps here
#endif  // LDS row stride (doubles) of the diagonal block: ≡16 mod 32

// Register-resident 128×128 diagonal-block kernels.  Thread t (ty = t>>4, tx = t&15)
// owns the 64 elements (ty + 16a, tx + 16b), a, b ∈ [0, 8), in VGPRs; per column
// step only the pivot column (or row) travels through a double-buffered 128-entry
// LDS vector, so each step is one barrier + ≤ 64 register FMAs, and block rows /
// columns outside the active triangle are skipped with wave-uniform branches.

// X = L⁻¹ by right-looking row elimination of LX = I.  L is read column-by-column
// from LDS (Ls, stride DSP); X is returned in r (same ownership map).
__device__ __forceinline__ void reg_trtri_lower(const double* __restrict__ Ls, double (&r)[8][8],
                                                double* __restrict__ buf, double* __restrict__ rdiag, int tid) {
  const int ty = tid >> 4, tx = tid & 15;
  if (tid < NB) rdiag[tid] = 1.0 / Ls[tid * DSP + tid];  // all pivots' reciprocals up front
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) r[a][b] = (ty + 16 * a == tx + 16 * b) ? 1.0 : 0.0;
  // kb is unrolled so that every block-level test below folds at compile time; kt runs.
#pragma unroll
  for (int kb = 0; kb < 8; ++kb)
  for (int kt = 0; kt < 16; ++kt) {
    const int k = 16 * kb + kt;
    double* rb = buf + (k & 1) * NB;
    const double rkk = rdiag[k];
    if (ty == kt) {  // owners of row k finalise X[k][:] = acc[k][:] / L[k][k] and publish it
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        if (a != kb) continue;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          r[a][b] *= rkk;
          rb[tx + 16 * b] = r[a][b];
        }
      }
    }
    __syncthreads();
    double xk[8], f[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) xk[b] = rb[tx + 16 * b];
#pragma unroll
    for (int a = 0; a < 8; ++a) f[a] = Ls[(ty + 16 * a) * DSP + k];
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      if (a < kb) continue;  // rows i < 16·kb ≤ k: untouched
      const int i = ty + 16 * a;
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        if (b > kb) continue;  // columns c ≥ 16·(kb+1) > k: untouched
        if (a > kb && b < kb) {  // interior block: i > k and c <= k for every lane
          r[a][b] = fma(-f[a], xk[b], r[a][b]);
        } else {
          const int c = tx + 16 * b;
          const double nv = fma(-f[a], xk[b], r[a][b]);
          r[a][b] = (i > k && c <= k) ? nv : r[a][b];
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void potrf_diag_kernel(double* __restrict__ A, int64_t lda, int k0,
                                                         double* __restrict__ dinv, int* info) {
  __shared__ double Ls[NB * DSP];
  __shared__ double buf[2 * NB];
  __shared__ double rdiag[NB];
  const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
  double* Ab = A + (int64_t)k0 * lda + k0;
  double r[8][8];
  GP2D_STAMP(0);
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int i = ty + 16 * a, k = tx + 16 * b;
      const double t = Ab[(int64_t)i * lda + k];  // unconditional: loads issue back-to-back
      r[a][b] = (k <= i) ? t : 0.0;
    }
  GP2D_STAMP(1);
  // right-looking Cholesky: column j is published by its owner lanes (tx == j & 15)
#pragma unroll
  for (int jb = 0; jb < 8; ++jb)
  for (int jt = 0; jt < 16; ++jt) {
    const int j = 16 * jb + jt;
    double* cb = buf + (j & 1) * NB;
    if (tx == jt) {
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        if (b != jb) continue;
#pragma unroll
        for (int a = 0; a < 8; ++a) cb[ty + 16 * a] = r[a][b];
      }
    }
    __syncthreads();
    const double d = cb[j];
    const double rd = sqrt(d);
    const double ird = 1.0 / rd;
    if (tid == 0 && !(d > 0.0) && info) atomicCAS(info, 0, k0 + j + 1);
    double li[8], lk[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) li[a] = cb[ty + 16 * a] * ird;
#pragma unroll
    for (int b = 0; b < 8; ++b) lk[b] = cb[tx + 16 * b] * ird;
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      if (a < jb) continue;
      const int i = ty + 16 * a;
#pragma unroll
      for (int b = 0; b <= a; ++b) {
        if (b < jb) continue;
        if (b > jb && b < a) {  // interior block: j < k < i for every lane
          r[a][b] = fma(-li[a], lk[b], r[a][b]);
        } else {
          const int k = tx + 16 * b;
          const double nv = fma(-li[a], lk[b], r[a][b]);
          r[a][b] = (k > j && k <= i) ? nv : r[a][b];
        }
      }
    }
    if (tx == jt) {
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        if (b != jb) continue;
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          const int i = ty + 16 * a;
          r[a][b] = (i > j) ? li[a] : ((i == j) ? rd : r[a][b]);
        }
      }
    }
  }
  GP2D_STAMP(2);
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int i = ty + 16 * a, k = tx + 16 * b;
      const double v = (k <= i) ? r[a][b] : 0.0;
      Ab[(int64_t)i * lda + k] = v;
      Ls[i * DSP + k] = v;
    }
  __syncthreads();
  GP2D_STAMP(3);
  reg_trtri_lower(Ls, r, buf, rdiag, tid);
  GP2D_STAMP(4);
  if (dinv) {
    double* D = dinv + (int64_t)(k0 / NB) * NB * NB;
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const int i = ty + 16 * a, k = tx + 16 * b;
        D[i * NB + k] = (k <= i) ? r[a][b] : 0.0;
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
  __shared__ double Ls[NB * DSP];
  __shared__ double buf[2 * NB];
  __shared__ double rdiag[NB];
  const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
  const int b0 = blockIdx.x;
  const double* Ab = A + (int64_t)b0 * NB * lda + (int64_t)b0 * NB;
  double r[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)  // batched loads into registers, then LDS
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int i = ty + 16 * a, k = tx + 16 * b;
      const double t = Ab[(int64_t)i * lda + k];  // unconditional: loads issue back-to-back
      r[a][b] = (k <= i) ? t : 0.0;
    }
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) Ls[(ty + 16 * a) * DSP + tx + 16 * b] = r[a][b];
  __syncthreads();
  reg_trtri_lower(Ls, r, buf, rdiag, tid);
  double* D = dinv + (int64_t)b0 * NB * NB;
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int i = ty + 16 * a, k = tx + 16 * b;
      D[i * NB + k] = (k <= i) ? r[a][b] : 0.0;
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
