// assemble.hpp — covariance assembly kernels.
//
// Replaces the reference's kernel builders:
//   GP_scripts.myKernel      GP_scripts.py:6-42   (vectorised mixed df/cf kernel)
//   GP_scripts.nonDivK       GP_scripts.py:57-69  (one 2×2 block, divFree ∈ {0,1,2})
//   GP_scripts.compute_K/_Ks GP_scripts.py:74-123 (component-major 2×2 layout)
//   myKernel.{myKernel,nonDivK,nonRotK}.K   myKernel.py:27-53, 159-176, 255-271
//   sklearn RBF(ARD)+White as built in krig.scikit_prior   krig.py:174-180
//
// One thread evaluates one (row point i, column point j) pair and writes its
// 2×2 block into the four component blocks; a wave covers 64 consecutive
// column points, so every store is a coalesced 512-byte row segment.  Work is
// exp-bound VALU; HBM traffic is the 32 B per pair written.
#pragma once
#include "common.hpp"
#include "../../include/gp2d.h"

namespace gp2d {

struct VecParams {
  int kind;
  int pdim;               // point stride: 2 (x1, x2), or 3 (t, x1, x2) for the spatio-temporal product
  double var_t, ilt2;     // temporal factor var_t·exp(−Δt²·ilt2/2) (pdim = 3)
  double il_df2, il_cf2;  // 1/ℓ²
  double l_df2;           // ℓ² (scalar kind: the σ² factor of GP_scripts.py:68)
  double ratio, cratio;   // ratio, 1 − ratio
  int same_len;           // ℓ_df == ℓ_cf: one exp serves both parts
};

struct ArdParams {
  int dim, nterms;
  double var[2];
  double ils[2][3];  // 1/ls
};

inline VecParams make_vec_params(const gp2d_kernel_t* k) {
  VecParams p;
  p.kind = k->kind;
  p.il_df2 = 1.0 / (k->l_df * k->l_df);
  p.il_cf2 = 1.0 / (k->l_cf * k->l_cf);
  p.l_df2 = k->l_df * k->l_df;
  p.ratio = k->ratio;
  p.cratio = 1.0 - k->ratio;
  p.same_len = (k->l_df == k->l_cf);
  p.pdim = (k->family == GP2D_FAMILY_VECTOR_ST) ? 3 : 2;
  p.var_t = (p.pdim == 3) ? k->var[0] : 1.0;
  p.ilt2 = (p.pdim == 3) ? 1.0 / (k->ls[0][0] * k->ls[0][0]) : 0.0;
  return p;
}

inline ArdParams make_ard_params(const gp2d_kernel_t* k) {
  ArdParams p;
  p.dim = k->dim;
  p.nterms = k->nterms;
  for (int t = 0; t < 2; ++t) {
    p.var[t] = k->var[t];
    for (int d = 0; d < 3; ++d) p.ils[t][d] = (k->ls[t][d] != 0.0) ? 1.0 / k->ls[t][d] : 0.0;
  }
  return p;
}

// 2×2 block of the SE vector kernels.
__device__ __forceinline__ void vec_block(const VecParams& p, double d1, double d2,
                                          double& k11, double& k12, double& k22) {
  const double r2 = d1 * d1 + d2 * d2;
  const double p11 = d1 * d1, p12 = d1 * d2, p22 = d2 * d2;
  if (p.kind == GP2D_KIND_SCALAR) {
    const double c = r2 * p.il_df2;
    const double s = p.il_df2 * exp(-0.5 * c) * p.l_df2;  // (1/σ²)·exp(−C/2)·σ²
    k11 = s; k12 = s; k22 = s;
    return;
  }
  double f11 = 0.0, f12 = 0.0, f22 = 0.0;
  double e_df = 0.0;
  if (p.kind == GP2D_KIND_DIVFREE || p.kind == GP2D_KIND_MIXED) {
    const double c = r2 * p.il_df2;
    e_df = exp(-0.5 * c);
    const double e = p.il_df2 * e_df;
    const double aux = 1.0 - c;  // (p−1) − C, p = 2
    f11 = e * (p11 * p.il_df2 + aux);
    f12 = e * (p12 * p.il_df2);
    f22 = e * (p22 * p.il_df2 + aux);
    if (p.kind == GP2D_KIND_DIVFREE) { k11 = f11; k12 = f12; k22 = f22; return; }
  }
  const double ccf = r2 * p.il_cf2;
  const double ecf = (p.kind == GP2D_KIND_MIXED && p.same_len) ? e_df : exp(-0.5 * ccf);
  const double e = p.il_cf2 * ecf;
  const double g11 = e * (1.0 - p11 * p.il_cf2);
  const double g12 = -e * (p12 * p.il_cf2);
  const double g22 = e * (1.0 - p22 * p.il_cf2);
  if (p.kind == GP2D_KIND_CURLFREE) { k11 = g11; k12 = g12; k22 = g22; return; }
  k11 = p.ratio * f11 + p.cratio * g11;
  k12 = p.ratio * f12 + p.cratio * g12;
  k22 = p.ratio * f22 + p.cratio * g22;
}

// Coordinates of vector-family point i: time (0 for the purely spatial family) and (x1, x2).
__device__ __forceinline__ void vec_point(const VecParams& p, const double* __restrict__ x, int64_t i, double& t,
                                          double& a, double& b) {
  if (p.pdim == 3) {
    t = x[3 * i]; a = x[3 * i + 1]; b = x[3 * i + 2];
  } else {
    t = 0.0; a = x[2 * i]; b = x[2 * i + 1];
  }
}

// Temporal factor of the spatio-temporal product (GPy RBF on t, myKernel.py:349-352); 1 otherwise.
__device__ __forceinline__ double time_factor(const VecParams& p, double dt) {
  return (p.pdim == 3) ? p.var_t * exp(-0.5 * dt * dt * p.ilt2) : 1.0;
}

// Full 2×2 block of a vector-family kernel: spatial block × temporal factor.
__device__ __forceinline__ void vec_block_st(const VecParams& p, double dt, double d1, double d2, double& k11,
                                             double& k12, double& k22) {
  vec_block(p, d1, d2, k11, k12, k22);
  if (p.pdim == 3) {
    const double f = time_factor(p, dt);
    k11 *= f; k12 *= f; k22 *= f;
  }
}

__device__ __forceinline__ double ard_value(const ArdParams& p, const double* a, const double* b) {
  double k = 0.0;
  for (int t = 0; t < p.nterms; ++t) {
    double s = 0.0;
    for (int d = 0; d < p.dim; ++d) {
      const double z = (a[d] - b[d]) * p.ils[t][d];
      s += z * z;
    }
    k += p.var[t] * exp(-0.5 * s);
  }
  return k;
}

// Block: 64 (column points) × 4 thread rows; each thread does ROWS_PER_THREAD
// row points so that the column point's coordinates are loaded once.
constexpr int ASM_ROWS = 16;
constexpr int ASM_LOWER = 2;   // `symmetric` mode: K_y's lower triangle only (gp2d_assemble)

// j_off / col_comp (gp2d_assemble_cols): column points start at j_off and only the columns of
// component col_comp (0: u, 1: v; −1: both) are written — the same per-element arithmetic.
//
// The workgroup's 64 column points are staged once through LDS (wave 0 loads the tile with one
// coalesced 1–1.5 KB read, every wave reads it back); the row point of a wave is wave-uniform
// (readfirstlane'd index: scalar loads).  symmetric = ASM_LOWER writes only the lower triangle
// (C ≤ R) of the n × n matrix (n = 2·na_pad, component-major) — all gp2d_potrf uses (its
// diagonal kernel loads the 32×32 sub-blocks whole but never uses, nor stores, their upper
// parts; the rest of the upper triangle it zeroes at its end) — i.e. K_uu's and K_vv's lower
// halves and all of K_vu: half the stores, n(n+1)/2 doubles (GP_scripts.py:80-88 likewise
// fills one triangle of compute_K and mirrors it).  Row segments wholly above the diagonal are
// skipped per wave (no kernel evaluation either when all four blocks' segments are).
__global__ __launch_bounds__(256) void assemble_vec_kernel(
    const double* __restrict__ xa, int64_t na, int64_t na_pad,
    const double* __restrict__ xb, int64_t nb, int64_t nb_pad,
    VecParams p, double diag_add, int symmetric, double* __restrict__ out, int64_t ld, int64_t j_off = 0,
    int col_comp = -1) {
  __shared__ double colpts[3 * 64];
  const int64_t jt = j_off + (int64_t)blockIdx.x * 64;   // the tile's first column point
  const int lane = threadIdx.x & 63;
  const int ty = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t j = jt + lane;
  const bool jv = j < nb;
  const bool lower = symmetric == ASM_LOWER;
  if (ty == 0) {
    for (int e = lane; e < p.pdim * 64; e += 64) {   // the tile's points, coalesced
      const int64_t g = jt * p.pdim + e;
      colpts[e] = (g < nb * p.pdim) ? xb[g] : 0.0;
    }
  }
  __syncthreads();
  double b0 = 0.0, b1 = 0.0, b2 = 0.0;
  if (p.pdim == 3) {
    b0 = colpts[3 * lane]; b1 = colpts[3 * lane + 1]; b2 = colpts[3 * lane + 2];
  } else {
    b1 = colpts[2 * lane]; b2 = colpts[2 * lane + 1];
  }
  // lower mode: matrix column C is kept in matrix row R iff C ≤ R; the wave's segments start at
  // column cu (u component) and cv (v component)
  const int64_t cu = jt, cv = nb_pad + jt;
#pragma unroll 1
  for (int q = 0; q < ASM_ROWS / 4; ++q) {
    const int64_t i = (int64_t)blockIdx.y * ASM_ROWS + ty + 4 * q;   // wave-uniform
    if (i >= na_pad) break;
    const int64_t R0 = i, R1 = na_pad + i;   // the pair's rows in the u and v components
    if (lower && cu > R1) continue;          // every segment of this row pair is above the diagonal
    const bool w_uu = !lower || cu + lane <= R0, w_uv = !lower || cv + lane <= R0;
    const bool w_vu = !lower || cu + lane <= R1, w_vv = !lower || cv + lane <= R1;
    double k11, k12, k22;
    if (jv && i < na) {
      double a0, a1, a2;
      vec_point(p, xa, i, a0, a1, a2);
      vec_block_st(p, a0 - b0, a1 - b1, a2 - b2, k11, k12, k22);
      if (symmetric && i == j) { k11 += diag_add; k22 += diag_add; }
    } else {
      const double dd = (symmetric && i == j) ? 1.0 : 0.0;  // padded points: identity rows
      k11 = dd; k12 = 0.0; k22 = dd;
    }
    double* r0 = out + i * ld;
    double* r1 = out + (na_pad + i) * ld;
    if (col_comp != 1) {
      if (w_uu) r0[j] = k11;
      if (w_vu) r1[j] = k12;
    }
    if (col_comp != 0) {
      if (w_uv) r0[nb_pad + j] = k12;
      if (w_vv) r1[nb_pad + j] = k22;
    }
  }
}

__global__ __launch_bounds__(256) void assemble_ard_kernel(
    const double* __restrict__ xa, int64_t na, int64_t na_pad,
    const double* __restrict__ xb, int64_t nb, int64_t nb_pad,
    ArdParams p, double diag_add, int symmetric, double* __restrict__ out, int64_t ld) {
  const int64_t j = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int ty = threadIdx.x >> 6;
  const bool jv = j < nb;
  double b[3] = {0.0, 0.0, 0.0};
  for (int d = 0; d < p.dim; ++d) b[d] = jv ? xb[j * p.dim + d] : 0.0;
#pragma unroll 1
  for (int q = 0; q < ASM_ROWS / 4; ++q) {
    const int64_t i = (int64_t)blockIdx.y * ASM_ROWS + ty + 4 * q;
    if (i >= na_pad) break;
    double k;
    if (jv && i < na) {
      double a[3] = {0.0, 0.0, 0.0};
      for (int d = 0; d < p.dim; ++d) a[d] = xa[i * p.dim + d];
      k = ard_value(p, a, b);
      if (symmetric && i == j) k += diag_add;
    } else {
      k = (symmetric && i == j) ? 1.0 : 0.0;
    }
    out[i * ld + j] = k;
  }
}

}  // namespace gp2d
