// lml.hpp — log marginal likelihood and its hyperparameter gradient.
//
// Replaces the objective GPy's model.optimize / optimize_restarts evaluates
// (krig.py:450, GP_plots.py:673-765: GPy exact Gaussian inference) and
// sklearn's log_marginal_likelihood(theta, eval_gradient=True) (_gpr.py:584-650):
//
//   LML      = −½ yᵀα − Σ_i log L_ii − (n_obs/2) log 2π          α = K_y⁻¹ y
//   ∂LML/∂θ  = ½ tr((ααᵀ − K_y⁻¹) ∂K_y/∂θ)
//
// From the fitted W = L⁻¹: log L_ii = −log W_ii, and K_y⁻¹ = WᵀW, formed as the
// lower tiles of the NN product Wᵀ·W on the FP64 MFMA GEMM (c_lower; Wᵀ upper
// triangular, so row block i only needs k ≥ i: a_upper; n³/3 flops).
//
// The trace is one fused pass: a thread per training-point pair (p, q) regenerates
// the 2×2 block ∂K/∂θ on the fly (no n×n derivative matrices are stored) and
// contracts it with the stored (row ≥ column) entries of ααᵀ − K_y⁻¹:
//   vu block (np+p, q): every pair, weight 2 (the uv block is its transpose);
//   uu, vv blocks: pairs p ≥ q, weight 2 off the diagonal, 1 on it.  Per-block partial sums are reduced in a fixed order, so the
// result is deterministic.
//
// The reference's own gradient (myKernel.update_gradients_full, myKernel.py:59-105)
// is not a derivative of its kernel (the (2ℓ²−Cℓ²)/ℓ⁵ term has the wrong sign and
// dA/dℓ lacks the 1/ℓ² factor; SURVEY.md §0.2 lists the gradient paths as broken).
// This file implements the exact derivative; DESIGN.md §3.2 documents the quirk.
#pragma once
#include "common.hpp"
#include "assemble.hpp"

namespace gp2d {

constexpr int LML_MAXG = 9;   // ARD: 2 variances + 2×3 length scales + noise
constexpr int LML_ROWS = 16;  // row points per block (4 per thread row)

// Wt = Wᵀ through a 64×65 LDS tile (both sides coalesced).
__global__ __launch_bounds__(256) void transpose_kernel(const double* __restrict__ W, int64_t n, int64_t ldw,
                                                        double* __restrict__ Wt) {
  __shared__ double t[64][65];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;  // source tile of W
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll 4
  for (int r = ty; r < 64; r += 4) t[r][tx] = W[(r0 + r) * ldw + c0 + tx];
  __syncthreads();
#pragma unroll 4
  for (int c = ty; c < 64; c += 4) Wt[(c0 + c) * n + r0 + tx] = t[tx][c];
}

// LML = −½ Σ y_i α_i + Σ log W_ii − (n_obs/2) log 2π (padded rows: W_ii = 1, y_i = 0) — one block,
// fixed order.
__global__ __launch_bounds__(256) void lml_terms_kernel(const double* __restrict__ W, int64_t n, int64_t ldw,
                                                        const double* __restrict__ alpha, const double* __restrict__ y,
                                                        int64_t nobs, double* __restrict__ out) {
  __shared__ double red[2][256];
  const int tid = threadIdx.x;
  double lw = 0.0, ya = 0.0;
  for (int64_t i = tid; i < n; i += 256) {
    lw += log(W[i * ldw + i]);
    ya += y[i] * alpha[i];
  }
  red[0][tid] = lw;
  red[1][tid] = ya;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) {
      red[0][tid] += red[0][tid + s];
      red[1][tid] += red[1][tid + s];
    }
    __syncthreads();
  }
  if (tid == 0) out[0] = -0.5 * red[1][0] + red[0][0] - 0.5 * (double)nobs * log(2.0 * M_PI);
}

// ∂/∂(ℓ_df, ℓ_cf, ratio) of the 2×2 block (k11, k12, k22) at separation (d1, d2).
// With u = 1/ℓ_df², E = exp(−r²u/2), Q = P·u + δ(1 − r²u) (P_ab = d_a d_b):
//   f = u E Q,   ∂f/∂u = E [Q (1 − u r²/2) + u (P − δ r²)],   ∂f/∂ℓ = ∂f/∂u · (−2u/ℓ);
// with v = 1/ℓ_cf², E' = exp(−r²v/2), G = δ − P·v:
//   g = v E' G,  ∂g/∂v = E' [G (1 − v r²/2) − v P],           ∂g/∂ℓ_cf = ∂g/∂v · (−2v/ℓ_cf);
// mixed K = ρ f + (1−ρ) g: ∂K/∂ℓ_df = ρ ∂f/∂ℓ, ∂K/∂ℓ_cf = (1−ρ) ∂g/∂ℓ_cf, ∂K/∂ρ = f − g.
// Scalar kind (σ = ℓ_df): K = exp(−r²/(2σ²)), ∂K/∂σ = K r²/σ³ (all four entries).
struct VecGradParams {
  VecParams p;
  double l_df, l_cf, l_t;
};

__device__ __forceinline__ void vec_block_grad(const VecGradParams& gp, double d1, double d2, double g[3][3]) {
  const VecParams& p = gp.p;
  const double r2 = d1 * d1 + d2 * d2;
  const double P[3] = {d1 * d1, d1 * d2, d2 * d2};
  const double D[3] = {1.0, 0.0, 1.0};
#pragma unroll
  for (int a = 0; a < 3; ++a) g[a][0] = g[a][1] = g[a][2] = 0.0;
  if (p.kind == GP2D_KIND_SCALAR) {
    const double u = p.il_df2;
    const double v = exp(-0.5 * r2 * u) * r2 * u / gp.l_df;
    g[0][0] = g[0][1] = g[0][2] = v;
    return;
  }
  double f[3] = {0.0, 0.0, 0.0}, df[3] = {0.0, 0.0, 0.0};
  if (p.kind == GP2D_KIND_DIVFREE || p.kind == GP2D_KIND_MIXED) {
    const double u = p.il_df2;
    const double E = exp(-0.5 * r2 * u);
    const double h = 1.0 - 0.5 * u * r2;
    const double s = -2.0 * u / gp.l_df;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const double Q = P[e] * u + D[e] * (1.0 - r2 * u);
      f[e] = u * E * Q;
      df[e] = E * (Q * h + u * (P[e] - D[e] * r2)) * s;
    }
  }
  double c[3] = {0.0, 0.0, 0.0}, dc[3] = {0.0, 0.0, 0.0};
  if (p.kind == GP2D_KIND_CURLFREE || p.kind == GP2D_KIND_MIXED) {
    const double v = p.il_cf2;
    const double E = exp(-0.5 * r2 * v);
    const double h = 1.0 - 0.5 * v * r2;
    const double s = -2.0 * v / gp.l_cf;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const double G = D[e] - P[e] * v;
      c[e] = v * E * G;
      dc[e] = E * (G * h - v * P[e]) * s;
    }
  }
  if (p.kind == GP2D_KIND_DIVFREE) {
#pragma unroll
    for (int e = 0; e < 3; ++e) g[0][e] = df[e];
  } else if (p.kind == GP2D_KIND_CURLFREE) {
#pragma unroll
    for (int e = 0; e < 3; ++e) g[1][e] = dc[e];
  } else {
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      g[0][e] = p.ratio * df[e];
      g[1][e] = p.cratio * dc[e];
      g[2][e] = f[e] - c[e];
    }
  }
}

template <int NV>
__device__ __forceinline__ void block_reduce_vec(const double* v, double (*red)[256], double* out) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int a = 0; a < NV; ++a) red[a][tid] = v[a];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) {
#pragma unroll
      for (int a = 0; a < NV; ++a) red[a][tid] += red[a][tid + s];
    }
    __syncthreads();
  }
  if (tid < NV) out[tid] = red[tid][0];
}

// Gradient accumulators live in fixed slots so that every index is a compile-time constant
// (no scratch): vector families 0 = l_df, 1 = l_cf, 2 = ratio, 3 = noise, 4 = var_t, 5 = l_t
// (spatio-temporal product); ARD t·4 = var_t, t·4+1+d = ls_td, 8 = noise.  SlotMap lists the
// slots in the output order.
struct SlotMap {
  int ng;
  int slot[LML_MAXG];
};

// Spatio-temporal product K = c_t(Δt)·K_s with c_t = var_t·exp(−Δt²/(2ℓ_t²)):
//   ∂K/∂θ_s = c_t ∂K_s/∂θ_s,  ∂K/∂var_t = exp(·)·K_s,  ∂K/∂ℓ_t = c_t·Δt²/ℓ_t³·K_s.
__device__ __forceinline__ void vec_grad_accum(const VecGradParams& gp, double dt, double d1, double d2, double w11,
                                               double w12, double w22, double* acc) {
  double g[3][3];
  vec_block_grad(gp, d1, d2, g);
  double ct = 1.0;
  if (gp.p.pdim == 3) {
    const double e = exp(-0.5 * dt * dt * gp.p.ilt2);
    ct = gp.p.var_t * e;
    double k11, k12, k22;
    vec_block(gp.p, d1, d2, k11, k12, k22);
    const double ws = w11 * k11 + w12 * k12 + w22 * k22;
    acc[4] += e * ws;
    acc[5] += ct * dt * dt * gp.p.ilt2 / gp.l_t * ws;
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) acc[a] += ct * (w11 * g[a][0] + w12 * g[a][1] + w22 * g[a][2]);
}

// ∂k/∂var_t = e_t, ∂k/∂ls_td = var_t·e_t·z_d²/ls_td (z_d = Δ_d/ls_td), weighted by w.
__device__ __forceinline__ void ard_grad_accum(const ArdParams& ap, const double* a, const double* b, double w,
                                               double* acc) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (t < ap.nterms) {
      double z2[3] = {0.0, 0.0, 0.0}, s = 0.0;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        if (d < ap.dim) {
          const double z = (a[d] - b[d]) * ap.ils[t][d];
          z2[d] = z * z;
          s += z2[d];
        }
      }
      const double e = exp(-0.5 * s);
      acc[t * 4] += w * e;
      const double we = w * ap.var[t] * e;
#pragma unroll
      for (int d = 0; d < 3; ++d)
        if (d < ap.dim) acc[t * 4 + 1 + d] += we * z2[d] * ap.ils[t][d];
    }
  }
}

__device__ __forceinline__ void load_point(const double* x, int64_t i, int dim, double* a) {
#pragma unroll
  for (int d = 0; d < 3; ++d) a[d] = (d < dim) ? x[i * dim + d] : 0.0;
}

// Vector family: partial[block][slots 0..3] = Σ over the block's pairs of
// (ααᵀ − K_y⁻¹) ⊙ ∂K/∂(ℓ_df, ℓ_cf, ratio) and the noise term Σ_diag (α_a² − K_y⁻¹_aa).
// Grid (ntr_pad/64, ceil(ntr/16)); C = K_y⁻¹, lower triangle, n × n.
__global__ __launch_bounds__(256) void lml_grad_vec_kernel(const double* __restrict__ C, int64_t n,
                                                           const double* __restrict__ alpha,
                                                           const double* __restrict__ x, int64_t ntr, int64_t np,
                                                           VecGradParams gp, double* __restrict__ partial) {
  __shared__ double red[6][256];
  const int64_t q = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int ty = threadIdx.x >> 6;
  double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  if (q < ntr) {
    double b0, b1, b2;
    vec_point(gp.p, x, q, b0, b1, b2);
    const double aqu = alpha[q], aqv = alpha[np + q];
#pragma unroll 1
    for (int r = 0; r < LML_ROWS / 4; ++r) {
      const int64_t p = (int64_t)blockIdx.y * LML_ROWS + ty + 4 * r;
      if (p >= ntr) break;
      const double apu = alpha[p], apv = alpha[np + p];
      const double* cu = C + p * n;          // row p (u)
      const double* cv = C + (np + p) * n;   // row np+p (v)
      // vu entry (np+p, q): always in the stored triangle; weight 2 (uv is its transpose)
      const double mvu = apv * aqu - cv[q];
      double w11 = 0.0, w22 = 0.0;
      if (p >= q) {
        const double wt = (p == q) ? 1.0 : 2.0;
        w11 = wt * (apu * aqu - cu[q]);
        w22 = wt * (apv * aqv - cv[np + q]);
        if (p == q) acc[3] += w11 + w22;
      }
      double a0, a1, a2;
      vec_point(gp.p, x, p, a0, a1, a2);
      vec_grad_accum(gp, a0 - b0, a1 - b1, a2 - b2, w11, 2.0 * mvu, w22, acc);
    }
  }
  block_reduce_vec<6>(acc, red, partial + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * LML_MAXG);
}

// ARD family (slots t·4 + {0: var, 1+d: ls_d}, 8: noise); pairs p ≥ q of the stored triangle.
__global__ __launch_bounds__(256) void lml_grad_ard_kernel(const double* __restrict__ C, int64_t n,
                                                           const double* __restrict__ alpha,
                                                           const double* __restrict__ x, int64_t ntr, ArdParams ap,
                                                           double* __restrict__ partial) {
  __shared__ double red[LML_MAXG][256];
  const int64_t q = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int ty = threadIdx.x >> 6;
  double acc[LML_MAXG];
#pragma unroll
  for (int a = 0; a < LML_MAXG; ++a) acc[a] = 0.0;
  if (q < ntr) {
    double b[3], a[3];
    load_point(x, q, ap.dim, b);
    const double aq = alpha[q];
#pragma unroll 1
    for (int r = 0; r < LML_ROWS / 4; ++r) {
      const int64_t p = (int64_t)blockIdx.y * LML_ROWS + ty + 4 * r;
      if (p >= ntr) break;
      if (p < q) continue;
      const double wt = ((p == q) ? 1.0 : 2.0) * (alpha[p] * aq - C[p * n + q]);
      load_point(x, p, ap.dim, a);
      ard_grad_accum(ap, a, b, wt, acc);
      if (p == q) acc[8] += wt;
    }
  }
  block_reduce_vec<LML_MAXG>(acc, red, partial + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * LML_MAXG);
}

// GPy Kern.update_gradients_full (myKernel.py:59-105, exact derivative): Σ_ab G_ab ∂K_ab/∂θ for a
// caller-supplied G = dL/dK, (bd·na) × (bd·nb) component-major without padding, leading dim ld.
// Grid (ceil(nb/64), ceil(na/16)).
__global__ __launch_bounds__(256) void kgrad_vec_kernel(const double* __restrict__ xa, int64_t na,
                                                        const double* __restrict__ xb, int64_t nb, VecGradParams gp,
                                                        const double* __restrict__ G, int64_t ld,
                                                        double* __restrict__ partial) {
  __shared__ double red[6][256];
  const int64_t q = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int ty = threadIdx.x >> 6;
  double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  if (q < nb) {
    double b0, b1, b2;
    vec_point(gp.p, xb, q, b0, b1, b2);
#pragma unroll 1
    for (int r = 0; r < LML_ROWS / 4; ++r) {
      const int64_t p = (int64_t)blockIdx.y * LML_ROWS + ty + 4 * r;
      if (p >= na) break;
      const double* g0 = G + p * ld;
      const double* g1 = G + (na + p) * ld;
      double a0, a1, a2;
      vec_point(gp.p, xa, p, a0, a1, a2);
      vec_grad_accum(gp, a0 - b0, a1 - b1, a2 - b2, g0[q], g0[nb + q] + g1[q], g1[nb + q], acc);
    }
  }
  block_reduce_vec<6>(acc, red, partial + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * LML_MAXG);
}

__global__ __launch_bounds__(256) void kgrad_ard_kernel(const double* __restrict__ xa, int64_t na,
                                                        const double* __restrict__ xb, int64_t nb, ArdParams ap,
                                                        const double* __restrict__ G, int64_t ld,
                                                        double* __restrict__ partial) {
  __shared__ double red[LML_MAXG][256];
  const int64_t q = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int ty = threadIdx.x >> 6;
  double acc[LML_MAXG];
#pragma unroll
  for (int a = 0; a < LML_MAXG; ++a) acc[a] = 0.0;
  if (q < nb) {
    double b[3], a[3];
    load_point(xb, q, ap.dim, b);
#pragma unroll 1
    for (int r = 0; r < LML_ROWS / 4; ++r) {
      const int64_t p = (int64_t)blockIdx.y * LML_ROWS + ty + 4 * r;
      if (p >= na) break;
      load_point(xa, p, ap.dim, a);
      ard_grad_accum(ap, a, b, G[p * ld + q], acc);
    }
  }
  block_reduce_vec<LML_MAXG>(acc, red, partial + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * LML_MAXG);
}

// out[g] = scale · Σ_blocks partial[block][slot[g]], fixed order (one 256-thread block per entry).
__global__ __launch_bounds__(256) void grad_sum_kernel(const double* __restrict__ partial, int64_t nblk, SlotMap sm,
                                                       double scale, double* __restrict__ out) {
  __shared__ double red[1][256];
  const int slot = sm.slot[blockIdx.x];
  double s = 0.0;
  for (int64_t b = threadIdx.x; b < nblk; b += 256) s += partial[b * LML_MAXG + slot];
  double tot = 0.0;
  block_reduce_vec<1>(&s, red, &tot);  // thread 0 receives the total
  if (threadIdx.x == 0) out[blockIdx.x] = scale * tot;
}

}  // namespace gp2d
