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
#include <utility>

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

// ---------------------------------------------------------------------------------------
// Blocked diagonal-block kernel.  The 128×128 block lives in LDS (130 KB, fp64, row pitch
// 130 doubles, so column-strided ds_read_b128 across 16 rows hit 16 distinct bank groups and
// every access is a per-row base plus an immediate offset).  The n sequential pivots of the whole
// factorisation are the critical path of POTRF, so each pivot must be cheap:
//   Cholesky, 4 panels of 32 columns: ONE wave factors the 128−32p × 32 panel with the
//     panel in registers (lane l: rows 32p+l and 32p+64+l) — per pivot a readlane of the
//     diagonal, a sqrt, one LDS write/broadcast-read of the pivot column and ≤ 62 FMAs,
//     no workgroup barrier; then all four waves apply the rank-32 update to the trailing
//     lower 32×32 blocks.
//   Inverse, W = L⁻¹ in place: each wave inverts one 32×32 diagonal block by forward
//     substitution (lane j owns column j, no cross-lane traffic), then block rows
//     i = 1..3:  T_ij = Σ_{p=j}^{i-1} L_ip W_pj,  W_ij = −W_ii T_ij.
constexpr int DP = NB + 2;  // row pitch (doubles): 1040 B ≡ 4 banks mod 64, so 16 rows → 16 bank groups
__device__ __forceinline__ int dsw(int r, int c) { return r * DP + c; }

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// sqrt(d) and 1/sqrt(d) from v_rsq_f64 + two Newton steps (≈ 1 ulp; the Cholesky needs
// accuracy, not correct rounding) — a third of the latency of sqrt() followed by a division,
// and the pivot chain is the critical path of the whole factorisation.
struct Pivot {
  double d, rd, ird;
  int bad;  // 1-based panel column of the first non-positive pivot (0: none)
};
__device__ __forceinline__ Pivot make_pivot(double d) {
  double y = __builtin_amdgcn_rsq(d);
  const double hd = 0.5 * d;
  y = y * fma(-hd * y, y, 1.5);
  y = y * fma(-hd * y, y, 1.5);
  return Pivot{d, d * y, y, 0};
}

// One pivot of the single-wave panel factorisation (K is a compile-time column index so
// that x0/x1 stay in registers).  Column K+1 is updated first and pivot K+1 is formed
// right after it, so its rsq/Newton chain overlaps the remaining FMAs of step K.
template <int K, bool X1>
__device__ __forceinline__ void panel_step(double (&x0)[32], double (&x1)[32], double* colbuf, int lane, int& bad,
                                           Pivot& pv) {
  bad = (bad == 0 && !(pv.d > 0.0)) ? K + 1 : bad;  // no branch: keeps the pivot chain schedulable
  x0[K] = (lane > K) ? x0[K] * pv.ird : ((lane == K) ? pv.rd : x0[K]);
  if constexpr (X1) x1[K] *= pv.ird;
  if constexpr (K < 31) {
    if (lane < 32) colbuf[lane] = x0[K];
    __builtin_amdgcn_wave_barrier();
    constexpr int C0 = (K + 1) & ~1;
    double lc[32];
#pragma unroll
    for (int c = C0; c < 32; c += 2) {
      const d2 t = *reinterpret_cast<const d2*>(colbuf + c);
      lc[c] = t.x;
      lc[c + 1] = t.y;
    }
    x0[K + 1] = fma(-x0[K], lc[K + 1], x0[K + 1]);
    asm volatile("" : "+v"(x0[K + 1]));
    pv = make_pivot(readlane_f64(x0[K + 1], K + 1));
    if constexpr (X1) {
      x1[K + 1] = fma(-x1[K], lc[K + 1], x1[K + 1]);
      asm volatile("" : "+v"(x1[K + 1]));
    }
#pragma unroll
    for (int c = K + 2; c < 32; ++c) {
      x0[c] = fma(-x0[K], lc[c], x0[c]);
      // pin the update here: otherwise the compiler sinks each column's updates to the
      // step that reads it and keeps every step's lc[] alive (hundreds of spilled VGPRs)
      asm volatile("" : "+v"(x0[c]));
      if constexpr (X1) {
        x1[c] = fma(-x1[K], lc[c], x1[c]);
        asm volatile("" : "+v"(x1[c]));
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}
// Returns the 1-based column of the first non-positive pivot of the panel (0: none).
template <bool X1, int... Ks>
__device__ __forceinline__ int panel_steps(std::integer_sequence<int, Ks...>, double (&x0)[32], double (&x1)[32],
                                           double* colbuf, int lane) {
  Pivot pv = make_pivot(readlane_f64(x0[0], 0));
  int bad = 0;
  (panel_step<Ks, X1>(x0, x1, colbuf, lane, bad, pv), ...);
  return bad;
}

// Column step K of the forward substitution L X = I, 32×32 block at b0 (lane ↔ column j
// of X): finalise x[K], then eliminate it from the rows below (pinned like panel_step).
template <int K>
__device__ __forceinline__ void inv_step(double (&x)[32], const double* S, int b0) {
  double lk[32];  // column K below the diagonal: all reads issued before the first use
#pragma unroll
  for (int i = K; i < 32; ++i) lk[i] = S[dsw(b0 + i, b0 + K)];
  x[K] = x[K] * lk[K];  // the diagonal holds 1/L_KK here (see below)
#pragma unroll
  for (int i = K + 1; i < 32; ++i) {
    x[i] = fma(-lk[i], x[K], x[i]);
    asm volatile("" : "+v"(x[i]));
  }
}
template <int... Ks>
__device__ __forceinline__ void inv_steps(std::integer_sequence<int, Ks...>, double (&x)[32], const double* S, int b0) {
  (inv_step<Ks>(x, S, b0), ...);
}

// 4×4 register tile of a 32×32 block product, one wave per block (lane → rows
// xr..xr+3, columns yc..yc+3):  acc[a][b] += Σ_{k<32} X[xr+a][xk+k] · Y(k, yc+b), with
// Y(k, c) = S[yk+k][c] (NT = false) or S[c][yk+k] (NT = true, i.e. Y = the transpose of
// rows yc..yc+3).  Fully unrolled so every LDS read is issued ahead of its FMAs; 16
// independent accumulator chains.
template <bool NT>
__device__ __forceinline__ void tile4x4(const double* __restrict__ S, int xr, int xk, int yk, int yc,
                                        double (&acc)[4][4]) {
#pragma unroll
  for (int k = 0; k < 32; k += 2) {
    d2 x[4], y[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) x[a] = *reinterpret_cast<const d2*>(S + dsw(xr + a, xk + k));
    if constexpr (NT) {
#pragma unroll
      for (int b = 0; b < 4; ++b) y[b] = *reinterpret_cast<const d2*>(S + dsw(yc + b, yk + k));
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          acc[a][b] = fma(x[a].x, y[b].x, acc[a][b]);
          acc[a][b] = fma(x[a].y, y[b].y, acc[a][b]);
        }
    } else {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        y[2 * u] = *reinterpret_cast<const d2*>(S + dsw(yk + k + u, yc));
        y[2 * u + 1] = *reinterpret_cast<const d2*>(S + dsw(yk + k + u, yc + 2));
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        acc[a][0] = fma(x[a].x, y[0].x, acc[a][0]);
        acc[a][1] = fma(x[a].x, y[0].y, acc[a][1]);
        acc[a][2] = fma(x[a].x, y[1].x, acc[a][2]);
        acc[a][3] = fma(x[a].x, y[1].y, acc[a][3]);
        acc[a][0] = fma(x[a].y, y[2].x, acc[a][0]);
        acc[a][1] = fma(x[a].y, y[2].y, acc[a][1]);
        acc[a][2] = fma(x[a].y, y[3].x, acc[a][2]);
        acc[a][3] = fma(x[a].y, y[3].y, acc[a][3]);
      }
    }
  }
}

__device__ __forceinline__ void tile4x4_zero(double (&acc)[4][4]) {
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
}

// S[r+a][c..c+3] = sgn·acc[a][..] + (accumulate ? S[r+a][c..c+3] : 0)
__device__ __forceinline__ void tile4x4_store(double* __restrict__ S, int r, int c, const double (&acc)[4][4],
                                              double sgn, bool accumulate) {
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    d2* o0 = reinterpret_cast<d2*>(S + dsw(r + a, c));
    d2* o1 = reinterpret_cast<d2*>(S + dsw(r + a, c + 2));
    const d2 b0 = accumulate ? *o0 : d2{0.0, 0.0}, b1 = accumulate ? *o1 : d2{0.0, 0.0};
    *o0 = d2{fma(sgn, acc[a][0], b0.x), fma(sgn, acc[a][1], b0.y)};
    *o1 = d2{fma(sgn, acc[a][2], b1.x), fma(sgn, acc[a][3], b1.y)};
  }
}

// inv_in_place (the fused factor + inverse, gp2d_potrf_inv): A's diagonal block receives
// W_kk = L_kk⁻¹ instead of L_kk (nothing reads L_kk from A after this kernel: the panel TRSM
// uses dinv), which is TRTRI's level 0.
__global__ __launch_bounds__(256) void potrf_diag_kernel(double* __restrict__ A, int64_t lda, int k0,
                                                         double* __restrict__ dinv, int* info, int inv_in_place) {
  __shared__ __attribute__((aligned(16))) double S[NB * DP];
  __shared__ __attribute__((aligned(16))) double colbuf[32];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  double* Ab = A + (int64_t)k0 * lda + k0;
  GP2D_STAMP(0);
  // load: 16-B vectors, rows coalesced, 8 loads in flight per thread
#pragma unroll 1
  for (int e0 = 0; e0 < (NB * NB / 2) / 256; e0 += 8) {
    d2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = tid + 256 * (e0 + u), r = idx >> 6, ch = idx & 63;
      v[u] = *reinterpret_cast<const d2*>(Ab + (int64_t)r * lda + 2 * ch);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = tid + 256 * (e0 + u), r = idx >> 6, ch = idx & 63;
      *reinterpret_cast<d2*>(S + dsw(r, 2 * ch)) = v[u];
    }
  }
  __syncthreads();
  GP2D_STAMP(1);
  // ---- Cholesky
  // row mapping inside the per-wave 32×32 tiles of the trailing update: 8 rows per wave,
  // 4 consecutive columns per lane
  const int tr4 = 4 * (lane >> 3), tc4 = 4 * (lane & 7);  // 4×4 tile of a 32×32 block
  for (int p = 0; p < 4; ++p) {
    const int c0 = 32 * p;
    if (wid == 0) {
      const int r0 = c0 + lane, r1 = c0 + 64 + lane;
      const bool v0 = r0 < NB, v1 = r1 < NB;
      // rows past the block read a clamped (valid) row and are never written back
      double* p0 = S + dsw(v0 ? r0 : NB - 1, c0);
      double* p1 = S + dsw(v1 ? r1 : NB - 1, c0);
      double x0[32], x1[32];
#pragma unroll
      for (int c = 0; c < 32; c += 2) {
        const d2 t0 = *reinterpret_cast<const d2*>(p0 + c);
        const d2 t1 = *reinterpret_cast<const d2*>(p1 + c);
        x0[c] = t0.x; x0[c + 1] = t0.y;
        x1[c] = t1.x; x1[c + 1] = t1.y;
      }
      // rows c0+64+lane exist only for the first two panels
      const int bad = (p < 2) ? panel_steps<true>(std::make_integer_sequence<int, 32>{}, x0, x1, colbuf, lane)
                              : panel_steps<false>(std::make_integer_sequence<int, 32>{}, x0, x1, colbuf, lane);
      if (bad && lane == 0 && info) atomicCAS(info, 0, k0 + c0 + bad);
      if (v0) {
#pragma unroll
        for (int c = 0; c < 32; c += 2) *reinterpret_cast<d2*>(p0 + c) = d2{x0[c], x0[c + 1]};
      }
      if (v1) {
#pragma unroll
        for (int c = 0; c < 32; c += 2) *reinterpret_cast<d2*>(p1 + c) = d2{x1[c], x1[c + 1]};
      }
    }
    __syncthreads();
    GP2D_STAMP(8 + 2 * p);
    // trailing update of the lower 32×32 blocks (bi, bj), p < bj <= bi < 4: one wave per
    // block, blocks dealt round-robin to the waves
    {
      const int t = 3 - p;  // trailing blocks per side
      const int nblk = t * (t + 1) / 2;
      for (int q = wid; q < nblk; q += 4) {
        // q → (bi, bj) in row-major lower order over the trailing t×t block triangle
        int bi = 0;
        while ((bi + 1) * (bi + 2) / 2 <= q) ++bi;
        const int bj = q - bi * (bi + 1) / 2;
        const int r = 32 * (p + 1 + bi) + tr4, cc = 32 * (p + 1 + bj) + tc4;
        double acc[4][4];
        tile4x4_zero(acc);
        tile4x4<true>(S, r, c0, c0, cc, acc);
        tile4x4_store(S, r, cc, acc, -1.0, true);
      }
    }
    __syncthreads();
    GP2D_STAMP(9 + 2 * p);
  }
  GP2D_STAMP(2);
  // ---- store L (zero strict upper)
#pragma unroll 1
  for (int e = 0; e < (inv_in_place ? 0 : (NB * NB / 2) / 256); ++e) {
    const int idx = tid + 256 * e, r = idx >> 6, c = 2 * (idx & 63);
    const d2 v = *reinterpret_cast<const d2*>(S + dsw(r, c));
    *reinterpret_cast<d2*>(Ab + (int64_t)r * lda + c) = d2{(c <= r) ? v.x : 0.0, (c + 1 <= r) ? v.y : 0.0};
  }
  GP2D_STAMP(3);
  if (!dinv) return;
  // ---- inverse: 32×32 diagonal blocks, wave w ↔ block w, lane j ↔ column j.  The LDS
  // diagonal is replaced by its reciprocals first (L is already stored), so each
  // substitution step is a multiply, not a division.
  __syncthreads();  // the L store above has read the diagonal
  if (tid < NB) S[dsw(tid, tid)] = 1.0 / S[dsw(tid, tid)];
  __syncthreads();
  GP2D_STAMP(5);
  {
    const int b0 = 32 * wid, j = lane & 31;
    double x[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) x[i] = (i == j) ? 1.0 : 0.0;
    inv_steps(std::make_integer_sequence<int, 32>{}, x, S, b0);
    __builtin_amdgcn_wave_barrier();
    if (lane < 32) {
#pragma unroll
      for (int i = 0; i < 32; ++i) S[dsw(b0 + i, b0 + j)] = x[i];  // lower part: x[i] = 0 for i < j
    }
  }
  __syncthreads();
  GP2D_STAMP(6);
  // ---- off-diagonal blocks by recursive doubling, W = [[W11, 0], [−W22·L21·W11, W22]]:
  //   level 1 (32 → 64): wave 0 forms W_10 = −W_11 (L_10 W_00), wave 1 W_32 = −W_33 (L_32 W_22);
  //   level 2 (64 → 128): T = L21·W11 (wave w ↔ block (2 + w/2, w%2)), stored over L21, then
  //   W21 = −W22·T.  Each 32×32 product is one wave's 4×4-per-lane register tile.
  {
    double acc[4][4];
    // level 1
    const int lb = 2 * wid;  // wave 0: blocks (1,0), 1: (3,2)
    const int r1 = 32 * (lb + 1) + tr4, c1 = 32 * lb + tc4;
    tile4x4_zero(acc);
    if (wid < 2) tile4x4<false>(S, r1, 32 * lb, 32 * lb, c1, acc);         // L_{lb+1,lb} W_{lb,lb}
    __syncthreads();
    if (wid < 2) tile4x4_store(S, r1, c1, acc, 1.0, false);
    __syncthreads();
    tile4x4_zero(acc);
    if (wid < 2) tile4x4<false>(S, r1, 32 * (lb + 1), 32 * (lb + 1), c1, acc);  // W_{lb+1,lb+1} T
    __syncthreads();
    if (wid < 2) tile4x4_store(S, r1, c1, acc, -1.0, false);
    __syncthreads();
    // level 2: T_ij = Σ_p L_ip W_pj over p ∈ {0,1} with W_pj = 0 for p < j
    const int bi = 2 + (wid >> 1), bj = wid & 1;
    const int r2 = 32 * bi + tr4, c2 = 32 * bj + tc4;
    tile4x4_zero(acc);
    for (int p = bj; p < 2; ++p) tile4x4<false>(S, r2, 32 * p, 32 * p, c2, acc);
    __syncthreads();
    tile4x4_store(S, r2, c2, acc, 1.0, false);
    __syncthreads();
    // W_ij = −Σ_{q=2}^{i} W_iq T_qj
    tile4x4_zero(acc);
    for (int q = 2; q <= bi; ++q) tile4x4<false>(S, r2, 32 * q, 32 * q, c2, acc);
    __syncthreads();
    tile4x4_store(S, r2, c2, acc, -1.0, false);
    __syncthreads();
  }
  GP2D_STAMP(4);
  double* D = dinv + (int64_t)(k0 / NB) * NB * NB;
#pragma unroll 1
  for (int e = 0; e < (NB * NB / 2) / 256; ++e) {
    const int idx = tid + 256 * e, r = idx >> 6, c = 2 * (idx & 63);
    const d2 v = *reinterpret_cast<const d2*>(S + dsw(r, c));
    const d2 w = d2{(c <= r) ? v.x : 0.0, (c + 1 <= r) ? v.y : 0.0};
    *reinterpret_cast<d2*>(D + (int64_t)r * NB + c) = w;
    if (inv_in_place) *reinterpret_cast<d2*>(Ab + (int64_t)r * lda + c) = w;
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
