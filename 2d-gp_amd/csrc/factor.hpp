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
// Blocked diagonal-block kernel.  The lower 128×128 block lives in LDS in a block-lower
// layout: 32-row block row rb keeps columns [0, 32(rb+1)) — the whole of its diagonal 32×32
// block, nothing right of it — at a row pitch of 32(rb+1) + 2 doubles (≡ 16 B mod 256 B, so
// column-strided ds_read_b128 across 16 rows hit 16 distinct bank groups).  82 KB instead of
// the 130 KB of a full-pitch square: the kernel then fits on a CU beside one workgroup of the
// trailing SYRK (72 KB), where the square needed an empty CU and waited up to 240 µs for one
// while the SYRK held every CU.  The n sequential pivots of the whole factorisation are the
// critical path of POTRF, so each pivot must be cheap:
//   Cholesky, 4 panels of 32 columns: ONE wave factors the 128−32p × 32 panel with the
//     panel in registers (lane l: rows 32p+l and 32p+64+l) — per pivot a readlane of the
//     diagonal, a sqrt, one LDS write/broadcast-read of the pivot column and ≤ 62 FMAs,
//     no workgroup barrier; then all four waves apply the rank-32 update to the trailing
//     lower 32×32 blocks.
//   Inverse, W = L⁻¹ in place: each wave inverts one 32×32 diagonal block by forward
//     substitution (lane j owns column j, no cross-lane traffic), then block rows
//     i = 1..3:  T_ij = Σ_{p=j}^{i-1} L_ip W_pj,  W_ij = −W_ii T_ij.
__host__ __device__ constexpr int dpitch(int rb) { return 32 * rb + 34; }   // doubles per row of block row rb
// first double of block row rb: 32 · Σ_{i<rb} dpitch(i)
__host__ __device__ constexpr int dbase(int rb) { return 512 * rb * (rb - 1) + 1088 * rb; }
constexpr int DS_DOUBLES = dbase(NB / 32);   // 10,496 doubles = 82 KB
static_assert(dbase(1) == 32 * dpitch(0) && dbase(2) == dbase(1) + 32 * dpitch(1) &&
                  dbase(3) == dbase(2) + 32 * dpitch(2) && DS_DOUBLES == dbase(3) + 32 * dpitch(3),
              "block-lower LDS layout");
__device__ __forceinline__ int dsw(int r, int c) {
  const int rb = r >> 5;
  return dbase(rb) + (r & 31) * dpitch(rb) + c;
}
__device__ __forceinline__ int drowlen(int r) { return 32 * ((r >> 5) + 1); }   // stored columns of row r

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
// The multipliers L[c][K] come through one LDS broadcast of the column.  (Taking the next 1, 2
// or 4 columns' multipliers straight from lane c's register by v_readlane instead, so the pivot
// chain K → K+1 carries no LDS round trip (git 00ed20f, GP2D_PANEL_RL), measured
// 54.4–54.9 µs per diagonal block against 54.0 µs — the panel wave is issue-bound on its
// 2·(31 − K) FMAs per pivot, not bound by the broadcast's latency; tools/microbench diag_bench_rl*.
// Round 5 took the chain itself off the issue stream — uniform-value pivot chain, bulk update one
// step late, broadcast under the next pivot — bit-identical and −1.2 %: a lone wave's issue of
// the whole step sets the pivot time; profiles/r05_diag_panel_ab.txt, git 9434024.)
template <int K, bool X1>
__device__ __forceinline__ void panel_step(double (&x0)[32], double (&x1)[32], double* colbuf, int lane, int& bad,
                                           Pivot& pv) {
  bad = (bad == 0 && !(pv.d > 0.0)) ? K + 1 : bad;  // no branch: keeps the pivot chain schedulable
  x0[K] = (lane >= K) ? x0[K] * pv.ird : x0[K];   // lane K: x0[K] = d, so d·(1/√d) = rd exactly
  if constexpr (X1) x1[K] *= pv.ird;
  if constexpr (K < 31) {
    double lc[32];
    constexpr int C0 = (K + 1) & ~1;
    if constexpr (C0 < 32) {
      colbuf[lane] = x0[K];   // all 64 lanes (entries 32–63 unread): no EXEC mask around the store
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int c = C0; c < 32; c += 2) {
        const d2 t = *reinterpret_cast<const d2*>(colbuf + c);
        if (c > K) lc[c] = t.x;
        lc[c + 1] = t.y;
      }
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

// 32×32 block products of the diagonal kernel on the f64 matrix core (round 5): one wave, 2×2
// tiles of v_mfma_f64_16x16x4f64, K = 32 in 8 steps of 4.  Operands: a = X[row l&15][k l>>4],
// b = Y(k l>>4, col l&15); acc[ti][tj][r] is C[16ti + (l>>4) + 4r][16tj + (l&15)].  A tenth of
// the LDS bytes per product of the FMA register tiles it replaced (16 vs 128 KB per wave; those
// are at git 00ed20f).
typedef d4 tileacc_t[2][2];
template <bool NT>
__device__ __forceinline__ void tile32_mfma(const double* __restrict__ S, int xr, int xk, int yk, int yc,
                                            tileacc_t& acc, int l16, int lk) {
#pragma unroll
  for (int k0 = 0; k0 < 32; k0 += 4) {
    double a[2], b[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      a[t] = S[dsw(xr + 16 * t + l16, xk + k0 + lk)];
      b[t] = NT ? S[dsw(yc + 16 * t + l16, yk + k0 + lk)] : S[dsw(yk + k0 + lk, yc + 16 * t + l16)];
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 2; ++tj) acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ti], b[tj], acc[ti][tj], 0, 0, 0);
  }
}
__device__ __forceinline__ void tile32_zero(tileacc_t& acc) {
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj) acc[ti][tj] = d4{0.0, 0.0, 0.0, 0.0};
}
// S[r0 + …][c0 + …] = sgn·acc + (accumulate ? S : 0), the MFMA output map
__device__ __forceinline__ void tile32_store(double* __restrict__ S, int r0, int c0, const tileacc_t& acc, double sgn,
                                             bool accumulate, int l16, int lk) {
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double* o = S + dsw(r0 + 16 * ti + lk + 4 * r, c0 + 16 * tj + l16);
        *o = fma(sgn, acc[ti][tj][r], accumulate ? *o : 0.0);
      }
}

// Column step K of the forward substitution of a 16×16 block at rows/cols rb0 (lane ↔ column
// j = lane & 15 of its half's block; rk = 1 / L_KK of that block): as inv_step, 16 wide.
template <int K>
__device__ __forceinline__ void inv16_step(double (&x)[16], const double* S, int rb0, double rk) {
  double lk[16];
#pragma unroll
  for (int i = K + 1; i < 16; ++i) lk[i] = S[dsw(rb0 + i, rb0 + K)];
  x[K] = x[K] * rk;
#pragma unroll
  for (int i = K + 1; i < 16; ++i) {
    x[i] = fma(-lk[i], x[K], x[i]);
    asm volatile("" : "+v"(x[i]));
  }
}
template <int... Ks>
__device__ __forceinline__ void inv16_steps(std::integer_sequence<int, Ks...>, double (&x)[16], const double* S, int rb0,
                                            double rl, int h) {
  (inv16_step<Ks>(x, S, rb0, h ? readlane_f64(rl, 16 + Ks) : readlane_f64(rl, Ks)), ...);
}

// inv_in_place (the fused factor + inverse, gp2d_potrf_inv): A's diagonal block receives
// W_kk = L_kk⁻¹ instead of L_kk (nothing reads L_kk from A after this kernel: the panel TRSM
// uses dinv), which is TRTRI's level 0.
// Problem batch (gp2d_potrf_batched): workgroup b factors problem b — A + b·sA, dinv + b·sD,
// info + b (one workgroup and sA = sD = 0 for a lone factorisation).
__global__ __launch_bounds__(256) void potrf_diag_kernel(double* __restrict__ A, int64_t lda, int k0,
                                                         double* __restrict__ dinv, int* info, int inv_in_place,
                                                         int64_t sA = 0, int64_t sD = 0) {
  __shared__ __attribute__((aligned(16))) double S[DS_DOUBLES];
  __shared__ __attribute__((aligned(16))) double colbuf[64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  A += blockIdx.x * sA;
  if (dinv) dinv += blockIdx.x * sD;
  if (info) info += blockIdx.x;
  double* Ab = A + (int64_t)k0 * lda + k0;
  GP2D_STAMP(0);
  // load the stored (block-lower) part: block row rb is 32 rows × 16(rb+1) 16-B vectors, rows
  // coalesced; all 20 loads of a thread in flight before the first LDS store
  {
    d2 v[20];
    auto each = [&](auto&& fn) {
      int u = 0;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int w = 0; w < 2 * (rb + 1); ++w, ++u) {
          const int idx = tid + 256 * w, rr = idx / (16 * (rb + 1)), ch = idx % (16 * (rb + 1));
          fn(u, 32 * rb + rr, dbase(rb) + rr * dpitch(rb) + 2 * ch, 2 * ch);
        }
    };
    each([&](int u, int r, int, int c) { v[u] = *reinterpret_cast<const d2*>(Ab + (int64_t)r * lda + c); });
    each([&](int u, int, int s, int) { *reinterpret_cast<d2*>(S + s) = v[u]; });
  }
  __syncthreads();
  GP2D_STAMP(1);
  // ---- Cholesky and inverse, overlapped.  Wave 0 factors the four 32-column panels (the
  // pivot chain); the trailing updates run with look-ahead (only the next panel's column
  // before it, the rest beside it), waves 1–3 store finished column blocks of L while wave 0
  // factors the next panel and invert the first three diagonal 32×32 blocks under the last
  // panel.  The inverse is W = L⁻¹ by recursive doubling over the 32-blocks, with the same
  // products summed in the same order as a level-by-level schedule:
  //   W_pp = L_pp⁻¹;  W10 = −W11 (L10 W00),  W32 = −W33 (L32 W22);
  //   T = L21·W11 (64-blocks: T20 = L20 W00 + L21 W10, T21 = L21 W11, T30, T31 alike), stored
  //   over L21;  W20 = −W22 T20, W21 = −W22 T21, W30 = −(W32 T20 + W33 T30), W31 likewise.
  // Each 32×32 product is one wave's matrix-core tile (tile32_mfma).
  // row mapping inside the per-wave 32×32 tiles: 8 rows per wave, 4 consecutive columns per lane
  const bool storeL = !inv_in_place;
  const bool inv = dinv != nullptr;
  auto panel = [&](int p) {   // wave 0
    const int c0 = 32 * p;
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
    if (p == 3 && storeL && v0) {   // the last diagonal 32×32 block of L straight from registers
      double* g = Ab + (int64_t)r0 * lda + c0;
#pragma unroll
      for (int c = 0; c < 32; c += 2)
        *reinterpret_cast<d2*>(g + c) = d2{(c0 + c <= r0) ? x0[c] : 0.0, (c0 + c + 1 <= r0) ? x0[c + 1] : 0.0};
    }
  };
  // A(bi, bj) −= L(bi, p) · L(bj, p)ᵀ  (32-block indices), one wave
  const int m16 = lane & 15, mk = lane >> 4;   // the MFMA operand / output map
  typedef tileacc_t acc_t;
  auto update = [&](int p, int bi, int bj) {
    acc_t acc;
    tile32_zero(acc);
    tile32_mfma<true>(S, 32 * bi, 32 * p, 32 * p, 32 * bj, acc, m16, mk);
    tile32_store(S, 32 * bi, 32 * bj, acc, -1.0, true, m16, mk);
  };
  // column block cb of L (all 128 rows, zeros above the diagonal) to A, by threads [t0, t0+nt)
  auto store_colblock = [&](int cb, int t0, int nt) {
    if (tid < t0 || tid >= t0 + nt) return;
    for (int e = tid - t0; e < NB * 16; e += nt) {
      const int r = e >> 4, c = 32 * cb + 2 * (e & 15);
      d2 v = d2{0.0, 0.0};
      if (r >= 32 * cb) v = *reinterpret_cast<const d2*>(S + dsw(r, c));
      *reinterpret_cast<d2*>(Ab + (int64_t)r * lda + c) = d2{(c <= r) ? v.x : 0.0, (c + 1 <= r) ? v.y : 0.0};
    }
  };
  // W(q,q) = L(q,q)⁻¹ in place in S, one wave (round 5): the two 16×16
  // diagonal blocks by forward substitution at once (lanes 0–15 the upper, 16–31 the lower one:
  // 16 serial steps instead of 32), then W21 = −W22·(L21·W11) as two 16×16×16 products on the
  // matrix core (T stored over L21, then W21 over T).
  auto inv_diag_mfma = [&](int q) {
    const int b0 = 32 * q, h = (lane >> 4) & 1, j = lane & 15, rb0 = b0 + 16 * h;
    const double rl = 1.0 / S[dsw(b0 + (lane & 31), b0 + (lane & 31))];   // lane i < 32: 1 / L_ii
    double x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = (i == j) ? 1.0 : 0.0;
    inv16_steps(std::make_integer_sequence<int, 16>{}, x, S, rb0, rl, h);
    if (lane < 32) {
#pragma unroll
      for (int i = 0; i < 16; ++i) S[dsw(rb0 + i, rb0 + j)] = x[i];   // x[i] = 0 above the diagonal
      if (h == 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) S[dsw(b0 + i, b0 + 16 + j)] = 0.0;   // W's upper right quarter
      }
    }
    asm volatile("" ::: "memory");
    d4 t = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k0 = 0; k0 < 16; k0 += 4)
      t = __builtin_amdgcn_mfma_f64_16x16x4f64(S[dsw(b0 + 16 + m16, b0 + k0 + mk)], S[dsw(b0 + k0 + mk, b0 + m16)], t,
                                               0, 0, 0);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int r = 0; r < 4; ++r) S[dsw(b0 + 16 + mk + 4 * r, b0 + m16)] = t[r];   // T over L21
    asm volatile("" ::: "memory");
    d4 w = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k0 = 0; k0 < 16; k0 += 4)
      w = __builtin_amdgcn_mfma_f64_16x16x4f64(S[dsw(b0 + 16 + m16, b0 + 16 + k0 + mk)],
                                               S[dsw(b0 + 16 + k0 + mk, b0 + m16)], w, 0, 0, 0);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int r = 0; r < 4; ++r) S[dsw(b0 + 16 + mk + 4 * r, b0 + m16)] = -w[r];   // W21 over T
  };
  // acc = Σ_{p in [p0, p1]} X(bi, p) · Y(p, bj)  (NN, 32-block indices)
  auto prod = [&](acc_t& acc, int bi, int bj, int p0, int p1) {
    tile32_zero(acc);
    for (int p = p0; p <= p1; ++p) tile32_mfma<false>(S, 32 * bi, 32 * p, 32 * p, 32 * bj, acc, m16, mk);
  };
  auto put = [&](int bi, int bj, const acc_t& acc, double sgn) {
    tile32_store(S, 32 * bi, 32 * bj, acc, sgn, false, m16, mk);
  };

  // P0
  if (wid == 0) panel(0);
  __syncthreads();
  GP2D_STAMP(2);
  // U0 on the next panel's column (and (2,2))
  update(0, wid == 0 ? 2 : wid, wid == 0 ? 2 : 1);
  __syncthreads();
  GP2D_STAMP(3);
  // P1 | U0 on (3,2), (3,3) | L column block 0
  if (wid == 0) panel(1);
  else if (wid < 3) update(0, 3, wid + 1);
  else if (storeL) store_colblock(0, 192, 64);
  __syncthreads();
  GP2D_STAMP(4);
  // U1 on (2,2), (3,2), (3,3)
  if (wid < 3) update(1, wid == 0 ? 2 : 3, wid == 2 ? 3 : 2);
  __syncthreads();
  GP2D_STAMP(5);
  // P2 | L column block 1
  if (wid == 0) panel(2);
  else if (storeL) store_colblock(1, 64, 192);
  __syncthreads();
  GP2D_STAMP(6);
  if (wid == 0) update(2, 3, 3);
  __syncthreads();
  GP2D_STAMP(7);
  // P3 | W00, W11 | L column block 2, then W22
  if (wid == 0) {
    panel(3);
  } else if (inv) {
    if (wid == 3 && storeL) store_colblock(2, 192, 64);
    inv_diag_mfma(wid - 1);
  } else if (storeL) {
    store_colblock(2, 64, 192);
  }
  __syncthreads();
  GP2D_STAMP(8);
  if (!inv) {
    if (storeL) store_colblock(3, 0, 256);
    return;
  }
  // B: W33 | T10 = L10 W00 → W10 = −W11 T10 | T32 = L32 W22 | L column block 3's zeros
  acc_t acc;
  if (wid == 0) {
    inv_diag_mfma(3);   // S(3,3) is nobody else's operand in B
  } else if (wid == 1) {
    prod(acc, 1, 0, 0, 0);
    put(1, 0, acc, 1.0);
    prod(acc, 1, 0, 1, 1);
    put(1, 0, acc, -1.0);
  } else if (wid == 2) {
    prod(acc, 3, 2, 2, 2);
    put(3, 2, acc, 1.0);
  } else if (storeL) {   // L's column block 3 above its diagonal block (rows 96–127 left panel 3)
    for (int e = lane; e < 96 * 16; e += 64) {
      const int r = e >> 4, c = 96 + 2 * (e & 15);
      *reinterpret_cast<d2*>(Ab + (int64_t)r * lda + c) = d2{0.0, 0.0};
    }
  }
  __syncthreads();
  GP2D_STAMP(9);
  // C: W33 → S, W32 = −W33 T32, then T31 | T20 | T21 | T30   (T kept in registers: one
  // accumulator set per wave — S(3,2) is nobody else's operand here)
  if (wid == 0) {
    prod(acc, 3, 2, 3, 3);
    put(3, 2, acc, -1.0);
    prod(acc, 3, 1, 1, 1);
  } else if (wid == 1) {
    prod(acc, 2, 0, 0, 1);
  } else if (wid == 2) {
    prod(acc, 2, 1, 1, 1);
  } else {
    prod(acc, 3, 0, 0, 1);
  }
  __syncthreads();
  if (wid == 0) put(3, 1, acc, 1.0);
  if (wid == 1) put(2, 0, acc, 1.0);
  if (wid == 2) put(2, 1, acc, 1.0);
  if (wid == 3) put(3, 0, acc, 1.0);
  __syncthreads();
  GP2D_STAMP(10);
  // E: W20 = −W22 T20, W21 = −W22 T21, W30 = −(W32 T20 + W33 T30), W31 = −(W32 T21 + W33 T31)
  const int ebi = 2 + (wid >> 1), ebj = wid & 1;
  prod(acc, ebi, ebj, 2, ebi);
  __syncthreads();
  put(ebi, ebj, acc, -1.0);
  __syncthreads();
  GP2D_STAMP(11);
  double* D = dinv + (int64_t)(k0 / NB) * NB * NB;
#pragma unroll 8
  for (int e = 0; e < (NB * NB / 2) / 256; ++e) {
    const int idx = tid + 256 * e, r = idx >> 6, c = 2 * (idx & 63);
    const d2 v = *reinterpret_cast<const d2*>(S + dsw(r, c));
    const d2 w = d2{(c <= r) ? v.x : 0.0, (c + 1 <= r) ? v.y : 0.0};
    *reinterpret_cast<d2*>(D + (int64_t)r * NB + c) = w;
    if (inv_in_place) *reinterpret_cast<d2*>(Ab + (int64_t)r * lda + c) = w;
  }
  GP2D_STAMP(12);
}

// Zero the strict upper triangle outside the diagonal blocks.
__global__ __launch_bounds__(256) void zero_upper_kernel(double* __restrict__ A, int64_t n, int64_t lda,
                                                         int64_t sA = 0) {   // problem blockIdx.z at A + z·sA
  A += blockIdx.z * sA;
  const int64_t i = blockIdx.y;
  const int64_t j = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
  const int64_t jstart = (i / NB + 1) * NB;
  if (j >= jstart && j < n) *reinterpret_cast<d2*>(A + i * lda + j) = d2{0.0, 0.0};
}

// Copy the inverted diagonal blocks into A's diagonal (TRTRI level 0).
__global__ __launch_bounds__(256) void put_diag_blocks_kernel(double* __restrict__ A, int64_t lda,
                                                              const double* __restrict__ dinv, int64_t sA = 0,
                                                              int64_t sD = 0) {   // problem blockIdx.z
  A += blockIdx.z * sA;
  dinv += blockIdx.z * sD;
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
