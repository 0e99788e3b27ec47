// ozaki.hpp — FP64-accurate variance contraction on the INT8 matrix cores
// (Ozaki scheme II: error-free integer splitting + Chinese-remainder reconstruction).
//
// The variance needs q_j = Σ_i V_ij² with V = W·K*ᵀ (W = L⁻¹, lower-triangular).  On
// MI355X the FP64 MFMA peak is 78.6 TF while the int8 MFMAs run at 4.7 POPS back to back
// (measured, tools/microbench/i8_mfma.hip), so the product is computed exactly in
// integers instead:
//   1. scale: Wint = rint(W_ik·2^{s_i}) (per-row power of two, |Wint| < 2^{pW}) and
//      Bint = rint(K*_jk·2^{s_B}) (one power of two from the analytic bound |K*| ≤ kss,
//      |Bint| < 2^{pB}); both are exact integers held in fp64 (pW = 49, pB = 45);
//   2. residues: for L pairwise-coprime moduli m_l ≤ 256 (Π m_l > n·2^{pW+pB}), the
//      centred residues of Wint / Bint fit int8; P_l = Wres_l · Bres_lᵀ is exact in
//      int32 (|P_l| ≤ n·128²) and reduced mod m_l in the GEMM epilogue (uint8 planes);
//   3. CRT: Pint/M = frac(Σ_l c_l·inv_l/m_l), evaluated with an exact high part
//      (inv_l/m_l rounded to 2^-33, products and sums exact in fp64) plus an fp64 low
//      part, so V_ij = (Pint/M)·M·2^{-s_i-s_B} carries ~2^-50 relative error before the
//      2^-p scaling error; the squares are summed per column in a fixed order.
// Parity is gated by the same 1e-10 tests as the FP64 path (tests/test_gpu_ozaki.py).
#pragma once
#include <type_traits>
#include "common.hpp"
#include "assemble.hpp"

namespace gp2d {

constexpr int OZ_MAXMOD = 20;   // a multiple of 4: the CRT kernel reads the constants in groups of four
#ifdef GP2D_OZ_P                   // one precision for both operands (dev builds)
#define GP2D_OZ_PW GP2D_OZ_P
#define GP2D_OZ_PB GP2D_OZ_P
#endif
#ifndef GP2D_OZ_PW
#define GP2D_OZ_PW 49
#endif
#ifndef GP2D_OZ_PB
#define GP2D_OZ_PB 45
#endif
// integer bits of the scaled operands: W rows (OZ_PW) and K* (OZ_PB); ≤ 52 keeps the
// scaled values exact in fp64, the moduli count follows OZ_PW + OZ_PB.  The rounding of W
// dominates the error, so 49 + 45 (12 moduli at the bench size) is more accurate than
// 47 + 47 and close to 50 + 50 (13 moduli); measured in DESIGN.md §3.1.
constexpr int OZ_PW = GP2D_OZ_PW;
constexpr int OZ_PB = GP2D_OZ_PB;
static_assert(OZ_PW <= 50 && OZ_PB <= 50, "ozaki: the one-part residues need |x| < 2^50");
// Both precisions are run-time choices per fit (the accuracy guard, gp2d_ozaki_guard_bits):
// OZ_PW / OZ_PB are the defaults; up to OZ_PW_MAX W bits the residue kernel splits
// Wint = xh·2^26 + xl; the K* residues stay one-part (|Bint| < 2^50) up to OZ_PB_MAX.
constexpr int OZ_PW_MAX = 60;
constexpr int OZ_PB_MAX = 50;
constexpr int OZ_SPLIT = 26;
constexpr int OZ_HBITS = 33;       // exact high part of inv_l / m_l

struct OzakiConsts {
  int nmod;
  int pw;                          // integer bits of the scaled W rows (OZ_PW .. OZ_PW_MAX)
  int pb;                          // integer bits of the scaled K* (OZ_PB .. OZ_PB_MAX)
  int m[OZ_MAXMOD];
  double c26[OZ_MAXMOD];           // 2^26 mod m_l, centred (the split residues of pw > 50)
  double md[OZ_MAXMOD];            // m_l as a double (the residue kernels' fma operand)
  double inv_m[OZ_MAXMOD];         // 1 / m_l
  double h[OZ_MAXMOD];             // inv_l / m_l rounded to a multiple of 2^-33
  double t[OZ_MAXMOD];             // inv_l / m_l − h_l
  double M;                        // Π m_l (rounded)
  int sB;                          // K* scale exponent
  double vlimit;                   // |V_ij| above this means the CRT range was exceeded
};

// Residue of an exact integer x (|x| < 2^50) modulo m as an int8 byte: q = rint(x/m) is exact
// (for odd m the fraction x/m is ≥ 1/(2m) away from ½, far above the product's rounding
// error; m = 256 divides exactly), so r = x − m·q ∈ [−m/2, m/2] and its low byte is the
// centred residue in [−128, 127] (r = ±128 only for m = 256, where 0x80 ≡ 128 ≡ −128).  No
// range fix-ups and no conversion: with xm = x + 1.5·2^52 (exact for |x| < 2^51; one add per
// x, shared by every modulus) fma(−m, q, xm) = 1.5·2^52 + r exactly (in [2^52, 2^53), ulp 1),
// whose mantissa is 2^51 + r, so the low 32 bits of the double are r in two's complement.
// 3 VALU operations per residue (4 with a cvt_i32_f64, 8 with the fix-ups).
constexpr double OZ_MAGIC52 = 6755399441055744.0;   // 1.5·2^52
__device__ __forceinline__ uint32_t residue_low_m(double x, double xm, double m, double inv_m) {
  return (uint32_t)__double_as_longlong(fma(-m, rint(x * inv_m), xm));   // low byte: the residue
}
// low bytes of a (byte 0) and b (byte 1); bytes 2, 3 zero — one v_perm_b32
__device__ __forceinline__ uint32_t pack2_lo(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x0c0c0400u); }
// bytes 0-1 of a, then bytes 0-1 of b
__device__ __forceinline__ uint32_t pack22(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x05040100u); }

// Slab-blocked residue planes (see the INT8 GEMM below): element (row, k) of a plane with K
// columns; a 256-row × 64-byte tile is one contiguous 16 KB.
__host__ __device__ __forceinline__ int64_t slab_offset(int64_t row, int64_t k, int64_t K) {
  return (((row >> 8) * (K >> 6) + (k >> 6)) << 14) + ((row & 255) << 6) + (k & 63);
}

// ------------------------------------------------------------------ W preparation
// Pass 1 (one workgroup per row i): row max (k ≤ i) → s_i (stored in rowscale[i]) and the
// row's L1 norm Σ_k |rint(W_ik·2^{s_i})| (stored in l1[i]).  The host turns max_i l1_i into
// the number of moduli: |Pint_ij| ≤ l1_i·max|Bint| < M/2 (a per-row bound, far tighter than
// the worst case n·2^{2p}).
__device__ __forceinline__ double block_reduce(double v, double* red, bool is_max) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] = is_max ? fmax(red[tid], red[tid + s]) : red[tid] + red[tid + s];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

// Row addressing of W: dense (row i at W + i·ldw) or the factor broadcast's packed lower block
// triangle (gp2d_pack_lower: 128-row block rb keeps columns [0, 128·(rb+1)), blocks one after the
// other), so a receiving rank prepares its planes straight from the payload.
struct WRows {
  int64_t ldw;   // 0: packed
  __device__ __forceinline__ int64_t off(int64_t i) const {
    if (ldw) return i * ldw;
    const int64_t rb = i >> 7;
    return ((rb * (rb + 1)) << 13) + (i & 127) * ((rb + 1) << 7);   // 128²·rb(rb+1)/2 + r·128(rb+1)
  }
  __device__ __forceinline__ int64_t len(int64_t i, int64_t n) const { return ldw ? n : ((i >> 7) + 1) << 7; }
};

__global__ __launch_bounds__(256) void ozaki_w_scale_kernel(const double* __restrict__ W, int64_t n, WRows wr, int pw,
                                                            double* __restrict__ rowscale, double* __restrict__ l1,
                                                            double M, int sB, int final_scale) {
  __shared__ double red[256];
  const int64_t i = blockIdx.x;
  const int tid = threadIdx.x;
  const double* w = W + wr.off(i);
  double mx = 0.0;
  for (int64_t k = tid; k <= i; k += 256) mx = fmax(mx, fabs(w[k]));
  mx = block_reduce(mx, red, true);
  const int e = (mx > 0.0) ? ilogb(mx) : 0;    // 2^e ≤ mx < 2^{e+1}
  const int si = pw - 1 - e;                   // |W·2^si| < 2^pw
  double sum = 0.0;
  if (l1 != nullptr) {   // the row's L1 norm (the data-driven moduli count only)
    for (int64_t k = tid; k <= i; k += 256) sum += fabs(rint(ldexp(w[k], si)));
    sum = block_reduce(sum, red, false);
  }
  if (tid == 0) {
    // final_scale: the CRT's row scale M·2^{−s_i−s_B} (s_i recoverable exactly by ilogb, as
    // ozaki_row_exp does); otherwise s_i itself, for the host's row bounds
    rowscale[i] = final_scale ? ldexp(M, -si - sB) : (double)si;
    if (l1 != nullptr) l1[i] = sum;
  }
}

// s_i → the final row scale M·2^{−s_i−s_B} (the data-driven path, once M is known)
__global__ __launch_bounds__(256) void ozaki_rowscale_final_kernel(double* __restrict__ rowscale, int64_t n, double M,
                                                                   int sB) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) rowscale[i] = ldexp(M, -(int)rowscale[i] - sB);
}

// s_i from the final row scale: ldexp keeps the mantissa, so the exponents differ by s_i + s_B
__device__ __forceinline__ int ozaki_row_exp(double rowscale_i, const OzakiConsts& oc) {
  return ilogb(oc.M) - ilogb(rowscale_i) - oc.sB;
}

// Pass 2: residue planes Wres[l] (int8, slab-blocked, zeros above the diagonal).  One
// workgroup per (256-row block bi, 64-wide k slab ks) with ks < 4·(bi+1) (the GEMM, a_lower,
// never reads past its diagonal tile): a wave covers 4 rows × 64 k per step — 16 lanes per row,
// 4 consecutive k per lane, 32 B of each row read contiguously — and writes, per modulus, the
// 4 rows' 64-B runs of the slab tile: 256 contiguous bytes per wave store (the per-row form
// wrote four 64-B pieces 16 KB apart).
__global__ __launch_bounds__(256) void ozaki_w_res_kernel(const double* __restrict__ W, int64_t n, WRows wr,
                                                          OzakiConsts oc, int8_t* __restrict__ wres,
                                                          const double* __restrict__ rowscale) {
  const int64_t bi = blockIdx.y, ks = blockIdx.x;
  if (ks * 64 >= (bi + 1) * 256) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t k0 = ks * 64 + 4 * (lane & 15);
  const int64_t plane = n * n;
#pragma unroll 1
  for (int it = 0; it < 16; ++it) {
    const int64_t i = bi * 256 + wv * 64 + it * 4 + (lane >> 4);
    const int si = ozaki_row_exp(rowscale[i], oc);
    const double* w = W + wr.off(i) + k0;
    d2 p0 = {0.0, 0.0}, p1 = {0.0, 0.0};
    if (k0 < wr.len(i, n)) {   // k0 and the row length are multiples of 4: all four or none stored
      p0 = *reinterpret_cast<const d2*>(w);
      p1 = *reinterpret_cast<const d2*>(w + 2);
    }
    const double v[4] = {p0.x, p0.y, p1.x, p1.y};
    double x[4], xm[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      x[u] = (k0 + u <= i) ? rint(ldexp(v[u], si)) : 0.0;
      xm[u] = x[u] + OZ_MAGIC52;
    }
    int8_t* dst = wres + slab_offset(i, k0, n);
    if (oc.pw <= 50) {   // uniform: |x| < 2^50, one exact residue per modulus
      for (int l = 0; l < oc.nmod; ++l) {
        const double m = oc.md[l], im = oc.inv_m[l];
        uint32_t r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) r[u] = residue_low_m(x[u], xm[u], m, im);
        *reinterpret_cast<uint32_t*>(dst + (int64_t)l * plane) = pack22(pack2_lo(r[0], r[1]), pack2_lo(r[2], r[3]));
      }
    } else {             // |x| < 2^60: x = xh·2^26 + xl exactly (|xl| ≤ 2^25, |xh| < 2^35), and
      //                    x ≡ rh·(2^26 mod m) + rl (mod m) with the centred residues rh, rl (|·| ≤ 128)
      double xh[4], xl[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        xh[u] = rint(ldexp(x[u], -OZ_SPLIT));
        xl[u] = x[u] - ldexp(xh[u], OZ_SPLIT);   // exact: an integer below 2^26 in magnitude
      }
      for (int l = 0; l < oc.nmod; ++l) {
        const double m = oc.md[l], im = oc.inv_m[l], c = oc.c26[l];
        uint32_t r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const double rh = fma(-m, rint(xh[u] * im), xh[u]), rl = fma(-m, rint(xl[u] * im), xl[u]);
          const double t = fma(rh, c, rl);         // exact: |t| ≤ 128·128 + 128
          r[u] = residue_low_m(t, t + OZ_MAGIC52, m, im);
        }
        *reinterpret_cast<uint32_t*>(dst + (int64_t)l * plane) = pack22(pack2_lo(r[0], r[1]), pack2_lo(r[2], r[3]));
      }
    }
  }
}

// ------------------------------------------------------------------ K*ᵀ residues + mean
// Block: 64 training points × 64 grid points (4 waves).  Lane l covers training points
// t = 64·bx + OZ_KS_PPL·(l mod LG) .. + OZ_KS_PPL − 1 (LG = 64 / OZ_KS_PPL lanes per grid row)
// and, in iteration q, grid point p = 64·by + RPI·q + RPW·wave + l / LG (RPW = 64 / LG rows per
// wave, RPI = 4·RPW rows per iteration).  One wave-wide store per (modulus, entry) then writes
// RPW consecutive rows × 64 B of one slab tile — contiguous bytes (the slab-blocked layout
// puts rows of a 256-row tile 64 B apart).  Writes the residue planes Bres[l] (rows j = grid
// components, columns k = training components, slab-blocked) and mean partials
// pm[bx][j] = Σ_{k in block} α_k·K*_jk (LG-lane shuffle reduction in a fixed order).
// alpha == nullptr: planes only; oc.nmod == 0: mean only (the planes were built earlier by
// gp2d_ozaki_kstar).
#ifndef GP2D_KS_OCC
#define GP2D_KS_OCC 5   // min workgroups per CU for ozaki_kstar_kernel: 5 waves per SIMD (102 VGPRs)
#endif
#ifndef GP2D_KS_PPL
#define GP2D_KS_PPL 2   // training points per lane (4: 44 VGPRs spill at 4 waves per SIMD, 3 % slower)
#endif
constexpr int OZ_KS_T = 64;   // training points per block
constexpr int OZ_KS_P = 64;   // grid points per block
constexpr int OZ_KS_PPL = GP2D_KS_PPL;
static_assert(OZ_KS_PPL == 2 || OZ_KS_PPL == 4, "2 or 4 training points per lane");

template <int PPL> struct packed_bytes;   // PPL residue bytes of one lane, stored at once
template <> struct packed_bytes<2> { typedef uint16_t type; };
template <> struct packed_bytes<4> { typedef uint32_t type; };

// OFF32: a plane (n·2·cp bytes) is below 2^31 (the launcher checks), so the stores are buffer
// stores — the plane in a scalar buffer resource, the 32-bit offsets computed once per grid
// point — instead of three 64-bit address additions per modulus.
template <bool OFF32>
__global__ __launch_bounds__(256, GP2D_KS_OCC) void ozaki_kstar_kernel(
    const double* __restrict__ xtr, int64_t ntr, int64_t npad, const double* __restrict__ xg, int64_t cv,
    int64_t cp, VecParams vp, const double* __restrict__ alpha, OzakiConsts oc, int8_t* __restrict__ bres,
    double* __restrict__ pm, uint8_t* __restrict__ flags) {
  constexpr int PPL = OZ_KS_PPL, LG = 64 / PPL, RPW = 64 / LG, RPI = 4 * RPW;
  typedef typename packed_bytes<PPL>::type pk_t;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int kg = lane % LG, r = lane / LG;
  const int64_t t0 = (int64_t)blockIdx.x * OZ_KS_T + PPL * kg;
  const int64_t n = 2 * npad, ncols = 2 * cp;
  double a1[PPL], a2[PPL], x0[PPL], x1[PPL], x2[PPL];
  bool tv[PPL];
#pragma unroll
  for (int u = 0; u < PPL; ++u) {
    const int64_t t = t0 + u;
    tv[u] = t < ntr;
    x0[u] = x1[u] = x2[u] = 0.0;
    if (tv[u]) vec_point(vp, xtr, t, x0[u], x1[u], x2[u]);
    a1[u] = (alpha != nullptr && t < npad) ? alpha[t] : 0.0;
    a2[u] = (alpha != nullptr && t < npad) ? alpha[npad + t] : 0.0;
  }
  const double scale = ldexp(1.0, oc.sB);
  bool nz = false;   // a nonzero scaled entry in this thread's part of the block
#pragma unroll 1
  for (int q = 0; q < OZ_KS_P / RPI; ++q) {
    const int64_t p = (int64_t)blockIdx.y * OZ_KS_P + RPI * q + RPW * wv + r;
    const bool pv = p < cv;
    double g0 = 0.0, g1 = 0.0, g2 = 0.0;
    if (pv) vec_point(vp, xg, p, g0, g1, g2);
    double k11[PPL], k12[PPL], k22[PPL];
    double mu = 0.0, mv = 0.0;
#pragma unroll
    for (int u = 0; u < PPL; ++u) {
      if (pv && tv[u]) {
        vec_block_st(vp, x0[u] - g0, x1[u] - g1, x2[u] - g2, k11[u], k12[u], k22[u]);
      } else {
        k11[u] = k12[u] = k22[u] = 0.0;
      }
      mu += a1[u] * k11[u] + a2[u] * k12[u];   // row j = p      (u component of the grid point)
      mv += a1[u] * k12[u] + a2[u] * k22[u];   // row j = cp + p (v component)
    }
    if (pm != nullptr) {
      // fixed-order reduction over the LG lanes of this grid point (this block's 64 points)
#pragma unroll
      for (int o = LG / 2; o > 0; o >>= 1) {
        mu += __shfl_xor(mu, o);
        mv += __shfl_xor(mv, o);
      }
      if (kg == 0 && p < cp) {
        pm[(int64_t)blockIdx.x * ncols + p] = mu;
        pm[(int64_t)blockIdx.x * ncols + cp + p] = mv;
      }
    }
    if (p >= cp || t0 >= npad) continue;   // npad is a multiple of 64: whole point groups
    // The (v,u) block equals the (u,v) block (k12 is symmetric in the 2×2 kernel block), so
    // only (u,u), (u,v) and (v,v) are stored: the GEMM reads (v,u) tiles from (u,v).
    double xi[3][PPL], xm[3][PPL];  // [entry: (u,u) (u,v) (v,v)][u]; xm = xi + 1.5·2^52
#pragma unroll
    for (int u = 0; u < PPL; ++u) {
      xi[0][u] = rint(k11[u] * scale);
      xi[1][u] = rint(k12[u] * scale);
      xi[2][u] = rint(k22[u] * scale);
      nz = nz || xi[0][u] != 0.0 || xi[1][u] != 0.0 || xi[2][u] != 0.0;
#pragma unroll
      for (int e = 0; e < 3; ++e) xm[e][u] = xi[e][u] + OZ_MAGIC52;
    }
    // (grid comp, train comp): (u,u) → row p, col t ; (u,v) → row p, col npad+t ;
    //                          (v,v) → row cp+p, col npad+t ; (v,u) not stored
    const int64_t o_uu = slab_offset(p, t0, n), o_uv = slab_offset(p, npad + t0, n),
                  o_vv = slab_offset(cp + p, npad + t0, n);
    const int64_t pstride = ncols * n;
    for (int l = 0; l < oc.nmod; ++l) {
      const double m = oc.md[l], im = oc.inv_m[l];
      pk_t pk[3];
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        uint32_t r[PPL];   // |xi| < 2^pB
#pragma unroll
        for (int u = 0; u < PPL; ++u) r[u] = residue_low_m(xi[e][u], xm[e][u], m, im);
        if constexpr (PPL == 2) pk[e] = (pk_t)pack2_lo(r[0], r[1]);
        else pk[e] = (pk_t)pack22(pack2_lo(r[0], r[1]), pack2_lo(r[2], r[3]));
      }
      int8_t* plane = bres + (int64_t)l * pstride;
      if constexpr (OFF32) {   // buffer stores: the plane in a scalar resource, 32-bit offsets
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(plane, (short)0, (int)pstride, 0x00020000);
        if constexpr (PPL == 2) {
          __builtin_amdgcn_raw_buffer_store_b16(pk[0], rs, (int)o_uu, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b16(pk[1], rs, (int)o_uv, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b16(pk[2], rs, (int)o_vv, 0, 0);
        } else {
          __builtin_amdgcn_raw_buffer_store_b32(pk[0], rs, (int)o_uu, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(pk[1], rs, (int)o_uv, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(pk[2], rs, (int)o_vv, 0, 0);
        }
      } else {
        *reinterpret_cast<pk_t*>(plane + o_uu) = pk[0];
        *reinterpret_cast<pk_t*>(plane + o_uv) = pk[1];
        *reinterpret_cast<pk_t*>(plane + o_vv) = pk[2];
      }
    }
  }
  // block flag (grid block by, training block bx): 0 iff every stored residue is zero, so the
  // int8 GEMM may skip the K slabs of this training block for this grid block
  if (flags != nullptr) {
    const int any = __syncthreads_or(nz ? 1 : 0);
    if (threadIdx.x == 0) flags[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = any ? 1 : 0;
  }
}

// Per 256-row B tile bj: the ascending list of K slabs whose K* tile is not all zero
// (list[bj][0..]) and cnt[bj][kb] = the number of listed slabs below slab 4·kb (kb ≤ K/256),
// from the K* kernel's block flags [cp/64][npad/64].  Rows bj < nbj/2 are the u components
// of grid tile bj, the rest the v components of tile bj − nbj/2; slab s covers training block
// s mod (npad/64) (u, then v components).  A slab is kept when any of the tile's four 64-point
// grid blocks has a nonzero entry with that training block (all component pairs share the flag).
// One wave per tile: ballot + popcount compaction in slab order.
__global__ __launch_bounds__(64) void ozaki_slab_list_kernel(const uint8_t* __restrict__ flags, int ntb, int nbj,
                                                             int kslabs, int* __restrict__ list,
                                                             int* __restrict__ cnt) {
  const int bj = blockIdx.x, lane = threadIdx.x;
  const int g = bj % (nbj / 2);
  const uint8_t* f = flags + (int64_t)(4 * g) * ntb;
  int* L = list + (int64_t)bj * kslabs;
  int* C = cnt + (int64_t)bj * (kslabs / 4 + 1);
  int c = 0;
  for (int s0 = 0; s0 < kslabs; s0 += 64) {
    const int sl = s0 + lane;
    bool keep = false;
    if (sl < kslabs) {
      const int tb = sl % ntb;
      keep = (f[tb] | f[ntb + tb] | f[2 * ntb + tb] | f[3 * ntb + tb]) != 0;
    }
    const uint64_t bal = __ballot(keep);
    const int below = c + __popcll(bal & ((1ull << lane) - 1ull));
    if (keep) L[below] = sl;
    if (sl < kslabs && (sl & 3) == 0) C[sl >> 2] = below;
    c += __popcll(bal);
  }
  if (lane == 0) C[kslabs >> 2] = c;
}

// Modular reduction of the biased GEMM sums, all in full-rate 24-bit VALU operations.
// The accumulators start at bias = m·⌈K·2^14 / m⌉ (≥ every |Σ a·b| with |a|, |b| ≤ 128), so
// a sum v, read as unsigned, lies in [0, 2^32) for K < 2^17 (the int32 MFMA accumulation
// wraps mod 2^32, the same bits).  With vh = v >> 20 (< 2^12) and c20 = 2^20 mod m,
//   y = v − vh·(2^20 − c20) = (v mod 2^20) + vh·c20 ≡ v (mod m),   0 ≤ y < 2^20 + 2^20 = 2^21
// (the 24-bit mad is exact mod 2^32 and its true result is below 2^21);
// q = ⌊8y · ⌈2^29/m⌉ / 2^32⌋ (v_mul_hi_u32_u24: 8y < 2^24, and ⌈2^29/m⌉ < 2^24 for m > 32) is
// exactly ⌊y/m⌋, since y·(⌈2^29/m⌉ − 2^29/m)/2^29 < 2^21/2^29 ≤ 1/m for m ≤ 256; r = y − q·m.
struct OzModConsts {
  int neg_c;       // −(2^20 − c20)
  int neg_m;       // −m
  uint32_t magic;  // ⌈2^29 / m⌉
};
__host__ __device__ inline uint32_t ozaki_acc_bias(int K, int m) {
  return (uint32_t)((((int64_t)K << 14) + m - 1) / m * m);
}
__device__ __forceinline__ OzModConsts ozaki_mod_consts(int m) {
  OzModConsts c;
  c.neg_c = -((1 << 20) - (1 << 20) % m);
  c.neg_m = -m;
  c.magic = (uint32_t)(((1u << 29) + (uint32_t)m - 1) / (uint32_t)m);
  return c;
}
__device__ __forceinline__ uint32_t ozaki_mod_u32(uint32_t v, const OzModConsts& c) {
  int y, r;
  uint32_t q;
  asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(y) : "v"(v >> 20), "s"(c.neg_c), "v"(v));
  asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(q) : "s"(c.magic), "v"(y << 3));
  asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(q), "s"(c.neg_m), "v"(y));
  return (uint32_t)r;
}

// ------------------------------------------------------------------ INT8 NT GEMM mod m
// C[i][j] = (Σ_k A[i][k]·B[j][k]) mod m, A lower-triangular (row block i0 needs k < i0+256).
//
// Operand layout ("slab-blocked"): residue planes are stored as 256-row × 64-byte tiles,
// each one contiguous 16 KB — element (row, k) of a plane with K columns lives at
//   ((row/256)·(K/64) + k/64)·16384 + (row%256)·64 + k%64.
// A K-slab of a 256-row operand panel is then ONE contiguous 16 KB read, and every 1 KB
// LDS-DMA piece is contiguous: with row-major planes the same slab is 256 scattered 64-B
// segments, one per DRAM page, and the L2-miss stream ran far below HBM bandwidth.
//
// 256×256 output tile per 512-thread workgroup: 8 waves as 2×4, two waves per SIMD, each
// wave 128×64 = 8×4 tiles of v_mfma_i32_16x16x64_i8 (128 accumulators).  While one wave of
// a SIMD issues its LDS-DMA pieces and fragment reads the other keeps the matrix core busy.
// K advances in 64-byte slabs loaded global→LDS directly (buffer_load_dwordx4 … lds) into a
// 4-stage ring with three slabs in flight; one barrier per slab, between the slab's two MFMA
// halves, publishes the next one.
// Lane l reads A[row l&15][k 16(l>>4)..+15]; a ds_read_b128 lane group covers rows
// {0-3,12-15} of one k-chunk and rows 4-11 of the next, so the LDS chunk index is swizzled
// chunk ^ g((row>>2)&3) with g = [0,2,3,1], which spreads every group over 16 distinct
// 4-bank slots.  The DMA writes LDS lane-linearly; the swizzle is applied on the global
// source address (an involution, so the same formula maps both ways).
constexpr int IBM = 256, IBN = 256, IBK = 64;
constexpr int I_OP = IBM * IBK;        // bytes per operand per stage (16 KB) = one layout tile
constexpr int I_STAGE = 2 * I_OP;      // A then B
constexpr int I_NSTAGE = 4;        // ring stages of the 256-wide shape (I_NSTAGE − 1 slabs in flight)


typedef int i4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// One 1 KB LDS-DMA piece per wave (buffer_load_dwordx4 … offen lds): 16 B per lane from the
// descriptor's base + the lane's 32-bit offset + the wave-uniform soffset into LDS at dst (M0).
// Against global_load_lds with 64-bit lane addresses it needs no per-piece address arithmetic:
// the lane offsets are the same for every K slab and the slab's offset is scalar (round 5:
// −4.5 % per unpipelined launch with the offset-field fragment reads, profiles/r05_bufbench_ab.txt).
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t r, lds_ptr_t dst, int voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)   // a gfx950 builtin: the host pass only needs the kernels' launch stubs
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 16, voff, soff, 0, 0);
#endif
}

__device__ __forceinline__ int swz16(int row, int chunk) {
  const int q = (row >> 2) & 3;
  const int g = (0x78 >> (2 * q)) & 3;  // 0x78 = 0b01_11_10_00 → g(0)=0, g(1)=2, g(2)=3, g(3)=1
  return chunk ^ g;
}

// s_waitcnt vmcnt(P·W) + lgkmcnt(0) + s_barrier: this wave's LDS-DMA pieces of all but the
// W youngest slabs (P pieces per slab per wave) have landed, then the workgroup syncs.
template <int P, int W>
__device__ __forceinline__ void vmwait_barrier(std::integral_constant<int, W>) {
  static_assert(P * W < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(P * W) : "memory");
}

// A: M×K plane, B: N×K plane (both slab-blocked); C: column-major N×M bytes (ldc ≥ M).
// B tiles (256-row layout block rb ≥ alias_rb, k slab s < alias_ks) are read from
// (rb − alias_rb, s + alias_ks): the K* planes store the (v,u) block only as its equal (u,v)
// block.  alias_rb = INT_MAX disables the aliasing.
// slist / scnt (optional, ozaki_slab_list_kernel, per 256-row B block): the K loop runs over
// the listed slabs only — the others have an all-zero K* tile and add exactly nothing.  A tile
// whose list is shorter than the ring's prologue runs dense.
//
// Two shapes (TBN = output columns per workgroup; rows are always 256 = IBM):
//   TBN = 256: 512 threads, 8 waves as 2×4, one workgroup per CU, 4-stage ring (128 KB).
//   TBN = 128: (alternative, measured slower; instantiated only in tools/microbench/igemm_bench.hip
//              (IG_TBN), numbers in DESIGN.md §3.6)
//              256 threads, 4 waves as 2×2, TWO workgroups per CU, 3-stage ring of 24 KB
//              stages (72 KB each).  Every wave computes the same 128×64 register tile as in
//              the 256 shape and a SIMD still holds two waves, but they belong to different
//              workgroups, so one workgroup's epilogue (modular reduction, LDS transpose,
//              64 KB of stores) and its successor's prologue run under the other's MFMAs
//              instead of idling the matrix cores (the epilogue alone is ≈ 17 % of a launch
//              on random residues, tools/microbench ablation).  Costs: 1.5× the LDS-DMA
//              pieces per MAC (the A slab is fetched by both column halves).
// Moduli batch: a launch with gridDim.z > 1 runs modulus z's product on planes A + z·sA,
// B + z·sB, C + z·sC with modulus m[z].  The dispatcher walks x, then y, then z, so one
// modulus's tiles go out before the next one's (the L2 working set of a single-modulus launch)
// and the next modulus's long-K tiles fill the previous one's tail instead of a launch gap.
struct IgemmZ {
  int64_t sA, sB, sC;
  int m[OZ_MAXMOD];
};
constexpr int64_t kIgemmZBatchMaxN = 4096;   // predict_ozaki_impl batches the moduli up to this n

template <int TBN, int NST>
__global__ __launch_bounds__(TBN * 2, (TBN == 256) ? 1 : 2) void igemm_nt_mod_kernel(
    const int8_t* __restrict__ A, const int8_t* __restrict__ B, uint8_t* __restrict__ C, int64_t ldc, int M, int N,
    int K, int a_lower, int modulus, int alias_rb, int alias_ks, const int* __restrict__ slist,
    const int* __restrict__ scnt, const IgemmZ zb) {
  if (gridDim.z > 1) {
    A += blockIdx.z * zb.sA;
    B += blockIdx.z * zb.sB;
    C += blockIdx.z * zb.sC;
    modulus = zb.m[blockIdx.z];
  }
  static_assert(TBN == 256 || TBN == 128, "tile width");
  static_assert(NST >= 3 && NST <= 5, "ring depth 3..5 (the tail is written out for these)");
  constexpr int NW = TBN / 32;                 // waves: 8 or 4
  constexpr int WC = TBN / 64;                 // wave columns: 4 or 2
  constexpr int B_OP = TBN * IBK;              // B bytes per stage
  constexpr int STG = I_OP + B_OP;             // stage bytes: A then B
  constexpr int AP = IBM / NW / 16;            // A pieces (16 rows × 64 B) per wave per slab: 2 or 4
  constexpr int BPW = TBN / NW / 16;           // B pieces per wave per slab: 2
  constexpr int PPW = AP + BPW;                // DMA pieces per wave per slab
  __shared__ __attribute__((aligned(16))) int8_t smem[NST * STG];
  const int bj = blockIdx.x;
  const int bi = (int)(gridDim.y - 1 - blockIdx.y);   // heavy (long-K) row blocks first
  const int i0 = bi * IBM, j0 = bj * TBN;
  const int jb = j0 / IBN, jr = j0 % IBN;             // 256-row B layout block, row offset in it
  const int ke = a_lower ? min(K, i0 + IBM) : K;
  // the wave index as a scalar: LDS-DMA destinations (M0) and piece offsets without v_readfirstlane
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WC, wc = wid % WC;
  const int l16 = lane & 15, lq = lane >> 4;
  const int64_t kslabs = K / IBK;
  const int8_t* Ap = A + (int64_t)bi * kslabs * I_OP;   // this row block's slab tiles
  const bool alias = jb >= alias_rb;
  const int8_t* Bp = B + (int64_t)jb * kslabs * I_OP + jr * IBK;
  const int8_t* Bq = B + ((int64_t)(alias ? jb - alias_rb : 0) * kslabs + alias_ks) * I_OP + jr * IBK;
  int nsl = ke / IBK;
  const int* sl = nullptr;   // slab list of this B block (nullptr: dense K loop)
  if (slist != nullptr) {
    const int c = scnt[(int64_t)jb * (kslabs / 4 + 1) + ke / IBM];
    if (c == 0 || c >= NST - 1) {
      nsl = c;
      sl = slist + (int64_t)jb * kslabs;
    }
  }

  // the accumulators start at a multiple of m above every |Σ_k a·b| ≤ K·128² (centred
  // residues), so the sums leave the MFMAs non-negative and ≡ the true sums (mod m)
  const int bias = (int)ozaki_acc_bias(K, modulus);   // the bit pattern of an unsigned value
  i4v acc[8][4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = i4v{bias, bias, bias, bias};

  // wave w moves A rows [16·AP·w, +16·AP) and B rows [32w, 32w+32): contiguous 1 KB pieces
  const int drow = lane >> 2, dchunk = lane & 3;
  // LDS-DMA through buffer descriptors over this row block's slab tiles (A) and the column
  // block's (B; Bq: the aliased (v,u) tiles): lane offsets fixed, the slab (ks·16 KB) in soffset
  const int rec = (int)(kslabs * I_OP);
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)Ap, (short)0, rec, 0x00020000);
  const __amdgpu_buffer_rsrc_t rBp = __builtin_amdgcn_make_buffer_rsrc((void*)Bp, (short)0, rec, 0x00020000);
  const __amdgpu_buffer_rsrc_t rBq = __builtin_amdgcn_make_buffer_rsrc((void*)Bq, (short)0, rec, 0x00020000);
  int voA[AP], voB[BPW];
#pragma unroll
  for (int h = 0; h < AP; ++h) {
    const int row = (wid * AP + h) * 16 + drow;
    voA[h] = row * IBK + 16 * swz16(row, dchunk);
  }
#pragma unroll
  for (int h = 0; h < BPW; ++h) {
    const int row = (wid * BPW + h) * 16 + drow;
    voB[h] = row * IBK + 16 * swz16(jr + row, dchunk);
  }
  auto issue = [&](int ks, int st) {
    int8_t* As = smem + st * STG;
    int8_t* Bs = As + I_OP;
    const int so = ks * I_OP;
#pragma unroll
    for (int h = 0; h < AP; ++h) lds_dma16(rA, (lds_ptr_t)(As + (wid * AP + h) * 16 * IBK), voA[h], so);
    const bool q = alias && ks < alias_ks;
#pragma unroll
    for (int h = 0; h < BPW; ++h) lds_dma16(q ? rBq : rBp, (lds_ptr_t)(Bs + (wid * BPW + h) * 16 * IBK), voB[h], so);
  };

  const uint32_t lds_base = (uint32_t)(size_t)(lds_ptr_t)smem;
  // one base VGPR per read group, the fragment in the offset field: the swizzle depends on
  // (row >> 2) & 3 = (l16 >> 2) & 3 only (fragment rows are 16-aligned; jr % 16 == 0)
  const uint32_t lane_a = (uint32_t)((wr * 128 + l16) * IBK + 16 * swz16(l16, lq));
  const uint32_t lane_b = (uint32_t)(I_OP + (wc * 64 + l16) * IBK + 16 * swz16(jr + l16, lq));
  auto reada = [&](int st, int half, i4v (&a)[4]) {  // A fragments mi = 4·half .. 4·half+3
    const uint32_t ad = lds_base + st * STG + lane_a;
    if (half == 0) {
      asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(a[0]) : "v"(ad) : "memory");
      asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(a[1]) : "v"(ad) : "memory");
      asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(a[2]) : "v"(ad) : "memory");
      asm volatile("ds_read_b128 %0, %1 offset:3072" : "=v"(a[3]) : "v"(ad) : "memory");
    } else {
      asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(a[0]) : "v"(ad) : "memory");
      asm volatile("ds_read_b128 %0, %1 offset:5120" : "=v"(a[1]) : "v"(ad) : "memory");
      asm volatile("ds_read_b128 %0, %1 offset:6144" : "=v"(a[2]) : "v"(ad) : "memory");
      asm volatile("ds_read_b128 %0, %1 offset:7168" : "=v"(a[3]) : "v"(ad) : "memory");
    }
  };
  auto readb = [&](int st, i4v (&b)[4]) {
    const uint32_t ad = lds_base + st * STG + lane_b;
    asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(b[0]) : "v"(ad) : "memory");
    asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(b[1]) : "v"(ad) : "memory");
    asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(b[2]) : "v"(ad) : "memory");
    asm volatile("ds_read_b128 %0, %1 offset:3072" : "=v"(b[3]) : "v"(ad) : "memory");
  };
  auto mfmas = [&](int half, const i4v (&a)[4], const i4v (&b)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        acc[4 * half + u][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u], b[ni], acc[4 * half + u][ni], 0, 0, 0);
  };
  // list lookups run one step ahead of their DMA: the load of step s's index is issued during
  // step s − 1.  Through the constant address space it is a scalar load (s_load, counted by
  // lgkmcnt); a vector load would need vmcnt(0), which also drains the slabs in flight.
  typedef const __attribute__((address_space(4))) int* const_int_ptr;
  auto slab = [&](int s) -> int { return sl ? ((const_int_ptr)sl)[min(s, nsl - 1)] : s; };
  if (nsl > 0) {
#pragma unroll
    for (int q = 0; q < NST - 1; ++q) issue(slab(q), q);
    int knext = slab(NST - 1);
    vmwait_barrier<PPW>(std::integral_constant<int, NST - 2>{});   // slab 0 landed (nsl ≥ NST − 1)
    // Per slab: MFMA half 0 (A rows 0-63 of the wave) → barrier publishing slab s+1 → reads
    // of slab s+1's B and A-half-0 fragments into the other register set → MFMA half 1.
    // Both waves of a workgroup on a SIMD leave the barrier together, so the next slab's first
    // fragments must already be in flight behind half 1's 16 MFMAs rather than be read after it.
    i4v bA[4], a0A[4], bB[4], a0B[4], a1[4];
    readb(0, bA);
    reada(0, 0, a0A);
    __builtin_amdgcn_sched_barrier(0);
    // Step kinds: FULL steps issue slab s + NST − 1 and publish s+1 leaving the younger
    // NST − 2 slabs in flight; the tail steps issue nothing and leave W = NST−3 .. 0 slabs in
    // flight; the LAST step has no barrier.  The steady-state loop runs only FULL steps,
    // unrolled by two for the register ping-pong, so it carries no per-slab branches.
    constexpr int LAST = -1;
    auto step = [&](auto dma_c, auto w_c, int s, i4v (&b)[4], i4v (&a0)[4], i4v (&bn)[4], i4v (&a0n)[4]) {
      constexpr bool dma = decltype(dma_c)::value;
      constexpr int w = decltype(w_c)::value;
      const int st = s % NST;
      // the stage written is slab s−1's: nobody reads it after the previous barrier
      if constexpr (dma) {
        issue(knext, (s + NST - 1) % NST);
        knext = slab(s + NST);
      }
      reada(st, 1, a1);
      asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");  // b, a0 landed
      __builtin_amdgcn_sched_barrier(0);
      mfmas(0, a0, b);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (w != LAST) {
        vmwait_barrier<PPW>(w_c);   // publish slab s+1 (lgkmcnt(0) inside: a1 landed)
        const int st1 = (s + 1) % NST;
        readb(st1, bn);
        reada(st1, 0, a0n);
        asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");  // nothing older than the 8 new reads
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      mfmas(1, a1, b);
      __builtin_amdgcn_sched_barrier(0);
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    using W_FULL = std::integral_constant<int, NST - 2>;
    const int m = nsl - (NST - 1);   // FULL steps
    int s = 0;
    for (; s + 1 < m; s += 2) {
      step(T_{}, W_FULL{}, s, bA, a0A, bB, a0B);
      step(T_{}, W_FULL{}, s + 1, bB, a0B, bA, a0A);
    }
    if (s < m) {   // odd number of FULL steps: one more, then move its fragments back to set A
      step(T_{}, W_FULL{}, s, bA, a0A, bB, a0B);
      ++s;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        bA[u] = bB[u];
        a0A[u] = a0B[u];
      }
    }
    // tail: NST − 1 steps, W = NST−3, ..., 0, then LAST
    if constexpr (NST == 5) {
      step(F_{}, std::integral_constant<int, 2>{}, s, bA, a0A, bB, a0B);
      step(F_{}, std::integral_constant<int, 1>{}, s + 1, bB, a0B, bA, a0A);
      step(F_{}, std::integral_constant<int, 0>{}, s + 2, bA, a0A, bB, a0B);
      step(F_{}, std::integral_constant<int, LAST>{}, s + 3, bB, a0B, bA, a0A);
    } else if constexpr (NST == 4) {
      step(F_{}, std::integral_constant<int, 1>{}, s, bA, a0A, bB, a0B);
      step(F_{}, std::integral_constant<int, 0>{}, s + 1, bB, a0B, bA, a0A);
      step(F_{}, std::integral_constant<int, LAST>{}, s + 2, bA, a0A, bB, a0B);
    } else {
      step(F_{}, std::integral_constant<int, 0>{}, s, bA, a0A, bB, a0B);
      step(F_{}, std::integral_constant<int, LAST>{}, s + 1, bB, a0B, bA, a0A);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // Epilogue: residues mod m, packed 4 rows per dword into an LDS image of Cᵀ [col][row]
  // (pitch 272 B), then written out as coalesced 16-B row runs of the column-major residue
  // plane.  Six full-rate VALU operations per residue (ozaki_mod_u32; no v_mul_lo_u32, no
  // float conversions, no range fix-ups).
  uint8_t* T = reinterpret_cast<uint8_t*>(smem);
  constexpr int TP = IBM + 16;
  static_assert(TBN * TP <= NST * STG, "epilogue image fits the ring");
  const OzModConsts mc = ozaki_mod_consts(modulus);
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      uint32_t pk = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) pk |= ozaki_mod_u32((uint32_t)acc[mi][ni][u], mc) << (8 * u);
      const int rloc = wr * 128 + mi * 16 + 4 * lq;
      const int cloc = wc * 64 + ni * 16 + l16;
      *reinterpret_cast<uint32_t*>(T + cloc * TP + rloc) = pk;
    }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < (IBM * TBN / 16) / (TBN * 2); ++p) {
    const int id = tid + TBN * 2 * p;
    const int cloc = id >> 4, ch = id & 15;
    // non-temporal: the planes are read once, by the CRT, past L2 (+0.3–0.5 %, profiles/r05_ntstore_ab.txt)
    const i4v v = *reinterpret_cast<const i4v*>(T + cloc * TP + 16 * ch);
    __builtin_nontemporal_store(v, reinterpret_cast<i4v*>(C + (int64_t)(j0 + cloc) * ldc + i0 + 16 * ch));
  }
}

// ------------------------------------------------------------------ accuracy guard statistics
// What the W precision must cover (gp2d_ozaki_guard_bits): the variance loses digits where the
// posterior variance is small against kss, and it is smallest at the observations.  At training
// point i the latent posterior variance is exact from the factor alone: with K_y = K + δI,
// [K − K·K_y⁻¹·K]_ii = δ − δ²·(K_y⁻¹)_ii and (K_y⁻¹)_ii = Σ_k W_ki² (a column norm of W = L⁻¹).
// Pass 1: per 256-row segment and column, Σ W_rc² and max |W_rc| (blocks above the diagonal skip).
constexpr int OZ_GUARD_RSEG = 256;
__global__ __launch_bounds__(256) void ozaki_guard_colsq_kernel(const double* __restrict__ W, int64_t n, int64_t ldw,
                                                                double* __restrict__ psum, double* __restrict__ pmax) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x, seg = blockIdx.y;
  const int64_t r0 = seg * OZ_GUARD_RSEG, r1 = min<int64_t>(n, r0 + OZ_GUARD_RSEG);
  if (c >= n) return;
  double sq = 0.0, mx = 0.0;
  if (r1 > (int64_t)blockIdx.x * 256) {   // the segment reaches this column block's diagonal
#pragma unroll 8
    for (int64_t r = r0; r < r1; ++r) {
      const double w = W[r * ldw + c];
      sq = fma(w, w, sq);
      mx = fmax(mx, fabs(w));
    }
  }
  psum[seg * n + c] = sq;
  pmax[seg * n + c] = mx;
}

// Pass 2 (one workgroup): (K_y⁻¹)_cc = Σ_seg psum in segment order (deterministic), the latent
// variance δ(1 − δ·(K_y⁻¹)_cc) at the observed components (c < ntr or npad ≤ c < npad + ntr),
// stats[0] = its minimum, stats[1] = max |W|.
__global__ __launch_bounds__(1024) void ozaki_guard_finish_kernel(const double* __restrict__ psum,
                                                                  const double* __restrict__ pmax, int64_t n,
                                                                  int64_t nseg, int64_t ntr, int64_t npad, double delta,
                                                                  double* __restrict__ stats) {
  __shared__ double red[2][16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double vmin = INFINITY, wmax = 0.0;
  for (int64_t c = tid; c < n; c += 1024) {
    double sq = 0.0, mx = 0.0;
    for (int64_t g = 0; g < nseg; ++g) {
      sq += psum[g * n + c];
      mx = fmax(mx, pmax[g * n + c]);
    }
    wmax = fmax(wmax, mx);
    const int64_t loc = c < npad ? c : c - npad;
    if (loc < ntr) vmin = fmin(vmin, delta * (1.0 - delta * sq));
  }
  for (int o = 32; o > 0; o >>= 1) {
    vmin = fmin(vmin, __shfl_xor(vmin, o));
    wmax = fmax(wmax, __shfl_xor(wmax, o));
  }
  if (lane == 0) { red[0][w] = vmin; red[1][w] = wmax; }
  __syncthreads();
  if (tid == 0) {
    for (int q = 1; q < 16; ++q) { vmin = fmin(vmin, red[0][q]); wmax = fmax(wmax, red[1][q]); }
    stats[0] = vmin;
    stats[1] = wmax;
  }
}

// ------------------------------------------------------------------ Morton order (point sorting)
// Bounding box of n points (dim 2 or 3): one 1024-thread workgroup, bbox[c] = min, bbox[3+c] = max.
__global__ __launch_bounds__(1024) void morton_bbox_kernel(const double* __restrict__ P, int64_t n, int dim,
                                                           double* __restrict__ bbox) {
  __shared__ double red[2][3][32];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int64_t i = tid; i < n; i += 1024)
    for (int c = 0; c < dim; ++c) {
      const double v = P[i * dim + c];
      lo[c] = fmin(lo[c], v);
      hi[c] = fmax(hi[c], v);
    }
  for (int c = 0; c < dim; ++c) {
    for (int o = 32; o > 0; o >>= 1) {
      lo[c] = fmin(lo[c], __shfl_xor(lo[c], o));
      hi[c] = fmax(hi[c], __shfl_xor(hi[c], o));
    }
    if (lane == 0) { red[0][c][w] = lo[c]; red[1][c][w] = hi[c]; }
  }
  __syncthreads();
  if (tid < dim) {
    double a = INFINITY, b = -INFINITY;
    for (int q = 0; q < 16; ++q) { a = fmin(a, red[0][tid][q]); b = fmax(b, red[1][tid][q]); }
    bbox[tid] = a;
    bbox[3 + tid] = b;
  }
}

__device__ __forceinline__ uint64_t spread2(uint64_t v) {   // 21 bits → every 2nd bit
  v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
  v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
  v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
  v = (v | (v << 2)) & 0x3333333333333333ull;
  return (v | (v << 1)) & 0x5555555555555555ull;
}
__device__ __forceinline__ uint64_t spread3(uint64_t v) {   // 21 bits → every 3rd bit
  v &= 0x1FFFFFull;
  v = (v | (v << 32)) & 0x001F00000000FFFFull;
  v = (v | (v << 16)) & 0x001F0000FF0000FFull;
  v = (v | (v << 8)) & 0x100F00F00F00F00Full;
  v = (v | (v << 4)) & 0x10C30C30C30C30C3ull;
  return (v | (v << 2)) & 0x1249249249249249ull;
}

// Z-order code of each point in its bounding box (21 bits per coordinate).
__global__ __launch_bounds__(256) void morton_code_kernel(const double* __restrict__ P, int64_t n, int dim,
                                                          const double* __restrict__ bbox,
                                                          int64_t* __restrict__ code) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint64_t c = 0;
  for (int k = 0; k < dim; ++k) {
    const double lo = bbox[k], span = fmax(bbox[3 + k] - lo, 1e-300);
    double q = rint((P[i * dim + k] - lo) / span * 2097151.0);
    q = fmin(fmax(q, 0.0), 2097151.0);
    const uint64_t v = (uint64_t)q;
    c |= (dim == 2 ? spread2(v) : spread3(v)) << k;
  }
  code[i] = (int64_t)c;
}

// ------------------------------------------------------------------ CRT + column Σ V²
// Residue planes are column-major ([j][i], ld = n).  One wave per OZ_CRT_COLS consecutive
// columns and a 64·RPL-row segment: lane l reconstructs rows RPL·l .. RPL·l + RPL − 1 (one
// RPL-byte load per plane and column), squares, and the wave reduces each column in a fixed
// shuffle order → partial[seg][j].  The lane's RPL row scales stay in registers across the
// wave's columns.
#ifndef GP2D_CRT_RPL
#define GP2D_CRT_RPL 16   // rows per lane: 16 (124 VGPRs, 4 waves per SIMD) or 8
#endif
constexpr int OZ_CRT_RPL = GP2D_CRT_RPL;
static_assert(OZ_CRT_RPL == 16 || OZ_CRT_RPL == 8, "CRT rows per lane: 16 or 8");
constexpr int OZ_CRT_ROWS = 64 * OZ_CRT_RPL;
constexpr int OZ_CRT_COLS = 4;    // columns per wave
constexpr int OZ_CRT_BCOLS = 4 * OZ_CRT_COLS;   // columns per 256-thread block

template <int RPL> struct crt_load;
template <> struct crt_load<16> { typedef uint4 type; };
template <> struct crt_load<8> { typedef uint2 type; };

#ifndef GP2D_CRT_OCC
#define GP2D_CRT_OCC 1   // min workgroups (= waves per SIMD) per CU the register budget must allow
#endif
__global__ __launch_bounds__(256, GP2D_CRT_OCC) void ozaki_crt_colsq_kernel(const uint8_t* __restrict__ cres, int64_t n,
                                                              int64_t ncols, OzakiConsts oc,
                                                              const double* __restrict__ rowscale,
                                                              double* __restrict__ P) {
  constexpr int RPL = OZ_CRT_RPL;
  typedef typename crt_load<RPL>::type ld_t;
  const int lane = threadIdx.x & 63;
  const int64_t jw = (int64_t)blockIdx.x * OZ_CRT_BCOLS + (threadIdx.x >> 6) * OZ_CRT_COLS;
  const int64_t seg = blockIdx.y;
  const int64_t i0 = seg * OZ_CRT_ROWS + RPL * lane;
  if (jw >= ncols) return;
  const bool rows_ok = i0 < n;
  double rs[RPL];
#pragma unroll
  for (int c = 0; c < RPL; ++c) rs[c] = rows_ok ? rowscale[i0 + c] : 0.0;
  const int64_t plane = n * ncols;
#pragma unroll 1
  for (int jc = 0; jc < OZ_CRT_COLS; ++jc) {
    const int64_t j = jw + jc;
    if (j >= ncols) break;
    double acc = 0.0;
    if (rows_ok) {
      double H[RPL], T[RPL];
#pragma unroll
      for (int c = 0; c < RPL; ++c) { H[c] = 0.0; T[c] = 0.0; }
      // planes in groups of 4 with the group's loads issued together; a group's planes past
      // nmod re-read plane nmod−1 (cached) and add nothing (h = t = 0 beyond nmod)
      const int nm1 = oc.nmod - 1;
      for (int l0 = 0; l0 < oc.nmod; l0 += 4) {
        ld_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          v[u] = *reinterpret_cast<const ld_t*>(cres + (int64_t)min(l0 + u, nm1) * plane + j * n + i0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t* w = reinterpret_cast<const uint32_t*>(&v[u]);
          const double h = oc.h[l0 + u], t = oc.t[l0 + u];
#pragma unroll
          for (int c = 0; c < RPL; ++c) {
            const double cl = (double)((w[c >> 2] >> (8 * (c & 3))) & 0xffu);
            H[c] = fma(cl, h, H[c]);   // exact: multiples of 2^-33 below 2^12
            T[c] = fma(cl, t, T[c]);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < RPL; ++c) {
        const double f = (H[c] - rint(H[c])) + T[c];   // Pint / M, centred
        const double vij = f * rs[c];
        acc = fma(vij, vij, acc);
        // |V_ij| ≤ ‖V_j‖₂ ≤ √kss: a value past the limit can only come from a CRT wrap-around
        // (|Pint| ≥ M/2, i.e. too few moduli) — poison the column instead of returning garbage
        if (fabs(vij) > oc.vlimit) acc = __builtin_nan("");
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) P[seg * ncols + j] = acc;
  }
}

}  // namespace gp2d
