// gemm_f64.hpp — FP64 MFMA GEMM core (v_mfma_f64_16x16x4_f64) for gfx950.
//
// One 128×128 output tile per 256-thread workgroup (4 waves as 2×2, each wave a
// 64×64 sub-tile = 4×4 MFMA tiles of 16×16, 64 fp64 accumulators per lane).
// K advances in BK=16 slabs staged through double-buffered LDS with register
// prefetch; one barrier per slab.  Used by every dense contraction of the path:
//   * Cholesky panel TRSM and trailing SYRK  (NT, c_lower)     — replaces LAPACK potrf
//     inside np.linalg.inv / GPy / sklearn (GP_laser.py:118, _gpr.py:349)
//   * TRTRI recursive doubling                (NN, a_lower / b_lower)
//   * predict variance V = L⁻¹·K*ᵀ with the column sum-of-squares fused in the
//     epilogue (NN, a_lower, EPI_COLSQ) — replaces Ks·Ki·Ksᵀ (GP_laser.py:129)
//     and solve_triangular+einsum (_gpr.py:454-475).
//
// MFMA f64 lane maps (verified on MI355X, tools/microbench/f64_rates.hip):
//   A: lane l holds A[l&15][l>>4]; B: lane l holds B[l>>4][l&15];
//   C/D: acc[r] of lane l is C[(l>>4) + 4r][l&15].
// LDS images: A as [BM][BK+2] and Bᵀ-stored B as [BN][BK+2] (stride ≡ 2 mod 32
// doubles: a 32-lane half reads 16 rows × 2 k-columns conflict-free); NN B as
// [BK][BN+16] (stride ≡ 16 mod 32: 2 rows × 16 columns conflict-free).
// Problem sizes are multiples of 128 (the engine pads), so there are no edge tiles.
#pragma once
#include "common.hpp"

namespace gp2d {

constexpr int GBM = 128, GBN = 128, GBK = 16;
constexpr int AS = GBK + 2;
constexpr int BS_NN = GBN + 16;
constexpr int BS_NT = GBK + 2;
constexpr int A_TILE = GBM * AS;                                            // 2304
constexpr int B_TILE = (GBK * BS_NN > GBN * BS_NT) ? GBK * BS_NN : GBN * BS_NT;  // 2304
constexpr int STAGE = A_TILE + B_TILE;

enum { EPI_STORE = 0, EPI_COLSQ = 1 };

struct GemmParams {
  const double* A; int64_t lda; int64_t sA;   // M×K row-major
  const double* B; int64_t ldb; int64_t sB;   // NN: K×N row-major; NT: N×K row-major
  double* C; int64_t ldc; int64_t sC;         // M×N
  int M, N, K;
  double alpha, beta;
  int a_lower;   // A lower-triangular: row block i0 only needs k < i0+BM
  int b_lower;   // (NN) B lower-triangular: column block j0 only needs k >= j0
  int a_upper;   // A upper-triangular: row block i0 only needs k >= i0
  int c_lower;   // enumerate lower tiles of a square C; diagonal tiles store i >= j
  int rev_rows;  // dispatch heavy (large i0) row blocks first (a_lower)
  int xcd_cols;  // 1-D grid: groups of 8 column tiles × all row blocks, column tile = XCD label
  int cols_first;  // 1-D grid, column blocks slow and ascending: heavy-first order for b_lower
  double* P; int64_t ldp; int64_t sP;         // EPI_COLSQ partials [M/BM][N]
  // Block-cyclic column tiles (the distributed factor, dfact.hpp): with jgrp > 0, column tile
  // bj sits jt = (bj / jgrp)·jgrp·jstep + bj % jgrp tiles from C's (and op(B)'s) first column
  // tile — groups of jgrp consecutive tiles, one group every jstep groups (a rank's super-
  // columns).  cyc_lower: only tiles with bi + mask_off ≥ jt run (the lower triangle in global
  // tile coordinates, mask_off = C's first global row tile − its first global column tile);
  // on bi + mask_off == jt the tile stores its lower triangle only.
  int jgrp, jstep;
  int cyc_lower, mask_off;
  // K split (EPI_STORE, beta = 0): with ksplit > 0 the launch carries 2·zcnt batch entries; a
  // tile whose K range is longer than ksplit is cut at its middle: entry z < zcnt sums the low
  // half into C, entry zcnt + z the high half into C2 (leading dimension ldc2, batch stride sC2;
  // zeros for an uncut tile) — one round of triangular long-K tiles becomes two rounds of
  // half-length ones; the caller adds C2 into C (add_into_kernel)
  int ksplit, zcnt;
  double* C2; int64_t ldc2; int64_t sC2;
  // Problem batch (batched factorisations, factor.hpp): launch_gemm(p, count, s, nprob) runs the
  // same product on nprob independent problems, problem q at A + q·pA, B + q·pB, C + q·pC,
  // C2 + q·pC2; grid.z = nprob × (entries per problem), zper = entries per problem (set by
  // launch_gemm; 0 = one problem).  Every problem's tiles sum in the same order as a lone launch.
  int zper;
  int64_t pA, pB, pC, pC2;
};

__host__ __device__ inline int cyc_tile(const GemmParams& p, int bj) {
  return p.jgrp > 0 ? (bj / p.jgrp) * p.jgrp * p.jstep + bj % p.jgrp : bj;
}

__device__ __forceinline__ void tri_tile(int t, int& bi, int& bj) {
  int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  bi = r;
  bj = t - r * (r + 1) / 2;
}

template <bool BT, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_f64_kernel(GemmParams p) {
  __shared__ double smem[2 * STAGE];

  int bi, bj;
  if (p.c_lower) {
    tri_tile(blockIdx.x, bi, bj);  // top rows first: the heavy ones under a_upper
  } else if (p.xcd_cols) {
    // Blocks b and b+8 share an XCD (round-robin dispatch).  Give every XCD one column
    // tile of the current group of 8 and all row blocks: the K*ᵀ column panel slabs are
    // then re-read from that XCD's L2 by all row blocks in step, and each W row panel is
    // read by 8 concurrent workgroups (one per XCD) through the Infinity Cache.
    const int nr = p.M / GBM;
    const int t = blockIdx.x;
    const int x = t & 7, q = t >> 3;
    const int g = q / nr, r = q - g * nr;
    bj = g * 8 + x;
    bi = nr - 1 - r;  // heavy (long-K) row blocks first
  } else if (p.cols_first) {
    const int nr = p.M / GBM;
    bj = (int)blockIdx.x / nr;
    bi = (int)blockIdx.x - bj * nr;
  } else {
    bj = blockIdx.x;
    bi = p.rev_rows ? (int)(gridDim.y - 1 - blockIdx.y) : (int)blockIdx.y;
  }
  int z = blockIdx.z, zq = 0;
  if (p.zper > 0) {   // problem zq of a problem batch
    zq = z / p.zper;
    z -= zq * p.zper;
  }
  const bool khigh = p.ksplit > 0 && z >= p.zcnt;   // the k ≥ ksplit half of a split product
  if (khigh) z -= p.zcnt;
  const int jt = cyc_tile(p, bj);
  if (p.cyc_lower && bi + p.mask_off < jt) return;   // strictly above the global diagonal
  const int i0 = bi * GBM, j0 = jt * GBN;
  const double* __restrict__ A = p.A + z * p.sA + zq * p.pA;
  const double* __restrict__ B = p.B + z * p.sB + zq * p.pB;

  int kb = max(p.b_lower ? j0 : 0, p.a_upper ? i0 : 0);
  int ke = p.a_lower ? min(p.K, i0 + GBM) : p.K;
  if (p.ksplit > 0) {   // tiles longer than ksplit: low half [kb, mid), high half [mid, ke)
    const int mid = (ke - kb > p.ksplit) ? kb + (((ke - kb) / 2) & ~(GBK - 1)) : ke;
    if (khigh) kb = mid;
    else ke = mid;
  }

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int lr = lane & 15, lk = lane >> 4;

  d4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = d4{0.0, 0.0, 0.0, 0.0};

  // global -> register prefetch mapping
  const int ar = tid >> 3, ac = (tid & 7) * 2;      // A / Bᵀ: 32 rows × 16 cols per pass
  const int br = tid >> 6, bc = (tid & 63) * 2;     // NN B:   4 rows × 128 cols per pass
  d2 ra[4], rb[4];

  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      ra[q] = *reinterpret_cast<const d2*>(A + (int64_t)(i0 + ar + 32 * q) * p.lda + k0 + ac);
    if (BT) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        rb[q] = *reinterpret_cast<const d2*>(B + (int64_t)(j0 + ar + 32 * q) * p.ldb + k0 + ac);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        rb[q] = *reinterpret_cast<const d2*>(B + (int64_t)(k0 + br + 4 * q) * p.ldb + j0 + bc);
    }
  };
  auto swrite = [&](int buf) {
    double* As = smem + buf * STAGE;
    double* Bs = As + A_TILE;
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<d2*>(As + (ar + 32 * q) * AS + ac) = ra[q];
    if (BT) {
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<d2*>(Bs + (ar + 32 * q) * BS_NT + ac) = rb[q];
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<d2*>(Bs + (br + 4 * q) * BS_NN + bc) = rb[q];
    }
  };

  if (kb < ke) {
    gload(kb);
    swrite(0);
    __syncthreads();
    int buf = 0;
    for (int k0 = kb; k0 < ke; k0 += GBK) {
      const bool has_next = (k0 + GBK) < ke;
      if (has_next) gload(k0 + GBK);
      const double* As = smem + buf * STAGE;
      const double* Bs = As + A_TILE;
#pragma unroll
      for (int kk = 0; kk < GBK; kk += 4) {
        double a[4], b[4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) a[mi] = As[(wr * 64 + mi * 16 + lr) * AS + kk + lk];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          if (BT) b[ni] = Bs[(wc * 64 + ni * 16 + lr) * BS_NT + kk + lk];
          else    b[ni] = Bs[(kk + lk) * BS_NN + wc * 64 + ni * 16 + lr];
        }
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
      }
      if (has_next) swrite(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  if (EPI == EPI_STORE) {
    double* __restrict__ C = khigh ? p.C2 + z * p.sC2 + zq * p.pC2 : p.C + z * p.sC + zq * p.pC;
    const int64_t ldc = khigh ? p.ldc2 : p.ldc;
    const bool diag_tile = (p.c_lower && bi == bj) || (p.cyc_lower && bi + p.mask_off == jt);
    const bool has_beta = p.beta != 0.0;
    // per 16-row group mi: 16 C loads, then the updates and stores (element-wise load → use →
    // store chains leave one HBM round trip per element).  With β ≠ 0 group mi+1's loads are
    // issued before group mi's updates, so a tile's C read costs one exposed round trip instead
    // of four; the per-element arithmetic is the same (round 3, profiles/r03_syrk_epilogue_ab.txt).
    auto cload = [&](int mi, double (&old)[4][4]) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i0 + wr * 64 + mi * 16 + lk + 4 * r;
          const int col = j0 + wc * 64 + ni * 16 + lr;
          old[ni][r] = __builtin_nontemporal_load(C + (int64_t)row * ldc + col);
        }
    };
    auto cstore = [&](int mi, const double (&old)[4][4]) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i0 + wr * 64 + mi * 16 + lk + 4 * r;
          const int col = j0 + wc * 64 + ni * 16 + lr;
          double v = p.alpha * acc[mi][ni][r];
          if (has_beta) v = fma(p.beta, old[ni][r], v);
          if (!(diag_tile && col - j0 > row - i0)) C[(int64_t)row * ldc + col] = v;
        }
    };
    if (has_beta) {
      double o0[4][4], o1[4][4];
      cload(0, o0);
      cload(1, o1);
      cstore(0, o0);
      cload(2, o0);
      cstore(1, o1);
      cload(3, o1);
      cstore(2, o0);
      cstore(3, o1);
    } else {
      const double none[4][4] = {};
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) cstore(mi, none);
    }
  } else {
    // column sums of squares of this 128-row slab of V, combined in a fixed order:
    // registers (rows (l>>4)+4r+16mi) -> lanes l, l^16, l^32, l^48 -> the two wave rows.
    double* red = smem;  // [2][128]
    double s[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      double t = 0.0;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) t += acc[mi][ni][r] * acc[mi][ni][r];
      t += __shfl_xor(t, 16);
      t += __shfl_xor(t, 32);
      s[ni] = t;
    }
    if (lane < 16) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) red[wr * 128 + wc * 64 + ni * 16 + lane] = s[ni];
    }
    __syncthreads();
    if (tid < 128) {
      double* __restrict__ P = p.P + z * p.sP + (int64_t)bi * p.ldp + j0;   // (no problem batch with COLSQ)
      P[tid] = red[tid] + red[128 + tid];
    }
  }
}

// Host-side launcher.  Returns 0 / negative error.
template <bool BT, int EPI>
inline int launch_gemm(const GemmParams& pin, int batch, hipStream_t s, int nprob = 1) {
  if (pin.M <= 0 || pin.N <= 0 || batch <= 0 || nprob <= 0) return 0;
  GemmParams p = pin;
  if (nprob > 1 && EPI != EPI_STORE) {
    set_error("gemm: a problem batch needs EPI_STORE");
    return -2;
  }
  if ((p.M % GBM) || (p.N % GBN) || (p.K % GBK)) {
    set_error("gemm: sizes must be multiples of 128/128/16");
    return -2;
  }
  dim3 grid;
  if (p.c_lower) {
    const int t = p.M / GBM;
    grid = dim3(t * (t + 1) / 2, 1, batch);
  } else if (p.xcd_cols) {
    if ((p.N / GBN) % 8) {
      set_error("gemm: xcd_cols needs a multiple of 8 column tiles");
      return -2;
    }
    grid = dim3((p.N / GBN) * (p.M / GBM), 1, batch);
  } else if (p.cols_first) {
    grid = dim3((p.N / GBN) * (p.M / GBM), 1, batch);
  } else {
    grid = dim3(p.N / GBN, p.M / GBM, batch);
  }
  if (p.ksplit > 0) {
    if (EPI != EPI_STORE || p.beta != 0.0 || p.c_lower || p.cyc_lower || p.C2 == nullptr || batch != p.zcnt) {
      set_error("gemm: K split needs EPI_STORE, beta = 0, no triangle mask, C2 and batch == zcnt");
      return -2;
    }
    grid.z = 2 * batch;
  }
  p.zper = nprob > 1 ? (int)grid.z : 0;
  grid.z *= (unsigned)nprob;
  if (grid.z > 65535u) {
    set_error("gemm: too many batch entries");
    return -2;
  }
  gemm_f64_kernel<BT, EPI><<<grid, 256, 0, s>>>(p);
  return check_launch("gemm_f64_kernel");
}

// C[z] += D[z] over an M×N block per batch entry (row strides ldc / ldd, batch strides sC / sD):
// the two halves of a K-split product (GemmParams::ksplit), summed in a fixed order.
// Problem batch: grid.z = nprob × count, problem q at C + q·pC, D + q·pD.
__global__ __launch_bounds__(256) void add_into_kernel(double* __restrict__ C, int64_t ldc, int64_t sC,
                                                       const double* __restrict__ D, int64_t ldd, int64_t sD,
                                                       int M, int N, int count, int64_t pC, int64_t pD) {
  const int zq = (int)blockIdx.z / count, z = (int)blockIdx.z - zq * count;
  const int row = blockIdx.y;
  double* c = C + z * sC + zq * pC + (int64_t)row * ldc;
  const double* d = D + z * sD + zq * pD + (int64_t)row * ldd;
  for (int j = (blockIdx.x * 256 + threadIdx.x) * 2; j < N; j += gridDim.x * 512) {
    const d2 a = *reinterpret_cast<const d2*>(c + j), b = *reinterpret_cast<const d2*>(d + j);
    *reinterpret_cast<d2*>(c + j) = d2{a.x + b.x, a.y + b.y};
  }
}

inline GemmParams gemm_params() {
  GemmParams p{};
  p.alpha = 1.0;
  p.beta = 0.0;
  return p;
}

// ---------------------------------------------------------------------------------------
// Skinny NT GEMM for the POTRF critical path (column update, panel TRSM):
//   C[M×128] = alpha · A[M×128] · B[128×128]ᵀ + beta · C,   M a multiple of R.
// With K = 128 the 128×128-tile kernel above spends most of each tile waiting for its
// next BK = 16 slab (≈ 45 µs per tile); here one workgroup owns an R-row × CB-column block of
// C and stages its operands in two K-halves of 64 — R A rows and the CB B rows of its columns
// (B is identical for every workgroup, so L2-resident) — with the second half's loads in
// flight during the first half's MFMAs; the 4 waves share the block's 16×16 tiles of
// v_mfma_f64_16x16x4.  LDS rows are 64 doubles with k XOR-swizzled by 2·(row & 15): the MFMA
// operand reads (16 rows × 2 k per 32-lane half) touch 64 distinct banks and 16-B pairs
// (k, k+1) stay adjacent.  Every 16×16 tile of C sums its K = 128 in the same order (k = 4ks +
// lane/16, ks ascending, the first half then the second) whatever R and CB, so all shapes give
// the same bits.
// Shapes (measured, tools/microbench/panel_bench.hip (git f1195df)): a launch costs ≈ 11 µs even for four
// workgroups — a workgroup's own 1 Mflop of f64 MFMAs at one wave per SIMD is ≈ 8k cycles — so
// the column update splits its 128 columns over four workgroups (R = 32, CB = 32; one tile per
// wave) and the in-place TRSM, whose workgroups must own whole rows, halves the rows (R = 16,
// CB = 128).
// C may alias A row for row only with CB = 128 (the in-place TRSM): a workgroup reads all of
// its A rows before it writes them, and no other workgroup touches those rows.
// Grid: (M / R, problems, 128 / CB).
constexpr int PNL_R = 32;
__device__ __forceinline__ int pnl_idx(int r, int k) { return r * 64 + (k ^ ((r & 15) << 1)); }

// Problem batch: problem blockIdx.y at A + y·pA, B + y·pB, C + y·pC (0 for a lone launch).
template <int R, int CB>
__global__ __launch_bounds__(256) void gemm_f64_panel_kernel(const double* A, int64_t lda, const double* __restrict__ B,
                                                             int64_t ldb, double* C, int64_t ldc, double alpha,
                                                             double beta, int64_t pA, int64_t pB, int64_t pC) {
  static_assert((R == 16 || R == 32) && (CB == 32 || CB == 64 || CB == 128), "panel block shape");
  constexpr int TJ = CB / 16;                  // column tiles of the block
  constexpr int TPW = (R / 16) * TJ / 4;       // 16×16 tiles per wave: 1, 2 or 4
  static_assert(TPW >= 1, "at least one tile per wave");
  constexpr int NLD = (R + CB) * 32 / 256;     // 16-B loads per thread per K-half
  __shared__ __attribute__((aligned(16))) double As[R * 64];
  __shared__ __attribute__((aligned(16))) double Bs[CB * 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  A += blockIdx.y * pA;
  B += blockIdx.y * pB;
  C += blockIdx.y * pC;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int c0 = (int)blockIdx.z * CB;
  auto load = [&](int h, d2 (&v)[NLD]) {
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int idx = tid + 256 * u;   // < (R + CB)·32
      if (idx < R * 32) {
        const int r = idx >> 5, c = 64 * h + 2 * (idx & 31);
        v[u] = *reinterpret_cast<const d2*>(A + (r0 + r) * lda + c);
      } else {
        const int j = idx - R * 32, r = j >> 5, c = 64 * h + 2 * (j & 31);
        v[u] = *reinterpret_cast<const d2*>(B + (int64_t)(c0 + r) * ldb + c);
      }
    }
  };
  auto stage = [&](const d2 (&v)[NLD]) {
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int idx = tid + 256 * u;
      if (idx < R * 32) {
        const int r = idx >> 5, c = 2 * (idx & 31);
        *reinterpret_cast<d2*>(As + pnl_idx(r, c)) = v[u];
      } else {
        const int j = idx - R * 32, r = j >> 5, c = 2 * (j & 31);
        *reinterpret_cast<d2*>(Bs + pnl_idx(r, c)) = v[u];
      }
    }
  };
  d4 acc[TPW];
#pragma unroll
  for (int u = 0; u < TPW; ++u) acc[u] = d4{0.0, 0.0, 0.0, 0.0};
  const int l16 = lane & 15, lk = lane >> 4;
  auto tile_i = [&](int u) { return (wid * TPW + u) / TJ; };   // row tile of the wave's u-th tile
  auto tile_j = [&](int u) { return (wid * TPW + u) % TJ; };   // column tile
  auto compute = [&]() {
#pragma unroll 4
    for (int ks = 0; ks < 16; ++ks) {
      const int k = 4 * ks + lk;
#pragma unroll
      for (int u = 0; u < TPW; ++u) {
        const double a = As[pnl_idx(16 * tile_i(u) + l16, k)], b = Bs[pnl_idx(16 * tile_j(u) + l16, k)];
        acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[u], 0, 0, 0);
      }
    }
  };
  {
    d2 v[NLD];
    load(0, v);
    stage(v);
    load(1, v);   // second half in flight during the first half's MFMAs
    __syncthreads();
    compute();
    __syncthreads();
    stage(v);
    __syncthreads();
    compute();
  }
  // f64 C/D map: acc[r] of lane l is C[(l>>4) + 4r][l&15].  C may alias A (CB = 128 only): this
  // workgroup's A rows were all read (into registers / LDS) before the barrier above.
#pragma unroll
  for (int u = 0; u < TPW; ++u)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t row = r0 + 16 * tile_i(u) + lk + 4 * q;
      const int col = c0 + 16 * tile_j(u) + l16;
      double* cp = C + row * ldc + col;
      const double old = (beta != 0.0) ? *cp : 0.0;
      *cp = fma(alpha, acc[u][q], beta * old);
    }
}

// The two shapes of the POTRF chain: column update (C ≠ A) and in-place panel TRSM (C = A).
constexpr int PNL_UPD_R = 32, PNL_UPD_CB = 32, PNL_TRSM_R = 16, PNL_TRSM_CB = 128;

}  // namespace gp2d
