// Persistent form of the POTRF trailing SYRK (dev experiment, round 3): one grid of 2 workgroups
// per CU walks the lower tiles statically (t, t + grid, ...); the last K slab of a tile issues the
// next tile's first-slab loads, so that global round trip runs under the C epilogue instead of
// after it.  Same per-tile arithmetic as gemm_f64_kernel<true, EPI_STORE> with c_lower.
#pragma once
#include "../../2d-gp_amd/csrc/gemm_f64.hpp"
namespace gp2d {
__global__ __launch_bounds__(256, 2) void syrk_persist_kernel(GemmParams p, int ntiles) {
  __shared__ double smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, lr = lane & 15, lk = lane >> 4;
  const int ar = tid >> 3, ac = (tid & 7) * 2;
  d2 ra[4], rb[4];
  auto gload = [&](int i0, int j0, int k0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) ra[q] = *reinterpret_cast<const d2*>(p.A + (int64_t)(i0 + ar + 32 * q) * p.lda + k0 + ac);
#pragma unroll
    for (int q = 0; q < 4; ++q) rb[q] = *reinterpret_cast<const d2*>(p.B + (int64_t)(j0 + ar + 32 * q) * p.ldb + k0 + ac);
  };
  auto swrite = [&](int buf) {
    double* As = smem + buf * STAGE;
    double* Bs = As + A_TILE;
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<d2*>(As + (ar + 32 * q) * AS + ac) = ra[q];
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<d2*>(Bs + (ar + 32 * q) * BS_NT + ac) = rb[q];
  };
  int t = blockIdx.x;
  if (t >= ntiles) return;
  int bi, bj;
  tri_tile(t, bi, bj);
  gload(bi * GBM, bj * GBN, 0);
  for (;;) {
    const int i0 = bi * GBM, j0 = bj * GBN;
    const int tn = t + (int)gridDim.x;
    int ni = 0, nj = 0;
    if (tn < ntiles) tri_tile(tn, ni, nj);
    swrite(0);
    __syncthreads();
    d4 acc[4][4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[mi][n] = d4{0.0, 0.0, 0.0, 0.0};
    int buf = 0;
    for (int k0 = 0; k0 < p.K; k0 += GBK) {
      const bool has_next = (k0 + GBK) < p.K;
      if (has_next) gload(i0, j0, k0 + GBK);
      else if (tn < ntiles) gload(ni * GBM, nj * GBN, 0);   // next tile's first slab, under the epilogue
      const double* As = smem + buf * STAGE;
      const double* Bs = As + A_TILE;
#pragma unroll
      for (int kk = 0; kk < GBK; kk += 4) {
        double a[4], b[4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) a[mi] = As[(wr * 64 + mi * 16 + lr) * AS + kk + lk];
#pragma unroll
        for (int n = 0; n < 4; ++n) b[n] = Bs[(wc * 64 + n * 16 + lr) * BS_NT + kk + lk];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int n = 0; n < 4; ++n)
            acc[mi][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi], b[n], acc[mi][n], 0, 0, 0);
      }
      if (has_next) swrite(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
    double* __restrict__ C = p.C;
    const bool diag_tile = bi == bj;
    auto cload = [&](int mi, double (&old)[4][4]) {
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          old[n][r] = __builtin_nontemporal_load(C + (int64_t)(i0 + wr * 64 + mi * 16 + lk + 4 * r) * p.ldc +
                                                 j0 + wc * 64 + n * 16 + lr);
    };
    auto cstore = [&](int mi, const double (&old)[4][4]) {
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i0 + wr * 64 + mi * 16 + lk + 4 * r, col = j0 + wc * 64 + n * 16 + lr;
          const double v = fma(p.beta, old[n][r], p.alpha * acc[mi][n][r]);
          if (!(diag_tile && col - j0 > row - i0)) C[(int64_t)row * p.ldc + col] = v;
        }
    };
    // one row group at a time (the prefetched slab holds 32 VGPRs through the epilogue)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      double old[4][4];
      cload(mi, old);
      cstore(mi, old);
    }
    if (tn >= ntiles) break;
    t = tn;
    bi = ni;
    bj = nj;
  }
}
inline int launch_syrk_persist(const GemmParams& q, hipStream_t s) {
  const int t = q.M / GBM, nt = t * (t + 1) / 2;
  syrk_persist_kernel<<<nt < 512 ? nt : 512, 256, 0, s>>>(q, nt);
  return 0;
}
}  // namespace gp2d
