// igemm_epi.hpp — DEV VARIANT (tools/microbench only) of ozaki.hpp's igemm_nt_mod_kernel<256, 4>
// (dense K loop) for timing the epilogue: EPI_LDS = the product's LDS-transposed column-major
// residue tile; default = the residues stored straight from the MFMA registers in a tile-blocked
// layout (no LDS image, no barrier) — a layout the CRT would have to read instead (the sampled
// check of igemm_bench then does not apply).
#pragma once
#include "../../2d-gp_amd/csrc/ozaki.hpp"
namespace gp2d {

template <int NST>
__global__ __launch_bounds__(512, 1) void igemm_epi_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ B,
                                                          uint8_t* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                          int a_lower, int modulus, int alias_rb, int alias_ks,
                                                          const int* __restrict__, const int* __restrict__) {
  static_assert(NST == 4, "4-stage ring");
  constexpr int TBN = 256, WC = 4, AP = 2, BPW = 2, PPW = AP + BPW;
  constexpr int STG = I_OP + TBN * IBK;
  __shared__ __attribute__((aligned(16))) int8_t smem[NST * STG];
  const int bj = blockIdx.x;
  const int bi = (int)(gridDim.y - 1 - blockIdx.y);
  const int i0 = bi * IBM, j0 = bj * TBN;
  const int jb = j0 / IBN, jr = j0 % IBN;
  const int ke = a_lower ? min(K, i0 + IBM) : K;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WC, wc = wid % WC;
  const int l16 = lane & 15, lq = lane >> 4;
  const int64_t kslabs = K / IBK;
  const int8_t* Ap = A + (int64_t)bi * kslabs * I_OP;
  const bool alias = jb >= alias_rb;
  const int8_t* Bp = B + (int64_t)jb * kslabs * I_OP + jr * IBK;
  const int8_t* Bq = B + ((int64_t)(alias ? jb - alias_rb : 0) * kslabs + alias_ks) * I_OP + jr * IBK;
  const int nsl = ke / IBK;   // dense K loop, ≥ 4 (K ≥ 256)
  const int bias = (int)ozaki_acc_bias(K, modulus);
  i4v acc[8][4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = i4v{bias, bias, bias, bias};

  const int drow = lane >> 2, dchunk = lane & 3;
  auto issue = [&](int ks, int st) {
    int8_t* As = smem + st * STG;
    int8_t* Bs = As + I_OP;
    const int8_t* Ag = Ap + (int64_t)ks * I_OP;
    const int8_t* Bg = ((alias && ks < alias_ks) ? Bq : Bp) + (int64_t)ks * I_OP;
#pragma unroll
    for (int h = 0; h < AP; ++h) {
      const int row = (wid * AP + h) * 16 + drow;
      __builtin_amdgcn_global_load_lds((const void*)(Ag + row * IBK + 16 * swz16(row, dchunk)),
                                       (lds_ptr_t)(As + (wid * AP + h) * 16 * IBK), 16, 0, 0);
    }
#pragma unroll
    for (int h = 0; h < BPW; ++h) {
      const int row = (wid * BPW + h) * 16 + drow;
      __builtin_amdgcn_global_load_lds((const void*)(Bg + row * IBK + 16 * swz16(jr + row, dchunk)),
                                       (lds_ptr_t)(Bs + (wid * BPW + h) * 16 * IBK), 16, 0, 0);
    }
  };
  const uint32_t lds_base = (uint32_t)(size_t)(lds_ptr_t)smem;
  auto reada = [&](int st, int half, i4v (&a)[4]) {
    const uint32_t As = lds_base + st * STG;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = wr * 128 + (4 * half + u) * 16 + l16;
      asm volatile("ds_read_b128 %0, %1" : "=v"(a[u]) : "v"(As + row * IBK + 16 * swz16(row, lq)) : "memory");
    }
  };
  auto readb = [&](int st, i4v (&b)[4]) {
    const uint32_t Bs = lds_base + st * STG + I_OP;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int row = wc * 64 + ni * 16 + l16;
      asm volatile("ds_read_b128 %0, %1" : "=v"(b[ni]) : "v"(Bs + row * IBK + 16 * swz16(jr + row, lq)) : "memory");
    }
  };
  auto mfmas = [&](int half, const i4v (&a)[4], const i4v (&b)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        acc[4 * half + u][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u], b[ni], acc[4 * half + u][ni], 0, 0, 0);
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
#pragma unroll
  for (int q = 0; q < NST - 1; ++q) issue(q, q);
  {
    // ---------------------------------------------------------------- early group: product order
    vmwait_barrier<PPW>(std::integral_constant<int, 2>{});   // slab 0 (own pieces), barrier −1
    i4v bA[4], a0A[4], bB[4], a0B[4], a1[4];
    readb(0, bA);
    reada(0, 0, a0A);
    __builtin_amdgcn_sched_barrier(0);
    constexpr int LAST = -1;
    auto step = [&](auto dma_c, auto w_c, int s, i4v (&b)[4], i4v (&a0)[4], i4v (&bn)[4], i4v (&a0n)[4]) {
      constexpr bool dma = decltype(dma_c)::value;
      constexpr int w = decltype(w_c)::value;
      const int st = s % NST;
      if constexpr (dma) issue(s + NST - 1, (s + NST - 1) % NST);
      reada(st, 1, a1);
      asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mfmas(0, a0, b);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (w != LAST) {
        vmwait_barrier<PPW>(w_c);   // barrier s: publish slab s+1
        const int st1 = (s + 1) % NST;
        readb(st1, bn);
        reada(st1, 0, a0n);
        asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      mfmas(1, a1, b);
      __builtin_amdgcn_sched_barrier(0);
    };
    const int m = nsl - (NST - 1);
    int s = 0;
    for (; s + 1 < m; s += 2) {
      step(T_{}, std::integral_constant<int, 2>{}, s, bA, a0A, bB, a0B);
      step(T_{}, std::integral_constant<int, 2>{}, s + 1, bB, a0B, bA, a0A);
    }
    if (s < m) {
      step(T_{}, std::integral_constant<int, 2>{}, s, bA, a0A, bB, a0B);
      ++s;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        bA[u] = bB[u];
        a0A[u] = a0B[u];
      }
    }
    step(F_{}, std::integral_constant<int, 1>{}, s, bA, a0A, bB, a0B);
    step(F_{}, std::integral_constant<int, 0>{}, s + 1, bB, a0B, bA, a0A);
    step(F_{}, std::integral_constant<int, LAST>{}, s + 2, bA, a0A, bB, a0B);
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
#ifdef EPI_LDS
  asm volatile("s_barrier" ::: "memory");
  uint8_t* T = reinterpret_cast<uint8_t*>(smem);
  constexpr int TP = IBM + 16;
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
    const uint4 v = *reinterpret_cast<const uint4*>(T + cloc * TP + 16 * ch);
    *reinterpret_cast<uint4*>(C + (int64_t)(j0 + cloc) * ldc + i0 + 16 * ch) = v;
  }
#else
  // direct stores of the MFMA layout (timing only: tile-blocked [tile][mi][ni][lane] dwords,
  // a wave's store of one (mi, ni) = 256 contiguous bytes); no LDS image, no barrier
  const OzModConsts mc = ozaki_mod_consts(modulus);
  uint32_t* Ct = reinterpret_cast<uint32_t*>(C) + ((int64_t)bj * gridDim.y + bi) * (IBM * TBN / 4);
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      uint32_t pk = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) pk |= ozaki_mod_u32((uint32_t)acc[mi][ni][u], mc) << (8 * u);
      Ct[((wid * 8 + mi) * 4 + ni) * 64 + lane] = pk;
    }
#endif
}
}  // namespace gp2d
