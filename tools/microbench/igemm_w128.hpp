// igemm_w128.hpp — DEV VARIANT of ozaki.hpp's igemm_nt_mod_kernel (tools/microbench only):
// the same 256×256 output tile per workgroup, but 4 waves (one per SIMD, 2×2) of 128×128 each
// (8×8 tiles of v_mfma_i32_16x16x64_i8, 256 accumulators per lane — held in AGPRs), instead of
// 8 waves (two per SIMD) of 128×64.  Per slab a wave reads 8 A + 8 B fragments (16 KB) instead
// of 8 + 4 (12 KB) for twice the MFMAs: the workgroup's LDS fragment reads fall from 96 KB to
// 64 KB per slab.  Each wave issues 8 LDS-DMA pieces per
// slab (4 A + 4 B) with no second wave on its SIMD to cover their issue.  Dense K loop (no slab
// list, no (v,u) aliasing): igemm_bench.hip's random-residue triangle.
#pragma once
#include "../../2d-gp_amd/csrc/ozaki.hpp"
namespace gp2d {

template <int NST>
__global__ __launch_bounds__(256, 1) void igemm_w128_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ B,
                                                            uint8_t* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                            int a_lower, int modulus, int, int, const int*,
                                                            const int*) {
  constexpr int PPW = 8;                       // DMA pieces per wave per slab (4 A, 4 B)
  __shared__ __attribute__((aligned(16))) int8_t smem[NST * I_STAGE];
  const int bj = blockIdx.x;
  const int bi = (int)(gridDim.y - 1 - blockIdx.y);
  const int i0 = bi * IBM, j0 = bj * IBN;
  const int ke = a_lower ? min(K, i0 + IBM) : K;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int l16 = lane & 15, lq = lane >> 4;
  const int64_t kslabs = K / IBK;
  const int8_t* Ap = A + (int64_t)bi * kslabs * I_OP;
  const int8_t* Bp = B + (int64_t)bj * kslabs * I_OP;
  const int nsl = ke / IBK;
  const int bias = (int)ozaki_acc_bias(K, modulus);
  i4v acc[8][8];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = i4v{bias, bias, bias, bias};
  const int drow = lane >> 2, dchunk = lane & 3;
  auto issue_piece = [&](int ks, int st, int p) {   // one 1 KB piece: A rows (p < 4) or B rows
    int8_t* dst = smem + st * I_STAGE + (p < 4 ? 0 : I_OP);
    const int8_t* src = (p < 4 ? Ap : Bp) + (int64_t)ks * I_OP;
    const int h = p & 3;
    const int row = (wid * 4 + h) * 16 + drow;
    __builtin_amdgcn_global_load_lds((const void*)(src + row * IBK + 16 * swz16(row, dchunk)),
                                     (lds_ptr_t)(dst + (wid * 4 + h) * 16 * IBK), 16, 0, 0);
  };
  auto issue = [&](int ks, int st) {
    int8_t* As = smem + st * I_STAGE;
    int8_t* Bs = As + I_OP;
    const int8_t* Ag = Ap + (int64_t)ks * I_OP;
    const int8_t* Bg = Bp + (int64_t)ks * I_OP;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int row = (wid * 4 + h) * 16 + drow;
      __builtin_amdgcn_global_load_lds((const void*)(Ag + row * IBK + 16 * swz16(row, dchunk)),
                                       (lds_ptr_t)(As + (wid * 4 + h) * 16 * IBK), 16, 0, 0);
    }
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int row = (wid * 4 + h) * 16 + drow;
      __builtin_amdgcn_global_load_lds((const void*)(Bg + row * IBK + 16 * swz16(row, dchunk)),
                                       (lds_ptr_t)(Bs + (wid * 4 + h) * 16 * IBK), 16, 0, 0);
    }
  };
  const uint32_t lds_base = (uint32_t)(size_t)(lds_ptr_t)smem;
  auto reada = [&](int st, int half, i4v (&a)[4]) {
    const uint32_t As = lds_base + st * I_STAGE;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = wr * 128 + (4 * half + u) * 16 + l16;
      const uint32_t ad = As + row * IBK + 16 * swz16(row, lq);
      asm volatile("ds_read_b128 %0, %1" : "=v"(a[u]) : "v"(ad) : "memory");
    }
  };
  auto readb = [&](int st, i4v (&b)[8]) {
    const uint32_t Bs = lds_base + st * I_STAGE + I_OP;
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      const int row = wc * 128 + ni * 16 + l16;
      const uint32_t ad = Bs + row * IBK + 16 * swz16(row, lq);
      asm volatile("ds_read_b128 %0, %1" : "=v"(b[ni]) : "v"(ad) : "memory");
    }
  };
  auto mfmas = [&](int half, const i4v (&a)[4], const i4v (&b)[8]) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int ni = 0; ni < 8; ++ni)
        acc[4 * half + u][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u], b[ni], acc[4 * half + u][ni], 0, 0, 0);
  };
#ifdef W128_SPREAD
  // the slab's DMA pieces spread through half 0's MFMAs: 2 pieces after every 8 MFMAs
  auto mfmas_dma = [&](const i4v (&a)[4], const i4v (&b)[8], int ks, int st) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int ni = 0; ni < 8; ++ni)
        acc[u][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u], b[ni], acc[u][ni], 0, 0, 0);
      issue_piece(ks, st, u);
      issue_piece(ks, st, 4 + u);
    }
  };
#endif
  if (nsl > 0) {
#pragma unroll
    for (int q = 0; q < NST - 1; ++q) issue(q, q);
    vmwait_barrier<PPW>(std::integral_constant<int, NST - 2>{});
    i4v bA[8], a0A[4], bB[8], a0B[4], a1[4];
    readb(0, bA);
    reada(0, 0, a0A);
    __builtin_amdgcn_sched_barrier(0);
    constexpr int LAST = -1;
    auto step = [&](auto dma_c, auto w_c, int s, i4v (&b)[8], i4v (&a0)[4], i4v (&bn)[8], i4v (&a0n)[4]) {
      constexpr bool dma = decltype(dma_c)::value;
      constexpr int w = decltype(w_c)::value;
      const int st = s % NST;
#ifndef W128_SPREAD
      if constexpr (dma) issue(s + NST - 1, (s + NST - 1) % NST);
#endif
      reada(st, 1, a1);
      asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");   // b, a0 landed
      __builtin_amdgcn_sched_barrier(0);
#ifdef W128_SPREAD
      if constexpr (dma) mfmas_dma(a0, b, s + NST - 1, (s + NST - 1) % NST);
      else mfmas(0, a0, b);
#else
      mfmas(0, a0, b);
#endif
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (w != LAST) {
        vmwait_barrier<PPW>(w_c);
        const int st1 = (s + 1) % NST;
        readb(st1, bn);
        reada(st1, 0, a0n);
        asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");   // a1 landed (older than the 12 new reads)
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
    const int m = nsl - (NST - 1);
    int s = 0;
    for (; s + 1 < m; s += 2) {
      step(T_{}, W_FULL{}, s, bA, a0A, bB, a0B);
      step(T_{}, W_FULL{}, s + 1, bB, a0B, bA, a0A);
    }
    if (s < m) {
      step(T_{}, W_FULL{}, s, bA, a0A, bB, a0B);
      ++s;
#pragma unroll
      for (int u = 0; u < 8; ++u) bA[u] = bB[u];
#pragma unroll
      for (int u = 0; u < 4; ++u) a0A[u] = a0B[u];
    }
    static_assert(NST == 4, "tail written for a 4-stage ring");
    step(F_{}, std::integral_constant<int, 1>{}, s, bA, a0A, bB, a0B);
    step(F_{}, std::integral_constant<int, 0>{}, s + 1, bB, a0B, bA, a0A);
    step(F_{}, std::integral_constant<int, LAST>{}, s + 2, bA, a0A, bB, a0B);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  uint8_t* T = reinterpret_cast<uint8_t*>(smem);
  constexpr int TP = IBM + 16;
  static_assert(IBN * TP <= NST * I_STAGE, "epilogue image fits the ring");
  const OzModConsts mc = ozaki_mod_consts(modulus);
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      uint32_t pk = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) pk |= ozaki_mod_u32((uint32_t)acc[mi][ni][u], mc) << (8 * u);
      const int rloc = wr * 128 + mi * 16 + 4 * lq;
      const int cloc = wc * 128 + ni * 16 + l16;
      *reinterpret_cast<uint32_t*>(T + cloc * TP + rloc) = pk;
    }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < (IBM * IBN / 16) / 256; ++p) {
    const int id = tid + 256 * p;
    const int cloc = id >> 4, ch = id & 15;
    const uint4 v = *reinterpret_cast<const uint4*>(T + cloc * TP + 16 * ch);
    *reinterpret_cast<uint4*>(C + (int64_t)(j0 + cloc) * ldc + i0 + 16 * ch) = v;
  }
}

}  // namespace gp2d
