// igemm_rot.hpp — DEV VARIANT of ozaki.hpp's igemm_nt_mod_kernel<256, 4> (tools/microbench only,
// dense K loop) with the late wave group (waves 4-7, the second wave on each SIMD) running its
// slab step rotated by half a step against the early group (waves 0-3, the product's order).
//
// The stamps show both waves of a SIMD leaving each barrier together and doing
// their fragment reads at the same time, so the matrix core idles while both wait on LDS.  Here,
// between barriers k and k+1:
//   early (product):  read b,a0 of slab k+1 | h1(k) | DMA k+3 | read a1(k+1) | h0(k+1) | wait
//   late  (rotated):  h0(k) | read b,a0 of slab k+1 | h1(k) | DMA k+4 | read a1(k+1) | wait
// so the late wave issues MFMAs straight out of the barrier while the early wave reads, and the
// two groups' read phases fall at different points of the interval.  The late wave carries every
// fragment of slab k into the interval (read before the barrier), so its MFMAs need no wait.
// Ordering (barrier k publishes slab k+1 in both groups):
//   RAW: the late wave reads slab k+1 after barrier k, having waited for its own pieces of slab
//        k+1 before it (vmcnt: the pieces of slabs issued after k+1 may stay in flight).
//   WAR: slab k's stage is rewritten only after barrier k: the early group issues slab k+4 into it
//        at its step k+1 (after barrier k), the late group in interval k (after barrier k); every
//        read of slab k (early: b, a0 after barrier k−1 and a1 before barrier k; late: all of it
//        in interval k−1) completed before barrier k (lgkmcnt(0) ahead of every barrier).
//   Barrier count: both groups meet nsl + 1 barriers (prologue, nsl − 1 publications, final).
#pragma once
#include "../../2d-gp_amd/csrc/ozaki.hpp"
namespace gp2d {

template <int NST>
__global__ __launch_bounds__(512, 1) void igemm_rot_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ B,
                                                          uint8_t* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                          int a_lower, int modulus, int alias_rb, int alias_ks,
                                                          const int* __restrict__, const int* __restrict__) {
  static_assert(NST == 4, "rotated schedule written for the 4-stage ring");
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
  const bool late = __builtin_amdgcn_readfirstlane(wid) >= 4 && nsl >= 4;

#pragma unroll
  for (int q = 0; q < NST - 1; ++q) issue(q, q);
  if (!late) {
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
  } else {
    // ---------------------------------------------------------------- late group: rotated
    issue(3, 3);
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(3 * PPW) : "memory");  // barrier −1
    // one a1 set (as the early group): a1 of slab k+1 is read over a1 of slab k once h1(k)'s
    // MFMAs have been issued (the same register reuse as the product's step)
#ifdef ROT_A1N   // own a1 set per slab: all 12 reads of slab k+1 go out right after h0(k)
    i4v bX[4], a0X[4], bY[4], a0Y[4], a1X[4], a1Y[4];
#define ROT_SETS_XY bX, a0X, a1X, bY, a0Y, a1Y
#define ROT_SETS_YX bY, a0Y, a1Y, bX, a0X, a1X
    i4v (&a1)[4] = a1X;
#else
    i4v bX[4], a0X[4], bY[4], a0Y[4], a1[4];
#define ROT_SETS_XY bX, a0X, a1, bY, a0Y, a1
#define ROT_SETS_YX bY, a0Y, a1, bX, a0X, a1
#endif
    readb(0, bX);
    reada(0, 0, a0X);
    reada(0, 1, a1);
    vmwait_barrier<PPW>(std::integral_constant<int, 2>{});   // barrier 0: own pieces of slab 1
    // interval k (after barrier k): W ≥ 0 ends with barrier k+1 publishing slab k+2 with W slabs
    // of own pieces still in flight; NOBAR reads slab k+1 but meets no barrier; LASTB only computes
    constexpr int NOBAR = -1, LASTB = -2;
    auto ivl = [&](auto dma_c, auto w_c, int k, i4v (&b)[4], i4v (&a0)[4], i4v (&a1c)[4], i4v (&bn)[4],
                   i4v (&a0n)[4], i4v (&a1n)[4]) {
      constexpr bool dma = decltype(dma_c)::value;
      constexpr int w = decltype(w_c)::value;
      const int st1 = (k + 1) % NST;
      __builtin_amdgcn_sched_barrier(0);
      mfmas(0, a0, b);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (w != LASTB) {
        readb(st1, bn);
        reada(st1, 0, a0n);
#ifdef ROT_A1N
        reada(st1, 1, a1n);
#endif
      }
      __builtin_amdgcn_sched_barrier(0);
      mfmas(1, a1c, b);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (dma) issue(k + 4, k % NST);
#ifndef ROT_A1N
      if constexpr (w != LASTB) reada(st1, 1, a1n);
#endif
      if constexpr (w >= 0) vmwait_barrier<PPW>(w_c);
      else if constexpr (w == NOBAR) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    const int m = nsl - 4;   // FULL intervals k = 0 .. nsl − 5
    int k = 0;
    for (; k + 1 < m; k += 2) {
      ivl(T_{}, std::integral_constant<int, 2>{}, k, ROT_SETS_XY);
      ivl(T_{}, std::integral_constant<int, 2>{}, k + 1, ROT_SETS_YX);
    }
    if (k < m) {
      ivl(T_{}, std::integral_constant<int, 2>{}, k, ROT_SETS_XY);
      ++k;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        bX[u] = bY[u];
        a0X[u] = a0Y[u];
#ifdef ROT_A1N
        a1X[u] = a1Y[u];
#endif
      }
    }
    ivl(F_{}, std::integral_constant<int, 1>{}, k, ROT_SETS_XY);
    ivl(F_{}, std::integral_constant<int, 0>{}, k + 1, ROT_SETS_YX);
    ivl(F_{}, std::integral_constant<int, NOBAR>{}, k + 2, ROT_SETS_XY);
    ivl(F_{}, std::integral_constant<int, LASTB>{}, k + 3, ROT_SETS_YX);
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  // Epilogue as the product kernel
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
}
}  // namespace gp2d
