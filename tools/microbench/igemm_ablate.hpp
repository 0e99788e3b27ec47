// igemm_ablate.hpp — DEV COPY of ozaki.hpp's igemm_nt_mod_kernel with ablation switches
// (tools/microbench only; the product kernel carries none):
//   -DGP2D_IGEMM_NO_DMA       no global→LDS DMA (MFMAs on stale LDS)
//   -DGP2D_IGEMM_NO_BARRIER   (with NO_DMA) no vmcnt wait / barrier per slab
//   -DGP2D_IGEMM_NO_LDSREAD   no fragment reads (MFMAs on constant registers)
//   -DGP2D_IGEMM_NO_MFMA      no MFMAs (one xor per step keeps the loads live)
//   -DGP2D_IGEMM_EPI_ONLY     no K loop at all (prologue-free: epilogue and stores only)
// Keep it in step with the product kernel when that changes (igemm_bench.hip checks both).
#pragma once
#include "../../2d-gp_amd/csrc/ozaki.hpp"
namespace gp2d {
// s_waitcnt vmcnt(4·W) + lgkmcnt(0) + s_barrier: this wave's LDS-DMA pieces of all but the
// W youngest slabs (4 pieces per slab per wave) have landed, then the workgroup syncs.
template <int W>
__device__ __forceinline__ void ab_vmwait_barrier(std::integral_constant<int, W>) {
#if defined(GP2D_IGEMM_NO_DMA) && defined(GP2D_IGEMM_NO_BARRIER)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
  if constexpr (W == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (W == 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (W == 2) asm volatile("s_waitcnt vmcnt(8)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (W == 3) asm volatile("s_waitcnt vmcnt(12)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#endif
}


// A: M×K plane, B: N×K plane (both slab-blocked); C: column-major N×M bytes (ldc ≥ M).
// B tiles (row block rb ≥ alias_rb, k slab s < alias_ks) are read from (rb − alias_rb,
// s + alias_ks): the K* planes store the (v,u) block only as its equal (u,v) block.
// alias_rb = INT_MAX disables the aliasing.
// slist / scnt (optional, ozaki_slab_list_kernel): the K loop of B tile bj runs over the listed
// slabs only — the others have an all-zero K* tile and add exactly nothing.  A tile whose list
// is shorter than the ring's prologue (1 or 2 slabs) runs dense.
__global__ __launch_bounds__(512, 1) void igemm_ablate_kernel(const int8_t* __restrict__ A,
                                                              const int8_t* __restrict__ B,
                                                              uint8_t* __restrict__ C, int64_t ldc, int M, int N,
                                                              int K, int a_lower, int modulus, double inv_mod,
                                                              int alias_rb, int alias_ks,
                                                              const int* __restrict__ slist,
                                                              const int* __restrict__ scnt) {
  __shared__ __attribute__((aligned(16))) int8_t smem[I_NSTAGE * I_STAGE];
  const int bj = blockIdx.x;
  const int bi = (int)(gridDim.y - 1 - blockIdx.y);   // heavy (long-K) row blocks first
  const int i0 = bi * IBM, j0 = bj * IBN;
  const int ke = a_lower ? min(K, i0 + IBM) : K;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int l16 = lane & 15, lq = lane >> 4;
  const int64_t kslabs = K / IBK;
  const int8_t* Ap = A + (int64_t)bi * kslabs * I_OP;   // this row block's slab tiles
  const bool alias = bj >= alias_rb;
  const int8_t* Bp = B + (int64_t)bj * kslabs * I_OP;
  const int8_t* Bq = B + ((int64_t)(alias ? bj - alias_rb : 0) * kslabs + alias_ks) * I_OP;
#ifdef GP2D_IGEMM_EPI_ONLY
  int nsl = 0;
#else
  int nsl = ke / IBK;
#endif
  const int* sl = nullptr;   // slab list of this B tile (nullptr: dense K loop)
  if (slist != nullptr) {
    const int c = scnt[(int64_t)bj * (kslabs / 4 + 1) + ke / IBM];
    if (c == 0 || c >= I_NSTAGE - 1) {
      nsl = c;
      sl = slist + (int64_t)bj * kslabs;
    }
  }

  i4v acc[8][4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = i4v{0, 0, 0, 0};

  // wave w moves rows [32w, 32w+32) of both operands: 2 contiguous 1 KB pieces each
  const int drow = lane >> 2, dchunk = lane & 3;
  // ks: the K slab (already mapped through the list) loaded into ring stage st
  auto issue = [&](int ks, int st) {
#ifdef GP2D_IGEMM_NO_DMA
    return;
#endif
    int8_t* As = smem + st * I_STAGE;
    int8_t* Bs = As + I_OP;
    const int8_t* Ag = Ap + (int64_t)ks * I_OP;
    const int8_t* Bg = ((alias && ks < alias_ks) ? Bq : Bp) + (int64_t)ks * I_OP;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = wid * 32 + h * 16 + drow;
      const int off = row * IBK + 16 * swz16(row, dchunk);
      __builtin_amdgcn_global_load_lds((const void*)(Ag + off), (lds_ptr_t)(As + (wid * 32 + h * 16) * IBK), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(Bg + off), (lds_ptr_t)(Bs + (wid * 32 + h * 16) * IBK), 16, 0, 0);
    }
  };
  const uint32_t lds_base = (uint32_t)(size_t)(lds_ptr_t)smem;
  auto reada = [&](int st, int half, i4v (&a)[4]) {  // A fragments mi = 4·half .. 4·half+3
#ifdef GP2D_IGEMM_NO_LDSREAD
    return;
#endif
    const uint32_t As = lds_base + st * I_STAGE;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = wr * 128 + (4 * half + u) * 16 + l16;
      const uint32_t ad = As + row * IBK + 16 * swz16(row, lq);
      asm volatile("ds_read_b128 %0, %1" : "=v"(a[u]) : "v"(ad) : "memory");
    }
  };
  auto readb = [&](int st, i4v (&b)[4]) {
#ifdef GP2D_IGEMM_NO_LDSREAD
    return;
#endif
    const uint32_t Bs = lds_base + st * I_STAGE + I_OP;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int row = wc * 64 + ni * 16 + l16;
      const uint32_t ad = Bs + row * IBK + 16 * swz16(row, lq);
      asm volatile("ds_read_b128 %0, %1" : "=v"(b[ni]) : "v"(ad) : "memory");
    }
  };
  auto mfmas = [&](int half, const i4v (&a)[4], const i4v (&b)[4]) {
#ifdef GP2D_IGEMM_NO_MFMA
    acc[0][0][0] += a[0][0] ^ b[0][0];
    return;
#endif
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
    for (int q = 0; q < I_NSTAGE - 1; ++q) issue(slab(q), q);
    int knext = slab(I_NSTAGE - 1);
    ab_vmwait_barrier(std::integral_constant<int, I_NSTAGE - 2>{});   // slab 0 landed (nsl ≥ 4 ≥ I_NSTAGE − 1)
    // Per slab: MFMA half 0 (A rows 0-63 of the wave) → barrier publishing slab s+1 → reads
    // of slab s+1's B and A-half-0 fragments into the other register set → MFMA half 1.
    // Both waves of a SIMD leave the barrier together, so the next slab's first fragments
    // must already be in flight behind half 1's 16 MFMAs rather than be read after it.
    i4v bA[4], a0A[4], bB[4], a0B[4], a1[4];
#ifdef GP2D_IGEMM_NO_LDSREAD
#pragma unroll
    for (int u = 0; u < 4; ++u) bA[u] = a0A[u] = bB[u] = a0B[u] = a1[u] = i4v{lane, u, wid, 1};
#endif
    readb(0, bA);
    reada(0, 0, a0A);
    __builtin_amdgcn_sched_barrier(0);
    // Step kinds: FULL steps issue slab s + I_NSTAGE − 1 and publish s+1 leaving the younger
    // I_NSTAGE − 2 slabs in flight; the tail steps issue nothing and leave W = I_NSTAGE−3 .. 0
    // slabs in flight; the LAST step has no barrier.  The steady-state loop runs only FULL
    // steps, unrolled by two for the register ping-pong, so it carries no per-slab branches.
    constexpr int LAST = -1;
    auto step = [&](auto dma_c, auto w_c, int s, i4v (&b)[4], i4v (&a0)[4], i4v (&bn)[4], i4v (&a0n)[4]) {
      constexpr bool dma = decltype(dma_c)::value;
      constexpr int w = decltype(w_c)::value;
      const int st = s % I_NSTAGE;
      // the stage written is slab s−1's: nobody reads it after the previous barrier
      if constexpr (dma) {
        issue(knext, (s + I_NSTAGE - 1) % I_NSTAGE);
        knext = slab(s + I_NSTAGE);
      }
      reada(st, 1, a1);
      asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");  // b, a0 landed
      __builtin_amdgcn_sched_barrier(0);
      mfmas(0, a0, b);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (w != LAST) {
        ab_vmwait_barrier(w_c);   // publish slab s+1 (lgkmcnt(0) inside: a1 landed)
        const int st1 = (s + 1) % I_NSTAGE;
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
    using W_FULL = std::integral_constant<int, I_NSTAGE - 2>;
    const int m = nsl - (I_NSTAGE - 1);   // FULL steps
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
    // tail: I_NSTAGE − 1 steps, W = I_NSTAGE−3, ..., 0, then LAST
    if constexpr (I_NSTAGE == 5) {
      step(F_{}, std::integral_constant<int, 2>{}, s, bA, a0A, bB, a0B);
      step(F_{}, std::integral_constant<int, 1>{}, s + 1, bB, a0B, bA, a0A);
      step(F_{}, std::integral_constant<int, 0>{}, s + 2, bA, a0A, bB, a0B);
      step(F_{}, std::integral_constant<int, LAST>{}, s + 3, bB, a0B, bA, a0A);
    } else {
      step(F_{}, std::integral_constant<int, 1>{}, s, bA, a0A, bB, a0B);
      step(F_{}, std::integral_constant<int, 0>{}, s + 1, bB, a0B, bA, a0A);
      step(F_{}, std::integral_constant<int, LAST>{}, s + 2, bA, a0A, bB, a0B);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // Epilogue: residues mod m, packed 4 rows per dword into an LDS image of Cᵀ [col][row]
  // (pitch 272 B), then written out as coalesced 16-B row runs of the column-major residue
  // plane.  Full-rate VALU only (no v_mul_lo_u32): v = vh·2^16 + vl with vl ∈ [0, 2^16), so
  // v ≡ y = vh·(2^16 mod m) + vl with |y| < 2^23 + 2^16 (|vh| < 2^15 for any int32 v): y is
  // exact in fp32 and both products fit the 24-bit multiplier; q = ⌊y/m⌋ from the fp32
  // quotient is off by at most one, so r = y − q·m ∈ [−m, 2m) and two unsigned-min steps
  // (r < 0 → r + m, then r ≥ m → r − m) finish the reduction.
  uint8_t* T = reinterpret_cast<uint8_t*>(smem);
  constexpr int TP = IBM + 16;
  const float fim = (float)inv_mod;
  const int c16 = 65536 % modulus;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      uint32_t pk = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int v = acc[mi][ni][u];
        int y, q, r;
        asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(y) : "v"(v >> 16), "s"(c16), "v"(v & 0xffff));
        asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(q) : "v"((float)y * fim));
        asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(q), "s"(-modulus), "v"(y));
        const uint32_t r0 = (uint32_t)r;
        const uint32_t r1 = min(r0, r0 + (uint32_t)modulus);
        const uint32_t res = min(r1, r1 - (uint32_t)modulus);
        pk |= res << (8 * u);
      }
      const int rloc = wr * 128 + mi * 16 + 4 * lq;
      const int cloc = wc * 64 + ni * 16 + l16;
      *reinterpret_cast<uint32_t*>(T + cloc * TP + rloc) = pk;
    }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < (IBM * IBN / 16) / 512; ++p) {
    const int id = tid + 512 * p;
    const int cloc = id >> 4, ch = id & 15;
    const uint4 v = *reinterpret_cast<const uint4*>(T + cloc * TP + 16 * ch);
    *reinterpret_cast<uint4*>(C + (int64_t)(j0 + cloc) * ldc + i0 + 16 * ch) = v;
  }
}

}  // namespace gp2d
