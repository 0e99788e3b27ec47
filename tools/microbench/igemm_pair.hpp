// igemm_pair.hpp — dev copy (tools/microbench only): the product's int8 GEMM
// (2d-gp_amd/csrc/ozaki.hpp igemm_nt_mod_kernel<256, 4>) with two K slabs per barrier.
#pragma once
#include "../../2d-gp_amd/csrc/ozaki.hpp"
namespace gp2d {
template <int TBN, int NST>
__global__ __launch_bounds__(TBN * 2, (TBN == 256) ? 1 : 2) void igemm_pair_kernel(
    const int8_t* __restrict__ A, const int8_t* __restrict__ B, uint8_t* __restrict__ C, int64_t ldc, int M, int N,
    int K, int a_lower, int modulus, int alias_rb, int alias_ks, const int* __restrict__ slist,
    const int* __restrict__ scnt) {
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
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
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
  const int bias = ozaki_acc_bias(K, modulus);
  i4v acc[8][4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = i4v{bias, bias, bias, bias};

  // wave w moves A rows [16·AP·w, +16·AP) and B rows [32w, 32w+32): contiguous 1 KB pieces
  const int drow = lane >> 2, dchunk = lane & 3;
  // ks: the K slab (already mapped through the list) loaded into ring stage st
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
      const int row = (wid * BPW + h) * 16 + drow;   // swizzle by the row within the 256 block
      __builtin_amdgcn_global_load_lds((const void*)(Bg + row * IBK + 16 * swz16(jr + row, dchunk)),
                                       (lds_ptr_t)(Bs + (wid * BPW + h) * 16 * IBK), 16, 0, 0);
    }
  };
  const uint32_t lds_base = (uint32_t)(size_t)(lds_ptr_t)smem;
  auto reada = [&](int st, int half, i4v (&a)[4]) {  // A fragments mi = 4·half .. 4·half+3
    const uint32_t As = lds_base + st * STG;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = wr * 128 + (4 * half + u) * 16 + l16;
      const uint32_t ad = As + row * IBK + 16 * swz16(row, lq);
      asm volatile("ds_read_b128 %0, %1" : "=v"(a[u]) : "v"(ad) : "memory");
    }
  };
  auto readb = [&](int st, i4v (&b)[4]) {
    const uint32_t Bs = lds_base + st * STG + I_OP;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int row = wc * 64 + ni * 16 + l16;
      const uint32_t ad = Bs + row * IBK + 16 * swz16(jr + row, lq);
      asm volatile("ds_read_b128 %0, %1" : "=v"(b[ni]) : "v"(ad) : "memory");
    }
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
    // Two slabs per barrier: the ring holds the pair being multiplied (s, s+1) and the next
    // pair (s+2, s+3) in flight; one vmcnt(0) + barrier per pair, in the second slab's middle.
    static_assert(NST == 4, "pair schedule: 4 stages");
    issue(slab(0), 0);
    if (nsl > 1) issue(slab(1), 1);
    int k2 = slab(2), k3 = slab(3);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    i4v bA[4], a0A[4], bB[4], a0B[4], a1[4];
    readb(0, bA);
    reada(0, 0, a0A);
    __builtin_amdgcn_sched_barrier(0);
    int s = 0;
    for (; s + 1 < nsl; s += 2) {
      const int st = s & 3, st1 = (s + 1) & 3, st2 = (s + 2) & 3;
      if (s + 2 < nsl) issue(k2, st2);   // (uniform branch; the vmcnt(0) below needs no count)
      k2 = slab(s + 4);
      // slab s (fragments in set A); slab s+1 was published by the previous pair's barrier
      reada(st, 1, a1);
      asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mfmas(0, a0A, bA);
      __builtin_amdgcn_sched_barrier(0);
      readb(st1, bB);
      reada(st1, 0, a0B);
      asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mfmas(1, a1, bA);
      __builtin_amdgcn_sched_barrier(0);
      // slab s+1 (set B); its middle publishes the next pair
      if (s + 3 < nsl) issue(k3, (s + 3) & 3);   // the stage of slab s−1: free since the last barrier
      k3 = slab(s + 5);
      reada(st1, 1, a1);
      asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mfmas(0, a0B, bB);
      __builtin_amdgcn_sched_barrier(0);
      // (past the end the reads fetch a stale stage: harmless, and no branch in the loop)
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      readb(st2, bA);
      reada(st2, 0, a0A);
      asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mfmas(1, a1, bB);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (s < nsl) {   // odd count: the last slab (fragments in set A)
      reada(s & 3, 1, a1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mfmas(0, a0A, bA);
      mfmas(1, a1, bA);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // Epilogue: residues mod m, packed 4 rows per dword into an LDS image of Cᵀ [col][row]
  // (pitch 272 B), then written out as coalesced 16-B row runs of the column-major residue
  // plane.  Six full-rate VALU operations per residue (ozaki_mod_u31; no v_mul_lo_u32, no
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
      for (int u = 0; u < 4; ++u) pk |= ozaki_mod_u31((uint32_t)acc[mi][ni][u], mc) << (8 * u);
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
