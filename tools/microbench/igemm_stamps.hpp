// igemm_stamps.hpp — DIAGNOSTIC COPY of ozaki.hpp's igemm_nt_mod_kernel<256, 4> with
// s_memtime stamps (tools/microbench only; read the SHARES, not the run time: every stamp
// drains lgkmcnt, so the build cannot overlap what the product kernel overlaps there).
// Per wave, 64-bit scalar sums of the cycles between consecutive stamps:
//   seg 0  work: after a barrier → the next step's vmcnt wait (fragment reads, h1 and h0 MFMAs, DMA issue)
//   seg 1  waiting for the wave's own LDS-DMA pieces of the next slab (s_waitcnt vmcnt)
//   seg 2  waiting at the per-slab s_barrier for the other waves
//   seg 3  the ring tail (NST − 1 steps without stamps)
//   seg 4  epilogue (mod m, LDS transpose, stores issued)
//   seg 5  prologue (launch → first fragments)
// Stamps are stored once per wave by lane 0 (vector store) into ig_stamp[block][wave][8]:
// slots 0-5 = segment sums, 6 = steady-state steps, 7 = tile start time.
#pragma once
#include "../../2d-gp_amd/csrc/ozaki.hpp"
namespace gp2d {
__device__ unsigned long long ig_stamp[2048 * 8 * 8];
__device__ __forceinline__ unsigned long long ig_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define ST_BEGIN()                                   \
  unsigned long long st_sum[6] = {0, 0, 0, 0, 0, 0}; \
  unsigned long long st_steps = 0;                   \
  const unsigned long long st_t0 = ig_now();         \
  unsigned long long st_last = st_t0
#define ST_SEG(i)                                  \
  do {                                             \
    const unsigned long long st_t = ig_now();      \
    st_sum[i] += st_t - st_last;                   \
    st_last = st_t;                                \
    if ((i) == 2) ++st_steps;                      \
  } while (0)
#define ST_END()                                                                          \
  do {                                                                                    \
    if ((threadIdx.x & 63) == 0) {                                                        \
      unsigned long long* o = ig_stamp + ((size_t)(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (threadIdx.x >> 6)) * 8; \
      for (int q = 0; q < 6; ++q) o[q] = st_sum[q];                                       \
      o[6] = st_steps;                                                                    \
      o[7] = st_t0;                                                                       \
    }                                                                                     \
  } while (0)
template <int TBN, int NST>
__global__ __launch_bounds__(TBN * 2, (TBN == 256) ? 1 : 2) void igemm_stamp_kernel(
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
  ST_BEGIN();
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
  const int bias = (int)ozaki_acc_bias(K, modulus);   // the bit pattern of an unsigned value
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
    ST_SEG(5);   // prologue (ring fill, first fragment reads drained by the stamp)
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
        ST_SEG(0);                  // work segment ends (lgkmcnt(0): a1 landed, as the barrier requires)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW * decltype(w_c)::value) : "memory");
        ST_SEG(1);                  // own DMA pieces of slab s+1 landed
        asm volatile("s_barrier" ::: "memory");
        ST_SEG(2);                  // barrier released
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
  ST_SEG(3);   // tail + last step (no stamps inside the tail's W = LAST step)
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
    const uint4 v = *reinterpret_cast<const uint4*>(T + cloc * TP + 16 * ch);
    *reinterpret_cast<uint4*>(C + (int64_t)(j0 + cloc) * ldc + i0 + 16 * ch) = v;
  }
  ST_SEG(4);   // epilogue issued
  ST_END();
}

}  // namespace gp2d
