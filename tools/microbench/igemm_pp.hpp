// DEV VARIANT (tools/microbench only; measured in round 5 and not kept — DESIGN.md §6 "int8 GEMM,
// ping-pong"; profiles/r05_igemm_pp_ab.txt, r05_ppbench_ab.txt): INT8 NT GEMM mod m with the two
// wave groups of a workgroup in ping-pong — the same product, tile, operand layout, ring and
// epilogue as igemm_nt_mod_kernel (2d-gp_amd/csrc/ozaki.hpp), a different schedule.
//
// igemm_nt_mod_kernel runs its 8 waves in lockstep — every wave issues its DMA pieces and
// fragment reads, then its MFMAs, then meets the others at the per-slab barrier — so both
// waves of a SIMD load at the same time and leave its matrix pipe idle while they do.  Here the
// wave groups G0 (waves 0-3, output rows 0-127 of the tile) and G1 (waves 4-7, rows 128-255),
// one wave of each per SIMD, alternate: between two consecutive barriers one group issues 16
// MFMAs (half of its slab) while the other issues its LDS-DMA pieces and the fragment reads of
// its next 16 — so the pipe always has a wave feeding it.  Four barriers per 64-byte K slab:
//
//   interval   G0                                     G1
//   I1         MFMA half 0 of slab s                  DMA A(s+3); read B(s), A0(s)
//   I2         DMA A(s+3); read A1(s)                 MFMA half 0 of slab s
//   I3         MFMA half 1 of slab s; vmcnt → s+1     DMA B(s+3); read A1(s); vmcnt → s+1
//   I4         DMA B(s+3); read B(s+1), A0(s+1)       MFMA half 1 of slab s
//
// RAW: slab s+1 is published by the barrier that ends I3 of slab s (every wave has waited for its
// own pieces of s+1 by then: its vmcnt leaves only slab s+2's pieces and its slab-(s+3) pieces
// of this cycle in flight); its first reads are G0's in I4.  WAR: slab s+3 goes to the stage of
// slab s−1, whose last reads (A1(s−1): G0 in I2, G1 in I3 of the previous cycle) were retired
// (lgkmcnt(0)) before that cycle's I3 barrier.  Every wave issues 4 DMA pieces per cycle; past the
// end of the list the pieces reload the last slab into the free stage (never read), so the
// counts stay those of the steady state.
#pragma once
#include "../../2d-gp_amd/csrc/ozaki.hpp"

// Schedule variants (tools/microbench/igemm_bench.hip builds them; the product uses the defaults):
//   IGPP_DMA   0: 2 DMA pieces in each read interval; 1: 1 in M1 (beside its 8 reads), 3 in M2
//   IGPP_PRIO  0: none; 1: s_setprio 1 around each MFMA cluster; 2: s_setprio 1 for G1 throughout
#ifndef IGPP_DMA
#define IGPP_DMA 0
#endif
#ifndef IGPP_PRIO
#define IGPP_PRIO 0
#endif

namespace gp2d {

__global__ __launch_bounds__(512, 1) void igemm_pp_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ B,
                                                          uint8_t* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                          int a_lower, int modulus, int alias_rb, int alias_ks,
                                                          const int* __restrict__ slist, const int* __restrict__ scnt,
                                                          const IgemmZ zb) {
  constexpr int NST = 4, TBN = 256;
  constexpr int STG = 2 * I_OP;   // stage bytes: A then B (one 64-byte slab of each)
  if (gridDim.z > 1) {
    A += blockIdx.z * zb.sA;
    B += blockIdx.z * zb.sB;
    C += blockIdx.z * zb.sC;
    modulus = zb.m[blockIdx.z];
  }
  __shared__ __attribute__((aligned(16))) int8_t smem[NST * STG];
  const int bj = blockIdx.x;
  const int bi = (int)(gridDim.y - 1 - blockIdx.y);   // heavy (long-K) row blocks first
  const int i0 = bi * IBM, j0 = bj * TBN;
  const int jb = j0 / IBN, jr = j0 % IBN;
  const int ke = a_lower ? min(K, i0 + IBM) : K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;   // wr: the wave's group (G0 / G1) and its 128 output rows
  const int l16 = lane & 15, lq = lane >> 4;
  const int64_t kslabs = K / IBK;
  const int8_t* Ap = A + (int64_t)bi * kslabs * I_OP;
  const bool alias = jb >= alias_rb;
  const int8_t* Bp = B + (int64_t)jb * kslabs * I_OP + jr * IBK;
  const int8_t* Bq = B + ((int64_t)(alias ? jb - alias_rb : 0) * kslabs + alias_ks) * I_OP + jr * IBK;
  int nsl = ke / IBK;
  const int* sl = nullptr;
  if (slist != nullptr) {
    const int c = scnt[(int64_t)jb * (kslabs / 4 + 1) + ke / IBM];
    if (c == 0 || c >= NST - 1) {   // a list shorter than the prologue's three slabs runs dense
      nsl = c;
      sl = slist + (int64_t)jb * kslabs;
    }
  }

  const int bias = (int)ozaki_acc_bias(K, modulus);
  i4v acc[8][4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = i4v{bias, bias, bias, bias};

  const int drow = lane >> 2, dchunk = lane & 3;
  // this wave's A pieces h0 .. h1−1 (rows 32·wid + 16h .. +15) of slab ks
  auto issue_a = [&](int ks, int st, int h0 = 0, int h1 = 2) {
    const int8_t* Ag = Ap + (int64_t)ks * I_OP;
    int8_t* As = smem + st * STG;
#pragma unroll
    for (int h = h0; h < h1; ++h) {
      const int row = (wid * 2 + h) * 16 + drow;
      __builtin_amdgcn_global_load_lds((const void*)(Ag + row * IBK + 16 * swz16(row, dchunk)),
                                       (lds_ptr_t)(As + (wid * 2 + h) * 16 * IBK), 16, 0, 0);
    }
  };
  auto issue_b = [&](int ks, int st) {   // this wave's 2 B pieces (rows 32·wid .. +31) of slab ks
    const int8_t* Bg = ((alias && ks < alias_ks) ? Bq : Bp) + (int64_t)ks * I_OP;
    int8_t* Bs = smem + st * STG + I_OP;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = (wid * 2 + h) * 16 + drow;
      __builtin_amdgcn_global_load_lds((const void*)(Bg + row * IBK + 16 * swz16(jr + row, dchunk)),
                                       (lds_ptr_t)(Bs + (wid * 2 + h) * 16 * IBK), 16, 0, 0);
    }
  };
  // Fragment reads: one base VGPR per read group (stage + the lane's row and swizzled chunk) and
  // the fragment in the instruction's offset field.  The swizzle depends on (row >> 2) & 3 =
  // (l16 >> 2) & 3 only (fragment rows are 16-aligned, B tiles start at j0 % 256 = 0), so every
  // fragment of a lane shares it — without this the compiler keeps an address VGPR per fragment
  // and stage and spills.
  const uint32_t lds_base = (uint32_t)(size_t)(lds_ptr_t)smem;
  const uint32_t lane_a = (uint32_t)((wr * 128 + l16) * IBK + 16 * swz16(l16, lq));
  const uint32_t lane_b = (uint32_t)(I_OP + (wc * 64 + l16) * IBK + 16 * swz16(jr + l16, lq));
  auto reada = [&](int st, int half, i4v (&a)[4]) {
    const uint32_t ad = lds_base + (uint32_t)(st * STG) + lane_a;
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
    const uint32_t ad = lds_base + (uint32_t)(st * STG) + lane_b;
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
  typedef const __attribute__((address_space(4))) int* const_int_ptr;
  // slab s of the K loop (past the end: the last one again — the tail's pieces land in a free stage)
  auto slab = [&](int s) -> int {
    const int q = min(s, nsl - 1);
    return sl ? ((const_int_ptr)sl)[q] : q;
  };
#define PP_BAR() asm volatile("s_barrier" ::: "memory")
#define PP_SB() __builtin_amdgcn_sched_barrier(0)

  if (nsl > 0) {
    issue_a(slab(0), 0);
    issue_b(slab(0), 0);
    issue_a(slab(1), 1);
    issue_b(slab(1), 1);
    issue_a(slab(2), 2);
    issue_b(slab(2), 2);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // slab 0 landed (this wave's pieces)
    PP_BAR();                                           // ... and everyone's: published
    // G1 runs the same body one interval behind G0: its first barrier pairs with the end of
    // G0's first read interval, and G0 makes up the count after the loop
    if (wr == 1) PP_BAR();
    if (IGPP_PRIO == 2 && wr == 1) __builtin_amdgcn_s_setprio(1);
    PP_SB();
    i4v a0[4], a1[4], bE[4], bO[4];
    auto cycle = [&](int s, i4v (&b)[4]) {
      const int k3 = slab(s + 3), st3 = (s + 3) % NST, st = s % NST;
      // M1: DMA A(s+3); read B(s), A0(s)
      if (IGPP_DMA == 0) issue_a(k3, st3);
      else issue_a(k3, st3, 0, 1);
      readb(st, b);
      reada(st, 0, a0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      PP_SB();
      PP_BAR();
      PP_SB();
      // C0
      if (IGPP_PRIO == 1) __builtin_amdgcn_s_setprio(1);
      mfmas(0, a0, b);
      if (IGPP_PRIO == 1) __builtin_amdgcn_s_setprio(0);
      PP_SB();
      PP_BAR();
      PP_SB();
      // M2: DMA B(s+3); read A1(s); this wave's pieces of slab s+1 landed (s+2's and s+3's 8 younger)
      if (IGPP_DMA != 0) issue_a(k3, st3, 1, 2);
      issue_b(k3, st3);
      reada(st, 1, a1);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_waitcnt vmcnt(8)" ::: "memory");
      PP_SB();
      PP_BAR();
      PP_SB();
      // C1
      if (IGPP_PRIO == 1) __builtin_amdgcn_s_setprio(1);
      mfmas(1, a1, b);
      if (IGPP_PRIO == 1) __builtin_amdgcn_s_setprio(0);
      PP_SB();
      PP_BAR();
      PP_SB();
    };
    int s = 0;
    for (; s + 2 <= nsl; s += 2) {   // B fragments alternate between two register sets: a cycle's
      cycle(s, bE);                  // reads never overwrite the set its predecessor's MFMAs use
      cycle(s + 1, bO);
    }
    if (s < nsl) cycle(s, bE);
    if (wr == 0) PP_BAR();
    // the tail's pieces land before the ring becomes the epilogue's image
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
#undef PP_BAR
#undef PP_SB
  // Epilogue: as igemm_nt_mod_kernel — residues mod m packed 4 rows per dword into an LDS image
  // of Cᵀ, then coalesced 16-byte row runs of the column-major residue plane
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
}

}  // namespace gp2d
