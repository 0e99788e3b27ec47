// igemm_lcnt.hpp — DEV VARIANT of ozaki.hpp's igemm_nt_mod_kernel<256, 4> (tools/microbench only)
// with the per-slab s_barrier replaced by LDS counters, so the 8 waves are coupled only by their
// data dependencies instead of meeting at every slab (the stamps put ≈ 180 cycles
// per slab at the barrier while a SIMD's older wave waits for its partner, and the two waves'
// non-MFMA phases line up because the barrier releases them together).
//
// Per ring stage st two monotonic LDS counters: landed[st] (one add per wave once its own
// LDS-DMA pieces of the stage's slab have arrived — its vmcnt wait) and freed[st] (one add per
// wave once its last fragment reads of the slab have returned — its lgkmcnt wait).  Slab s is the
// (s / NST + 1)-th use of stage s % NST, so both reach NW · (s / NST + 1) when every wave is done.
//   RAW: a wave reads slab s+1 only after landed[(s+1) % NST] reached its target; each wave adds
//        to landed at the TOP of step s (its pieces of slab s+1 were issued two steps earlier), so
//        a wave waits for the others' step tops, not for the end of their MFMAs.
//   WAR: a wave issues slab s+NST−1 into the stage of slab s−1 only after freed[(s−1) % NST]
//        reached its target.
// Visibility: the adding wave's vmcnt wait retires its DMA writes into LDS before its ds_add is
// issued; a reader issues its fragment ds_reads only after its counter read returned the add, so
// the LDS array has executed the writes before the reads (one LDS per CU, in-order execution).
// Every spin is bounded; an exhausted spin sets ig_lcnt_err (the bench then reports wrong tiles)
// instead of hanging the workgroup.
#pragma once
#include "../../2d-gp_amd/csrc/ozaki.hpp"
namespace gp2d {
__device__ int ig_lcnt_err;

__device__ __forceinline__ void lcnt_add(uint32_t addr, int lane) {
  if (lane == 0) asm volatile("ds_add_u32 %0, %1" ::"v"(addr), "v"(1u) : "memory");
}
// wait until the counter at addr reaches target (drains lgkmcnt: call with no counted reads in
// flight); after one exhausted spin the wave stops waiting altogether (dead = true), so a protocol
// error costs one bounded spin per wave, not one per slab
__device__ __forceinline__ void lcnt_wait(uint32_t addr, uint32_t target, bool& dead) {
  if (dead) return;
  for (int it = 0; it < (1 << 20); ++it) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    if (__builtin_amdgcn_readfirstlane(v) >= target) return;
  }
  dead = true;
  ig_lcnt_err = 1;
}

template <int NST>
__global__ __launch_bounds__(512, 1) void igemm_lcnt_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ B,
                                                           uint8_t* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                           int a_lower, int modulus, int alias_rb, int alias_ks,
                                                           const int* __restrict__, const int* __restrict__) {
  constexpr int TBN = 256, NW = 8, WC = 4, AP = 2, BPW = 2, PPW = AP + BPW;
  constexpr int STG = I_OP + TBN * IBK;
  __shared__ __attribute__((aligned(16))) int8_t smem[NST * STG + 64];
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
  const int nsl = ke / IBK;   // dense K loop, ≥ NST − 1 (K ≥ 256)
  const int bias = (int)ozaki_acc_bias(K, modulus);
  i4v acc[8][4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = i4v{bias, bias, bias, bias};
  const uint32_t lds_base = (uint32_t)(size_t)(lds_ptr_t)smem;
  const uint32_t landed = lds_base + NST * STG, freed = landed + 4 * NST;
  if (tid < 2 * NST) reinterpret_cast<uint32_t*>(smem + NST * STG)[tid] = 0u;
  __syncthreads();
  bool dead = false;

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
  auto target = [](int s) { return (uint32_t)(NW * (s / NST + 1)); };

#pragma unroll
  for (int q = 0; q < NST - 1; ++q) issue(q, q);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW * (NST - 2)) : "memory");   // own pieces of slab 0
  lcnt_add(landed + 4 * 0, lane);
  lcnt_wait(landed + 4 * 0, target(0), dead);
  i4v b[4], a0[4], a1[4];
  readb(0, b);
  reada(0, 0, a0);
  for (int s = 0; s < nsl; ++s) {
    const int st = s % NST;
    // own pieces of slab s+1 (issued two steps ago): signal them now, at the step top
    if (s + 1 < nsl) {
      if (s + 2 < nsl) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lcnt_add(landed + 4 * ((s + 1) % NST), lane);
    }
    if (s + NST - 1 < nsl) {   // slab s+NST−1 into slab s−1's stage once every wave has left it
      if (s >= 1) lcnt_wait(freed + 4 * ((s - 1) % NST), target(s - 1), dead);
      issue(s + NST - 1, (s + NST - 1) % NST);
    }
    reada(st, 1, a1);
    asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");   // b, a0 of slab s landed
    __builtin_amdgcn_sched_barrier(0);
    mfmas(0, a0, b);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // a1 landed: this wave has left slab s
    lcnt_add(freed + 4 * st, lane);
    i4v bn[4], a0n[4];
    if (s + 1 < nsl) {
      lcnt_wait(landed + 4 * ((s + 1) % NST), target(s + 1), dead);
      readb((s + 1) % NST, bn);
      reada((s + 1) % NST, 0, a0n);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfmas(1, a1, b);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      b[u] = bn[u];
      a0[u] = a0n[u];
    }
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
