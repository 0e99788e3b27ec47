// igemm_persist.hpp — dev copy (tools/microbench only): the persistent form of the product's
// int8 GEMM (2d-gp_amd/csrc/ozaki.hpp igemm_nt_mod_kernel<256, 4>).  Measured:
// on the random-residue microbench a tie (851k vs 855k cycles), on zero operands 14 % / 7 % /
// 1 % faster at K = 256 / 1024 / 4096 (the per-tile ring fill and launch hidden); in the bench
// 1.7 % faster unpipelined but no gain (one workgroup per CU) or a tie (two tiles per
// workgroup) with job pipelining, where the concurrent fit's kernels only find CUs when
// workgroups retire.  Kept here as a measured alternative; the product keeps the one-tile form.
#pragma once
#include "../../2d-gp_amd/csrc/ozaki.hpp"
#include <climits>
namespace gp2d {
// ------------------------------------------------------------------ INT8 NT GEMM mod m, persistent
// The same 256×256 tile, ring and fragment schedule as igemm_nt_mod_kernel<256, NST>, but one
// workgroup per CU walks a fixed sequence of tiles and its LDS-DMA ring never drains: the K
// slabs of all its tiles form one stream, so the next tile's first NST − 1 slabs are in flight
// while the current tile's last slabs are multiplied and its epilogue runs (the one-tile-per-
// workgroup form pays a ring fill and a workgroup launch per tile).
//   * Tile sequence: round k of workgroup w is tile k·G + w (k even) or k·G + G − 1 − w (k odd)
//     in the heavy-first order of the one-tile form (row blocks descending, column tiles
//     ascending), G = gridDim.x: the snake pairs long and short row blocks.
//   * LIST: K slabs from the slab lists (a tile with an empty list runs slab 0, which is all
//     zero, so every tile has ≥ 1 slab); otherwise dense.  Past the end of the stream the DMA
//     cursor sits on a dummy tile (slab 0 of A re-read into the stage being freed), so every
//     step has the same vmcnt arithmetic and the common step path has no branch but the
//     (not taken) tile switch.
//   * Epilogue in the stage that the tile's last slab occupied (free once every wave passed the
//     step's barrier; the next DMA into it is issued only after the epilogue's last barrier).
template <int NST, bool LIST>
__global__ __launch_bounds__(512, 1) void igemm_nt_mod_persist_kernel(
    const int8_t* __restrict__ A, const int8_t* __restrict__ B, uint8_t* __restrict__ C, int64_t ldc, int M, int N,
    int K, int a_lower, int modulus, int alias_rb, int alias_ks, const int* __restrict__ slist,
    const int* __restrict__ scnt) {
  static_assert(NST == 4, "ring depth (the post-epilogue wait assumes 4)");
  constexpr int WC = 4, AP = 2, BPW = 2, PPW = AP + BPW;
  constexpr int STG = 2 * I_OP;
  __shared__ __attribute__((aligned(16))) int8_t smem[NST * STG];
  const int nbj = N / IBN, nbi = M / IBM, T = nbi * nbj, G = (int)gridDim.x, w = (int)blockIdx.x;
  const int kslabs = K / IBK, cstride = kslabs / 4 + 1;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WC, wc = wid % WC;
  const int l16 = lane & 15, lq = lane >> 4;
  typedef const __attribute__((address_space(4))) int* const_int_ptr;

  auto tile_id = [&](int k) -> int {
    const int t = k * G + ((k & 1) ? G - 1 - w : w);
    return t < T ? t : -1;
  };
  auto tile_ke = [&](int t) -> int { return a_lower ? min(K, (nbi - t / nbj) * IBM) : K; };
  // slabs of tile t (≥ 1; 0 for t < 0); LIST: one scalar load
  auto tile_nsl = [&](int t) -> int {
    if (t < 0) return 0;
    const int ke = tile_ke(t);
    if (!LIST) return ke / IBK;
    const int c = scnt[(t % nbj) * cstride + ke / IBM];
    return c > 0 ? c : 1;
  };
  if (tile_id(0) < 0) return;   // more workgroups than tiles

  // ---- DMA cursor
  const int8_t* dAp;    // A slab tiles of the DMA tile's row block
  const int8_t* dBp;    // B slab tiles of its column block
  const int8_t* dBq;    // aliased B source for slabs < dalim
  const int* dsl;       // LIST: its slab list
  int dalim, dnsl, dmask, ds = 0, dks = 0, dk = 0;
  int nx_c = 0;         // LIST: the next tile's raw list count (loaded one tile ahead)
  auto dma_enter = [&](int t, int c) {   // make tile t (−1: the dummy) the DMA tile
    if (t < 0) {
      dAp = A; dBp = A; dBq = A; dsl = scnt; dalim = 0; dnsl = INT_MAX; dmask = 0;
      return;
    }
    const int bi = nbi - 1 - t / nbj, jb = t % nbj;
    dAp = A + (int64_t)bi * kslabs * I_OP;
    dBp = B + (int64_t)jb * kslabs * I_OP;
    const bool al = jb >= alias_rb;
    dBq = B + ((int64_t)(al ? jb - alias_rb : 0) * kslabs + alias_ks) * I_OP;
    dalim = al ? alias_ks : 0;
    dmask = -1;
    if (LIST) {
      dnsl = c > 0 ? c : 1;
      dsl = c > 0 ? slist + (int64_t)jb * kslabs : scnt + (int64_t)jb * cstride;   // scnt[jb][0] = 0: slab 0
    } else {
      dnsl = tile_ke(t) / IBK;
      dsl = nullptr;
    }
  };
  auto raw_count = [&](int t) -> int { return (LIST && t >= 0) ? scnt[(t % nbj) * cstride + tile_ke(t) / IBM] : 0; };
  {
    const int t0 = tile_id(0);
    dma_enter(t0, raw_count(t0));
    nx_c = raw_count(tile_id(1));
    dks = LIST ? ((const_int_ptr)dsl)[0] : 0;
  }

  const int drow = lane >> 2, dchunk = lane & 3;
  auto dma_step = [&](int st) {
    int8_t* As = smem + st * STG;
    int8_t* Bs = As + I_OP;
    const int8_t* Ag = dAp + (int64_t)dks * I_OP;
    const int8_t* Bg = (dks < dalim ? dBq : dBp) + (int64_t)dks * I_OP;
#pragma unroll
    for (int h = 0; h < AP; ++h) {
      const int row = (wid * AP + h) * 16 + drow;
      __builtin_amdgcn_global_load_lds((const void*)(Ag + row * IBK + 16 * swz16(row, dchunk)),
                                       (lds_ptr_t)(As + (wid * AP + h) * 16 * IBK), 16, 0, 0);
    }
#pragma unroll
    for (int h = 0; h < BPW; ++h) {
      const int row = (wid * BPW + h) * 16 + drow;
      __builtin_amdgcn_global_load_lds((const void*)(Bg + row * IBK + 16 * swz16(row, dchunk)),
                                       (lds_ptr_t)(Bs + (wid * BPW + h) * 16 * IBK), 16, 0, 0);
    }
    if (__builtin_expect(++ds == dnsl, 0)) {   // next tile of the sequence (or the dummy)
      ++dk;
      ds = 0;
      dma_enter(tile_id(dk), nx_c);
      nx_c = raw_count(tile_id(dk + 1));
    }
    dks = LIST ? ((const_int_ptr)dsl)[ds & dmask] : (ds & dmask);
  };

  const int bias = ozaki_acc_bias(K, modulus);
  i4v acc[8][4];
  auto reset_acc = [&]() {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = i4v{bias, bias, bias, bias};
  };
  reset_acc();

  const uint32_t lds_base = (uint32_t)(size_t)(lds_ptr_t)smem;
  auto reada = [&](int st, int half, i4v (&a)[4]) {
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
      const uint32_t ad = Bs + row * IBK + 16 * swz16(row, lq);
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

  const OzModConsts mc = ozaki_mod_consts(modulus);
  // epilogue of tile t into the free stage st, in two passes over the wave's row halves
  // (mi 0-3, then 4-7): each pass reduces and writes 16 dwords per lane into a 256-column ×
  // 128-B image of Cᵀ (16-B chunk index ^ (column & 7)), then 512 threads store it as 64-B row
  // runs.  Ends with a barrier (the stage is reused by the next step's DMA).
  auto epilogue = [&](int st, int t) {
    const int i0 = (nbi - 1 - t / nbj) * IBM, j0 = (t % nbj) * IBN;
    // lane indices re-derived behind an opaque copy: the compiler would otherwise hoist the
    // epilogue's per-lane addresses out of the K loop and spill the fragment registers
    int tl = tid;
    asm volatile("" : "+v"(tl));
    const int lane = tl & 63, wid = tl >> 6, wr = wid / WC, wc = wid % WC, l16 = lane & 15, lq = lane >> 4;
    uint8_t* Tm = reinterpret_cast<uint8_t*>(smem) + st * STG;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int m4 = 0; m4 < 4; ++m4)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          uint32_t p = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) p |= ozaki_mod_u31((uint32_t)acc[4 * pass + m4][ni][u], mc) << (8 * u);
          const int rl = wr * 64 + m4 * 16 + 4 * lq;   // row within this pass's 128
          const int cloc = wc * 64 + ni * 16 + l16;
          *reinterpret_cast<uint32_t*>(Tm + cloc * 128 + (((rl >> 4) ^ (cloc & 7)) << 4) + (rl & 15)) = p;
        }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int id = tl + 512 * q;
        const int cloc = id >> 3, ch = id & 7;
        const uint4 v = *reinterpret_cast<const uint4*>(Tm + cloc * 128 + ((ch ^ (cloc & 7)) << 4));
        const int row = (ch >> 2) * 128 + 64 * pass + (ch & 3) * 16;
        *reinterpret_cast<uint4*>(C + (int64_t)(j0 + cloc) * ldc + i0 + row) = v;
      }
      __syncthreads();
    }
  };

  // ---- prologue: NST − 1 slabs of the stream in flight, slab 0 landed
#pragma unroll
  for (int q = 0; q < NST - 1; ++q) dma_step(q);
  vmwait_barrier<PPW>(std::integral_constant<int, NST - 2>{});
  i4v bA[4], a0A[4], bB[4], a0B[4], a1[4];
  readb(0, bA);
  reada(0, 0, a0A);
  __builtin_amdgcn_sched_barrier(0);
  // one step = one slab of the stream (issues one slab or dummy, publishes slab g+1).  POST:
  // the tile's first step after an epilogue, whose 8 global stores per thread sit between the
  // older slabs and this step's pieces (vmcnt counts in issue order): they stay outstanding too.
  auto step = [&](auto post_c, int g, i4v (&b)[4], i4v (&a0)[4], i4v (&bn)[4], i4v (&a0n)[4]) {
    constexpr bool post = decltype(post_c)::value;
    const int st = g & (NST - 1);
    dma_step((g + NST - 1) & (NST - 1));
    reada(st, 1, a1);
    asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mfmas(0, a0, b);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (post)
      vmwait_barrier<PPW>(std::integral_constant<int, NST>{});
    else
      vmwait_barrier<PPW>(std::integral_constant<int, NST - 2>{});
    const int st1 = (g + 1) & (NST - 1);
    readb(st1, bn);
    reada(st1, 0, a0n);
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mfmas(1, a1, b);
    __builtin_amdgcn_sched_barrier(0);
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  int g = 0;   // stream position of the current tile's first slab
  int ck = 0, ct = tile_id(0);
  int cnsl = tile_nsl(ct);
  while (ct >= 0) {
    const int m = cnsl;
    const int ct_next = tile_id(ck + 1);
    cnsl = tile_nsl(ct_next);   // LIST: a scalar load, used after this tile's slabs
    // slab 0 (after an epilogue: the post wait), set A → B
    if (g > 0)
      step(T_{}, g, bA, a0A, bB, a0B);
    else
      step(F_{}, g, bA, a0A, bB, a0B);
    int s = 1;
    for (; s + 1 < m; s += 2) {
      step(F_{}, g + s, bB, a0B, bA, a0A);
      step(F_{}, g + s + 1, bA, a0A, bB, a0B);
    }
    if (s < m) {   // one more: B → A
      step(F_{}, g + s, bB, a0B, bA, a0A);
    } else {       // next fragments are in set B: back to A
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        bA[u] = bB[u];
        a0A[u] = a0B[u];
      }
    }
    g += m;
    // the tile's last slab's stage is free: every wave passed that step's barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    epilogue((g - 1) & (NST - 1), ct);
    reset_acc();
    ++ck;
    ct = ct_next;
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

}  // namespace gp2d
