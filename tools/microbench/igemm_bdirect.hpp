// igemm_bdirect.hpp — DEV EXPERIMENT: the int8 NT GEMM of ozaki.hpp with the B operand (the
// K* residue planes) read straight from global memory into MFMA fragment registers instead of
// LDS-DMA + ds_read: a wave's B fragment for one 16-row group is one contiguous 1 KB run of the
// slab-blocked plane (lane l: row l&15, 16-byte chunk l>>4), so each is a single
// global_load_dwordx4.  Only A goes through the LDS ring (16 KB stages).  Per slab a wave
// issues its B loads for the NEXT slab first, then its A DMA pieces; the next slab's B lands
// during this slab's MFMAs (vmcnt(PA) at the end of the step leaves only the A pieces just
// issued in flight).
#pragma once
#include "../../2d-gp_amd/csrc/ozaki.hpp"
namespace gp2d {

template <int NST>
__global__ __launch_bounds__(512, 1) void igemm_bdirect_kernel(
    const int8_t* __restrict__ A, const int8_t* __restrict__ B, uint8_t* __restrict__ C, int64_t ldc, int M, int N,
    int K, int a_lower, int modulus, double inv_mod, int alias_rb, int alias_ks, const int* __restrict__ slist,
    const int* __restrict__ scnt) {
  constexpr int TBN = 256;
  constexpr int STG = I_OP;               // A only
  constexpr int PA = 2;                   // A DMA pieces per wave per slab
  __shared__ __attribute__((aligned(16))) int8_t smem[NST * STG > 256 * (IBM + 16) ? NST * STG : 256 * (IBM + 16)];
  const int bj = blockIdx.x;
  const int bi = (int)(gridDim.y - 1 - blockIdx.y);
  const int i0 = bi * IBM, j0 = bj * TBN;
  const int ke = a_lower ? min(K, i0 + IBM) : K;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int l16 = lane & 15, lq = lane >> 4;
  const int64_t kslabs = K / IBK;
  const int8_t* Ap = A + (int64_t)bi * kslabs * I_OP;
  const bool alias = bj >= alias_rb;
  const int8_t* Bp = B + (int64_t)bj * kslabs * I_OP;
  const int8_t* Bq = B + ((int64_t)(alias ? bj - alias_rb : 0) * kslabs + alias_ks) * I_OP;
  int nsl = ke / IBK;
  const int* sl = nullptr;
  if (slist != nullptr) {
    const int c = scnt[(int64_t)bj * (kslabs / 4 + 1) + ke / IBM];
    if (c == 0 || c >= NST - 1) {
      nsl = c;
      sl = slist + (int64_t)bj * kslabs;
    }
  }
  i4v acc[8][4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = i4v{0, 0, 0, 0};
  const int drow = lane >> 2, dchunk = lane & 3;
  auto issue_a = [&](int ks, int st) {
    int8_t* As = smem + st * STG;
    const int8_t* Ag = Ap + (int64_t)ks * I_OP;
#pragma unroll
    for (int h = 0; h < PA; ++h) {
      const int row = wid * 32 + h * 16 + drow;
      __builtin_amdgcn_global_load_lds((const void*)(Ag + row * IBK + 16 * swz16(row, dchunk)),
                                       (lds_ptr_t)(As + (wid * 32 + h * 16) * IBK), 16, 0, 0);
    }
  };
  // this lane's byte offset inside a B slab tile for fragment ni: row wc·64 + ni·16 + l16, chunk lq.
  // Buffer loads (descriptor in SGPRs, 32-bit lane offset) keep the address out of VGPRs: the
  // B plane of one modulus is < 2^31 bytes.
  const int boff = (wc * 64 + l16) * IBK + 16 * lq;
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc((void*)B, 0, 0x7fffffff, 0x00020000);
  const int bp_off = (int)(Bp - B), bq_off = (int)(Bq - B);
  auto load_b = [&](int ks, i4v (&b)[4]) {
    const int sbase = ((alias && ks < alias_ks) ? bq_off : bp_off) + ks * I_OP;   // wave-uniform
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
      b[ni] = __builtin_bit_cast(i4v, __builtin_amdgcn_raw_buffer_load_b128(brs, boff + ni * 16 * IBK, sbase, 0));
  };
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
  auto mfmas = [&](int half, const i4v (&a)[4], const i4v (&b)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        acc[4 * half + u][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u], b[ni], acc[4 * half + u][ni], 0, 0, 0);
  };
  typedef const __attribute__((address_space(4))) int* const_int_ptr;
  auto slab = [&](int s) -> int { return sl ? ((const_int_ptr)sl)[min(s, nsl - 1)] : s; };
  if (nsl > 0) {
    i4v bA[4], bB[4], a0A[4], a0B[4], a1[4];
    load_b(slab(0), bA);
#pragma unroll
    for (int q = 0; q < NST - 1; ++q) issue_a(slab(q), q);
    int kan = slab(NST - 1), kbn = slab(1);
    // slab 0's A (PA·(NST−1) pieces issued after B(0)... all must land) and B(0)
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(PA * (NST - 2)) : "memory");
    reada(0, 0, a0A);
    __builtin_amdgcn_sched_barrier(0);
    constexpr int LAST = -1;
    // step s: B(s+1) loads, then A(s+NST−1) DMA; A half 1 of s; MFMA half 0; barrier publishing
    // A(s+1) (vmcnt leaves B(s+1) and this step's A pieces in flight); A half 0 of s+1; MFMA
    // half 1; then vmcnt leaves only this step's A pieces: B(s+1) is in registers for step s+1
    auto step = [&](auto dma_c, auto nb_c, int s, i4v (&b)[4], i4v (&a0)[4], i4v (&bn)[4], i4v (&a0n)[4]) {
      constexpr bool dma = decltype(dma_c)::value;
      constexpr bool nextb = decltype(nb_c)::value;
      const int st = s % NST;
      if constexpr (nextb) {
        load_b(kbn, bn);
        kbn = slab(s + 2);
      }
      if constexpr (dma) {
        issue_a(kan, (s + NST - 1) % NST);
        kan = slab(s + NST);
      }
      reada(st, 1, a1);
      asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");   // a0 landed
      __builtin_amdgcn_sched_barrier(0);
      mfmas(0, a0, b);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (nextb) {
        if constexpr (dma) asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(4 + PA) : "memory");
        else asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        reada((s + 1) % NST, 0, a0n);
        asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      mfmas(1, a1, b);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (nextb) {
        if constexpr (dma) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PA) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    const int m = nsl - (NST - 1);   // steps that still issue an A slab
    int s = 0;
    for (; s + 1 < m; s += 2) {
      step(T_{}, T_{}, s, bA, a0A, bB, a0B);
      step(T_{}, T_{}, s + 1, bB, a0B, bA, a0A);
    }
    if (s < m) {
      step(T_{}, T_{}, s, bA, a0A, bB, a0B);
      ++s;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        bA[u] = bB[u];
        a0A[u] = a0B[u];
      }
    }
    // tail: exactly NST − 1 slabs left (s .. s+NST−2), written out like ozaki.hpp's kernel
    if constexpr (NST == 5) {
      step(F_{}, T_{}, s, bA, a0A, bB, a0B);
      step(F_{}, T_{}, s + 1, bB, a0B, bA, a0A);
      step(F_{}, T_{}, s + 2, bA, a0A, bB, a0B);
      step(F_{}, F_{}, s + 3, bB, a0B, bA, a0A);
    } else if constexpr (NST == 4) {
      step(F_{}, T_{}, s, bA, a0A, bB, a0B);
      step(F_{}, T_{}, s + 1, bB, a0B, bA, a0A);
      step(F_{}, F_{}, s + 2, bA, a0A, bB, a0B);
    } else {
      step(F_{}, T_{}, s, bA, a0A, bB, a0B);
      step(F_{}, F_{}, s + 1, bB, a0B, bA, a0A);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
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
        pk |= min(r1, r1 - (uint32_t)modulus) << (8 * u);
      }
      *reinterpret_cast<uint32_t*>(T + (wc * 64 + ni * 16 + l16) * TP + wr * 128 + mi * 16 + 4 * lq) = pk;
    }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < (IBM * TBN / 16) / 512; ++p) {
    const int id = tid + 512 * p;
    const int cloc = id >> 4, ch = id & 15;
    const uint4 v = *reinterpret_cast<const uint4*>(T + cloc * TP + 16 * ch);
    *reinterpret_cast<uint4*>(C + (int64_t)(j0 + cloc) * ldc + i0 + 16 * ch) = v;
  }
}


// Variant 2: B two slabs ahead in three register sets, A fragments in two sets (half 1 of a
// slab is read into the registers half 0 just used).  Every step issues the same VMEM ops —
// B(s+2) (4 loads) then A(s+NST−1) (PA DMA pieces) — with clamped dummies past the end (and
// in the prologue's virtual steps), so every wait count is a constant:
//   mid-step (A(s+1) published): vmcnt((NST−2)·(4+PA));  end of step (B(s+1) landed): vmcnt(4+2·PA).
template <int NST>
__global__ __launch_bounds__(512, 1) void igemm_bdirect2_kernel(
    const int8_t* __restrict__ A, const int8_t* __restrict__ B, uint8_t* __restrict__ C, int64_t ldc, int M, int N,
    int K, int a_lower, int modulus, double inv_mod, int alias_rb, int alias_ks, const int* __restrict__ slist,
    const int* __restrict__ scnt) {
  constexpr int TBN = 256;
  constexpr int STG = I_OP;
  constexpr int PA = 2;
  constexpr int OPS = 4 + PA;
  __shared__ __attribute__((aligned(16))) int8_t smem[NST * STG > 256 * (IBM + 16) ? NST * STG : 256 * (IBM + 16)];
  const int bj = blockIdx.x;
  const int bi = (int)(gridDim.y - 1 - blockIdx.y);
  const int i0 = bi * IBM, j0 = bj * TBN;
  const int ke = a_lower ? min(K, i0 + IBM) : K;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int l16 = lane & 15, lq = lane >> 4;
  const int64_t kslabs = K / IBK;
  const int8_t* Ap = A + (int64_t)bi * kslabs * I_OP;
  const bool alias = bj >= alias_rb;
  int nsl = ke / IBK;
  const int* sl = nullptr;
  if (slist != nullptr) {
    const int c = scnt[(int64_t)bj * (kslabs / 4 + 1) + ke / IBM];
    if (c == 0 || c >= NST - 1) {
      nsl = c;
      sl = slist + (int64_t)bj * kslabs;
    }
  }
  i4v acc[8][4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = i4v{0, 0, 0, 0};
  const int drow = lane >> 2, dchunk = lane & 3;
  typedef const __attribute__((address_space(4))) int* const_int_ptr;
  auto slab = [&](int s) -> int { return sl ? ((const_int_ptr)sl)[max(0, min(s, nsl - 1))] : max(0, min(s, nsl - 1)); };
  auto issue_a = [&](int ks, int st) {
    int8_t* As = smem + st * STG;
    const int8_t* Ag = Ap + (int64_t)ks * I_OP;
#pragma unroll
    for (int h = 0; h < PA; ++h) {
      const int row = wid * 32 + h * 16 + drow;
      __builtin_amdgcn_global_load_lds((const void*)(Ag + row * IBK + 16 * swz16(row, dchunk)),
                                       (lds_ptr_t)(As + (wid * 32 + h * 16) * IBK), 16, 0, 0);
    }
  };
  const int boff = (wc * 64 + l16) * IBK + 16 * lq;
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc((void*)B, 0, 0x7fffffff, 0x00020000);
  const int bp_off = (int)((int64_t)bj * kslabs * I_OP);
  const int bq_off = (int)(((int64_t)(alias ? bj - alias_rb : 0) * kslabs + alias_ks) * I_OP);
  auto load_b = [&](int ks, i4v (&b)[4]) {
    const int sbase = ((alias && ks < alias_ks) ? bq_off : bp_off) + ks * I_OP;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
      b[ni] = __builtin_bit_cast(i4v, __builtin_amdgcn_raw_buffer_load_b128(brs, boff + ni * 16 * IBK, sbase, 0));
  };
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
  auto mfmas = [&](int half, const i4v (&a)[4], const i4v (&b)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        acc[4 * half + u][ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u], b[ni], acc[4 * half + u][ni], 0, 0, 0);
  };
  if (nsl > 0) {
    i4v b0[4], b1[4], b2[4], ac[4], an[4];
    // prologue = virtual steps t = −(NST−1) .. −1: B(t+2) (a clamped dummy below 0) into set
    // (t+2) mod 3, then A(t+NST−1) into its stage
#pragma unroll
    for (int t = -(NST - 1); t < 0; ++t) {
      const int sb = t + 2;
      const int set = ((sb % 3) + 3) % 3;
      if (set == 0) load_b(slab(sb), b0);
      else if (set == 1) load_b(slab(sb), b1);
      else load_b(slab(sb), b2);
      issue_a(slab(t + NST - 1), (t + NST - 1) % NST);
    }
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(4 + 2 * PA) : "memory");  // B(0), A(0)
    reada(0, 0, ac);
    auto step = [&](int s, i4v (&bc)[4], i4v (&b2n)[4]) {
      const int st = s % NST;
      load_b(slab(s + 2), b2n);                          // B(s+2) (a dummy past the end)
      issue_a(slab(s + NST - 1), (s + NST - 1) % NST);   // A(s+NST−1) (ditto)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // ac (half 0 of slab s) landed
      __builtin_amdgcn_sched_barrier(0);
      mfmas(0, ac, bc);
      __builtin_amdgcn_sched_barrier(0);
      reada(st, 1, ac);                                  // half 1 of slab s into the same registers
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"((NST - 2) * OPS) : "memory");
      reada((s + 1) % NST, 0, an);                       // half 0 of slab s+1
      __builtin_amdgcn_sched_barrier(0);
      mfmas(1, ac, bc);
      __builtin_amdgcn_sched_barrier(0);
      // B(s+1) landed; `an` (read by inline asm, so invisible to the compiler's waits) landed
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"(4 + 2 * PA) : "memory");
#pragma unroll
      for (int u = 0; u < 4; ++u) ac[u] = an[u];
    };
    int s = 0;
    for (; s + 2 < nsl; s += 3) {
      step(s, b0, b2);
      step(s + 1, b1, b0);
      step(s + 2, b2, b1);
    }
    if (s < nsl) step(s, b0, b2);
    if (s + 1 < nsl) step(s + 1, b1, b0);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // dummies drained
  }
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
        pk |= min(r1, r1 - (uint32_t)modulus) << (8 * u);
      }
      *reinterpret_cast<uint32_t*>(T + (wc * 64 + ni * 16 + l16) * TP + wr * 128 + mi * 16 + 4 * lq) = pk;
    }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < (IBM * TBN / 16) / 512; ++p) {
    const int id = tid + 512 * p;
    const int cloc = id >> 4, ch = id & 15;
    const uint4 v = *reinterpret_cast<const uint4*>(T + cloc * TP + 16 * ch);
    *reinterpret_cast<uint4*>(C + (int64_t)(j0 + cloc) * ldc + i0 + 16 * ch) = v;
  }
}

}  // namespace gp2d
