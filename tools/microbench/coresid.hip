// Can the CRT pass run beside the int8 GEMM instead of after it? (dev tool, round 6)
//
// The predict stream runs, per 8192-point chunk, K* → 12 int8 GEMM launches → CRT + column Σ V².
// The GEMM is MFMA-bound with HBM to spare, the CRT is a memory-bound VALU pass: side by side
// they would overlap — but only if a CRT wave fits on a CU beside the GEMM's workgroup.  The
// product GEMM allocates 254 VGPRs × 2 waves per SIMD (the whole 512-entry file), so nothing
// co-resides; a third wave needs the GEMM at ≤ 224 and the companion at ≤ 64, and this
// compiler ignores amdgpu_num_vgpr below its own allocation (the GEMM stays at 250–254 with
// the attribute at 200–232, with one A-fragment set instead of two at 250).  Companion kernels:
// the product CRT (RPL = 16, 124 VGPRs) and crt4 (4 rows per lane, 64 VGPRs).  Prints each alone
// and each pair side by side (the GEMM's 12 launches on stream A, the CRT of another chunk's
// planes on stream B): what the dispatcher's workgroup-level time slicing gives.
#include "../../2d-gp_amd/csrc/ozaki.hpp"
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include <cmath>
namespace gp2d { void set_error(const std::string&) {} }
using namespace gp2d;

constexpr int C4_COLS = 4;                 // columns per wave
constexpr int C4_BCOLS = 4 * C4_COLS;      // per 256-thread block
constexpr int C4_ROWS = 256;               // rows per segment (4 per lane)
__global__ __launch_bounds__(256) void crt4_kernel(
    const uint8_t* __restrict__ cres, int64_t n, int64_t ncols, OzakiConsts oc, const double* __restrict__ rowscale,
    double* __restrict__ P) {
  const int lane = threadIdx.x & 63;
  const int64_t jw = (int64_t)blockIdx.x * C4_BCOLS + (threadIdx.x >> 6) * C4_COLS;
  const int64_t seg = blockIdx.y;
  const int64_t i0 = seg * C4_ROWS + 4 * lane;
  if (jw >= ncols) return;
  double rs[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) rs[c] = rowscale[i0 + c];
  const int64_t plane = n * ncols;
#pragma unroll 1
  for (int jc = 0; jc < C4_COLS; ++jc) {
    const int64_t j = jw + jc;
    double H[4] = {0, 0, 0, 0}, T[4] = {0, 0, 0, 0};
    const uint8_t* base = cres + j * n + i0;
#pragma unroll 1
    for (int l0 = 0; l0 < oc.nmod; l0 += 4) {
      uint32_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint32_t*>(base + (int64_t)min(l0 + u, oc.nmod - 1) * plane);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double h = oc.h[l0 + u], t = oc.t[l0 + u];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const double cl = (double)((v[u] >> (8 * c)) & 0xffu);
          H[c] = fma(cl, h, H[c]);
          T[c] = fma(cl, t, T[c]);
        }
      }
    }
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const double f = (H[c] - rint(H[c])) + T[c];
      const double vij = f * rs[c];
      acc = fma(vij, vij, acc);
      if (fabs(vij) > oc.vlimit) acc = __builtin_nan("");
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) P[seg * ncols + j] = acc;
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int n = 8192, nc = 16384, nmod = 12, reps = argc > 1 ? atoi(argv[1]) : 5;
  std::mt19937 rng(23);
  std::vector<int8_t> A((size_t)n * n, 0), B((size_t)nc * n);
  for (int i = 0; i < n; ++i)
    for (int k = 0; k <= i; ++k) A[slab_offset(i, k, n)] = (int8_t)(rng() & 0xff);
  for (int j = 0; j < nc; ++j)
    for (int k = 0; k < n; ++k) B[slab_offset(j, k, n)] = (int8_t)(rng() & 0xff);
  int8_t *dA, *dB;
  uint8_t *dC, *dR;
  double *drs, *dP, *dP4;
  const size_t plane = (size_t)n * nc;
  CK(hipMalloc(&dA, A.size()));
  CK(hipMalloc(&dB, B.size()));
  CK(hipMalloc(&dC, plane * nmod));   // the GEMM's output planes (this chunk)
  CK(hipMalloc(&dR, plane * nmod));   // the previous chunk's planes (the CRT's input)
  CK(hipMalloc(&drs, n * sizeof(double)));
  CK(hipMalloc(&dP, (size_t)(n / OZ_CRT_ROWS) * nc * sizeof(double)));
  CK(hipMalloc(&dP4, (size_t)(n / C4_ROWS) * nc * sizeof(double)));
  CK(hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice));
  {
    std::vector<uint8_t> R(plane * nmod);
    for (auto& v : R) v = (uint8_t)(rng() % 241);
    CK(hipMemcpy(dR, R.data(), R.size(), hipMemcpyHostToDevice));
    std::vector<double> rs(n);
    for (auto& v : rs) v = 1e-3 * (1 + (rng() % 1000) / 1000.0);
    CK(hipMemcpy(drs, rs.data(), n * sizeof(double), hipMemcpyHostToDevice));
  }
  OzakiConsts oc{};
  oc.nmod = nmod;
  for (int l = 0; l < OZ_MAXMOD; ++l) {
    oc.m[l] = 251 - 2 * l;
    oc.h[l] = std::ldexp((double)(rng() % (1u << 20)), -33);
    oc.t[l] = std::ldexp((double)(rng() % 1000), -60);
  }
  oc.vlimit = 1e300;
  hipStream_t sA, sB;
  CK(hipStreamCreateWithFlags(&sA, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sB, hipStreamNonBlocking));
  const dim3 gg(nc / 256, n / IBM);
  auto gemms = [&](hipStream_t s) {
    for (int l = 0; l < nmod; ++l)
      igemm_nt_mod_kernel<256, 4><<<gg, 512, 0, s>>>(dA, dB, dC + l * plane, n, n, nc, n, 1, 251 - 2 * l, 1 << 30, 0,
                                                      nullptr, nullptr, IgemmZ{});
  };
  auto crt16 = [&](hipStream_t s) {
    ozaki_crt_colsq_kernel<<<dim3(nc / OZ_CRT_BCOLS, n / OZ_CRT_ROWS), 256, 0, s>>>(dR, n, nc, oc, drs, dP);
  };
  auto crt4 = [&](hipStream_t s) { crt4_kernel<<<dim3(nc / C4_BCOLS, n / C4_ROWS), 256, 0, s>>>(dR, n, nc, oc, drs, dP4); };
  hipEvent_t e0, eA, eB;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&eA));
  CK(hipEventCreate(&eB));
  auto alone = [&](auto f, hipStream_t s) {
    f(s);
    CK(hipStreamSynchronize(s));
    float tot = 0;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0, s));
      f(s);
      CK(hipEventRecord(eA, s));
      CK(hipEventSynchronize(eA));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, eA));
      tot += ms;
    }
    return tot / reps;
  };
  auto pair = [&](auto fb, float* spanA, float* spanB) {
    float ta = 0, tb = 0;
    for (int r = 0; r < reps + 1; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, sA));
      CK(hipStreamWaitEvent(sB, e0, 0));
      gemms(sA);
      fb(sB);
      CK(hipEventRecord(eA, sA));
      CK(hipEventRecord(eB, sB));
      CK(hipEventSynchronize(eA));
      CK(hipEventSynchronize(eB));
      float a, b;
      CK(hipEventElapsedTime(&a, e0, eA));
      CK(hipEventElapsedTime(&b, e0, eB));
      if (r > 0) { ta += a; tb += b; }
    }
    *spanA = ta / reps;
    *spanB = tb / reps;
  };
  const float tg = alone(gemms, sA), t16 = alone(crt16, sB), t4 = alone(crt4, sB);
  float a16, b16, a4, b4;
  pair(crt16, &a16, &b16);
  pair(crt4, &a4, &b4);
  // crt4 against the product CRT: the same Σ V² per column (different summation order)
  std::vector<double> P((size_t)(n / OZ_CRT_ROWS) * nc), P4((size_t)(n / C4_ROWS) * nc);
  CK(hipMemcpy(P.data(), dP, P.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(P4.data(), dP4, P4.size() * 8, hipMemcpyDeviceToHost));
  double worst = 0;
  for (int j = 0; j < nc; ++j) {
    double s = 0, s4 = 0;
    for (int g = 0; g < n / OZ_CRT_ROWS; ++g) s += P[(size_t)g * nc + j];
    for (int g = 0; g < n / C4_ROWS; ++g) s4 += P4[(size_t)g * nc + j];
    worst = std::max(worst, std::fabs(s - s4) / std::fabs(s));
  }
  printf("{\"gemm12_alone_ms\": %.4f, \"crt16_alone_ms\": %.4f, "
         "\"crt4_alone_ms\": %.4f, \"pair_crt16\": {\"gemm_span_ms\": %.4f, \"crt_span_ms\": %.4f}, "
         "\"pair_crt4\": {\"gemm_span_ms\": %.4f, \"crt_span_ms\": %.4f}, \"serial_crt16_ms\": %.4f, "
         "\"crt4_vs_crt16_max_rel\": %.3e}\n",
         tg, t16, t4, a16, b16, a4, b4, tg + t16, worst);
  return 0;
}
