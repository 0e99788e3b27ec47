// The twelve per-modulus int8 GEMM launches of one predict chunk (gp2d.hip predict_ozaki_impl)
// against ONE launch with the moduli on blockIdx.z (the kernel's IgemmZ batch), dev tool: time per chunk's
// twelve products, back to back, at config B's (n = 2048) and the headline's (n = 8192) shapes
// with 16,384 columns, random residues, W lower-triangular (dense K loop); every output byte of
// the batched launch compared with the per-modulus launches on the device.
#include "../../2d-gp_amd/csrc/ozaki.hpp"
#include <cstdio>
#include <random>
#include <vector>
namespace gp2d { void set_error(const std::string&) {} }
using namespace gp2d;
__global__ void count_diff(const uint8_t* a, const uint8_t* b, int64_t n, unsigned long long* bad) {
  unsigned long long c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    c += a[i] != b[i];
  if (c) atomicAdd(bad, c);
}
int main() {
  const int nmod = 12, nc = 16384;
  const int mods[12] = {256, 255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217};
  for (int n : {2048, 8192}) {
    std::mt19937 rng(5 + n);
    std::vector<int8_t> A((size_t)n * n, 0), B((size_t)nc * n);
    for (int i = 0; i < n; ++i)
      for (int k = 0; k <= i; ++k) A[slab_offset(i, k, n)] = (int8_t)(rng() & 0xff);
    for (int j = 0; j < nc; ++j)
      for (int k = 0; k < n; ++k) B[slab_offset(j, k, n)] = (int8_t)(rng() & 0xff);
    const int64_t pa = (int64_t)n * n, pb = (int64_t)nc * n, pc = (int64_t)n * nc;
    int8_t *dA, *dB;
    uint8_t *dC1, *dC2;
    (void)hipMalloc(&dA, pa * nmod); (void)hipMalloc(&dB, pb * nmod);
    (void)hipMalloc(&dC1, pc * nmod); (void)hipMalloc(&dC2, pc * nmod);
    for (int l = 0; l < nmod; ++l) {
      (void)hipMemcpy(dA + l * pa, A.data(), pa, hipMemcpyHostToDevice);
      (void)hipMemcpy(dB + l * pb, B.data(), pb, hipMemcpyHostToDevice);
    }
    (void)hipMemset(dC1, 0, pc * nmod); (void)hipMemset(dC2, 1, pc * nmod);
    const dim3 g(nc / 256, n / IBM), gz(nc / 256, n / IBM, nmod);
    auto per_mod = [&]() {
      for (int l = 0; l < nmod; ++l)
        igemm_nt_mod_kernel<256, 4><<<g, 512>>>(dA + l * pa, dB + l * pb, dC1 + l * pc, n, n, nc, n, 1, mods[l],
                                                1 << 30, 0, nullptr, nullptr, IgemmZ{});
    };
    auto batched = [&]() {
      IgemmZ zb{pa, pb, pc, {}};
      for (int l = 0; l < nmod; ++l) zb.m[l] = mods[l];
      igemm_nt_mod_kernel<256, 4><<<gz, 512>>>(dA, dB, dC2, n, n, nc, n, 1, mods[0], 1 << 30, 0, nullptr, nullptr, zb);
    };
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 4; ++rep) {
      for (int v = 0; v < 2; ++v) {
        for (int w = 0; w < 2; ++w) v ? batched() : per_mod();
        (void)hipDeviceSynchronize();
        const int reps = n == 2048 ? 100 : 10;
        (void)hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) v ? batched() : per_mod();
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        printf("n=%d %s: %.4f ms per chunk (12 moduli)\n", n, v ? "one launch, moduli on z" : "12 launches      ",
               ms / reps);
      }
    }
    unsigned long long* dbad;
    (void)hipMalloc(&dbad, 8); (void)hipMemset(dbad, 0, 8);
    count_diff<<<1024, 256>>>(dC1, dC2, pc * nmod, dbad);
    unsigned long long bad = 0;
    (void)hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost);
    printf("n=%d: %llu of %lld output bytes differ between the two\n", n, bad, (long long)(pc * nmod));
    (void)hipFree(dA); (void)hipFree(dB); (void)hipFree(dC1); (void)hipFree(dC2); (void)hipFree(dbad);
  }
  return 0;
}
