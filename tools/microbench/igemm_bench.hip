// int8 NT GEMM kernels of ozaki.hpp in isolation on random residues (dev tool):
// one wave per SIMD (igemm_nt_mod_kernel) vs two (igemm_nt_mod_w8_kernel); outputs compared.
// Build variants with -DGP2D_IGEMM_NO_DMA / -DGP2D_IGEMM_NO_MFMA (see Makefile).
#include "../../2d-gp_amd/csrc/ozaki.hpp"
#include <cstdio>
#include <vector>
namespace gp2d { void set_error(const std::string&) {} }
using namespace gp2d;
__global__ void fill(int8_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = (int8_t)(h & 0xff);
  }
}
int main() {
  const int n = 8192, nc = 16384;
  int8_t *A, *B; uint8_t *C1, *C2;
  (void)hipMalloc(&A, (size_t)n * n); (void)hipMalloc(&B, (size_t)nc * n);
  (void)hipMalloc(&C1, (size_t)n * nc); (void)hipMalloc(&C2, (size_t)n * nc);
  fill<<<4096, 256>>>(A, (size_t)n * n, 17u); fill<<<4096, 256>>>(B, (size_t)nc * n, 91u);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const int tri = 1;
  for (int xg = 1; xg >= 0; --xg)
  for (int v = 0; v < 2; ++v) {
    dim3 g = xg ? dim3((n / 256) * (nc / 256)) : dim3(nc / 256, n / 256);
    auto launch = [&]() {
      if (v == 0) igemm_nt_mod_kernel<<<g, 256>>>(A, n, B, n, C1, n, n, nc, n, tri, 251, 1.0 / 251, xg);
      else igemm_nt_mod_w8_kernel<<<g, 512>>>(A, n, B, n, C2, n, n, nc, n, tri, 251, 1.0 / 251, xg);
    };
    for (int w = 0; w < 3; ++w) launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 20; ++r) launch();
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double ops = 2.0 * ((double)n * n / 2 + n * 128.0) * nc;
    printf("%s %s xcd=%d: %.3f ms/launch, %.0f TOPs\n", VARIANT, v ? "w8" : "w4", xg, ms / 20, ops / (ms / 20) / 1e9);
  }
  std::vector<uint8_t> h1((size_t)n * nc), h2((size_t)n * nc);
  (void)hipMemcpy(h1.data(), C1, h1.size(), hipMemcpyDeviceToHost);
  (void)hipMemcpy(h2.data(), C2, h2.size(), hipMemcpyDeviceToHost);
  size_t diff = 0;
  for (size_t i = 0; i < h1.size(); ++i) diff += h1[i] != h2[i];
  printf("%s w4 vs w8 differing bytes: %zu\n", VARIANT, diff);
  return 0;
}
