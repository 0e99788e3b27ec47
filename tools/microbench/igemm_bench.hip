// int8 NT GEMM (ozaki.hpp) in isolation: full kernel vs DMA-only vs MFMA-only (dev tool).
#include "../../2d-gp_amd/csrc/ozaki.hpp"
#include <cstdio>
namespace gp2d { void set_error(const std::string&) {} }
using namespace gp2d;
int main() {
  const int n = 8192, nc = 16384;
  int8_t *A, *B; uint8_t* C;
  (void)hipMalloc(&A, (size_t)n * n); (void)hipMalloc(&B, (size_t)nc * n); (void)hipMalloc(&C, (size_t)n * nc);
  (void)hipMemset(A, 3, (size_t)n * n); (void)hipMemset(B, 5, (size_t)nc * n);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (int tri = 1; tri >= 0; --tri)
  for (int xg = 0; xg < 2; ++xg) {
    dim3 g = xg ? dim3((n / 256) * (nc / 256)) : dim3(nc / 256, n / 256);
    for (int w = 0; w < 2; ++w) igemm_nt_mod_kernel<<<g, 256>>>(A, n, B, n, C, n, n, nc, n, tri, 251, 1.0 / 251, xg);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) igemm_nt_mod_kernel<<<g, 256>>>(A, n, B, n, C, n, n, nc, n, tri, 251, 1.0 / 251, xg);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double ops = tri ? 2.0 * ((double)n * n / 2 + n * 128.0) * nc : 2.0 * (double)n * n * nc;
    printf("%s tri=%d xcd=%d: %.3f ms/launch, %.0f TOPs\n", VARIANT, tri, xg, ms / 10, ops / (ms / 10) / 1e9);
  }
  return 0;
}
