// The POTRF trailing update (SYRK, K = 128, lower tiles, beta = 1) in isolation (dev tool):
// time per launch at the N_train = 4096 (n = 8192) step-0 size and at the N = 16384 sizes,
// and a sampled check against a CPU dot product.
#include "../../2d-gp_amd/csrc/gemm_f64.hpp"
#include <cstdio>
#include <random>
#include <vector>
namespace gp2d { void set_error(const std::string&) {} }
using namespace gp2d;
#ifndef SYRK_LAUNCH
#define SYRK_LAUNCH(q, s) launch_gemm<true, EPI_STORE>(q, 1, s)
#endif
int main() {
  for (int m : {8064, 4096, 1024, 32640}) {
#ifndef SYRK_K
#define SYRK_K 128
#endif
    const int K = SYRK_K, ld = m + SYRK_K;
    std::mt19937_64 rng(5);
    std::uniform_real_distribution<double> U(-1, 1);
    std::vector<double> A((size_t)m * ld), C((size_t)m * ld);
    for (auto& v : A) v = U(rng);
    for (auto& v : C) v = U(rng);
    double *dA, *dC;
    (void)hipMalloc(&dA, A.size() * 8); (void)hipMalloc(&dC, C.size() * 8);
    (void)hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
    GemmParams q = gemm_params();
    q.A = dA; q.lda = ld; q.B = dA; q.ldb = ld; q.C = dC; q.ldc = ld;
    q.M = m; q.N = m; q.K = K; q.alpha = -1.0; q.beta = 1.0; q.c_lower = 1;
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)SYRK_LAUNCH(q, 0);
    (void)hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
    (void)SYRK_LAUNCH(q, 0);   // checked launch: C ← C − A·Aᵀ (lower tiles)
    std::vector<double> R((size_t)m * ld);
    (void)hipMemcpy(R.data(), dC, R.size() * 8, hipMemcpyDeviceToHost);
    double err = 0;
    for (int t = 0; t < 2000; ++t) {
      const int i = rng() % m, j = rng() % (i + 1);
      double s = C[(size_t)i * ld + j];
      for (int k = 0; k < K; ++k) s -= A[(size_t)i * ld + k] * A[(size_t)j * ld + k];
      err = std::max(err, std::abs(s - R[(size_t)i * ld + j]));
    }
    const int reps = m > 20000 ? 5 : 20;
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) (void)SYRK_LAUNCH(q, 0);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double fl = (double)m * (m + 128) * K;   // lower tiles incl. diagonal tiles
    printf("%s m=%d: %.1f us/launch, %.1f TF/s, max err %.2e\n", VARIANT, m, 1e3 * ms / reps,
           fl / (ms / reps * 1e-3) / 1e12, err);
    (void)hipFree(dA); (void)hipFree(dC);
  }
  return 0;
}
