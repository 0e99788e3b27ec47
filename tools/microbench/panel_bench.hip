// The POTRF critical-path skinny GEMM (gemm_f64_panel_kernel: C[M×128] += alpha·A[M×128]·B[128×128]ᵀ,
// the column update and the panel TRSM) in isolation (dev tool): time per launch, back to back
// (independent launches on one stream) and with a one-element dependency between consecutive
// launches' buffers (each launch reads what the previous wrote: the chain's situation), for
// M from one block row to the N_train = 4096 step-0 size; a sampled CPU check.
#include "../../2d-gp_amd/csrc/gemm_f64.hpp"
#include <cstdio>
#include <random>
#include <vector>
namespace gp2d { void set_error(const std::string&) {} }
using namespace gp2d;
__global__ void empty_kernel(int* p) { if (threadIdx.x == 1023 && p) *p = 0; }
int main() {
  {   // back-to-back launch cost of a one-workgroup empty kernel on one stream
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int w = 0; w < 10; ++w) empty_kernel<<<1, 256>>>(nullptr);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 200; ++r) empty_kernel<<<1, 256>>>(nullptr);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    printf("empty kernel: %.2f us/launch back to back\n", 1e3 * ms / 200);
  }
  const int lda = 8192 + 128;
  for (int m : {128, 1024, 4096, 8064}) {
    std::mt19937_64 rng(9);
    std::uniform_real_distribution<double> U(-1, 1);
    std::vector<double> A((size_t)m * lda), B(128 * 128);
    for (auto& v : A) v = U(rng);
    for (auto& v : B) v = U(rng);
    double *dA, *dB, *dC;
    (void)hipMalloc(&dA, A.size() * 8); (void)hipMalloc(&dB, B.size() * 8); (void)hipMalloc(&dC, A.size() * 8);
    (void)hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dC, A.data(), A.size() * 8, hipMemcpyHostToDevice);
    for (int shape = 0; shape < 5; ++shape) {
    static const int SR[5] = {32, 32, 16, 32, 16}, SC[5] = {128, 32, 128, 64, 64};
    auto launch = [&](double* C) {
      const dim3 g((unsigned)(m / SR[shape]), 1, (unsigned)(128 / SC[shape]));
      switch (shape) {
        case 0: gemm_f64_panel_kernel<32, 128><<<g, 256>>>(dA, lda, dB, 128, C, lda, -1.0, 1.0, 0, 0, 0); break;
        case 1: gemm_f64_panel_kernel<32, 32><<<g, 256>>>(dA, lda, dB, 128, C, lda, -1.0, 1.0, 0, 0, 0); break;
        case 2: gemm_f64_panel_kernel<16, 128><<<g, 256>>>(dA, lda, dB, 128, C, lda, -1.0, 1.0, 0, 0, 0); break;
        case 3: gemm_f64_panel_kernel<32, 64><<<g, 256>>>(dA, lda, dB, 128, C, lda, -1.0, 1.0, 0, 0, 0); break;
        default: gemm_f64_panel_kernel<16, 64><<<g, 256>>>(dA, lda, dB, 128, C, lda, -1.0, 1.0, 0, 0, 0); break;
      }
    };
    (void)hipMemcpy(dC, A.data(), A.size() * 8, hipMemcpyHostToDevice);
    launch(dC);
    std::vector<double> R((size_t)m * lda);
    (void)hipMemcpy(R.data(), dC, R.size() * 8, hipMemcpyDeviceToHost);
    double err = 0;
    for (int t = 0; t < 1000; ++t) {
      const int i = rng() % m, j = rng() % 128;
      double s = A[(size_t)i * lda + j];
      for (int k = 0; k < 128; ++k) s -= A[(size_t)i * lda + k] * B[(size_t)j * 128 + k];
      err = std::max(err, std::abs(s - R[(size_t)i * lda + j]));
    }
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int reps = 50;
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) launch(dC);   // same stream: each launch starts after the previous ends
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double fl = 2.0 * m * 128 * 128;
    printf("%s %dx%d m=%d: %.1f us/launch (%d workgroups), %.2f TF/s, max err %.2e\n", VARIANT, SR[shape],
           SC[shape], m, 1e3 * ms / reps, (m / SR[shape]) * (128 / SC[shape]), fl / (ms / reps * 1e-3) / 1e12, err);
    }
    (void)hipFree(dA); (void)hipFree(dB); (void)hipFree(dC);
  }
  return 0;
}
