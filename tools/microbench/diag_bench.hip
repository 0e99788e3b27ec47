// Times the 128×128 diagonal-block kernels in isolation (dev tool).
__device__ unsigned long long g_stamps[16];
#define GP2D_STAMP(slot) do { if (threadIdx.x == 0) g_stamps[slot] = __builtin_amdgcn_s_memtime(); } while (0)
#include "../../2d-gp_amd/csrc/factor.hpp"
#include <cstdio>
#include <vector>
#include <cmath>
namespace gp2d { void set_error(const std::string&) {} }
using namespace gp2d;
__global__ void noop_kernel(double* p) { if (threadIdx.x == 9999) p[0] = 1; }
__global__ __launch_bounds__(256) void barrier_only(double* p) {
  __shared__ double S[128];
  for (int j = 0; j < 256; ++j) { if (threadIdx.x == 0) S[j & 127] = j; __syncthreads(); }
  if (threadIdx.x == 0) p[0] = S[5];
}
__global__ __launch_bounds__(256) void sqrtdiv_only(double* p) {
  double x = p[threadIdx.x];
  for (int j = 0; j < 128; ++j) { double r = sqrt(x); x = 1.0 / r + 1.0; }
  p[threadIdx.x] = x;
}
int main() {
  const int n = 128;
  std::vector<double> K(n * n);
  for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) K[i * n + j] = (i == j ? n : 0) + 1.0 / (1 + std::abs(i - j));
  double *A, *A0, *D; int* info;
  hipMalloc(&A, n * n * 8); hipMalloc(&A0, n * n * 8); hipMalloc(&D, n * n * 8); hipMalloc(&info, 4);
  hipMemcpy(A0, K.data(), n * n * 8, hipMemcpyHostToDevice);
  hipMemset(info, 0, 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float ms;
  auto timeit = [&](const char* name, auto fn) {
    for (int w = 0; w < 3; ++w) fn();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 50; ++r) fn();
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %9.2f us/launch\n", name, 1e3 * ms / 50);
  };
  timeit("noop", [&] { noop_kernel<<<1, 256>>>(A); });
  timeit("barrier x256", [&] { barrier_only<<<1, 256>>>(A); });
  timeit("sqrt+div x128 (chain)", [&] { sqrtdiv_only<<<1, 256>>>(D); });
  timeit("potrf_diag_reg (chol+inv)", [&] { hipMemcpyAsync(A, A0, n * n * 8, hipMemcpyDeviceToDevice); potrf_diag_reg_kernel<<<1, 256>>>(A, n, 0, D, info); });
  std::vector<double> Lr(n * n), Dr(n * n), Lb(n * n), Db(n * n);
  hipMemcpy(Lr.data(), A, n * n * 8, hipMemcpyDeviceToHost); hipMemcpy(Dr.data(), D, n * n * 8, hipMemcpyDeviceToHost);
  timeit("potrf_diag blocked (chol+inv)", [&] { hipMemcpyAsync(A, A0, n * n * 8, hipMemcpyDeviceToDevice); potrf_diag_kernel<<<1, 256>>>(A, n, 0, D, info); });
  hipMemcpy(Lb.data(), A, n * n * 8, hipMemcpyDeviceToHost); hipMemcpy(Db.data(), D, n * n * 8, hipMemcpyDeviceToHost);
  double eL = 0, eD = 0, mL = 0, mD = 0;
  for (int i = 0; i < n * n; ++i) { eL = std::max(eL, std::abs(Lr[i] - Lb[i])); eD = std::max(eD, std::abs(Dr[i] - Db[i])); mL = std::max(mL, std::abs(Lr[i])); mD = std::max(mD, std::abs(Dr[i])); }
  printf("blocked vs reg: L max rel diff %.2e, inv max rel diff %.2e\n", eL / mL, eD / mD);
  timeit("memcpy only", [&] { hipMemcpyAsync(A, A0, n * n * 8, hipMemcpyDeviceToDevice); });
  timeit("trti2_diag (inv only)", [&] { trti2_diag_kernel<<<1, 256>>>(A, n, D); });
  potrf_diag_kernel<<<1, 256>>>(A, n, 0, D, info); (void)hipDeviceSynchronize();
  unsigned long long st[16]; (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st));
  printf("phases (cycles): load %llu, chol %llu, store L %llu, rdiag %llu, diag-inv %llu, offdiag-inv %llu\n", st[1]-st[0], st[2]-st[1], st[3]-st[2], st[5]-st[3], st[6]-st[5], st[4]-st[6]);
  printf("panels/trailing (cycles):"); for (int p = 0; p < 4; ++p) printf(" p%d %llu/%llu", p, st[8 + 2 * p] - (p ? st[7 + 2 * p] : st[1]), st[9 + 2 * p] - st[8 + 2 * p]); printf("\n");
  int h; hipMemcpy(&h, info, 4, hipMemcpyDeviceToHost);
  printf("info=%d\n", h);
  return 0;
}
