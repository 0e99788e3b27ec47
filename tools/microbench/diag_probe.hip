// Cycle-stamped variants of the register-resident inversion loop (dev tool).
#include "../../2d-gp_amd/csrc/factor.hpp"
#include <cstdio>
#include <vector>
#include <cmath>
namespace gp2d { void set_error(const std::string&) {} }
using namespace gp2d;

template <int VAR>
__global__ __launch_bounds__(256) void inv_variant(const double* __restrict__ A, double* __restrict__ D, unsigned long long* stamps) {
  __shared__ double Ls[NB * DSP];
  __shared__ double buf[2 * NB];
  const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
  for (int idx = tid; idx < NB * NB; idx += 256) { const int i = idx >> 7, j = idx & (NB - 1); Ls[i * DSP + j] = (j <= i) ? A[i * NB + j] : 0.0; }
  __syncthreads();
  double r[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) r[a][b] = (ty + 16 * a == tx + 16 * b) ? 1.0 : 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
  for (int k = 0; k < NB; ++k) {
    const int kb = k >> 4, kt = k & 15;
    double* rb = buf + (k & 1) * NB;
    const double rkk = (VAR == 3) ? Ls[k * DSP + k] : 1.0 / Ls[k * DSP + k];
    if (ty == kt) {
#pragma unroll
      for (int a = 0; a < 8; ++a) { if (a != kb) continue;
#pragma unroll
        for (int b = 0; b < 8; ++b) { r[a][b] *= rkk; rb[tx + 16 * b] = r[a][b]; } }
    }
    if (VAR != 1) __syncthreads();
    double xk[8], f[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) xk[b] = rb[tx + 16 * b];
#pragma unroll
    for (int a = 0; a < 8; ++a) f[a] = Ls[(ty + 16 * a) * DSP + k];
    if (VAR != 2) {
#pragma unroll
    for (int a = 0; a < 8; ++a) { if (a < kb) continue; const int i = ty + 16 * a;
#pragma unroll
      for (int b = 0; b < 8; ++b) { if (b > kb) continue; const int c = tx + 16 * b;
        const double nv = fma(-f[a], xk[b], r[a][b]); r[a][b] = (i > k && c <= k) ? nv : r[a][b]; } }
    } else {
#pragma unroll
      for (int a = 0; a < 8; ++a) r[a][0] += f[a] * xk[a];
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) { stamps[0] = t1 - t0; stamps[1] = rt1 - rt0; }
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) { const int i = ty + 16 * a, k = tx + 16 * b; D[i * NB + k] = r[a][b]; }
}

int main() {
  const int n = 128;
  std::vector<double> K(n * n, 0.0);
  for (int i = 0; i < n; ++i) for (int j = 0; j <= i; ++j) K[i * n + j] = (i == j ? 2.0 : 0.01);
  double *A, *D; unsigned long long* st;
  (void)hipMalloc(&A, n * n * 8); (void)hipMalloc(&D, n * n * 8); (void)hipMalloc(&st, 16);
  (void)hipMemcpy(A, K.data(), n * n * 8, hipMemcpyHostToDevice);
  const char* names[] = {"full", "no barrier", "no update", "no divide"};
  for (int v = 0; v < 4; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      if (v == 0) inv_variant<0><<<1, 256>>>(A, D, st);
      if (v == 1) inv_variant<1><<<1, 256>>>(A, D, st);
      if (v == 2) inv_variant<2><<<1, 256>>>(A, D, st);
      if (v == 3) inv_variant<3><<<1, 256>>>(A, D, st);
      (void)hipDeviceSynchronize();
    }
    unsigned long long h[2]; (void)hipMemcpy(h, st, 16, hipMemcpyDeviceToHost);
    printf("%-12s cycles %8llu  real %8.2f us  clock %.2f GHz  cycles/step %.0f\n", names[v], h[0], h[1] / 100.0, h[0] / (h[1] * 10.0) , h[0] / 128.0);
  }
  return 0;
}
