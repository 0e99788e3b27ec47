// int8 MFMA on gfx950: operand/accumulator lane maps (exact integer check) and throughput.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef int i4 __attribute__((ext_vector_type(4)));
typedef int i16v __attribute__((ext_vector_type(16)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

// A: 16x64 row-major int8, B: 64x16 row-major int8.  Hypothesis: lane l holds A[l&15][16(l>>4)+j], B[16(l>>4)+j][l&15]
__global__ void lay16(const signed char* A, const signed char* B, int* D) {
  int l = threadIdx.x;
  signed char a[16], b[16];
  for (int j = 0; j < 16; ++j) { a[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j]; b[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)]; }
  i4 av, bv; __builtin_memcpy(&av, a, 16); __builtin_memcpy(&bv, b, 16);
  i4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = acc[r];
}
// A: 32x32, B: 32x32. Hypothesis: lane l holds A[l&31][16(l>>5)+j], B[16(l>>5)+j][l&31]
__global__ void lay32(const signed char* A, const signed char* B, int* D) {
  int l = threadIdx.x;
  signed char a[16], b[16];
  for (int j = 0; j < 16; ++j) { a[j] = A[(l & 31) * 32 + 16 * (l >> 5) + j]; b[j] = B[(16 * (l >> 5) + j) * 32 + (l & 31)]; }
  i4 av, bv; __builtin_memcpy(&av, a, 16); __builtin_memcpy(&bv, b, 16);
  i16v acc = {0};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, acc, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[l * 16 + r] = acc[r];
}
template <int NACC>
__global__ void rate16(int iters, int seed, int* out) {
  i4 a = {seed, seed + 1, seed + 2, seed + 3}, b = {seed * 3, 7, 11, 13};
  i4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = i4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
  int s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int NACC>
__global__ void rate32(int iters, int seed, int* out) {
  i4 a = {seed, seed + 1, seed + 2, seed + 3}, b = {seed * 3, 7, 11, 13};
  i16v acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = i16v{0};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
  int s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
  std::vector<signed char> A(64 * 64), B(64 * 64);
  for (int i = 0; i < 64 * 64; ++i) { A[i] = (signed char)((i * 37 + 11) % 251 - 125); B[i] = (signed char)((i * 53 + 5) % 241 - 120); }
  signed char *dA, *dB; int* dD;
  CK(hipMalloc(&dA, 4096)); CK(hipMalloc(&dB, 4096)); CK(hipMalloc(&dD, 64 * 16 * 4));
  CK(hipMemcpy(dA, A.data(), 4096, hipMemcpyHostToDevice)); CK(hipMemcpy(dB, B.data(), 4096, hipMemcpyHostToDevice));
  std::vector<int> D(64 * 16);
  lay16<<<1, 64>>>(dA, dB, dD); CK(hipMemcpy(D.data(), dD, 64 * 4 * 4, hipMemcpyDeviceToHost));
  int bad_a = 0, bad_b = 0;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
    int col = l & 15;
    int rowa = 4 * (l >> 4) + r, rowb = (l >> 4) + 4 * r;
    long sa = 0, sb = 0;
    for (int k = 0; k < 64; ++k) { sa += A[rowa * 64 + k] * B[k * 16 + col]; sb += A[rowb * 64 + k] * B[k * 16 + col]; }
    bad_a += (sa != D[l * 4 + r]); bad_b += (sb != D[l * 4 + r]);
  }
  printf("{\"16x16x64 mismatches row=4(l>>4)+r\": %d, \"row=(l>>4)+4r\": %d}\n", bad_a, bad_b);
  lay32<<<1, 64>>>(dA, dB, dD); CK(hipMemcpy(D.data(), dD, 64 * 16 * 4, hipMemcpyDeviceToHost));
  int bad32 = 0;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) {
    int col = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    long s = 0;
    for (int k = 0; k < 32; ++k) s += A[row * 32 + k] * B[k * 32 + col];
    bad32 += (s != D[l * 16 + r]);
  }
  printf("{\"32x32x32 mismatches row=(r&3)+8(r>>2)+4(l>>5)\": %d}\n", bad32);
  int* out; CK(hipMalloc(&out, 1 << 24));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int nblk = 1024, iters = 20000; float ms;
  for (int rep = 0; rep < 2; ++rep) {
    rate16<4><<<nblk, 256>>>(10, 1, out); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); rate16<4><<<nblk, 256>>>(iters, 1, out); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\":\"mfma_i32_16x16x64_i8\", \"TOPs\": %.1f}\n", (double)nblk * 4 * iters * 4 * 32768.0 / ms / 1e9);
    rate32<2><<<nblk, 256>>>(10, 1, out); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); rate32<2><<<nblk, 256>>>(iters, 1, out); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\":\"mfma_i32_32x32x32_i8\", \"TOPs\": %.1f}\n", (double)nblk * 4 * iters * 2 * 65536.0 / ms / 1e9);
  }
  return 0;
}
