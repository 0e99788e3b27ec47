// The int8 NT GEMM of ozaki.hpp in isolation on random residues (dev tool): time per
// 8192×16384×8192 lower-triangular launch, and 4096 sampled outputs checked against a
// CPU dot product.  FULL = the product kernel; the ablation variants build the dev copy
// (igemm_ablate.hpp) with -DGP2D_IGEMM_NO_DMA / NO_MFMA / NO_LDSREAD / EPI_ONLY.
#include "igemm_ablate.hpp"
#include <cstdio>
#include <random>
#include <vector>
#include <climits>
#include <cstdlib>
namespace gp2d { void set_error(const std::string&) {} }
using namespace gp2d;
#ifndef IG_TBN
#define IG_TBN 256
#endif
#ifndef IG_NST
#define IG_NST 4
#endif
#ifndef IGEMM_KERNEL
#define IGEMM_KERNEL igemm_nt_mod_kernel<IG_TBN, IG_NST>
#define IGEMM_EXTRA , nullptr, nullptr, gp2d::IgemmZ{}   // dense K loop (no slab list), one modulus
#endif
#ifndef IGEMM_EXTRA
#define IGEMM_EXTRA
#endif
#ifndef IGEMM_THREADS
#define IGEMM_THREADS (2 * IG_TBN)
#endif
#ifndef IGEMM_INV   // the dev copies still take 1/m (the product kernel reduces without it)
#define IGEMM_INV
#endif
int main() {
  const int n = 8192, nc = 16384, mod = 251;
  std::mt19937 rng(17);
  std::vector<int8_t> A((size_t)n * n), B((size_t)nc * n), Ab(A.size()), Bb(B.size());
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < n; ++k) A[(size_t)i * n + k] = (k <= i) ? (int8_t)(rng() & 0xff) : 0;
  for (auto& v : B) v = (int8_t)(rng() & 0xff);
  if (getenv("IGEMM_ZERO")) { for (auto& v : A) v = 0; for (auto& v : B) v = 0; }
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < n; ++k) Ab[slab_offset(i, k, n)] = A[(size_t)i * n + k];
  for (int j = 0; j < nc; ++j)
    for (int k = 0; k < n; ++k) Bb[slab_offset(j, k, n)] = B[(size_t)j * n + k];
  int8_t *dA, *dB; uint8_t* dC;
  (void)hipMalloc(&dA, A.size()); (void)hipMalloc(&dB, B.size()); (void)hipMalloc(&dC, (size_t)n * nc);
  (void)hipMemcpy(dA, Ab.data(), A.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, Bb.data(), B.size(), hipMemcpyHostToDevice);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const dim3 g(nc / IG_TBN, n / IBM);
  // IGEMM_K=k: dense (not triangular) launches with K = k on the same planes — per-tile vs
  // per-slab cost (time = tiles·a + slabs·b); the sampled check then does not apply
  const int kx = getenv("IGEMM_K") ? atoi(getenv("IGEMM_K")) : n, low = getenv("IGEMM_K") ? 0 : 1;
#ifdef IGEMM_GRID
  const dim3 gl(IGEMM_GRID);
#else
  const dim3 gl = g;
#endif
  auto launch = [&]() { IGEMM_KERNEL<<<gl, IGEMM_THREADS>>>(dA, dB, dC, n, n, nc, kx, low, mod IGEMM_INV, 1 << 30, 0 IGEMM_EXTRA); };
  for (int w = 0; w < 3; ++w) launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 20; ++r) launch();
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  const double ops = 2.0 * ((double)n * n / 2 + n * 128.0) * nc;
  if (!low) {
    printf("%s: K=%d dense: %.4f ms/launch\n", VARIANT, kx, ms / 20);
    return 0;
  }
  printf("%s: %.3f ms/launch, %.0f TOPs\n", VARIANT, ms / 20, ops / (ms / 20) / 1e9);
  std::vector<uint8_t> C((size_t)n * nc);
  (void)hipMemcpy(C.data(), dC, C.size(), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int t = 0; t < 4096; ++t) {
    const int i = rng() % n, j = rng() % nc;
    long long sacc = 0;
    for (int k = 0; k <= i; ++k) sacc += (long long)A[(size_t)i * n + k] * B[(size_t)j * n + k];
    const int want = (int)(((sacc % mod) + mod) % mod);
    bad += C[(size_t)j * n + i] != want;
  }
  printf("%s: %d of 4096 sampled outputs differ from the CPU dot product\n", VARIANT, bad);
#ifdef IG_STAMPS
  // igemm_stamps.hpp: per-wave segment sums of the last launch → shares and per-step cycles
  std::vector<unsigned long long> st(2048 * 8 * 8);
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(ig_stamp), st.size() * 8);
  double seg[6] = {0}, steps = 0, waves = 0;
  for (size_t w = 0; w < st.size() / 8; ++w) {
    for (int q = 0; q < 6; ++q) seg[q] += (double)st[w * 8 + q];
    steps += (double)st[w * 8 + 6];
    waves += 1;
  }
  const char* nm[6] = {"work (reads, h1+h0 MFMAs, DMA issue)", "vmcnt wait (own DMA of next slab)", "s_barrier wait",
                       "ring tail", "epilogue", "prologue"};
  double tot = 0;
  for (int q = 0; q < 6; ++q) tot += seg[q];
  printf("stamps: %.0f waves, %.1f stamped steps per wave, %.0f wave-cycles per wave\n", waves, steps / waves, tot / waves);
  for (int q = 0; q < 6; ++q)
    printf("  seg %d %-40s share %.3f  per wave %.0f  per step %.1f\n", q, nm[q], seg[q] / tot, seg[q] / waves,
           q < 3 ? seg[q] / steps : 0.0);
#endif
  return 0;
}
