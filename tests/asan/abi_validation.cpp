// Host AddressSanitizer / UndefinedBehaviorSanitizer run of the C ABI's argument validation
// (SURVEY.md §5): every entry point of include/gp2d.h is called with the malformed arguments a
// caller can pass (NULL descriptors and buffers, non-multiple sizes, bad enums, undersized
// workspaces, out-of-range kernel parameters) and must return < 0 with a message in
// gp2d_last_error() — before any device work, so this runs on a CPU-only host.  The pure host
// functions (sizes, moduli counts, kernel diagonal) are exercised on valid arguments too.
// Built by tests/asan/Makefile with -fsanitize=address,undefined on the host side only
// (libgp2d's device code is compiled as usual); run by tests/test_host_asan.py.
#include "../../include/gp2d.h"
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

static int g_fail = 0, g_checks = 0;
#define EXPECT_ERR(call)                                                                      \
  do {                                                                                        \
    ++g_checks;                                                                               \
    const int rc_ = (call);                                                                   \
    const char* m_ = gp2d_last_error();                                                       \
    if (rc_ >= 0 || m_ == nullptr || std::strlen(m_) == 0) {                                  \
      std::printf("FAIL %s:%d rc=%d msg='%s' : %s\n", __FILE__, __LINE__, rc_, m_ ? m_ : "", #call); \
      ++g_fail;                                                                               \
    }                                                                                         \
  } while (0)
#define EXPECT(cond)                                                                          \
  do {                                                                                        \
    ++g_checks;                                                                               \
    if (!(cond)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #cond); ++g_fail; }      \
  } while (0)

static gp2d_kernel_t vec(int kind, double ldf, double lcf, double ratio) {
  gp2d_kernel_t k;
  std::memset(&k, 0, sizeof k);
  k.family = GP2D_FAMILY_VECTOR2D;
  k.kind = kind;
  k.l_df = ldf;
  k.l_cf = lcf;
  k.ratio = ratio;
  return k;
}

int main() {
  EXPECT(gp2d_abi_version() == GP2D_ABI_VERSION);
  // ---- pure host functions on valid and edge arguments
  EXPECT(gp2d_padded_points(1) == 64 && gp2d_padded_points(64) == 64 && gp2d_padded_points(65) == 128);
  EXPECT(gp2d_padded_points(0) == 64 && gp2d_padded_points(-5) == 64);
  gp2d_kernel_t df = vec(GP2D_KIND_DIVFREE, 5.0, 5.0, 1.0), mixed = vec(GP2D_KIND_MIXED, 4.0, 3.0, 0.3);
  EXPECT(gp2d_block_dim(&df) == 2 && gp2d_block_dim(nullptr) == 2);
  EXPECT(std::fabs(gp2d_kernel_diag(&df) - 0.04) < 1e-15);
  EXPECT(std::fabs(gp2d_kernel_diag(&mixed) - (0.3 / 16 + 0.7 / 9)) < 1e-15);
  EXPECT(gp2d_kernel_diag(nullptr) == 0.0);
  gp2d_kernel_t ard;
  std::memset(&ard, 0, sizeof ard);
  ard.family = GP2D_FAMILY_ARD_RBF; ard.dim = 3; ard.nterms = 2;
  ard.var[0] = 0.8; ard.var[1] = 0.2;
  for (int t = 0; t < 2; ++t) for (int d = 0; d < 3; ++d) ard.ls[t][d] = 1.0 + t + d;
  EXPECT(gp2d_block_dim(&ard) == 1 && std::fabs(gp2d_kernel_diag(&ard) - 1.0) < 1e-15);
  for (int64_t n : {256, 1024, 8192, 32768}) {
    EXPECT(gp2d_ozaki_nmod(n) > 0 && gp2d_ozaki_nmod(n) <= 20);
    EXPECT(gp2d_ozaki_wres_bytes(n) > 0);
    EXPECT(gp2d_potrf_inv_workspace(n) > 0 && gp2d_trtri_workspace(n) > 0 && gp2d_potrs_workspace(n) > 0);
    EXPECT(gp2d_predict_workspace(n, 8192, 2) > 0 && gp2d_predict_ozaki_workspace(n, 8192) > 0);
    EXPECT(gp2d_lml_grad_workspace(n) > 0 && gp2d_predict_ozaki_planes_workspace(n, 8192) > 0);
    const int a = gp2d_ozaki_nmod_apriori(n, &df, 0.0025, 0, 0);
    EXPECT(a > 0 && a <= 20 && a <= gp2d_ozaki_nmod(n));
  }
  EXPECT(gp2d_potrf_inv_workspace(128) == 0);
  EXPECT(gp2d_ozaki_kstar_bytes(8192, 65536, 8192, 12) > 0);
  EXPECT(gp2d_kernel_grad_workspace(100, 100) > 0);
  EXPECT(gp2d_lml_grad_count(&df) > 0 && gp2d_kernel_grad_count(&mixed) > 0 && gp2d_lml_grad_count(&ard) > 0);

  // ---- malformed kernel descriptors
  double buf[64] = {0};
  double buf2[64] = {0};   // a second, distinct buffer (aliasing checks)
  gp2d_kernel_t bad = df;
  EXPECT_ERR(gp2d_assemble(buf, 1, 64, buf, 1, 64, nullptr, 0.0, 1, buf, 128, nullptr));
  bad.kind = 7;
  EXPECT_ERR(gp2d_assemble(buf, 1, 64, buf, 1, 64, &bad, 0.0, 1, buf, 128, nullptr));
  bad = df; bad.l_df = 0.0;
  EXPECT_ERR(gp2d_assemble(buf, 1, 64, buf, 1, 64, &bad, 0.0, 1, buf, 128, nullptr));
  bad = df; bad.l_df = -1.0;
  EXPECT_ERR(gp2d_assemble(buf, 1, 64, buf, 1, 64, &bad, 0.0, 1, buf, 128, nullptr));
  bad = mixed; bad.l_cf = 0.0;
  EXPECT_ERR(gp2d_assemble(buf, 1, 64, buf, 1, 64, &bad, 0.0, 1, buf, 128, nullptr));
  bad = df; bad.family = 9;
  EXPECT_ERR(gp2d_assemble(buf, 1, 64, buf, 1, 64, &bad, 0.0, 1, buf, 128, nullptr));
  gp2d_kernel_t bard = ard; bard.dim = 4;
  EXPECT_ERR(gp2d_assemble(buf, 1, 64, buf, 1, 64, &bard, 0.0, 1, buf, 64, nullptr));
  bard = ard; bard.nterms = 3;
  EXPECT_ERR(gp2d_assemble(buf, 1, 64, buf, 1, 64, &bard, 0.0, 1, buf, 64, nullptr));
  bard = ard; bard.ls[1][2] = 0.0;
  EXPECT_ERR(gp2d_assemble(buf, 1, 64, buf, 1, 64, &bard, 0.0, 1, buf, 64, nullptr));
  gp2d_kernel_t st = df; st.family = GP2D_FAMILY_VECTOR_ST; st.var[0] = 0.0; st.ls[0][0] = 1.0;
  EXPECT_ERR(gp2d_assemble(buf, 1, 64, buf, 1, 64, &st, 0.0, 1, buf, 128, nullptr));
  // ---- assembly sizes
  EXPECT_ERR(gp2d_assemble(buf, 1, 63, buf, 1, 64, &df, 0.0, 1, buf, 128, nullptr));   // pad not ×64
  EXPECT_ERR(gp2d_assemble(buf, 65, 64, buf, 1, 64, &df, 0.0, 1, buf, 128, nullptr));  // n > pad
  EXPECT_ERR(gp2d_assemble(buf, -1, 64, buf, 1, 64, &df, 0.0, 1, buf, 128, nullptr));
  EXPECT_ERR(gp2d_assemble(buf, 1, 64, buf, 1, 64, &df, 0.0, 1, buf, 127, nullptr));   // ld < 2·64
  // ---- fit
  int info = 0;
  EXPECT_ERR(gp2d_potrf(buf, 100, 100, buf, &info, nullptr, 0, nullptr));        // n not ×128
  EXPECT_ERR(gp2d_potrf(buf, 0, 128, buf, &info, nullptr, 0, nullptr));
  EXPECT_ERR(gp2d_potrf(buf, 128, 127, buf, &info, nullptr, 0, nullptr));        // lda < n
  EXPECT_ERR(gp2d_potrf(buf, 128, 129, buf, &info, nullptr, 0, nullptr));        // lda odd
  EXPECT_ERR(gp2d_potrf(buf, 128, 128, nullptr, &info, nullptr, 0, nullptr));    // no dinv
  EXPECT_ERR(gp2d_potrf_inv(buf, 200, 200, buf, &info, buf, 64, nullptr));
  EXPECT_ERR(gp2d_potrf_inv(buf, 256, 256, buf, &info, nullptr, 0, nullptr));    // workspace
  EXPECT_ERR(gp2d_potrf_inv(buf, 256, 256, buf, &info, buf, gp2d_potrf_inv_workspace(256) - 8, nullptr));
  EXPECT_ERR(gp2d_trtri(buf, 130, 130, nullptr, buf, 64, nullptr));
  EXPECT_ERR(gp2d_trtri(buf, 256, 256, nullptr, nullptr, 0, nullptr));
  EXPECT_ERR(gp2d_trtri(buf, 256, 256, nullptr, buf, gp2d_trtri_workspace(256) - 1, nullptr));
  EXPECT_ERR(gp2d_potrs_inv(buf, 100, 100, buf, buf, buf, 1 << 20, nullptr));
  EXPECT_ERR(gp2d_potrs_inv(buf, 128, 128, buf, buf, nullptr, 0, nullptr));
  // ---- predict (f64 engine)
  const size_t pw = gp2d_predict_workspace(256, 128, 2);
  EXPECT_ERR(gp2d_predict(buf, 256, 256, buf, buf, 64, 64, buf, 10, &df, 0, 0.0, 1, buf, buf, 128, buf, pw, nullptr)); // n ≠ 2·pad
  EXPECT_ERR(gp2d_predict(buf, 256, 256, buf, buf, 100, 128, buf, 10, &df, 0, 0.0, 1, buf, buf, 100, buf, pw, nullptr)); // chunk
  EXPECT_ERR(gp2d_predict(buf, 256, 256, buf, buf, 100, 128, buf, 10, &df, 0, 0.0, 1, buf, buf, 128, buf, pw - 8, nullptr));
  EXPECT_ERR(gp2d_predict(buf, 256, 256, buf, buf, 100, 128, buf, 10, &df, 5, 0.0, 1, buf, buf, 128, buf, pw, nullptr)); // var_mode
  EXPECT_ERR(gp2d_predict(buf, 256, 256, buf, buf, 100, 128, buf, 10, nullptr, 0, 0.0, 1, buf, buf, 128, buf, pw, nullptr));
  // ---- Ozaki engine
  int nmod = 0;
  int8_t* wb = reinterpret_cast<int8_t*>(buf);
  EXPECT_ERR(gp2d_ozaki_prepare(buf, 384, 384, &df, 0, 0, wb, buf, &nmod, nullptr));               // n not ×256
  EXPECT_ERR(gp2d_ozaki_prepare_async(buf, 384, 384, &df, 0.0025, 0, 0, wb, buf, &nmod, nullptr));
  gp2d_kernel_t mbad = mixed; mbad.ratio = 1.5;                                              // ratio ∉ [0, 1]
  EXPECT_ERR(gp2d_ozaki_prepare_async(buf, 256, 256, &mbad, 0.0025, 0, 0, wb, buf, &nmod, nullptr));
  mbad.ratio = -0.1;
  EXPECT_ERR(gp2d_ozaki_prepare(buf, 256, 256, &mbad, 0, 0, wb, buf, &nmod, nullptr));
  EXPECT_ERR(gp2d_ozaki_prepare_async(buf, 256, 256, &ard, 0.0025, 0, 0, wb, buf, &nmod, nullptr)); // vector only
  EXPECT(gp2d_ozaki_nmod_apriori(256, &mbad, 0.0025, 0, 0) < 0);
  EXPECT(gp2d_ozaki_nmod_apriori(256, &df, 0.0025, 61, 0) < 0 && gp2d_ozaki_nmod_apriori(256, &df, 0.0025, 48, 0) < 0);
  EXPECT(gp2d_ozaki_nmod_apriori(256, &df, 0.0025, 0, 51) < 0 && gp2d_ozaki_nmod_apriori(256, &df, 0.0025, 0, 44) < 0);
  EXPECT_ERR(gp2d_ozaki_prepare_async(buf, 256, 256, &df, 0.0025, 61, 0, wb, buf, &nmod, nullptr));  // wbits
  EXPECT_ERR(gp2d_ozaki_prepare_async(buf, 256, 256, &df, 0.0025, 0, 51, wb, buf, &nmod, nullptr));  // kbits
  EXPECT(gp2d_ozaki_nmod_apriori(8192, &df, 0.0025, 60, 50) > gp2d_ozaki_nmod_apriori(8192, &df, 0.0025, 49, 45));
  EXPECT(gp2d_ozaki_nmod_apriori(8192, &df, 0.0025, 60, 50) <= gp2d_ozaki_nmod(8192));   // the workspace covers it
  // the accuracy guard's policy (host arithmetic only)
  int gw = 0, gk = 0;   // the bench's own setting keeps the defaults; a hard one needs both raised
  EXPECT(gp2d_ozaki_guard_bits(0.04, 0.04 * 1.2e-3, 1e-10, &gw, &gk) == 1 && gw == 49 && gk == 45);
  EXPECT(gp2d_ozaki_guard_bits(0.04, 0.04 * 6e-5, 1e-10, &gw, &gk) == 1 && gw > 52 && gk > 45 && gw <= 60 && gk <= 50);
  EXPECT(gp2d_ozaki_guard_bits(0.04, 0.04 * 1e-7, 1e-10, &gw, &gk) == 0 && gp2d_ozaki_guard_bits(0.04, 0.0, 1e-10, &gw, &gk) == 0);
  EXPECT(gp2d_ozaki_guard_bits(0.04, 0.01, 0.0, &gw, &gk) == -1 && gp2d_ozaki_guard_bits(0.04, 0.01, 1e-10, nullptr, &gk) == -1);
  EXPECT(gp2d_ozaki_error_model(0.04, 0.001, 50, 45) < gp2d_ozaki_error_model(0.04, 0.001, 49, 45));
  EXPECT(gp2d_ozaki_error_model(0.04, 0.001, 49, 46) < gp2d_ozaki_error_model(0.04, 0.001, 49, 45));
  EXPECT(gp2d_ozaki_guard_workspace(8192) > 0 && gp2d_ozaki_guard_workspace(0) == 0);
  EXPECT_ERR(gp2d_ozaki_guard(buf, 256, 256, 200, 128, 0.0025, buf, buf, 16, nullptr));   // workspace
  EXPECT_ERR(gp2d_ozaki_guard(buf, 256, 256, 200, 128, 0.0025, buf, buf, 1 << 20, nullptr)); // ntr > npad
  EXPECT_ERR(gp2d_ozaki_guard(buf, 256, 256, 100, 128, INFINITY, buf, buf, 1 << 20, nullptr));  // diag_add
  const size_t ow = gp2d_predict_ozaki_workspace(256, 128);
  EXPECT_ERR(gp2d_predict_ozaki(wb, buf, 12, 0, 256, buf, buf, 100, 128, buf, 10, &df, 0, 0.0, 1, buf, buf, nullptr, 100, buf, ow, nullptr)); // chunk
  EXPECT_ERR(gp2d_predict_ozaki(wb, buf, 12, 0, 384, buf, buf, 100, 192, buf, 10, &df, 0, 0.0, 1, buf, buf, nullptr, 128, buf, ow, nullptr)); // n
  const size_t ow12 = gp2d_predict_ozaki_workspace_nmod(256, 128, 12);   // what a 12-moduli fit needs
  EXPECT(ow12 > 0 && ow12 <= ow && gp2d_predict_ozaki_workspace_nmod(256, 128, 0) == 0 &&
         gp2d_predict_ozaki_workspace_nmod(256, 128, 99) == 0 &&
         gp2d_predict_ozaki_workspace_nmod(256, 128, 11) < ow12);
  EXPECT_ERR(gp2d_predict_ozaki(wb, buf, 12, 0, 256, buf, buf, 100, 128, buf, 10, &df, 0, 0.0, 1, buf, buf, nullptr, 128, buf, ow12 - 8, nullptr));
  EXPECT_ERR(gp2d_predict_ozaki(wb, buf, 0, 0, 256, buf, buf, 100, 128, buf, 10, &df, 0, 0.0, 1, buf, buf, nullptr, 128, buf, ow, nullptr)); // nmod
  EXPECT_ERR(gp2d_predict_ozaki(wb, buf, 17, 0, 256, buf, buf, 100, 128, buf, 10, &df, 0, 0.0, 1, buf, buf, nullptr, 128, buf, ow, nullptr));
  EXPECT_ERR(gp2d_ozaki_kstar(buf, 100, 128, buf, 10, &df, 12, 0, 100, wb, 1 << 20, nullptr));     // chunk
  EXPECT_ERR(gp2d_ozaki_kstar(buf, 100, 128, buf, 10, &df, 12, 0, 128, wb, 16, nullptr));          // bres too small
  EXPECT_ERR(gp2d_morton_codes(buf, 10, 4, buf, nullptr, nullptr));                               // dim
  EXPECT_ERR(gp2d_ozaki_prepare_packed(buf, 200, &df, 0.0025, 0, 0, wb, buf, &nmod, nullptr));     // n not ×128
  EXPECT_ERR(gp2d_ozaki_prepare_packed(buf, 256, &df, 0.0025, 0, 0, wb, buf, nullptr, nullptr));  // nmod_out
  int64_t* ib = reinterpret_cast<int64_t*>(buf);
  const size_t sw = gp2d_morton_sort_workspace(100);
  EXPECT(sw > 0 && gp2d_morton_sort_workspace(0) == 0);
  EXPECT_ERR(gp2d_morton_sort(buf, 100, 1, buf, ib, buf, sw, nullptr));                          // dim
  EXPECT_ERR(gp2d_morton_sort(buf, 0, 2, buf, ib, buf, sw, nullptr));                            // n
  EXPECT_ERR(gp2d_morton_sort(buf, 100, 2, buf, ib, buf, sw - 8, nullptr));                      // workspace
  EXPECT_ERR(gp2d_morton_sort(buf, 100, 2, buf, nullptr, buf, sw, nullptr));                     // order
  EXPECT_ERR(gp2d_gather_rows(buf, ib, 10, 0, buf2, nullptr));                                   // dim
  EXPECT_ERR(gp2d_gather_rows(buf, ib, 10, 2, buf, nullptr));                                    // aliasing
  EXPECT_ERR(gp2d_obs_pad(buf, 70, 64, 2, nullptr, buf2, nullptr));                              // npad < ntr
  EXPECT_ERR(gp2d_obs_pad(buf, 10, 64, 3, nullptr, buf2, nullptr));                              // bd
  EXPECT_ERR(gp2d_status_flip(nullptr, 4, nullptr));
  EXPECT(gp2d_status_flip(reinterpret_cast<int*>(buf), 0, nullptr) == 0);                      // nothing to do
  // ---- likelihood, gradients, products
  EXPECT_ERR(gp2d_lml(buf, 100, 100, buf, buf, 10, buf, nullptr));
  EXPECT_ERR(gp2d_lml_grad(buf, 256, 256, buf, buf, 100, 128, &df, buf, nullptr, 0, nullptr));
  EXPECT_ERR(gp2d_kernel_grad(buf, 10, buf, 10, &df, buf, 19, buf, nullptr, 0, nullptr));
  EXPECT_ERR(gp2d_gemm(0, -1, 4, 4, 1.0, buf, 4, buf, 4, 0.0, buf, 4, nullptr));
  EXPECT_ERR(gp2d_gemm(2, 4, 4, 4, 1.0, buf, 4, buf, 4, 0.0, buf, 4, nullptr));
  EXPECT_ERR(gp2d_gemm(0, 4, 4, 4, 1.0, buf, 3, buf, 4, 0.0, buf, 4, nullptr));
  EXPECT_ERR(gp2d_transpose(buf, 100, 100, buf, nullptr));
  // ---- timing hooks (host state only)
  gp2d_timing_enable(1);
  double ms = -1, fl = -1;
  int64_t cnt = -1;
  EXPECT(gp2d_timing_read(&ms, &cnt, &fl) == 0 && cnt == 0 && ms == 0.0);
  // ---- factor broadcast: argument checks run before RCCL is resolved
  EXPECT(gp2d_bcast(nullptr, 0, 0, nullptr, nullptr) == 0);
  EXPECT_ERR(gp2d_bcast(buf, 8, 0, nullptr, nullptr));
  EXPECT_ERR(gp2d_bcast(buf, 8, -1, buf, nullptr));
  gp2d_timing_enable(0);
  gp2d_ozaki_set_skip(1);
  std::printf("%d checks, %d failed\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
