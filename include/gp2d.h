/*
 * gp2d.h — C ABI of libgp2d.so, the MI355X (gfx950) GP-kriging engine.
 *
 * Drop-in boundary for rafaelcgon/2D-GP's hot path.  Every
 * entry point below replaces one numpy/GPy/sklearn call of the reference;
 * the replaced call site is cited per function.  All array pointers are
 * caller-owned DEVICE buffers (e.g. torch-ROCm tensors' data_ptr()), fp64,
 * row-major.  `stream` is a hipStream_t passed as void* (NULL = default).
 * No function allocates device memory: callers size workspaces with the
 * *_workspace() queries.
 *
 * Return value: 0 on success; < 0 on an argument or HIP launch error
 * (gp2d_last_error() gives the message).  Numerical failure of the Cholesky
 * factorisation is reported LAPACK-style through *info_dev (device int):
 * 0 = success, k > 0 = the leading minor of order k is not positive definite.
 *
 * Layouts:
 *   points          (N, dim) row-major; dim = 2 for the vector kernels (x1, x2),
 *                   3 for VECTOR_ST (t, x1, x2), 1..3 for the scalar ARD family (T, Y, X order);
 *   vector kernels  component-major 2Np × 2Np: [[K_uu, K_uv], [K_vu, K_vv]]
 *                   (GP_scripts.py:89-95), Np = gp2d_padded_points(N);
 *   observations    y = [u_1..u_N, 0.., v_1..v_N, 0..] (2Np; GP_laser.py:98-99);
 *   predictions     mean/var = [u_1..u_M, v_1..v_M] (GP_laser.py:134-136).
 * Padded training points carry identity rows in K_y and zero cross-covariance,
 * so they change nothing.
 */
#ifndef GP2D_H
#define GP2D_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GP2D_ABI_VERSION 11

/* kernel families */
#define GP2D_FAMILY_VECTOR2D 0   /* 2×2 matrix-valued SE kernels on (x1, x2)          */
#define GP2D_FAMILY_ARD_RBF  1   /* scalar Σ var·exp(−½Σ_d (Δ_d/ls_d)²) (krig.py:174-180) */
#define GP2D_FAMILY_VECTOR_ST 2  /* spatio-temporal product Kt(t) × vector2d(y, x) on (T, Y, X) points:
                                    var[0]·exp(−Δt²/(2·ls[0][0]²)) times the 2×2 block of `kind`
                                    (scratch.py:506-508 kt * nonDivK; myKernel.py:337-360 Kt)    */

/* vector2d kinds — the reference's divFree flag (GP_scripts.py:57-69) */
#define GP2D_KIND_SCALAR   0     /* divFree=0: scalar SE broadcast into the 2×2 block  */
#define GP2D_KIND_DIVFREE  1     /* divFree=1 (nonDivK, myKernel.py:159-176)           */
#define GP2D_KIND_CURLFREE 2     /* divFree=2 (nonRotK, myKernel.py:255-271)           */
#define GP2D_KIND_MIXED    3     /* ratio·K_df + (1−ratio)·K_cf (myKernel.py:27-53)    */

/* predictive-variance conventions */
#define GP2D_VAR_LATENT  0       /* Kss − k*ᵀK_y⁻¹k* (GP_laser.py:128-131)             */
#define GP2D_VAR_NOISY   1       /* + likelihood noise (GPy model.predict)             */
#define GP2D_VAR_CLIPPED 2       /* + noise, negatives clipped to 0 (sklearn _gpr.py:473-485) */

typedef struct gp2d_kernel {
    int32_t family;      /* GP2D_FAMILY_*                                              */
    int32_t kind;        /* GP2D_KIND_* (vector2d)                                     */
    double  l_df;        /* div-free length scale (σ for KIND_SCALAR)                  */
    double  l_cf;        /* curl-free length scale                                     */
    double  ratio;       /* weight of the div-free part (myKernel `ratio`, GP_laser `rate`) */
    int32_t dim;         /* ARD: input dimension, 1..3                                 */
    int32_t nterms;      /* ARD: number of RBF terms, 1..2                             */
    double  var[2];      /* ARD: term variances; VECTOR_ST: var[0] = temporal variance */
    double  ls[2][3];    /* ARD: term length scales per dimension; VECTOR_ST: ls[0][0] = ℓ_t */
} gp2d_kernel_t;

/* ---- sizes ------------------------------------------------------------------- */
int     gp2d_abi_version(void);
const char* gp2d_build_info(void);   /* "release gfx950 abi=… oz_pw=… …": the build's tuning constants */
int64_t gp2d_padded_points(int64_t n);                 /* round up to the 64-point tile */
int     gp2d_block_dim(const gp2d_kernel_t* k);        /* 2 for vector2d, 1 for ARD      */
double  gp2d_kernel_diag(const gp2d_kernel_t* k);      /* k(x,x) per component: myKernel.Kdiag, myKernel.py:55-57 */

/* ---- covariance assembly -----------------------------------------------------
 * Replaces GP_scripts.myKernel (GP_scripts.py:6-42), compute_K / compute_Ks
 * (GP_scripts.py:74-123) and the GPy Kern.K methods (myKernel.py:27-53,
 * 159-176, 255-271).  out is (bd·nb_pad) × (bd·... ) with leading dim ld:
 * rows index xa's components, columns xb's.  diag_add (noise + jitter) is added
 * on the diagonal when xa == xb (GP_laser.py:114-115); padded rows/columns are
 * identity (when diag_add is used) or zero.
 * symmetric: 0 = cross-covariance K(xa, xb) (compute_Ks); 1 = K_y = K(x, x) + diag_add·I
 * in full (compute_K); 2 = K_y's lower triangle only (vector families: entries (R, C) with
 * C ≤ R, the rest left unwritten) — all gp2d_potrf uses, n(n+1)/2 stores instead of n² (the
 * fit's assembly; GP_scripts.py:80-88 also builds one triangle and mirrors it).    */
int gp2d_assemble(const double* xa, int64_t na, int64_t na_pad,
                  const double* xb, int64_t nb, int64_t nb_pad,
                  const gp2d_kernel_t* k, double diag_add, int symmetric,
                  double* out, int64_t ld, void* stream);

/* ---- fit ---------------------------------------------------------------------
 * gp2d_potrf: in-place lower Cholesky of the n×n SPD matrix A (n a multiple of
 * 128).  Replaces np.linalg.inv(K) (GP_laser.py:118, GP_scripts.py:50) and the
 * Cholesky inside GPy / sklearn (_gpr.py:349).  On return the strict upper
 * triangle is zero.  If dinv != NULL it receives the (n/128) inverted 128×128
 * diagonal blocks (input to gp2d_trtri).  *info_dev as LAPACK potrf (the call resets it to
 * 0 on `stream` first; the batched form resets all nprob words).
 * Concurrency: the factorisation runs on internal streams joined to `stream` at both
 * ends.  By default every call shares one set of internal streams per device;
 * gp2d_factor_sets(k) (k ≤ 4, returns the previous k) puts k sets in use — a caller
 * stream keeps the set it first drew — so factorisations issued on different caller
 * streams run concurrently, their latency-bound chains interleaved (engine.krige_jobs
 * fits_ahead).  Each set's enqueue is serialised by its own lock (thread-safe).
 * A call with k > 1 starts a new batch: the caller-stream → set map is cleared, so the
 * next k caller streams get sets 0..k−1 in order of first use.                       */
int gp2d_factor_sets(int k);
/* gp2d_factor_warm(k, stream): put one empty kernel on `stream` (the caller's predict stream),
 *   then create the current device's internal factor stream sets 0..k−1 and put one empty kernel
 *   on each of their streams.  HIP binds a stream to a hardware queue at its first command; on
 *   one MI355X a job stream ran 53.1–53.9 ms per headline job when its predict stream, then the
 *   factor streams, then its side streams were first used in that order, and 56.4–56.7 ms in the
 *   other orders measured (tools/probe_first_fit.py, DESIGN.md §6 "bench state").
 *   engine.warm_streams calls it once per device before any engine stream is used.            */
int gp2d_factor_warm(int nsets, void* stream);
/* gp2d_factor_set_of: the internal stream set `stream`'s factorisations currently draw
 * (0..k−1), or −1 if the stream has none in use (diagnostics and tests).            */
int gp2d_factor_set_of(void* stream);
/* gp2d_factor_join(1): this thread's later gp2d_potrf / gp2d_potrf_inv calls wait on the
 * host for the factorisation's chain before they enqueue the caller stream's join, so the
 * caller's hardware queue holds no pending wait while the chain runs (a pending wait there
 * slows the chain by up to 40 %).  For callers that block on the result
 * anyway (a synchronous fit, a job stream's first fit); 0 (default) keeps the calls
 * asynchronous.  A negative argument only queries; returns the previous mode.          */
int gp2d_factor_join(int host);
size_t gp2d_potrf_workspace(int64_t n);
int gp2d_potrf(double* A, int64_t n, int64_t lda, double* dinv, int* info_dev,
               void* work, size_t work_bytes, void* stream);

/* gp2d_trtri: in-place inverse of the lower-triangular L (L → W = L⁻¹), using the
 * diagonal-block inverses from gp2d_potrf (dinv) or computing them if NULL.     */
size_t gp2d_trtri_workspace(int64_t n);
int gp2d_trtri(double* A, int64_t n, int64_t lda, const double* dinv,
               void* work, size_t work_bytes, void* stream);

/* gp2d_potrf_inv: the fit's factor in one call — A (SPD, n a multiple of 128) is
 * replaced by W = L⁻¹ (lower, strict upper zero), the result of gp2d_potrf followed
 * by gp2d_trtri, with the inverse's GEMMs overlapped with the factorisation (each is
 * issued as soon as the block column that finalises its inputs is factored).
 * Replaces np.linalg.inv(K) (GP_laser.py:118) on the fit path.  dinv (n/128 blocks of
 * 128×128) receives the diagonal-block inverses; *info_dev as LAPACK potrf.        */
size_t gp2d_potrf_inv_workspace(int64_t n);
int gp2d_potrf_inv(double* A, int64_t n, int64_t lda, double* dinv, int* info_dev,
                   void* work, size_t work_bytes, void* stream);

/* gp2d_potrf_batched / gp2d_trtri_batched: nprob independent fits of one size in one
 * chain — problem q's SPD matrix at A + q·sA (sA ≥ n·lda elements), its diagonal-block
 * inverses at dinv + q·n·128, its info word at info_dev[q].  Each launch carries every
 * problem, so a sweep's settings (runKrig.py:14-17's hyperparameter table) or a job
 * stream's next fits pay the latency-bound diagonal chain once.  Problem q's results are
 * bit for bit those of gp2d_potrf / gp2d_trtri on it alone.  nprob ≤ 64.             */
int gp2d_potrf_batched(double* A, int64_t n, int64_t lda, int64_t sA, int nprob, double* dinv,
                       int* info_dev, void* stream);
size_t gp2d_trtri_batched_workspace(int64_t n, int nprob);
int gp2d_trtri_batched(double* A, int64_t n, int64_t lda, int64_t sA, int nprob, const double* dinv,
                       void* work, size_t work_bytes, void* stream);

/* gp2d_potrs_inv: alpha = Wᵀ (W y) = K_y⁻¹ y given W = L⁻¹.  Replaces
 * np.dot(Ki, y) (GP_scripts.py:45) / cho_solve (_gpr.py:360).                    */
size_t gp2d_potrs_workspace(int64_t n);
int gp2d_potrs_inv(const double* W, int64_t n, int64_t ldw, const double* y, double* alpha,
                   void* work, size_t work_bytes, void* stream);

/* ---- predict ------------------------------------------------------------------
 * Posterior mean and variance at m points.  Replaces compute_Ks + getMean +
 * the Kss − Ks·Ki·Ksᵀ diagonal (GP_laser.py:122-136), GPy model.predict
 * (krig.py:543-544) and sklearn predict(return_std=True) (_gpr.py:436-490).
 * W: n×n inverse Cholesky factor, n = bd·ntr_pad; alpha: n; xtr (ntr, dim);
 * xg (m, dim).  mean, var: bd·m outputs ([u..., v...] for vector2d).
 * var_mode: GP2D_VAR_*; noise is added for NOISY/CLIPPED.  The grid is
 * processed in chunks of `chunk` points (multiple of 64); the workspace
 * depends on (n, chunk).  Deterministic: no atomics, fixed reduction order, so
 * results do not depend on how the grid is sharded across GPUs.                  */
size_t gp2d_predict_workspace(int64_t n, int64_t chunk, int bd);
int gp2d_predict(const double* W, int64_t n, int64_t ldw, const double* alpha,
                 const double* xtr, int64_t ntr, int64_t ntr_pad,
                 const double* xg, int64_t m, const gp2d_kernel_t* k,
                 int var_mode, double noise, int compute_var,
                 double* mean, double* var, int64_t chunk,
                 void* work, size_t work_bytes, void* stream);

/* ---- predict, FP64-accurate variance on the INT8 matrix cores (Ozaki scheme II) -----
 * Same results contract as gp2d_predict (1e-10 relative parity gate) for the vector2d
 * family; the variance contraction ‖W k*‖² runs as nmod exact int8 GEMMs
 * (v_mfma_i32_16x16x64_i8) on residues modulo pairwise-coprime m_l ≤ 256, followed by
 * a Chinese-remainder reconstruction in fp64.  Requires n % 256 == 0.
 * gp2d_ozaki_prepare: once per fit, W → residue planes wres (≤ gp2d_ozaki_wres_bytes(n)
 * bytes) and per-row scales rowscale (n doubles); *nmod_out receives the number of moduli
 * the data needs (from per-row L1 bounds of the scaled W; synchronises the stream once).
 * wbits / kbits: integer bits per scaled W row, 0 (the default, 49) or 49..60, and of the scaled
 * K*, 0 (45) or 45..50 — the accuracy guard's choice (gp2d_ozaki_guard_bits; more bits cost about
 * one modulus per 8).  The row scales carry wbits; every later call that makes or reads K* planes
 * for this fit takes its kbits.  gp2d_ozaki_nmod(n) is the worst-case count (60 + 50 bits), used
 * for sizing.                                                                            */
int    gp2d_ozaki_nmod(int64_t n);
size_t gp2d_ozaki_wres_bytes(int64_t n);
int    gp2d_ozaki_prepare(const double* W, int64_t n, int64_t ldw, const gp2d_kernel_t* k, int wbits, int kbits,
                          int8_t* wres, double* rowscale, int* nmod_out, void* stream);
/* gp2d_ozaki_prepare_async: as gp2d_ozaki_prepare without the host round trip — the moduli
 * count is gp2d_ozaki_nmod_apriori(n, k, diag_add, wbits, kbits) (diag_add = the noise + jitter on K_y's
 * diagonal), which bounds the data-driven count for any fit of these hyperparameters.     */
int    gp2d_ozaki_prepare_async(const double* W, int64_t n, int64_t ldw, const gp2d_kernel_t* k,
                                double diag_add, int wbits, int kbits, int8_t* wres, double* rowscale,
                                int* nmod_out, void* stream);
/* gp2d_ozaki_prepare_packed: gp2d_ozaki_prepare_async reading W from the factor broadcast's
 * payload (gp2d_pack_lower's packed lower block triangle, gp2d_pack_lower_doubles(n) doubles):
 * a rank that receives a job's factor only to predict with the ozaki engine builds its planes
 * without unpacking W into an n×n matrix.  Same planes and row scales, bit for bit.          */
int    gp2d_ozaki_prepare_packed(const double* packed, int64_t n, const gp2d_kernel_t* k, double diag_add,
                                 int wbits, int kbits, int8_t* wres, double* rowscale, int* nmod_out, void* stream);
/* Accuracy guard.  The int8 engine rounds each W row to `wbits` integer bits and K* to `kbits`:
 * the variance kss − ‖W k*‖² then carries an elementwise relative error that grows where the
 * posterior variance is small against kss — at the observations.
 * gp2d_ozaki_guard: stats_dev[0] = the smallest latent posterior variance at the observed
 *   training components, δ − δ²·(K_y⁻¹)_ii with (K_y⁻¹)_ii = Σ_k W_ki² and δ = diag_add (the
 *   noise + jitter on K_y's diagonal; GP_laser.py:114-115; δ ≤ 0 gives stats_dev[0] ≤ 0, which the
 *   policy sends to the FP64 engine), stats_dev[1] = max |W_ik|
 *   (device doubles; workspace gp2d_ozaki_guard_workspace(n) bytes; fixed reduction order).
 * gp2d_ozaki_error_model: the modelled elementwise error A·2^(49 − wbits)·X^1.5 + B·2^(45 − kbits)·X,
 *   X = kss/v_min (A, B fitted to full-grid measurements).
 * gp2d_ozaki_guard_bits: the cheapest (*wbits, *kbits) (fewest total bits) whose modelled error is
 *   ≤ target (the north-star gate is 1e-10): returns 1; 0 if none (use the FP64 engine,
 *   gp2d_predict); −1 on bad input.
 * Replaces nothing in the reference (its variance is fp64 throughout, GP_laser.py:128-131): it
 * keeps the emulation inside the reference's accuracy contract for any hyperparameters.     */
size_t gp2d_ozaki_guard_workspace(int64_t n);
int    gp2d_ozaki_guard(const double* W, int64_t n, int64_t ldw, int64_t ntr, int64_t npad, double diag_add,
                        double* stats_dev, void* work, size_t work_bytes, void* stream);
double gp2d_ozaki_error_model(double kss, double vmin, int wbits, int kbits);
int    gp2d_ozaki_guard_bits(double kss, double vmin, double target, int* wbits, int* kbits);
size_t gp2d_predict_ozaki_workspace(int64_t n, int64_t chunk);
/* gp2d_predict_ozaki_workspace(n, chunk) and gp2d_predict_ozaki_planes_workspace(n, chunk) are
 * the worst case (the most moduli any W / K* precision can need at this n);
 * gp2d_predict_ozaki_workspace_nmod(n, chunk, nmod) is what either predict entry needs for a fit
 * prepared with nmod moduli (the entries check against that; 0 if nmod is out of range) — at
 * config D's n = 32,768 the worst case is 1.5× the 13 moduli the guard takes there.  Likewise the
 * residue planes of a fit take nmod·n² bytes of the gp2d_ozaki_wres_bytes(n) worst case (the
 * async preparations' nmod is gp2d_ozaki_nmod_apriori's, known before the call).          */
size_t gp2d_predict_ozaki_workspace_nmod(int64_t n, int64_t chunk, int nmod);
/* The variance GEMMs skip K slabs (64 training components) whose K* tile is exactly zero for
 * a 256-row grid tile — exact, such slabs add nothing.  gp2d_ozaki_set_skip(0) runs them
 * dense (A/B measurement and the bit-identity test); default on.                       */
void   gp2d_ozaki_set_skip(int on);
/* Z-order (Morton) codes of n points (dim 2 or 3) in their bounding box, 21 bits per
 * coordinate (bbox: 6 doubles of device scratch).  The ozaki engine sorts training and grid
 * points by these codes so that all-zero K* tiles cluster into skippable slabs.          */
int    gp2d_morton_codes(const double* pts, int64_t n, int dim, double* bbox, int64_t* codes, void* stream);
/* gp2d_morton_sort: the engine's point order — Morton codes, a stable LSD radix sort of them
 *   (8-bit digits; equal codes keep their input order, so the permutation is deterministic) into
 *   order[n] (int64: sorted point j is input point order[j]) and, if `sorted` is not NULL, the
 *   points gathered into that order (n × dim).  Workspace: gp2d_morton_sort_workspace(n) bytes.
 * gp2d_gather_rows: dst[j] = src[order[j]] for rows of `dim` doubles (no aliasing).
 * gp2d_obs_pad: a fit's observation vector — out[c·npad + i] = y[c·ntr + perm[i]] for i < ntr
 *   (perm NULL: the identity), 0 for the padded points; y is the reference's stacking
 *   [u_1..u_N, v_1..v_N] (GP_laser.py:98-99; krig.py:375-394 for bd = 2), out has bd·npad doubles.
 * There is no reference call these replace: the reference never reorders points;
 * they keep the ozaki engine's ordering off any framework kernel.                          */
size_t gp2d_morton_sort_workspace(int64_t n);
int    gp2d_morton_sort(const double* pts, int64_t n, int dim, double* sorted, int64_t* order, void* work,
                        size_t work_bytes, void* stream);
int    gp2d_gather_rows(const double* src, const int64_t* order, int64_t n, int64_t dim, double* dst,
                        void* stream);
int    gp2d_obs_pad(const double* y, int64_t ntr, int64_t npad, int bd, const int64_t* perm, double* out,
                    void* stream);
/* gp2d_predict_ozaki / _planes need n < 131072 (N_train < 65536): the int8 GEMM's biased
 * 32-bit sums must stay below 2^32 (the FP64 engine, gp2d_predict, has no such bound).
 * out_order (optional, int64[m]): xg is the caller's grid permuted (gp2d_morton_sort's sorted
 * points, so K*'s zero tiles cluster); the outputs of point j go to position out_order[j] of
 * mean / var — the caller's own order, scattered in the epilogue.  NULL: xg's order.      */
int    gp2d_predict_ozaki(const int8_t* wres, const double* rowscale, int nmod, int kbits, int64_t n,
                          const double* alpha, const double* xtr, int64_t ntr, int64_t ntr_pad,
                          const double* xg, int64_t m, const gp2d_kernel_t* k,
                          int var_mode, double noise, int compute_var,
                          double* mean, double* var, const int64_t* out_order, int64_t chunk,
                          void* work, size_t work_bytes, void* stream);
/* K* residue planes ahead of the fit.  The int8 residues of K* depend only on the training
 * points, the grid and the kernel, so they can be generated before / concurrently with the
 * fit (e.g. while a rank waits for the factor broadcast):
 * gp2d_ozaki_nmod_apriori: a moduli count that bounds gp2d_ozaki_prepare's data-driven one
 *   for any fit of this kernel with diagonal K_y,ii = kdiag + diag_add at W precision wbits
 *   (0 = default; −1 on bad input);
 * gp2d_ozaki_kstar: the planes of every chunk of the m grid points (per chunk: nmod planes
 *   of n·2·⌈chunk/256⌉·256 bytes, then the K* block flags the GEMMs' zero-slab skipping
 *   reads; size gp2d_ozaki_kstar_bytes);
 * gp2d_predict_ozaki_planes: gp2d_predict_ozaki (compute_var = 1) with the variance GEMMs
 *   reading those planes; the mean K*α is evaluated in fp64 as in gp2d_predict_ozaki, so
 *   both outputs are bit-identical to it.  Returns −3 if the fit needs more moduli than
 *   nmod_b, or another K* precision than the planes' kbits_b (the caller regenerates).
 * Replaces the same reference calls as gp2d_predict_ozaki (compute_Ks + getMean + the
 * variance diagonal, GP_laser.py:122-136).                                              */
int    gp2d_ozaki_nmod_apriori(int64_t n, const gp2d_kernel_t* k, double diag_add, int wbits, int kbits);
size_t gp2d_ozaki_kstar_bytes(int64_t n, int64_t m, int64_t chunk, int nmod);
int    gp2d_ozaki_kstar(const double* xtr, int64_t ntr, int64_t ntr_pad, const double* xg, int64_t m,
                        const gp2d_kernel_t* k, int nmod, int kbits, int64_t chunk, int8_t* bres,
                        size_t bres_bytes, void* stream);
size_t gp2d_predict_ozaki_planes_workspace(int64_t n, int64_t chunk);
int    gp2d_predict_ozaki_planes(const int8_t* wres, const double* rowscale, int nmod, int kbits, int64_t n,
                                 const double* alpha, const double* xtr, int64_t ntr, int64_t ntr_pad,
                                 const double* xg, int64_t m, const gp2d_kernel_t* k, int var_mode,
                                 double noise, const int8_t* bres, int nmod_b, int kbits_b, double* mean, double* var,
                                 const int64_t* out_order, int64_t chunk, void* work, size_t work_bytes,
                                 void* stream);

/* ---- hyperparameters: log marginal likelihood and its gradient -----
 * Replaces the objective of GPy model.optimize / optimize_restarts (krig.py:450,
 * GP_plots.py:673-765) and sklearn log_marginal_likelihood(theta, eval_gradient=True)
 * (_gpr.py:584-650), evaluated from a fit (W = L⁻¹, alpha = K_y⁻¹y, y the padded
 * observations of gp2d_potrs_inv):
 * gp2d_lml: *lml_dev (device double) = −½ yᵀα + Σ log W_ii − (nobs/2) log 2π,
 *   nobs = observed entries (bd·N).
 * gp2d_lml_grad: grad_dev (device, gp2d_lml_grad_count(k) doubles) = ½ tr((ααᵀ − K_y⁻¹) ∂K_y/∂θ)
 *   in natural units, θ = vector2d: (l_df, l_cf, ratio, noise) — entries a kind does not
 *   use are 0, KIND_SCALAR's σ is l_df; VECTOR_ST: (l_df, l_cf, ratio, var_t, l_t, noise); ARD, per term t: (var[t], ls[t][0..D)), then noise —
 *   GPy's param_array order (krig.py:459-466).
 *   K_y⁻¹ = WᵀW is formed in the workspace (gp2d_lml_grad_workspace(n) bytes, ≈ 2n² doubles).
 *   The reference's myKernel.update_gradients_full (myKernel.py:59-105) is not the
 *   derivative of its kernel; this is the exact one.                  */
int    gp2d_lml(const double* W, int64_t n, int64_t ldw, const double* alpha, const double* y,
                int64_t nobs, double* lml_dev, void* stream);
int    gp2d_lml_grad_count(const gp2d_kernel_t* k);
size_t gp2d_lml_grad_workspace(int64_t n);
int    gp2d_lml_grad(const double* W, int64_t n, int64_t ldw, const double* alpha,
                     const double* xtr, int64_t ntr, int64_t ntr_pad, const gp2d_kernel_t* k,
                     double* grad_dev, void* work, size_t work_bytes, void* stream);

/* gp2d_kernel_grad: the GPy Kern.update_gradients_full contraction (myKernel.py:59-105,
 * exact derivative): grad_dev[g] = Σ_ab dL_dK[a][b] · ∂K(xa, xb)_ab/∂θ_g for a caller-supplied
 * dL_dK (device, (bd·na) × (bd·nb) component-major WITHOUT padding — the reference layout —
 * leading dim ld).  θ as gp2d_lml_grad without the noise entry
 * (gp2d_kernel_grad_count(k) = gp2d_lml_grad_count(k) − 1 values).                      */
int    gp2d_kernel_grad_count(const gp2d_kernel_t* k);
size_t gp2d_kernel_grad_workspace(int64_t na, int64_t nb);
int    gp2d_kernel_grad(const double* xa, int64_t na, const double* xb, int64_t nb,
                        const gp2d_kernel_t* k, const double* dL_dK, int64_t ld,
                        double* grad_dev, void* work, size_t work_bytes, void* stream);

/* ---- dense helpers (the GP_scripts functional API on explicit matrices) ------------
 * gp2d_gemm: C = alpha·A·op(B) + beta·C on the FP64 MFMA GEMM core; op(B) = B (transb = 0,
 *   B is k×n) or Bᵀ (transb = 1, B is n×k); row-major; m, n multiples of 128, k of 16 (the
 *   Python layer pads).  Replaces the np.dot chains of GP_scripts.getMean (GP_scripts.py:44-46)
 *   and getCov (GP_scripts.py:48-54, Ks·Ki·Ksᵀ).
 * gp2d_transpose: At = Aᵀ for an n×n matrix (n a multiple of 64, At with leading dim n).
 *   Forms K⁻¹ = WᵀW from W = L⁻¹ in place of np.linalg.inv (GP_scripts.py:50).           */
int gp2d_gemm(int transb, int64_t m, int64_t n, int64_t k, double alpha, const double* A, int64_t lda,
              const double* B, int64_t ldb, double beta, double* C, int64_t ldc, void* stream);
int gp2d_transpose(const double* A, int64_t n, int64_t lda, double* At, void* stream);

/* ---- multi-GPU: one job's factor over P GPUs -----------
 * Replaces, for one large job, the single-GPU gp2d_potrf + gp2d_trtri pair (np.linalg.inv,
 * GP_laser.py:118; the factor of GPy's GPRegression inside krig.py:411 / :541-557, whose
 * D-sized grid the reference predicts slice by slice).  1-D block-cyclic over SB-column
 * super-blocks (SB = gp2d_dfact_sb() = 512): rank s mod P owns super-column s.  Every rank
 * holds the whole n×n K_y (n a multiple of SB, assembled by gp2d_assemble) and touches only
 * its own super-columns; the caller broadcasts one panel per step (any transport: RCCL,
 * gloo, gp2d_bcast).  Step s:
 *   owner of s:  gp2d_dfact_panel(A, n, lda, s, panel, info, work, ...)
 *                → panel = [D_s = L_ss⁻¹ (SB×SB, lower); L21 = L[(s+1)·SB.., s] ((n−s·SB−SB)×SB)],
 *                  row-major with leading dim SB, gp2d_dfact_panel_doubles(n) doubles at most;
 *                  *info_dev (device int) receives the global order of a non-PD minor (LAPACK style);
 *   broadcast the first (n − SB·s)·SB doubles of `panel` from rank s mod P;
 *   every rank:  gp2d_dfact_update(A, n, lda, s, panel, P, rank, t_lo, t_hi, ...)
 *                  POTRF trailing update (K = SB) of the owned super-columns t ∈ [max(t_lo, s+1), t_hi)
 *                  (the next owner updates t = s+1 first, a look-ahead);
 *                gp2d_dfact_invstep(A, n, lda, s, panel, P, rank, work, work_bytes, ...)
 *                  TRTRI step: the owned W columns J ≤ s (column block s reset to E_s first):
 *                  X[s] = D_s·R[s] and R[t > s] −= L21·X[s], both K = SB products; `work` as for
 *                  gp2d_dfact_panel (gp2d_dfact_workspace(n) bytes, ≈ SB·n doubles).
 * After the last step every owned super-column holds its columns of W = L⁻¹, zero above its
 * diagonal block.  Per-element arithmetic is independent of P (P = 2 gives the bits of P = 1).
 * gp2d_copy2d: dst[rows×cols] = src (leading dims in doubles; hipMemcpy2DAsync) — the panel and
 *   W-column packing of the caller.  gp2d_zero_upper: zero the strict upper triangle of A outside
 *   its 128×128 diagonal blocks.
 * gp2d_pack_lower: the factor broadcast's payload (any fit mode that sends W = L⁻¹): row block
 *   rb of the lower-triangular n×n W keeps columns [0, 128·(rb+1)), blocks stored one after the
 *   other (gp2d_pack_lower_doubles(n) = 128²·nb(nb+1)/2 doubles, ≈ n²/2); unpack = 1 writes them
 *   back (the rest of W is left as it is).                                                  */
int gp2d_dfact_sb(void);
size_t gp2d_dfact_panel_doubles(int64_t n);
size_t gp2d_dfact_workspace(int64_t n);
int gp2d_dfact_panel(double* A, int64_t n, int64_t lda, int s, double* panel, int* info_dev, void* work,
                     size_t work_bytes, void* stream);
int gp2d_dfact_update(double* A, int64_t n, int64_t lda, int s, const double* panel, int nranks, int rank,
                      int t_lo, int t_hi, void* stream);
int gp2d_dfact_invstep(double* A, int64_t n, int64_t lda, int s, const double* panel, int nranks, int rank,
                       void* work, size_t work_bytes, void* stream);
/* α = K_y⁻¹y = Wᵀ(W y) from the owned super-columns (each rank reads only its columns of W),
 * for the `count` super-columns t = t0 + q·dt in one launch each:
 * gp2d_dfact_zpart: zpart[q][i] = Σ_{k in super-column t, k ≤ i} W[i][k]·y[k] (count × n; 0 above
 *   the super-block); z = Σ_t zpart_t summed in t order by gp2d_dfact_zsum (gather every rank's
 *   partials first).
 * gp2d_dfact_alpha_blocks: alpha[q][c] = Σ_{i ≥ t·SB+c} W[i][t·SB+c]·z[i], c < SB (work:
 *   gp2d_dfact_alpha_workspace(n, count) bytes).  Both orders are fixed, so any P gives the bits
 *   of P = 1.
 * gp2d_assemble_cols: columns [c0, c0+ncols) of the symmetric K_y = K(x, x) + diag_add·I (vector
 *   families; c0, ncols multiples of 64, inside one component) — the same arithmetic as
 *   gp2d_assemble(symmetric = 1); a rank of the distributed factor assembles only its columns.  */
int gp2d_dfact_zpart(const double* W, int64_t n, int64_t ldw, int t0, int dt, int count, const double* y,
                     double* zpart, void* stream);
int gp2d_dfact_zsum(const double* parts, int nparts, int64_t n, double* z, void* stream);  /* z = Σ parts[p] in p order */
size_t gp2d_dfact_alpha_workspace(int64_t n, int count);
int gp2d_dfact_alpha_blocks(const double* W, int64_t n, int64_t ldw, int t0, int dt, int count, const double* z,
                            double* alpha, void* work, size_t work_bytes, void* stream);
int gp2d_assemble_cols(const double* x, int64_t n, int64_t n_pad, const gp2d_kernel_t* k, double diag_add,
                       double* out, int64_t ld, int64_t c0, int64_t ncols, void* stream);
int gp2d_copy2d(double* dst, int64_t ldd, const double* src, int64_t lds, int64_t rows, int64_t cols,
                void* stream);
int gp2d_zero_upper(double* A, int64_t n, int64_t lda, void* stream);
size_t gp2d_pack_lower_doubles(int64_t n);
int gp2d_pack_lower(double* W, int64_t n, int64_t ldw, double* packed, int unpack, void* stream);

/* ---- multi-GPU: the library's own RCCL communicator ----------------
 * The reference is single-process; its parallelism is the job array runKrig.py:7,14-17 and the
 * per-slice predict krig.py:541-557.  These entries carry the multi-GPU data path over RCCL on
 * xGMI — a job's packed factor W = L⁻¹ + α + training points (gp2d/distributed.py
 * broadcast_fit), the distributed factor's panels, its W column all-gather and its status
 * all-reduce — on a communicator the library creates, driven on the caller's HIP stream.  RCCL
 * is resolved at first call (no link-time dependency); every entry returns −100 − ncclResult_t
 * on an RCCL failure.
 * gp2d_comm_id_bytes / gp2d_comm_unique_id: the ncclUniqueId (128 bytes) rank 0 makes and the
 *   caller hands to every rank over its own host channel (the Python layer: torch.distributed's
 *   TCP store).
 * gp2d_comm_init: ncclCommInitRank on HIP device `device` (−1: the current one); collective over
 *   the nranks processes.  gp2d_comm_destroy frees it; gp2d_comm_size reads (nranks, rank).
 * gp2d_bcast: in-place ncclBroadcast of `bytes` bytes from rank `root` (any communicator of the
 *   resolved RCCL, including the caller's own).
 * gp2d_allgather: ncclAllGather of bytes_per_rank bytes per rank, rank order.
 * gp2d_allreduce: in-place ncclAllReduce of `count` INT32 / FLOAT64 values, op SUM / MAX / MIN.
 * gp2d_sendrecv: one grouped ncclSend (send → send_peer) + ncclRecv (recv ← recv_peer) of
 *   `bytes` bytes; either pointer may be NULL; a rank may name itself (an RCCL copy kernel).
 * gp2d_stream_create_cumask: a HIP stream whose kernels use only the CUs of mask bits
 *   [first, first + count) (hipExtStreamCreateWithCUMask; the driver deals the bits over the
 *   XCDs, bit i → XCD i mod 8) — e.g. a communication stream on a few CUs of every XCD beside a
 *   predict stream on the rest; gp2d_stream_destroy.                                        */
enum { GP2D_COMM_INT32 = 2, GP2D_COMM_FLOAT64 = 8 };
enum { GP2D_COMM_SUM = 0, GP2D_COMM_MAX = 1, GP2D_COMM_MIN = 2 };
size_t gp2d_comm_id_bytes(void);
int gp2d_comm_unique_id(void* id);
int gp2d_comm_init(void** comm, int nranks, const void* id, int rank, int device);
int gp2d_comm_destroy(void* comm);
int gp2d_comm_size(void* comm, int* nranks, int* rank);
int gp2d_bcast(void* buf, size_t bytes, int root, void* comm, void* stream);
int gp2d_allgather(const void* send, void* recv, size_t bytes_per_rank, void* comm, void* stream);
int gp2d_allreduce(void* buf, size_t count, int dtype, int op, void* comm, void* stream);
int gp2d_sendrecv(const void* send, int send_peer, void* recv, int recv_peer, size_t bytes, void* comm,
                  void* stream);
int gp2d_stream_create_cumask(int first, int count, void** stream);
int gp2d_stream_destroy(void* stream);
/* gp2d_status_flip: 0 ↔ INT32_MAX on `count` device status words (an involution).  Applied
 *   before and after an all-reduce MIN of LAPACK-style info words (0 = success, k > 0 = first
 *   non-PD minor), it makes the reduction return the FIRST failing minor over the ranks, or 0 —
 *   the one-rank answer (the distributed factor's status, gp2d/distributed.py).              */
int gp2d_status_flip(int* status, int count, void* stream);

/* ---- instrumentation ------------------------------------------------------------
 * When enabled, every launch of the predict variance kernel (the dominant
 * kernel) is bracketed by hipEvents on its stream; gp2d_timing_read()
 * synchronises those events and returns the summed milliseconds, the launch
 * count and the summed algorithmic flop count, then resets the counters.        */
void gp2d_timing_enable(int on);
/* gp2d_trace_mark: one empty kernel (trace_mark_kernel) on `stream` — a marker a rocprofv3 kernel
 * trace shows, so a tool can list the kernels that ran between two of them (bench.py's timed
 * region, GP2D_TRACE_MARKS=1).                                                              */
int  gp2d_trace_mark(int tag, void* stream);
int  gp2d_timing_read(double* total_ms, int64_t* launches, double* flops);

const char* gp2d_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* GP2D_H */
