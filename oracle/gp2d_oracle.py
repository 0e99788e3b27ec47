"""CPU oracle (numpy restatement) of rafaelcgon/2D-GP's GP-kriging hot path.

TEST INFRASTRUCTURE ONLY.  This module is the checker for the HIP path and the
``cpu_baseline`` leg of ``bench.py``.  The product package never imports it.

Parity status: PINNED.  ``tests/test_oracle_golden.py`` checks every function
here against golden vectors in ``tests/golden/``.  ``oracle/make_golden.py``
made those vectors by exec'ing the reference's own ``GP_scripts.py:1-142``
(``myKernel``, ``nonDivK``, ``compute_K``, ``compute_Ks``, ``getMean``,
``getCov``), by running the reference's numpy expressions verbatim (split
indices, grids), and by running scikit-learn (config A, the
``krig.scikit_prior`` recipe).

Conventions:
  * points are (N, 2) arrays of (x1, x2) in km;
  * vector-kernel matrices are component-major, i.e. ``[[K_uu, K_uv], [K_vu, K_vv]]``
    with N×N blocks (GP_scripts.py:89-95, :117-122);
  * observations are ``y = [u_1..u_N, v_1..v_N]`` (GP_laser.py:98-99);
  * predictions are ``f[:M]`` = u and ``f[M:]`` = v (GP_laser.py:134-136).
"""
from __future__ import annotations

import numpy as np

KIND_SCALAR, KIND_DIVFREE, KIND_CURLFREE, KIND_MIXED = 0, 1, 2, 3

_KIND_NAMES = {"scalar": KIND_SCALAR, "isotropic": KIND_SCALAR, "sq": KIND_SCALAR,
               "df": KIND_DIVFREE, "divfree": KIND_DIVFREE, "div-free": KIND_DIVFREE,
               "cf": KIND_CURLFREE, "curlfree": KIND_CURLFREE, "curl-free": KIND_CURLFREE,
               "mixed": KIND_MIXED}


def kind_code(kind) -> int:
    if isinstance(kind, str):
        return _KIND_NAMES[kind.lower()]
    return int(kind)


def _block_terms(d1, d2, length, which):
    """Entries (k11, k12, k22) of one 2×2 SE vector-kernel block.

    div-free  : (1/ℓ²)·exp(−r²/2ℓ²)·[d dᵀ/ℓ² + ((p−1) − r²/ℓ²)·I]  GP_scripts.py:26-28,40 ; :63-64,69
    curl-free : (1/ℓ²)·exp(−r²/2ℓ²)·[I − d dᵀ/ℓ²]                    GP_scripts.py:32-33,41 ; :65-66
    scalar    : (1/σ²)·exp(−r²/2σ²)·σ² (same value in all 4 entries)  GP_scripts.py:67-69 with the
                2×2 broadcast that compute_K does at GP_scripts.py:84.
    """
    l2 = np.square(length)
    c = (np.square(d1) + np.square(d2)) / l2
    e = np.square(1.0 / length) * np.exp(-c / 2.0)
    if which == KIND_DIVFREE:
        aux = 1.0 - c  # (p-1) - C with p = 2
        return e * (d1 * d1 / l2 + aux), e * (d1 * d2 / l2), e * (d2 * d2 / l2 + aux)
    if which == KIND_CURLFREE:
        return e * (1.0 - d1 * d1 / l2), -e * (d1 * d2 / l2), e * (1.0 - d2 * d2 / l2)
    if which == KIND_SCALAR:
        s = e * l2
        return s, s, s
    raise ValueError(which)


def vector_kernel(xa, xb, kind=KIND_DIVFREE, l_df=1.0, l_cf=1.0, ratio=1.0):
    """Component-major (2Na, 2Nb) cross-covariance K(xa, xb).

    Vectorised restatement of GP_scripts.myKernel (GP_scripts.py:6-42) and the
    GPy plugin myKernel.K (myKernel.py:27-53); for kind=scalar it follows
    compute_K/compute_Ks with divFree=0 (GP_scripts.py:74-123), which broadcasts
    the scalar SE value into all four entries of each 2×2 block.
    For kind=mixed the result is ratio·K_df(l_df) + (1−ratio)·K_cf(l_cf)
    (GP_scripts.py:42; GP_laser.py:113,122).  kind=df uses l_df, kind=cf uses
    l_cf, kind=scalar uses l_df as σ.
    """
    kind = kind_code(kind)
    xa = np.asarray(xa, dtype=np.float64).reshape(-1, 2)
    xb = np.asarray(xb, dtype=np.float64).reshape(-1, 2)
    d1 = xa[:, 0][:, None] - xb[:, 0]
    d2 = xa[:, 1][:, None] - xb[:, 1]
    if kind == KIND_MIXED:
        a11, a12, a22 = _block_terms(d1, d2, l_df, KIND_DIVFREE)
        b11, b12, b22 = _block_terms(d1, d2, l_cf, KIND_CURLFREE)
        k11 = ratio * a11 + (1 - ratio) * b11
        k12 = ratio * a12 + (1 - ratio) * b12
        k22 = ratio * a22 + (1 - ratio) * b22
    else:
        length = l_cf if kind == KIND_CURLFREE else l_df
        k11, k12, k22 = _block_terms(d1, d2, length, kind)
    return np.block([[k11, k12], [k12, k22]])


def kernel_diag(kind=KIND_DIVFREE, l_df=1.0, l_cf=1.0, ratio=1.0):
    """k(x, x) on the u (or v) diagonal: myKernel.Kdiag (myKernel.py:55-57), nonDivK.Kdiag
    (:178-180), nonRotK.Kdiag (:273-275).  For scalar it is (1/σ²)·σ² (GP_scripts.py:67-69)."""
    kind = kind_code(kind)
    if kind == KIND_MIXED:
        return ratio * (1.0 / l_df ** 2) + (1 - ratio) * (1.0 / l_cf ** 2)
    if kind == KIND_SCALAR:
        return np.square(1.0 / l_df) * np.square(l_df)
    if kind == KIND_CURLFREE:
        return 1.0 / l_cf ** 2
    return 1.0 / l_df ** 2


def vector_kernel_chunked(xa, xb, chunk=2048, **kw):
    """Same as vector_kernel but bounded memory for large Nb (yields column chunks)."""
    xb = np.asarray(xb, dtype=np.float64).reshape(-1, 2)
    for s in range(0, xb.shape[0], chunk):
        yield s, vector_kernel(xa, xb[s:s + chunk], **kw)


# --------------------------------------------------------------------------------------
# Fit and predict (GP_laser.py:113-140; sklearn _gpr.py:345-365, 436-490)
# --------------------------------------------------------------------------------------
class OracleFit:
    def __init__(self, x, y, kind, l_df, l_cf, ratio, noise, method="chol", jitter=0.0):
        import scipy.linalg as sla
        self.x = np.asarray(x, dtype=np.float64).reshape(-1, 2)
        self.kw = dict(kind=kind_code(kind), l_df=l_df, l_cf=l_cf, ratio=ratio)
        self.noise = float(noise)
        n = 2 * self.x.shape[0]
        K = vector_kernel(self.x, self.x, **self.kw)
        K[np.diag_indices(n)] += self.noise + jitter          # GP_laser.py:114-115
        self.method = method
        y = np.asarray(y, dtype=np.float64).reshape(-1)
        if method == "inv":                                   # GP_laser.py:118, GP_scripts.py:44-46
            self.Ki = np.linalg.inv(K)
            self.alpha = self.Ki @ y
        else:                                                 # _gpr.py:349-360 (cho_solve)
            self.L = np.linalg.cholesky(K)
            self.alpha = sla.cho_solve((self.L, True), y)

    def predict(self, xg, var_mode="latent", chunk=2048):
        """mean (2M,) = [u; v]; var (2M,) = [uvar; vvar].

        var_mode: 'latent'  — Kss − K* K_y⁻¹ K*ᵀ diagonal (GP_laser.py:128-131)
                  'gpy'     — latent + likelihood noise (GPy model.predict default)
                  'sklearn' — latent + noise, negatives clipped to 0 (_gpr.py:473-485)
        """
        import scipy.linalg as sla
        xg = np.asarray(xg, dtype=np.float64).reshape(-1, 2)
        M = xg.shape[0]
        kss = kernel_diag(**self.kw)
        mu = np.empty(2 * M)
        var = np.empty(2 * M)
        for s in range(0, M, chunk):
            e = min(M, s + chunk)
            Ks = vector_kernel(xg[s:e], self.x, **self.kw)       # (2m, 2N), GP_laser.py:122
            f = Ks @ self.alpha                                  # GP_scripts.py:45
            m = e - s
            mu[s:e], mu[M + s:M + e] = f[:m], f[m:]
            if self.method == "inv":
                q = np.einsum("ij,ij->i", Ks, Ks @ self.Ki)      # diag(Ks Ki Ksᵀ), GP_laser.py:129
            else:
                V = sla.solve_triangular(self.L, Ks.T, lower=True)   # _gpr.py:454
                q = np.einsum("ij,ij->j", V, V)
            v = kss - q
            if var_mode in ("gpy", "sklearn"):
                v = v + self.noise
            if var_mode == "sklearn":
                v = np.where(v < 0, 0.0, v)
            var[s:e], var[M + s:M + e] = v[:m], v[m:]
        return mu, var


def fit_predict(x, y, xg, kind="df", l_df=5.0, l_cf=5.0, ratio=1.0, noise=0.0025,
                method="chol", var_mode="latent", chunk=2048):
    fit = OracleFit(x, y, kind, l_df, l_cf, ratio, noise, method=method)
    return fit.predict(xg, var_mode=var_mode, chunk=chunk)


# --------------------------------------------------------------------------------------
# Scalar ARD-RBF (+RBF) + White GP — the krig.scikit_prior recipe (krig.py:174-194), config A
# --------------------------------------------------------------------------------------
def ard_rbf(xa, xb, variances, lengthscales):
    xa = np.atleast_2d(np.asarray(xa, dtype=np.float64))
    xb = np.atleast_2d(np.asarray(xb, dtype=np.float64))
    K = np.zeros((xa.shape[0], xb.shape[0]))
    for v, ls in zip(variances, lengthscales):
        ls = np.asarray(ls, dtype=np.float64)
        a = xa / ls
        b = xb / ls
        d2 = (np.sum(a * a, 1)[:, None] + np.sum(b * b, 1)[None, :]) - 2 * a @ b.T
        d2 = np.maximum(d2, 0.0)
        K += v * np.exp(-0.5 * d2)
    return K


def ard_rbf_exact(xa, xb, variances, lengthscales):
    """Difference-based ARD RBF (no ‖a‖²+‖b‖²−2ab cancellation), the form the HIP kernel uses."""
    xa = np.atleast_2d(np.asarray(xa, dtype=np.float64))
    xb = np.atleast_2d(np.asarray(xb, dtype=np.float64))
    K = np.zeros((xa.shape[0], xb.shape[0]))
    for v, ls in zip(variances, lengthscales):
        d2 = np.zeros_like(K)
        for d in range(xa.shape[1]):
            t = (xa[:, d][:, None] - xb[:, d][None, :]) / ls[d]
            d2 += t * t
        K += v * np.exp(-0.5 * d2)
    return K


def ard_fit_predict(X, y, Xg, variances, lengthscales, noise, jitter=1e-10):
    """sklearn GaussianProcessRegressor(kernel=Σ v·RBF(ls) + White(noise), optimizer=None)
    fit (_gpr.py:345-365, alpha=1e-10 jitter) and predict(return_std=True) (_gpr.py:436-490)."""
    import scipy.linalg as sla
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    K = ard_rbf_exact(X, X, variances, lengthscales)
    K[np.diag_indices_from(K)] += noise + jitter
    L = np.linalg.cholesky(K)
    alpha = sla.cho_solve((L, True), y)
    Ks = ard_rbf_exact(Xg, X, variances, lengthscales)
    mean = Ks @ alpha
    V = sla.solve_triangular(L, Ks.T, lower=True)
    var = float(np.sum(variances)) + noise - np.einsum("ij,ij->j", V, V)
    var = np.where(var < 0, 0.0, var)
    return mean, np.sqrt(var)


# --------------------------------------------------------------------------------------
# Spatio-temporal product kernel
# --------------------------------------------------------------------------------------
def vector_st_kernel(xa, xb, kind=KIND_DIVFREE, l_df=1.0, l_cf=1.0, ratio=1.0, var_t=1.0, l_t=1.0):
    """Kt(var_t, l_t) × vector kernel on (T, Y, X) rows: GPy's product `kt * nonDivK(2, [1, 2], ℓ)`
    (scratch.py:506-508) with Kt.K = the GPy RBF on t broadcast into all four blocks
    (myKernel.py:347-355); the product is elementwise (GPy Prod).  Components follow the
    spatial coordinate order (Y, X), i.e. obs = [v; u] (krig.py:390)."""
    xa = np.asarray(xa, dtype=np.float64).reshape(-1, 3)
    xb = np.asarray(xb, dtype=np.float64).reshape(-1, 3)
    C = var_t * np.exp(-0.5 * np.square(xa[:, 0][:, None] - xb[:, 0][None, :]) / l_t ** 2)
    K = vector_kernel(xa[:, 1:], xb[:, 1:], kind=kind, l_df=l_df, l_cf=l_cf, ratio=ratio)
    return K * np.block([[C, C], [C, C]])


def st_fit_predict(x, y, xg, kind="df", l_df=5.0, l_cf=5.0, ratio=1.0, var_t=1.0, l_t=1.0, noise=0.0025,
                   var_mode="latent"):
    """Posterior mean / variance of the spatio-temporal GP (Cholesky; GP_laser.py:113-131 recipe)."""
    import scipy.linalg as sla
    kw = dict(kind=kind_code(kind), l_df=l_df, l_cf=l_cf, ratio=ratio, var_t=var_t, l_t=l_t)
    K = vector_st_kernel(x, x, **kw)
    K[np.diag_indices_from(K)] += noise
    L = np.linalg.cholesky(K)
    alpha = sla.cho_solve((L, True), np.asarray(y, dtype=np.float64).reshape(-1))
    xg = np.asarray(xg, dtype=np.float64).reshape(-1, 3)
    M = xg.shape[0]
    Ks = vector_st_kernel(xg, x, **kw)
    f = Ks @ alpha
    V = sla.solve_triangular(L, Ks.T, lower=True)
    kss = var_t * kernel_diag(kind_code(kind), l_df=l_df, l_cf=l_cf, ratio=ratio)
    v = kss - np.einsum("ij,ij->j", V, V)
    if var_mode in ("gpy", "sklearn"):
        v = v + noise
    if var_mode == "sklearn":
        v = np.where(v < 0, 0.0, v)
    return f, v


def vector_st_lml(x, y, kind="df", l_df=5.0, l_cf=5.0, ratio=1.0, var_t=1.0, l_t=1.0, noise=0.0025,
                  eval_gradient=False, rel_step=1e-4):
    """LML of the spatio-temporal GP; gradient (l_df, l_cf, ratio, var_t, l_t, noise) as in
    vector_lml (4-point stencil on the kernel matrix, ∂/∂noise = I)."""
    kw = dict(kind=kind, l_df=l_df, l_cf=l_cf, ratio=ratio, var_t=var_t, l_t=l_t)
    K = vector_st_kernel(x, x, **kw)
    K[np.diag_indices_from(K)] += noise
    val, L, alpha = lml_from_K(K, y)
    if not eval_gradient:
        return val
    code = kind_code(kind)
    uses = {KIND_SCALAR: ("l_df",), KIND_DIVFREE: ("l_df",), KIND_CURLFREE: ("l_cf",),
            KIND_MIXED: ("l_df", "l_cf", "ratio")}[code] + ("var_t", "l_t")
    names = ("l_df", "l_cf", "ratio", "var_t", "l_t")
    g = np.zeros(6)
    for i, name in enumerate(names):
        if name not in uses:
            continue
        h = rel_step * (abs(kw[name]) if name != "ratio" else 1.0)
        Ks = []
        for t in (-2, -1, 1, 2):
            k2 = dict(kw)
            k2[name] = kw[name] + t * h
            Ks.append(vector_st_kernel(x, x, **k2))
        g[i] = _trace_grad(L, alpha, (Ks[0] - 8 * Ks[1] + 8 * Ks[2] - Ks[3]) / (12 * h))
    g[5] = _trace_grad(L, alpha, np.eye(K.shape[0]))
    return val, g


# --------------------------------------------------------------------------------------
# Log marginal likelihood and its gradient
# --------------------------------------------------------------------------------------
def lml_from_K(K, y):
    """−½ yᵀK⁻¹y − Σ log L_ii − (n/2) log 2π via Cholesky (sklearn _gpr.py:612-628; GPy
    ExactGaussianInference, the objective of model.optimize at krig.py:450)."""
    import scipy.linalg as sla
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    L = np.linalg.cholesky(K)
    alpha = sla.cho_solve((L, True), y)
    return -0.5 * y @ alpha - np.sum(np.log(np.diag(L))) - 0.5 * y.size * np.log(2 * np.pi), L, alpha


def _trace_grad(L, alpha, dK):
    """½ tr((ααᵀ − K⁻¹) dK) (sklearn _gpr.py:631-642)."""
    import scipy.linalg as sla
    Ki = sla.cho_solve((L, True), np.eye(L.shape[0]))
    return 0.5 * np.einsum("ij,ji->", np.outer(alpha, alpha) - Ki, dK)


VECTOR_PARAMS = ("l_df", "l_cf", "ratio", "noise")


def vector_lml(x, y, kind="df", l_df=5.0, l_cf=5.0, ratio=1.0, noise=0.0025, jitter=0.0,
               eval_gradient=False, rel_step=1e-4):
    """LML of the vector-kernel GP (K_y = vector_kernel + (noise+jitter)·I).

    The gradient (l_df, l_cf, ratio, noise) differentiates the kernel MATRIX numerically —
    a 4-point central stencil on vector_kernel, independent of the HIP kernel's closed-form
    derivative — and contracts it as ½ tr((ααᵀ − K_y⁻¹) ∂K). Parameters a kind does not use
    get 0 (scalar kind: σ = l_df).  ∂K_y/∂noise = I."""
    x = np.asarray(x, dtype=np.float64).reshape(-1, 2)
    kw = dict(kind=kind, l_df=l_df, l_cf=l_cf, ratio=ratio)
    K = vector_kernel(x, x, **kw)
    K[np.diag_indices_from(K)] += noise + jitter
    val, L, alpha = lml_from_K(K, y)
    if not eval_gradient:
        return val
    code = kind_code(kind)
    uses = {KIND_SCALAR: ("l_df",), KIND_DIVFREE: ("l_df",), KIND_CURLFREE: ("l_cf",),
            KIND_MIXED: ("l_df", "l_cf", "ratio")}[code]
    g = np.zeros(4)
    for i, name in enumerate(VECTOR_PARAMS[:3]):
        if name not in uses:
            continue
        h = rel_step * (abs(kw[name]) if name != "ratio" else 1.0)
        Ks = []
        for t in (-2, -1, 1, 2):
            k2 = dict(kw)
            k2[name] = kw[name] + t * h
            Ks.append(vector_kernel(x, x, **k2))
        dK = (Ks[0] - 8 * Ks[1] + 8 * Ks[2] - Ks[3]) / (12 * h)
        g[i] = _trace_grad(L, alpha, dK)
    g[3] = _trace_grad(L, alpha, np.eye(K.shape[0]))
    return val, g


def ard_lml(X, y, variances, lengthscales, noise, jitter=0.0, eval_gradient=False):
    """LML of Σ_t var_t·RBF(ls_t) + White(noise) (the krig.scikit_prior model, krig.py:174-180)
    with the analytic gradient in GPy's param_array order: per term (var_t, ls_t[0..D)), then
    noise.  ∂k/∂var_t = e_t, ∂k/∂ls_td = var_t·e_t·Δ_d²/ls_td³ (sklearn kernels.RBF.__call__
    gradient, divided by ls to leave log-space)."""
    X = np.atleast_2d(np.asarray(X, dtype=np.float64))
    K = ard_rbf_exact(X, X, variances, lengthscales)
    K[np.diag_indices_from(K)] += noise + jitter
    val, L, alpha = lml_from_K(K, y)
    if not eval_gradient:
        return val
    g = []
    for v, ls in zip(variances, lengthscales):
        e = ard_rbf_exact(X, X, [1.0], [ls])
        g.append(_trace_grad(L, alpha, e))
        for d in range(X.shape[1]):
            D2 = np.square(X[:, d][:, None] - X[:, d][None, :])
            g.append(_trace_grad(L, alpha, v * e * D2 / ls[d] ** 3))
    g.append(_trace_grad(L, alpha, np.eye(K.shape[0])))
    return val, np.array(g)


def reference_mykernel_gradient(x, dL_dK, l_df, l_cf, ratio):
    """The reference's myKernel.update_gradients_full (myKernel.py:59-105), restated to document
    SURVEY.md §0.2's quirk: its l_df / l_cf entries are NOT the derivative of myKernel.K
    (myKernel.py:27-53) — the A·(2ℓ²−Cℓ²)/ℓ⁵ term has the opposite sign and dA/dℓ lacks
    the 1/ℓ² factor.  Its ratio entry is right.  Returns (g_ldf, g_lcf, g_ratio)."""
    x = np.asarray(x, dtype=np.float64).reshape(-1, 2)
    d1 = x[:, 0][:, None] - x[:, 0]
    d2 = x[:, 1][:, None] - x[:, 1]
    B11, B12, B22 = d1 * d1, d1 * d2, d2 * d2
    r2 = B11 + B22

    def blk(a, b, c):
        return np.block([[a, b], [b, c]])

    ld2 = l_df ** 2
    Cd = r2 / ld2
    Ad = blk(B11 / ld2 + 1 - Cd, B12 / ld2, B22 / ld2 + 1 - Cd)
    dAd = (2 / l_df ** 3) * blk(r2 - B11, -B12, r2 - B22)
    Cd4 = blk(Cd, Cd, Cd)
    g_df = ratio * np.exp(-Cd4 / 2) * (dAd + Ad * (2 * ld2 - Cd4 * ld2) / l_df ** 5)
    lc2 = l_cf ** 2
    Cc = r2 / lc2
    Ac = blk(1 - B11 / lc2, -B12 / lc2, 1 - B22 / lc2)
    dAc = (2 / l_cf ** 3) * blk(B11, B12, B22)
    Cc4 = blk(Cc, Cc, Cc)
    g_cf = (1 - ratio) * np.exp(-Cc4 / 2) * (dAc + Ac * (2 * lc2 - Cc4 * lc2) / l_cf ** 5)
    dr = np.exp(-Cd4 / 2) * Ad / ld2 - np.exp(-Cc4 / 2) * Ac / lc2
    return np.sum(g_df * dL_dK), np.sum(g_cf * dL_dK), np.sum(dr * dL_dK)


# --------------------------------------------------------------------------------------
# Index / grid work (bit-exact)
# --------------------------------------------------------------------------------------
def split_indices(n, step):
    """Train/test split of GP_laser.py:80-83 and krig.py:335-337:
    samples = arange(0, n, step); test = np.array(list(set(arange(n)) - set(samples))).
    The test order is CPython's set iteration order, reproduced by doing the same
    set arithmetic (hash(np.int64(k)) == hash(k))."""
    samples = np.arange(0, n, step)
    test = set(range(n)) - set(range(0, n, step))
    return samples, np.array(list(test), dtype=np.int64)


def laser_grid(xo, yo, xt, yt, dx=0.5, pad=5.0):
    """GP_laser.py:102-109: x = arange(min−5, max+5, dx) over obs ∪ test; meshgrid(x, y)
    flattened row-major (point p = iy·nx + ix)."""
    x = np.arange(np.min([xo.min(), xt.min()]) - pad, np.max([xo.max(), xt.max()]) + pad, dx)
    y = np.arange(np.min([yo.min(), yt.min()]) - pad, np.max([yo.max(), yt.max()]) + pad, dx)
    X, Y = np.meshgrid(x, y)
    return x, y, np.reshape(X, [X.size]), np.reshape(Y, [Y.size])


def get_grid(to, yo, xo, dt=0.5, dx=0.5, xL=40, yL=40):
    """krig.getGrid (krig.py:648-678): window clip, arange extents, meshgrid(yg, tg, xg)
    flattened T-major then Y then X; returns (X (M,3) in T,Y,X order, tg, yg, xg)."""
    if (np.max(xo) - np.min(xo)) > xL:
        xmin = np.mean(xo) - xL / 2
        xmax = np.mean(xo) + xL / 2
    else:
        xmin = np.min(xo) - dx
        xmax = np.max(xo) + dx
    if (np.max(yo) - np.min(yo)) > yL:
        ymin = np.mean(yo) - yL / 2
        ymax = np.mean(yo) + yL / 2
    else:
        ymin = np.min(yo) - dx
        ymax = np.max(yo) + dx
    xg = np.arange(xmin, xmax, dx)
    yg = np.arange(ymin, ymax, dx)
    tg = np.arange(np.min(to), np.max(to), dt)
    Yg, Tg, Xg = np.meshgrid(yg, tg, xg)
    X = np.concatenate([np.reshape(Tg, [Tg.size, 1]), np.reshape(Yg, [Yg.size, 1]),
                        np.reshape(Xg, [Xg.size, 1])], axis=1)
    return X, tg, yg, xg
