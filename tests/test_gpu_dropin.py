"""The drop-in surfaces through the HIP engine: the GP_scripts functional module
(GP_scripts.py:1-142) replayed on the reference's own call sequences, and Krig checkpoints
restored without a refit (krig.py:478-483).

Tolerances: covariance entries 1e-13 relative to the matrix max-norm; posterior mean /
variance 1e-10 relative (normwise per output vector, north_star)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

import GP_scripts as GS  # noqa: E402
import krig  # noqa: E402
from gp2d import engine as E  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def test_functional_kernels_golden(golden):
    g = golden("gp_scripts_small.npz")
    s = float(g["sigma"])
    for kind in (0, 1, 2):
        assert rel(GS.compute_K(g["x1"], g["x2"], s, kind), g[f"K_{kind}"]) < 1e-13
        assert rel(GS.compute_Ks(g["x1"], g["x2"], g["x1s"], g["x2s"], s, kind), g[f"Ks_{kind}"]) < 1e-13
    xa = np.stack([g["x1"], g["x2"]], 1)
    xb = np.stack([g["x1s"], g["x2s"]], 1)
    l_df, l_cf, r = g["myK_params"]
    assert rel(GS.myKernel(xa, xa, l_df, l_cf, r), g["myK_mixed_aa"]) < 1e-13
    assert rel(GS.myKernel(xa, xb, l_df, l_cf, r), g["myK_mixed_ab"]) < 1e-13
    # one 2×2 block and the scalar case of nonDivK (GP_scripts.py:57-69)
    K1 = g["K_1"]
    n = g["x1"].size
    blk = GS.nonDivK(np.array([g["x1"][0], g["x2"][0]]), np.array([g["x1"][3], g["x2"][3]]), s, 1)
    ref = np.array([[K1[0, 3], K1[0, n + 3]], [K1[n, 3], K1[n, n + 3]]])
    assert np.allclose(blk, ref, rtol=1e-13, atol=1e-16)
    sc = GS.nonDivK(np.array([g["x1"][0], g["x2"][0]]), np.array([g["x1"][3], g["x2"][3]]), s, 0)
    assert np.isscalar(sc) or np.ndim(sc) == 0
    assert abs(float(sc) - g["K_0"][0, 3]) <= 1e-15


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_getmean_replays_laser_sequence(golden, kind):
    """The caller-side sequence of GP_laser.py:113-134 on the module: K (+noise·I), Ki, Ks,
    getMean(Ks, Ki, obs), Cov = Kss − Ks·Ki·Ksᵀ — Ki by the caller's own np.linalg.inv."""
    g = golden("gp_scripts_small.npz")
    s, noise = float(g["sigma"]), float(g["noise"])
    K = GS.compute_K(g["x1"], g["x2"], s, kind)
    K = K + np.identity(K.shape[0]) * noise
    Ki = np.linalg.inv(K)
    Ks = GS.compute_Ks(g["x1"], g["x2"], g["x1s"], g["x2s"], s, kind)
    f = GS.getMean(Ks, Ki, g["y"][:, None])
    assert f.shape == g[f"mean_{kind}"].shape
    assert rel(f, g[f"mean_{kind}"]) < 1e-10


@pytest.mark.parametrize("kind", [1, 2])
def test_getcov_golden(golden, kind):
    """Noise-free getCov (GP_scripts.py:48-54): diag(ML), Ki·K = I, Ks."""
    g = golden("gp_scripts_small.npz")
    s = float(g["sigma"])
    ML, Ki, Ks = GS.getCov(g["x1"], g["x2"], g["x1s"], g["x2s"], s, kind)
    M = g["x1s"].size
    assert ML.shape == (2 * M, 2 * M) and np.allclose(ML, ML.T, rtol=0, atol=1e-12 * np.abs(ML).max())
    K = g[f"K_{kind}"]
    assert rel(Ks, g[f"Ks_{kind}"]) < 1e-13
    # the noise-free K is ill-conditioned: compare Ki through its defining identity and
    # diag(ML) at the accuracy its condition number allows (both sides are fp64 inverses)
    cond = np.linalg.cond(K)
    assert np.max(np.abs(Ki @ K - np.eye(K.shape[0]))) < 1e-15 * cond * 10
    assert rel(np.diag(ML), g[f"getCov_diag_{kind}"]) < max(1e-10, 1e-15 * cond)


def test_getcov_non_pd_raises():
    x = np.array([0.0, 0.0, 1.0])
    y = np.array([0.0, 0.0, 1.0])   # a repeated point: K is singular without noise
    # sigma = 0.5 makes K_ii = 1/sigma^2 = 4 a perfect square, so the second pivot is
    # 4 - (4/2)^2 = 0 exactly (with another sigma it rounds to a tiny value of either sign)
    with pytest.raises(np.linalg.LinAlgError):
        GS.getCov(x, y, x, y, 0.5, 1)


def test_laser_recipe_through_module(golden):
    """GP_laser.py:113-136 verbatim in structure, with every kernel and product on the GPU
    module and the caller's own np.linalg.inv, against the exec'd-reference fixture."""
    g = golden("laser_mixed_N256.npz")
    xo, yo, uo, vo = g["xo"], g["yo"], g["uo"], g["vo"]
    l_df, l_cf, rate, noise = (float(g[k]) for k in ("l_df", "l_cf", "rate", "noise"))
    X, Y = np.meshgrid(g["x"], g["y"])
    Xs, Ys = X.reshape(X.size), Y.reshape(Y.size)
    obs = np.concatenate([uo, vo]).reshape(-1, 1)
    K = rate * GS.compute_K(xo, yo, l_df, 1) + (1 - rate) * GS.compute_K(xo, yo, l_cf, 2)
    K = K + np.identity(K.shape[0]) * noise
    Ki = np.linalg.inv(K)
    Ks = rate * GS.compute_Ks(xo, yo, Xs, Ys, l_df, 1) + (1 - rate) * GS.compute_Ks(xo, yo, Xs, Ys, l_cf, 2)
    Kst = rate * GS.compute_Ks(xo, yo, g["xt"], g["yt"], l_df, 1) + \
        (1 - rate) * GS.compute_Ks(xo, yo, g["xt"], g["yt"], l_cf, 2)
    Kss = rate * GS.compute_K(Xs, Ys, l_df, 1) + (1 - rate) * GS.compute_K(Xs, Ys, l_cf, 2)
    KiKsT = E.gemm(Ki, Ks, transb=True)
    Cov = E.gemm(Ks, KiKsT, alpha=-1.0, C=Kss, beta=1.0).cpu().numpy()   # Kss − Ks·Ki·Ksᵀ
    ny = g["y"].size
    uvar = np.reshape(np.diag(Cov[:X.size, :X.size]), [ny, -1])
    vvar = np.reshape(np.diag(Cov[X.size:, X.size:]), [ny, -1])
    f = GS.getMean(Ks, Ki, obs)
    ft = GS.getMean(Kst, Ki, obs)
    half = f.size // 2
    assert rel(np.reshape(f[:half], [ny, -1]), g["uf"]) < 1e-10
    assert rel(np.reshape(f[half:], [ny, -1]), g["vf"]) < 1e-10
    assert rel(ft[:ft.size // 2], g["uft"]) < 1e-10 and rel(ft[ft.size // 2:], g["vft"]) < 1e-10
    assert rel(uvar, g["uvar"]) < 1e-10 and rel(vvar, g["vvar"]) < 1e-10


def test_rbf_and_sqexp():
    rng = np.random.default_rng(3)
    x1, x2 = rng.uniform(0, 5, 40), rng.uniform(0, 5, 40)
    K = GS.rbf(x1, x2, l=1.3, sigma=0.8, noise=0.01)
    ref = 0.8 ** 2 * np.exp(-np.square(x2[None, :] - x1[:, None]) / (2 * 1.3 ** 2)) + np.identity(40) * 0.01
    assert rel(K, ref) < 1e-14
    a, b, c, d = (rng.uniform(0, 5, k) for k in (7, 7, 11, 11))
    S = GS.sqExp(a, b, c, d, 0.9)
    R = np.exp(-((a[:, None] - c[None, :]) ** 2 + (b[:, None] - d[None, :]) ** 2) / (2 * 0.81))
    assert S.shape == (7, 11) and rel(S, R) < 1e-14


@pytest.mark.parametrize("m,n,k,transb", [(1, 1, 1, False), (130, 257, 33, True), (300, 1, 513, False)])
def test_gemm_any_shape(m, n, k, transb):
    rng = np.random.default_rng(m + n + k)
    A = rng.normal(size=(m, k))
    B = rng.normal(size=(n, k) if transb else (k, n))
    C = rng.normal(size=(m, n))
    out = E.gemm(A, B, transb=transb, alpha=-0.5, C=C, beta=2.0).cpu().numpy()
    ref = -0.5 * A @ (B.T if transb else B) + 2.0 * C
    assert np.max(np.abs(out - ref)) < 1e-13 * max(1.0, np.abs(ref).max()) * np.sqrt(k)


@pytest.mark.parametrize("variance", ["f64", "ozaki"])
def test_krig_checkpoint_restores_without_refit(tmp_path, variance, monkeypatch):
    rng = np.random.default_rng(11)
    x = np.stack([rng.uniform(0, 30, 300), rng.uniform(0, 20, 300)], 1)
    y = np.concatenate([np.sin(x[:, 1] / 5), np.cos(x[:, 0] / 6)]) + rng.normal(0, 0.05, 600)
    xg = np.stack([rng.uniform(-2, 32, 700), rng.uniform(-2, 22, 700)], 1)
    k = krig.Krig("mixed", l_df=4.0, l_cf=3.0, ratio=0.6, noise=0.0025, variance=variance).fit(x, y)
    mu, var = k.predict(xg)
    p = str(tmp_path / "model.npz")
    k.save(p, with_factor=True)

    def no_fit(*a, **kw):
        raise AssertionError("Krig.load refitted a checkpoint that carries the factor")
    monkeypatch.setattr(E, "fit", no_fit)
    k2 = krig.Krig.load(p)
    assert k2.variance == variance
    mu2, var2 = k2.predict(xg)
    assert np.array_equal(mu, mu2) and np.array_equal(var, var2)
    assert k2.log_likelihood() == pytest.approx(k.log_likelihood(), rel=1e-13)


@pytest.mark.parametrize("variance", ["f64", "ozaki"])
def test_krig_checkpoint_of_jitchol_rescued_fit(tmp_path, variance, monkeypatch):
    """A fit that needed GPy's jitchol jitter (repeated points, no noise), saved with its factor
    and loaded: bit-identical predictions (the Ozaki planes take the moduli count of the jittered
    diagonal); saved without the factor, the refit keeps the jitchol setting and succeeds."""
    rng = np.random.default_rng(4)
    x = rng.uniform(0, 20, (60, 2))
    x = np.concatenate([x, x[:5]])
    y = rng.normal(size=2 * x.shape[0])
    xg = rng.uniform(0, 20, (300, 2))
    k = krig.Krig("df", l_df=3.0, noise=0.0, variance=variance, jitchol=5).fit(x, y)
    used = k.gp.extra["jitchol"]
    assert used > 0
    mu, var = k.predict(xg)
    p, q = str(tmp_path / "model.npz"), str(tmp_path / "model_nofactor.npz")
    k.save(p, with_factor=True)
    k.save(q)
    k3 = krig.Krig.load(q)   # refit from the inputs: needs jitchol again
    assert k3.jitchol == 5 and k3.gp.extra["jitchol"] == used
    mu3, var3 = k3.predict(xg)
    assert np.array_equal(mu, mu3) and np.array_equal(var, var3, equal_nan=True)

    def no_fit(*a, **kw):
        raise AssertionError("Krig.load refitted a checkpoint that carries the factor")
    monkeypatch.setattr(E, "fit", no_fit)
    k2 = krig.Krig.load(p)
    assert k2.gp.extra["jitchol"] == used
    if variance == "ozaki":   # the reload reaches the guard's decision again (here: jitter, no noise)
        assert k2.gp.extra["guard"]["engine"] == k.gp.extra["guard"]["engine"]
        assert k2.gp.extra["guard"]["wbits"] == k.gp.extra["guard"]["wbits"]
        assert k2.gp.extra["guard"]["kbits"] == k.gp.extra["guard"]["kbits"]
        if "ozaki" in k.gp.extra:
            assert k2.gp.extra["ozaki"][2] == k.gp.extra["ozaki"][2]
    mu2, var2 = k2.predict(xg)
    assert np.array_equal(mu, mu2) and np.array_equal(var, var2, equal_nan=True)
