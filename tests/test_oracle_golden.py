"""Pin the CPU oracle (oracle/gp2d_oracle.py) against the reference's own outputs.

Golden vectors were produced by oracle/make_golden.py from the reference
(GP_scripts.py:1-142 exec'd, GP_laser.py recipe, krig.getGrid, sklearn).
Tolerances: kernel entries 1e-13 relative to the matrix max-norm; posterior
mean/var 1e-10 relative (north_star gate), measured normwise on each output.
Index work is bit-exact.
"""
import numpy as np
import pytest

from oracle import gp2d_oracle as O


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_compute_K_Ks_layout(golden, kind):
    g = golden("gp_scripts_small.npz")
    xa = np.stack([g["x1"], g["x2"]], 1)
    xb = np.stack([g["x1s"], g["x2s"]], 1)
    s = float(g["sigma"])
    K = O.vector_kernel(xa, xa, kind=kind, l_df=s, l_cf=s)
    Ks = O.vector_kernel(xb, xa, kind=kind, l_df=s, l_cf=s)
    assert rel_err(K, g[f"K_{kind}"]) < 1e-13
    assert rel_err(Ks, g[f"Ks_{kind}"]) < 1e-13
    assert np.allclose(np.full(2 * xb.shape[0], O.kernel_diag(kind, l_df=s, l_cf=s)), g[f"Kssdiag_{kind}"], rtol=1e-15, atol=0)


@pytest.mark.parametrize("kind", [0, 1, 2])
@pytest.mark.parametrize("method", ["inv", "chol"])
def test_small_posterior(golden, kind, method):
    g = golden("gp_scripts_small.npz")
    xa = np.stack([g["x1"], g["x2"]], 1)
    xb = np.stack([g["x1s"], g["x2s"]], 1)
    fit = O.OracleFit(xa, g["y"], kind, float(g["sigma"]), float(g["sigma"]), 1.0, float(g["noise"]),
                      method=method)
    mu, var = fit.predict(xb)
    M = xb.shape[0]
    assert rel_err(mu, g[f"mean_{kind}"]) < 1e-10
    assert rel_err(var[:M], g[f"uvar_{kind}"]) < 1e-10
    assert rel_err(var[M:], g[f"vvar_{kind}"]) < 1e-10


def test_vectorised_mykernel_mixed(golden):
    g = golden("gp_scripts_small.npz")
    xa = np.stack([g["x1"], g["x2"]], 1)
    xb = np.stack([g["x1s"], g["x2s"]], 1)
    l_df, l_cf, r = g["myK_params"]
    assert rel_err(O.vector_kernel(xa, xa, "mixed", l_df, l_cf, r), g["myK_mixed_aa"]) < 1e-14
    assert rel_err(O.vector_kernel(xa, xb, "mixed", l_df, l_cf, r), g["myK_mixed_ab"]) < 1e-14


@pytest.mark.parametrize("method", ["inv", "chol"])
def test_laser_recipe_mixed_N256(golden, method):
    g = golden("laser_mixed_N256.npz")
    # split indices reproduce the reference's CPython set order bit-exactly
    s, t = O.split_indices(int(g["n_raw"]), 3)
    assert np.array_equal(s, g["samples"]) and np.array_equal(t, g["test"])
    xo = np.stack([g["xo"], g["yo"]], 1)
    obs = np.concatenate([g["uo"], g["vo"]])
    x, y, Xs, Ys = O.laser_grid(g["xo"], g["yo"], g["xt"], g["yt"], dx=1.0)
    assert np.array_equal(x, g["x"]) and np.array_equal(y, g["y"])
    fit = O.OracleFit(xo, obs, "mixed", float(g["l_df"]), float(g["l_cf"]), float(g["rate"]),
                      float(g["noise"]), method=method)
    mu, var = fit.predict(np.stack([Xs, Ys], 1))
    M = Xs.size
    ny = y.size
    assert rel_err(mu[:M].reshape(ny, -1), g["uf"]) < 1e-10
    assert rel_err(mu[M:].reshape(ny, -1), g["vf"]) < 1e-10
    assert rel_err(var[:M].reshape(ny, -1), g["uvar"]) < 1e-10
    assert rel_err(var[M:].reshape(ny, -1), g["vvar"]) < 1e-10
    mt, _ = fit.predict(np.stack([g["xt"], g["yt"]], 1))
    Mt = g["xt"].size
    assert rel_err(mt[:Mt], g["uft"]) < 1e-10 and rel_err(mt[Mt:], g["vft"]) < 1e-10


@pytest.mark.parametrize("fixture,kind,ratio", [("mykernel_mixed_N1024.npz", "mixed", 0.5),
                                                ("mykernel_divfree_N1024.npz", "df", 1.0)])
def test_mykernel_N1024(golden, fixture, kind, ratio):
    g = golden(fixture)
    x = np.stack([g["x"], g["y"]], 1)
    obs = np.concatenate([g["u"], g["v"]])
    mu, var = O.fit_predict(x, obs, g["xg"], kind=kind, l_df=float(g["l_df"]), l_cf=5.0, ratio=ratio,
                            noise=float(g["noise"]))
    assert rel_err(mu, g["mean"]) < 1e-10
    assert rel_err(var, g["var"]) < 1e-10
    if "K_rows" in g.files:
        K = O.vector_kernel(x, x, kind, 5.0, 5.0, ratio)
        K[np.diag_indices_from(K)] += float(g["noise"])
        assert rel_err(K[g["K_rows_idx"]], g["K_rows"]) < 1e-14


def test_sklearn_config_A(golden):
    g = golden("sklearn_ard_N128.npz")
    HP = g["HP"]
    mean, std = O.ard_fit_predict(g["X"], g["u"], g["Xp"], [HP[0], HP[4]], [HP[1:4], HP[5:8]], HP[8])
    assert rel_err(mean, g["mean"]) < 1e-10
    assert rel_err(std, g["std"]) < 1e-10


def test_split_indices_bit_exact(golden):
    g = golden("split_indices.npz")
    for step in (2, 3, 5):
        for n in g["sizes"]:
            _, t = O.split_indices(int(n), step)
            assert np.array_equal(t, g[f"test_{step}_{n}"]), (step, n)


def test_get_grid_bit_exact(golden):
    g = golden("grids.npz")
    for i in range(int(g["ncases"])):
        X, tg, yg, xg = O.get_grid(g[f"c{i}_to"], g[f"c{i}_yo"], g[f"c{i}_xo"], float(g[f"c{i}_dt"]),
                                   float(g[f"c{i}_dx"]), float(g[f"c{i}_xL"]), float(g[f"c{i}_yL"]))
        assert np.array_equal(X, g[f"c{i}_X"]) and np.array_equal(tg, g[f"c{i}_tg"])
        assert np.array_equal(yg, g[f"c{i}_yg"]) and np.array_equal(xg, g[f"c{i}_xg"])


def test_known_answers():
    # k(x,x) = I/ℓ²; plots/Cov_divFree.png peaks at 25 = 1/0.2²
    K = O.vector_kernel([[0.3, -1.2]], [[0.3, -1.2]], "df", 0.2)
    assert np.allclose(K, np.eye(2) * 25.0, rtol=0, atol=1e-12)
    K = O.vector_kernel([[0.3, -1.2]], [[0.3, -1.2]], "cf", 0.2, 0.2)
    assert np.allclose(K, np.eye(2) * 25.0, rtol=0, atol=1e-12)
    # single observation at the origin, no noise: mean at origin = observation (GP_plots.py:457-484)
    for kind in ("df", "cf"):
        mu, var = O.fit_predict([[0.0, 0.0]], [1.0, 0.0], [[0.0, 0.0]], kind=kind, l_df=0.1, l_cf=0.1, noise=0.0,
                                method="inv")
        assert np.allclose(mu, [1.0, 0.0], atol=1e-12)
        assert np.allclose(var, 0.0, atol=1e-9)


# ------------------------------------------------------------------ LML
@pytest.mark.parametrize("name,kind", [("df", "df"), ("cf", "cf"), ("mixed", "mixed")])
def test_vector_lml_golden(golden, name, kind):
    """Oracle LML / gradient vs the fixture built on the reference's own myKernel
    (GP_scripts.py:6-42): value 1e-10 relative; gradient (both finite-difference based,
    4-point stencils) 1e-6 relative to the largest entry."""
    g = golden("lml_vector_N300.npz")
    x = np.stack([g["x"], g["y"]], 1)
    y = np.concatenate([g["u"], g["v"]])
    l_df, l_cf, rate, noise = g[f"{name}_params"]
    val, grad = O.vector_lml(x, y, kind=kind, l_df=l_df, l_cf=l_cf, ratio=rate, noise=noise, eval_gradient=True)
    assert abs(val - float(g[f"{name}_lml"])) <= 1e-10 * abs(float(g[f"{name}_lml"]))
    assert rel_err(grad, g[f"{name}_grad"]) < 1e-6


@pytest.mark.parametrize("T", [1, 2])
def test_ard_lml_sklearn(golden, T):
    """Oracle ARD LML / analytic gradient vs scikit-learn's log_marginal_likelihood
    (_gpr.py:584-650, alpha=1e-10 jitter) — value and gradient 1e-10 relative."""
    g = golden("lml_sklearn_ard_N128.npz")
    HP = g[f"T{T}_HP"]
    var = [HP[0]] + ([HP[4]] if T == 2 else [])
    ls = [tuple(HP[1:4])] + ([tuple(HP[5:8])] if T == 2 else [])
    val, grad = O.ard_lml(g["X"], g["u"], var, ls, HP[-1], jitter=1e-10, eval_gradient=True)
    assert abs(val - float(g[f"T{T}_lml"])) <= 1e-10 * abs(float(g[f"T{T}_lml"]))
    assert rel_err(grad, g[f"T{T}_grad"]) < 1e-10


def test_reference_gradient_quirk():
    """the reference's myKernel.update_gradients_full (myKernel.py:59-105) is not
    the derivative of myKernel.K — its length-scale entries disagree with finite differences,
    while its ratio entry agrees.  The build implements the exact derivative."""
    import scipy.linalg as sla
    rng = np.random.default_rng(5)
    n = 80
    x = np.stack([rng.uniform(0, 30, n), rng.uniform(0, 20, n)], 1)
    y = rng.normal(0, 1, 2 * n)
    kw = dict(kind="mixed", l_df=4.0, l_cf=6.0, ratio=0.3, noise=0.01)
    _, g = O.vector_lml(x, y, eval_gradient=True, **kw)
    K = O.vector_kernel(x, x, kind="mixed", l_df=4.0, l_cf=6.0, ratio=0.3) + 0.01 * np.eye(2 * n)
    L = np.linalg.cholesky(K)
    a = sla.cho_solve((L, True), y)
    dL_dK = 0.5 * (np.outer(a, a) - sla.cho_solve((L, True), np.eye(2 * n)))
    r_df, r_cf, r_ratio = O.reference_mykernel_gradient(x, dL_dK, 4.0, 6.0, 0.3)
    assert abs(r_ratio - g[2]) < 1e-6 * abs(g[2])
    assert abs(r_df - g[0]) > 1e-2 * abs(g[0])
    assert abs(r_cf - g[1]) > 1e-2 * abs(g[1])


# ------------------------------------------------------ spatio-temporal product (§8f.2)
@pytest.mark.parametrize("name,kind", [("df", "df"), ("mixed", "mixed")])
def test_st_product_golden(golden, name, kind):
    """Oracle Kt × vector kernel and its posterior vs the fixture built from the reference's
    myKernel (GP_scripts.py:6-42) times the GPy-RBF temporal factor (myKernel.py:347-355)."""
    g = golden("st_product_N150.npz")
    X = np.stack([g["t"], g["y"], g["x"]], 1)
    ldf, lcf, rate, var_t, l_t, noise = g[f"{name}_params"]
    kw = dict(kind=kind, l_df=ldf, l_cf=lcf, ratio=rate, var_t=var_t, l_t=l_t)
    K = O.vector_st_kernel(X, X, **kw) + noise * np.eye(2 * X.shape[0])
    N = X.shape[0]
    assert rel_err(K[[0, 1, N, 2 * N - 1]], g[f"{name}_K_rows"]) < 1e-13
    mean, var = O.st_fit_predict(X, g["obs"], g["G"], noise=noise, **kw)
    assert rel_err(mean, g[f"{name}_mean"]) < 1e-10
    assert rel_err(var, g[f"{name}_var"]) < 1e-10
