"""Spatio-temporal product kernel Kt × vector kernel on (T, Y, X),
through the C ABI (family GP2D_FAMILY_VECTOR_ST).

Tolerances: kernel entries 1e-13 relative to the matrix max-norm; posterior mean / variance
1e-10 relative normwise (the north_star gate) for both variance engines; LML 1e-10 relative,
gradient 1e-6 relative to the finite-difference oracle.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from gp2d import engine as E  # noqa: E402
from gp2d import hyper as H  # noqa: E402
from oracle import gp2d_oracle as O  # noqa: E402


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def st_tracks(n, seed=5):
    rng = np.random.default_rng(seed)
    X = np.stack([rng.uniform(0, 6, n), rng.uniform(0, 45, n), rng.uniform(0, 60, n)], 1)
    v = np.cos(X[:, 2] / 9) + 0.1 * X[:, 0] + rng.normal(0, 0.05, n)
    u = np.sin(X[:, 1] / 7) - 0.05 * X[:, 0] + rng.normal(0, 0.05, n)
    return X, np.concatenate([v, u])


def spec(kind, ratio, var_t=2.0, l_t=1.5, l_df=5.0, l_cf=4.0):
    return E.KernelSpec(family="vector_st", kind=kind, l_df=l_df, l_cf=l_cf, ratio=ratio, var_t=var_t, l_t=l_t)


@pytest.mark.parametrize("kind,ratio", [("df", 1.0), ("cf", 0.0), ("mixed", 0.3), ("scalar", 1.0)])
@pytest.mark.parametrize("na,nb", [(1, 1), (37, 100), (130, 64)])
def test_st_assemble(kind, ratio, na, nb):
    rng = np.random.default_rng(na + 7 * nb)
    xa = np.stack([rng.uniform(0, 3, na), rng.uniform(0, 10, na), rng.uniform(0, 10, na)], 1)
    xb = np.stack([rng.uniform(0, 3, nb), rng.uniform(0, 10, nb), rng.uniform(0, 10, nb)], 1)
    ks = spec(kind, ratio, l_df=2.5, l_cf=3.5)
    K = E.assemble(ks, xa, xb).cpu().numpy()
    ref = O.vector_st_kernel(xa, xb, kind=kind, l_df=2.5, l_cf=3.5, ratio=ratio, var_t=2.0, l_t=1.5)
    assert rel(K, ref) < 1e-13
    assert ks.kdiag() == pytest.approx(2.0 * O.kernel_diag(O.kind_code(kind), l_df=2.5, l_cf=3.5, ratio=ratio),
                                       rel=1e-15)


@pytest.mark.parametrize("name", ["df", "mixed"])
@pytest.mark.parametrize("engine", ["f64", "ozaki"])
def test_st_golden_posterior(golden, name, engine):
    g = golden("st_product_N150.npz")
    X = np.stack([g["t"], g["y"], g["x"]], 1)
    ldf, lcf, rate, var_t, l_t, noise = (float(v) for v in g[f"{name}_params"])
    ks = E.KernelSpec(family="vector_st", kind=name, l_df=ldf, l_cf=lcf, ratio=rate, var_t=var_t, l_t=l_t)
    gp = E.fit(ks, X, g["obs"], noise, variance=engine)
    mu, var = E.predict(gp, g["G"])
    assert rel(mu.cpu().numpy(), g[f"{name}_mean"]) < 1e-10
    assert rel(var.cpu().numpy(), g[f"{name}_var"]) < 1e-10


@pytest.mark.parametrize("kind,ratio", [("df", 1.0), ("cf", 0.0), ("mixed", 0.35)])
@pytest.mark.parametrize("n", [300, 1000])
def test_st_fit_predict_vs_oracle(kind, ratio, n):
    X, y = st_tracks(n, seed=n)
    rng = np.random.default_rng(1)
    G = np.stack([rng.uniform(-1, 7, 700), rng.uniform(-5, 50, 700), rng.uniform(-5, 65, 700)], 1)
    ks = spec(kind, ratio)
    mo, vo = O.st_fit_predict(X, y, G, kind=kind, l_df=5.0, l_cf=4.0, ratio=ratio, var_t=2.0, l_t=1.5, noise=0.01)
    for engine in ("f64", "ozaki"):
        gp = E.fit(ks, X, y, 0.01, variance=engine)
        mu, var = E.predict(gp, G, chunk=256)
        assert rel(mu.cpu().numpy(), mo) < 1e-10, engine
        assert rel(var.cpu().numpy(), vo) < 1e-10, engine


@pytest.mark.parametrize("kind,ratio", [("df", 1.0), ("mixed", 0.35), ("cf", 0.0)])
def test_st_lml_grad(kind, ratio):
    X, y = st_tracks(300, seed=12)
    ks = spec(kind, ratio)
    gp = E.fit(ks, X, y, 0.01)
    val, grad = E.log_marginal_likelihood(gp, eval_gradient=True)
    oval, og = O.vector_st_lml(X, y, kind=kind, l_df=5.0, l_cf=4.0, ratio=ratio, var_t=2.0, l_t=1.5, noise=0.01,
                               eval_gradient=True)
    assert E.param_names(ks) == ("l_df", "l_cf", "ratio", "var_t", "l_t", "noise")
    assert abs(val - oval) <= 1e-10 * abs(oval)
    assert rel(grad, og) < 1e-6, (grad, og)


def test_st_kernel_grad_dense():
    rng = np.random.default_rng(3)
    xa = np.stack([rng.uniform(0, 3, 40), rng.uniform(0, 10, 40), rng.uniform(0, 10, 40)], 1)
    xb = np.stack([rng.uniform(0, 3, 90), rng.uniform(0, 10, 90), rng.uniform(0, 10, 90)], 1)
    G = rng.normal(0, 1, (80, 180))
    kw = dict(kind="mixed", l_df=3.0, l_cf=4.0, ratio=0.35, var_t=2.0, l_t=1.5)
    g = E.kernel_grad(spec("mixed", 0.35, l_df=3.0, l_cf=4.0), xa, G, xb)
    ref = []
    for name in ("l_df", "l_cf", "ratio", "var_t", "l_t"):
        h = 1e-4 * (kw[name] if name != "ratio" else 1.0)
        Ks = []
        for t in (-2, -1, 1, 2):
            k2 = dict(kw)
            k2[name] += t * h
            Ks.append(O.vector_st_kernel(xa, xb, **k2))
        ref.append(np.sum(G * (Ks[0] - 8 * Ks[1] + 8 * Ks[2] - Ks[3]) / (12 * h)))
    assert rel(g, ref) < 1e-7


def test_st_optimize_improves():
    X, y = st_tracks(200, seed=4)
    ks = spec("df", 1.0, var_t=1.0, l_t=1.0)
    start = E.log_marginal_likelihood(E.fit(ks, X, y, 0.02))
    res = H.optimize(ks, X, y, 0.02, maxiter=60)
    assert res.lml > start
    gp = E.fit(res.kernel, X, y, res.noise)
    assert E.log_marginal_likelihood(gp) == pytest.approx(res.lml, rel=1e-12)
