"""Log marginal likelihood + gradient on the GPU, through the C ABI.

Tolerances: LML value 1e-10 relative (fp64; the same gate as mean / variance).
Gradients: 1e-6 relative to the largest entry against finite-difference references
(the golden fixture built on the reference's myKernel, the oracle's 4-point stencil on
the kernel matrix), 1e-9 against scikit-learn's analytic ARD gradient, 1e-10 against
the oracle's analytic ARD contraction.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from gp2d import engine as E  # noqa: E402
from gp2d import hyper as H  # noqa: E402
from gp2d import kern, krig  # noqa: E402
from oracle import gp2d_oracle as O  # noqa: E402


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def tracks(n, seed=2016):
    rng = np.random.default_rng(seed)
    x = np.stack([rng.uniform(0, 60, n), rng.uniform(0, 45, n)], 1)
    u = np.sin(x[:, 1] / 7) + rng.normal(0, 0.05, n)
    v = np.cos(x[:, 0] / 9) + rng.normal(0, 0.05, n)
    return x, np.concatenate([u, v])


@pytest.mark.parametrize("name", ["df", "cf", "mixed"])
def test_lml_golden_vector(golden, name):
    g = golden("lml_vector_N300.npz")
    x = np.stack([g["x"], g["y"]], 1)
    y = np.concatenate([g["u"], g["v"]])
    l_df, l_cf, rate, noise = (float(v) for v in g[f"{name}_params"])
    ks = E.KernelSpec(kind=name, l_df=l_df, l_cf=l_cf, ratio=rate)
    gp = E.fit(ks, x, y, noise)
    val, grad = E.log_marginal_likelihood(gp, eval_gradient=True)
    ref = float(g[f"{name}_lml"])
    assert abs(val - ref) <= 1e-10 * abs(ref), (val, ref)
    assert rel(grad, g[f"{name}_grad"]) < 1e-6, (grad, g[f"{name}_grad"])


@pytest.mark.parametrize("T", [1, 2])
def test_lml_ard_sklearn(golden, T):
    g = golden("lml_sklearn_ard_N128.npz")
    HP = [float(v) for v in g[f"T{T}_HP"]]
    var = [HP[0]] + ([HP[4]] if T == 2 else [])
    ls = [tuple(HP[1:4])] + ([tuple(HP[5:8])] if T == 2 else [])
    ks = E.KernelSpec(family="ard", variances=tuple(var), lengthscales=tuple(ls))
    gp = E.fit(ks, g["X"], g["u"], HP[-1], jitter=1e-10)
    val, grad = E.log_marginal_likelihood(gp, eval_gradient=True)
    ref = float(g[f"T{T}_lml"])
    assert abs(val - ref) <= 1e-10 * abs(ref), (val, ref)
    assert rel(grad, g[f"T{T}_grad"]) < 1e-9, (grad, g[f"T{T}_grad"])
    _, og = O.ard_lml(g["X"], g["u"], var, ls, HP[-1], jitter=1e-10, eval_gradient=True)
    assert rel(grad, og) < 1e-10


@pytest.mark.parametrize("kind,ratio", [("df", 1.0), ("cf", 0.0), ("mixed", 0.35), ("scalar", 1.0)])
@pytest.mark.parametrize("n", [1, 37, 300, 1000])
def test_lml_vs_oracle(kind, ratio, n):
    x, y = tracks(n, seed=n)
    kw = dict(l_df=4.5, l_cf=6.5, ratio=ratio)
    noise = 0.01
    gp = E.fit(E.KernelSpec(kind=kind, **kw), x, y, noise)
    val, grad = E.log_marginal_likelihood(gp, eval_gradient=True)
    oval, ograd = O.vector_lml(x, y, kind=kind, noise=noise, eval_gradient=True, **kw)
    assert abs(val - oval) <= 1e-10 * max(abs(oval), 1.0), (val, oval)
    assert rel(grad, ograd) < 1e-6, (grad, ograd)
    assert E.log_marginal_likelihood(gp) == val


def test_lml_grad_deterministic():
    x, y = tracks(700, seed=3)
    gp = E.fit(E.KernelSpec(kind="mixed", l_df=5.0, l_cf=4.0, ratio=0.6), x, y, 0.0025)
    a = E.log_marginal_likelihood(gp, eval_gradient=True)
    b = E.log_marginal_likelihood(gp, eval_gradient=True)
    assert a[0] == b[0] and np.array_equal(a[1], b[1])


def test_lml_grad_full_size_fd():
    """Headline / config C size (N=4096, div-free): the analytic gradient against a central difference of
    the GPU LML itself (size-independent property; step 1e-5 relative)."""
    x, y = tracks(4096, seed=11)
    noise = 0.0025
    ks = E.KernelSpec(kind="df", l_df=5.0)
    gp = E.fit(ks, x, y, noise)
    val, grad = E.log_marginal_likelihood(gp, eval_gradient=True)
    del gp
    for i, (name, base) in enumerate((("l_df", 5.0), ("noise", noise))):
        h = 1e-5 * base
        f = []
        for t in (-1, 1):
            k2 = E.KernelSpec(kind="df", l_df=base + t * h) if name == "l_df" else ks
            nz = noise + t * h if name == "noise" else noise
            g2 = E.fit(k2, x, y, nz)
            f.append(E.log_marginal_likelihood(g2))
            del g2
        fd = (f[1] - f[0]) / (2 * h)
        gi = grad[0] if name == "l_df" else grad[3]
        assert abs(fd - gi) < 1e-5 * abs(gi) + 1e-6 * abs(val), (name, fd, gi)


@pytest.mark.parametrize("kind,ratio", [("df", 1.0), ("cf", 0.0), ("mixed", 0.35), ("scalar", 1.0)])
def test_kernel_grad_dense(kind, ratio):
    rng = np.random.default_rng(9)
    xa = rng.uniform(0, 12, (37, 2))
    xb = rng.uniform(0, 12, (100, 2))
    G = rng.normal(0, 1, (74, 200))
    kw = dict(l_df=3.0, l_cf=4.0, ratio=ratio)
    g = E.kernel_grad(E.KernelSpec(kind=kind, **kw), xa, G, xb)
    ref = np.zeros(3)
    for i, name in enumerate(("l_df", "l_cf", "ratio")):
        h = 1e-4 * (kw[name] if name != "ratio" else 1.0)
        Ks = []
        for t in (-2, -1, 1, 2):
            k2 = dict(kw)
            k2[name] += t * h
            Ks.append(O.vector_kernel(xa, xb, kind=kind, **k2))
        dK = (Ks[0] - 8 * Ks[1] + 8 * Ks[2] - Ks[3]) / (12 * h)
        ref[i] = np.sum(G * dK)
    used = {"df": [0], "scalar": [0], "cf": [1], "mixed": [0, 1, 2]}[kind]
    mask = np.zeros(3, bool)
    mask[used] = True
    assert rel(g[mask], ref[mask]) < 1e-7
    assert np.all(g[~mask] == 0.0)


def test_kernel_grad_ard_dense():
    rng = np.random.default_rng(10)
    xa = rng.uniform(0, 5, (50, 3))
    xb = rng.uniform(0, 5, (70, 3))
    G = rng.normal(0, 1, (50, 70))
    var, ls = (0.7, 0.2), ((1.0, 2.0, 3.0), (4.0, 0.5, 1.5))
    g = E.kernel_grad(E.KernelSpec(family="ard", variances=var, lengthscales=ls), xa, G, xb)
    ref = []
    for v, l in zip(var, ls):
        e = O.ard_rbf_exact(xa, xb, [1.0], [l])
        ref.append(np.sum(G * e))
        for d in range(3):
            D2 = np.square(xa[:, d][:, None] - xb[:, d][None, :])
            ref.append(np.sum(G * v * e * D2 / l[d] ** 3))
    assert rel(g, ref) < 1e-12


def test_kern_update_gradients_full():
    rng = np.random.default_rng(4)
    X = rng.uniform(0, 20, (60, 2))
    G = rng.normal(0, 1, (120, 120))
    k = kern.myKernel(l_df=3.0, l_cf=5.0, ratio=0.4)
    k.update_gradients_full(G, X)
    g = E.kernel_grad(E.KernelSpec(kind="mixed", l_df=3.0, l_cf=5.0, ratio=0.4), X, G)
    assert (k.length_df.gradient, k.length_cf.gradient, k.ratio.gradient) == tuple(g)
    assert float(k.length_df) == 3.0
    kd = kern.nonDivK(length=2.0)
    kd.update_gradients_full(G, X)
    assert kd.length.gradient == E.kernel_grad(E.KernelSpec(kind="df", l_df=2.0), X, G)[0]
    kc = kern.nonRotK(l=2.0)
    kc.update_gradients_full(G, X)
    assert kc.length.gradient == E.kernel_grad(E.KernelSpec(kind="cf", l_df=2.0, l_cf=2.0), X, G)[1]


def _sample(n, kind, l_df, l_cf, ratio, noise, seed):
    rng = np.random.default_rng(seed)
    x = np.stack([rng.uniform(0, 40, n), rng.uniform(0, 30, n)], 1)
    K = O.vector_kernel(x, x, kind=kind, l_df=l_df, l_cf=l_cf, ratio=ratio) + noise * np.eye(2 * n)
    y = np.linalg.cholesky(K) @ rng.normal(0, 1, 2 * n)
    return x, y


def test_optimize_matches_oracle_optimum():
    """L-BFGS-B on the GPU LML reaches the optimum scipy finds on the oracle LML."""
    from scipy.optimize import minimize
    x, y = _sample(250, "df", 6.0, 6.0, 1.0, 0.01, seed=21)
    res = H.optimize(E.KernelSpec(kind="df", l_df=3.0), x, y, 0.05)
    assert res.success, res.message

    def f(z):
        return -O.vector_lml(x, y, kind="df", l_df=np.exp(z[0]), noise=np.exp(z[1]))

    ref = minimize(f, np.log([3.0, 0.05]), method="Nelder-Mead", options=dict(xatol=1e-10, fatol=1e-12,
                                                                               maxiter=4000))
    assert abs(res.lml - (-ref.fun)) < 1e-6 * abs(ref.fun)
    assert abs(res.kernel.l_df - np.exp(ref.x[0])) < 1e-3 * np.exp(ref.x[0])
    assert abs(res.noise - np.exp(ref.x[1])) < 1e-3 * np.exp(ref.x[1])
    gp = E.fit(res.kernel, x, y, res.noise)
    _, g = E.log_marginal_likelihood(gp, eval_gradient=True)
    assert abs(g[0] * res.kernel.l_df) < 1e-2 and abs(g[3] * res.noise) < 1e-2


def test_optimize_restarts_mixed_and_fix():
    x, y = _sample(200, "mixed", 5.0, 3.0, 0.7, 0.01, seed=22)
    ks = E.KernelSpec(kind="mixed", l_df=4.0, l_cf=4.0, ratio=0.5)
    start = E.log_marginal_likelihood(E.fit(ks, x, y, 0.02))
    res = H.optimize_restarts(ks, x, y, 0.02, num_restarts=3, seed=1)
    assert len(res.runs) == 3 and res.lml >= max(r[1] for r in res.runs) - 1e-9
    assert res.lml > start and 0.0 < res.kernel.ratio < 1.0
    fixed = H.optimize(ks, x, y, 0.02, fix=("ratio", "noise"))
    assert fixed.kernel.ratio == 0.5 and fixed.noise == 0.02


@pytest.mark.parametrize("concurrent", [1, 2, 3])
def test_sweep_matches_individual_fits(concurrent):
    """concurrent > 1 queues several settings' fit + LML chains on separate streams with no host
    round trip; a non-PD setting still gives -inf (the last setting's negative noise)."""
    x, y = tracks(500, seed=8)
    ks = E.KernelSpec(kind="df", l_df=5.0)
    settings = [dict(l_df=l, noise=nz) for l in (3.0, 5.0, 8.0) for nz in (0.0025, 0.01)] + [dict(noise=-50.0)]
    vals, grads = H.sweep(ks, x, y, settings, noise=0.0025, eval_gradient=True, concurrent=concurrent)
    assert vals[-1] == -np.inf
    vals, grads, settings = vals[:-1], grads[:-1], settings[:-1]
    for s, v, g in zip(settings, vals, grads):
        gp = E.fit(E.KernelSpec(kind="df", l_df=s["l_df"]), x, y, s["noise"])
        rv, rg = E.log_marginal_likelihood(gp, eval_gradient=True)
        assert v == rv and np.array_equal(g, rg)


def test_krig_optimize_and_runRestarts(tmp_path):
    x, y = _sample(150, "df", 6.0, 6.0, 1.0, 0.01, seed=23)
    k = krig.Krig("df", l_df=3.0, noise=0.05).fit(x, y)
    before = k.log_likelihood()
    res = k.optimize()
    assert k.log_likelihood() == pytest.approx(res.lml, rel=1e-12) and res.lml > before
    path = os.path.join(tmp_path, "model")
    krig.Krig("df", l_df=3.0, noise=0.05).fit(x, y).save(path + ".npz")
    r2 = krig.runRestarts(path, nres=2)
    k2 = krig.Krig.load(path + ".npz")
    assert k2.param_array[0] == pytest.approx(r2.kernel.l_df, rel=1e-12)
    assert k2.log_likelihood() >= res.lml - 1e-6 * abs(res.lml)
