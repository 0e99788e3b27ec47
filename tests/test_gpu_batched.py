"""Batched factorisations (gp2d_potrf_batched / gp2d_trtri_batched, engine.fit_batch,
hyper.sweep(batch=...)): several fits of one size in one chain.

Every launch of the batched chain carries all problems with the lone launch's tiles, K ranges
and summation order, so the gate is bit identity with engine.fit / gp2d_potrf + gp2d_trtri on
each problem alone (W, α, the INT8 residue planes, LML and gradient); the lone path itself is
pinned against the reference fixtures elsewhere (test_gpu_parity.py, test_gpu_configs.py).
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from gp2d import _native as N  # noqa: E402
from gp2d import engine as E  # noqa: E402
from gp2d import hyper as H  # noqa: E402


def tracks(n, seed=2016):
    rng = np.random.default_rng(seed)
    x = np.stack([rng.uniform(0, 60, n), rng.uniform(0, 45, n)], 1)
    u = np.sin(x[:, 1] / 7) + rng.normal(0, 0.05, n)
    v = np.cos(x[:, 0] / 9) + rng.normal(0, 0.05, n)
    return x, np.concatenate([u, v])


def same(a, b):
    return torch.equal(a, b)


@pytest.mark.parametrize("ntr,kind,variance", [(500, "df", "f64"), (1000, "mixed", "ozaki"), (64, "cf", "f64"),
                                               (2048, "df", "ozaki")])
def test_fit_batch_settings_bit_identical(ntr, kind, variance):
    """One training set, several (l, noise) settings — config E's shape — ragged point counts
    (500: 8 block columns of 128 after padding, 64: a single block column)."""
    x, y = tracks(ntr, seed=ntr)
    settings = [(3.0, 0.0025), (5.0, 0.01), (8.0, 0.0025)]
    probs = [(E.KernelSpec(kind=kind, l_df=l, l_cf=l + 1.0, ratio=0.6), x, y, nz) for l, nz in settings]
    fits = E.fit_batch(probs, variance=variance)
    for (k, _, _, nz), gb in zip(probs, fits):
        g1 = E.fit(k, x, y, nz, variance=variance)
        assert same(gb.W, g1.W) and same(gb.alpha, g1.alpha)
        if variance == "ozaki":
            _, rb, mb, kb = gb.extra["ozaki"]   # (the residue buffers' tiles above the diagonal are never written)
            _, r1, m1, k1 = g1.extra["ozaki"]
            assert mb == m1 and kb == k1 and same(rb, r1)
            xg = np.stack([np.linspace(-5, 65, 300), np.linspace(-5, 50, 300)], 1)
            mu_b, var_b = E.predict(gb, xg)
            mu_1, var_1 = E.predict(g1, xg)
            assert same(mu_b, mu_1) and same(var_b, var_1)


def test_fit_batch_jobs_bit_identical():
    """Different training sets of one size — a job stream's next fits (config B's shape)."""
    probs = []
    for j in range(4):
        x, y = tracks(1024, seed=100 + j)
        probs.append((E.KernelSpec(kind="df", l_df=5.0), x, y, 0.0025))
    fits = E.fit_batch(probs, variance="ozaki", check=False)
    for (k, x, y, nz), gb in zip(probs, fits):
        gb.check()
        g1 = E.fit(k, x, y, nz, variance="ozaki")
        assert same(gb.W, g1.W) and same(gb.alpha, g1.alpha) and same(gb.perm, g1.perm)


def test_fit_batch_non_spd_problem():
    x, y = tracks(300, seed=5)
    k = E.KernelSpec(kind="df", l_df=5.0)
    probs = [(k, x, y, 0.0025), (k, x, y, -50.0), (k, x, y, 0.01)]
    with pytest.raises(np.linalg.LinAlgError, match="problem 1"):
        E.fit_batch(probs)
    fits = E.fit_batch(probs, check=False)
    fits[0].check()
    fits[2].check()
    with pytest.raises(np.linalg.LinAlgError):
        fits[1].check()
    assert same(fits[2].W, E.fit(k, x, y, 0.01).W)


def test_fit_batch_rejects_mixed_sizes():
    x1, y1 = tracks(300, seed=1)
    x2, y2 = tracks(700, seed=2)
    k = E.KernelSpec(kind="df", l_df=5.0)
    with pytest.raises(ValueError, match="same matrix order"):
        E.fit_batch([(k, x1, y1, 0.01), (k, x2, y2, 0.01)])


def test_potrf_trtri_batched_abi_matches_lone_calls():
    """The C ABI directly: nprob = 3 matrices with a padded problem stride vs gp2d_potrf +
    gp2d_trtri on each, and nprob = 1 with stride 0."""
    L = N.lib()
    dev = torch.device("cuda:0")
    s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    n, lda, B = 768, 768, 3
    rng = np.random.default_rng(3)
    mats = []
    for b in range(B):
        G = rng.normal(size=(n, n))
        mats.append(G @ G.T / n + (0.5 + b) * np.eye(n))
    stride = n * lda + 4096
    buf = torch.zeros(B * stride, dtype=torch.float64, device=dev)
    for b in range(B):
        buf[b * stride:b * stride + n * lda] = torch.tensor(mats[b].ravel(), device=dev)
    dinv = torch.empty((B, n // 128, 128, 128), dtype=torch.float64, device=dev)
    info = torch.zeros(B, dtype=torch.int32, device=dev)
    p = ctypes.c_void_p
    N.check(L.gp2d_potrf_batched(p(buf.data_ptr()), n, lda, stride, B, p(dinv.data_ptr()), p(info.data_ptr()), s),
            "gp2d_potrf_batched")
    wb = int(L.gp2d_trtri_batched_workspace(n, B))
    work = torch.empty(wb // 8 + 1, dtype=torch.float64, device=dev)
    N.check(L.gp2d_trtri_batched(p(buf.data_ptr()), n, lda, stride, B, p(dinv.data_ptr()), p(work.data_ptr()), wb, s),
            "gp2d_trtri_batched")
    assert info.cpu().tolist() == [0] * B
    for b in range(B):
        A = torch.tensor(mats[b], device=dev).contiguous()
        d1 = torch.empty((n // 128, 128, 128), dtype=torch.float64, device=dev)
        i1 = torch.zeros(1, dtype=torch.int32, device=dev)
        N.check(L.gp2d_potrf(p(A.data_ptr()), n, n, p(d1.data_ptr()), p(i1.data_ptr()), None, 0, s), "gp2d_potrf")
        w1 = int(L.gp2d_trtri_workspace(n))
        k1 = torch.empty(w1 // 8 + 1, dtype=torch.float64, device=dev)
        N.check(L.gp2d_trtri(p(A.data_ptr()), n, n, p(d1.data_ptr()), p(k1.data_ptr()), w1, s), "gp2d_trtri")
        got = buf[b * stride:b * stride + n * lda].view(n, lda)
        assert same(got, A) and same(dinv[b], d1)
        W = A.cpu().numpy()
        assert np.max(np.abs(W @ np.linalg.cholesky(mats[b]) - np.eye(n))) < 1e-10


def test_sweep_batched_matches_individual_fits():
    x, y = tracks(500, seed=8)
    ks = E.KernelSpec(kind="df", l_df=5.0)
    settings = [dict(l_df=l, noise=nz) for l in (3.0, 5.0, 8.0) for nz in (0.0025, 0.01)] + [dict(noise=-50.0)]
    vals, grads = H.sweep(ks, x, y, settings, noise=0.0025, eval_gradient=True, batch=3)
    assert vals[-1] == -np.inf
    for s, v, g in zip(settings[:-1], vals[:-1], grads[:-1]):
        gp = E.fit(E.KernelSpec(kind="df", l_df=s["l_df"]), x, y, s["noise"])
        rv, rg = E.log_marginal_likelihood(gp, eval_gradient=True)
        assert v == rv and np.array_equal(g, rg)
    v2, g2 = H.sweep(ks, x, y, settings, noise=0.0025, eval_gradient=True)   # the default (auto batch)
    assert np.array_equal(v2, vals) and np.array_equal(g2, grads)


def test_fit_batch_single_and_mixed_kinds():
    """B = 1 is engine.fit; one batch may mix kernel families of one matrix order (df, cf,
    mixed, different noise) — each problem keeps its own bits."""
    x, y = tracks(640, seed=77)
    k = E.KernelSpec(kind="mixed", l_df=4.0, l_cf=6.0, ratio=0.3)
    (g1,) = E.fit_batch([(k, x, y, 0.004)], variance="ozaki")
    ref = E.fit(k, x, y, 0.004, variance="ozaki")
    assert same(g1.W, ref.W) and same(g1.alpha, ref.alpha)
    probs = [(E.KernelSpec(kind="df", l_df=3.0), x, y, 0.0025), (E.KernelSpec(kind="cf", l_cf=7.0), x, y, 0.01),
             (k, x, y, 0.004)]
    for (kk, _, _, nz), gb in zip(probs, E.fit_batch(probs)):
        g = E.fit(kk, x, y, nz)
        assert same(gb.W, g.W) and same(gb.alpha, g.alpha)
