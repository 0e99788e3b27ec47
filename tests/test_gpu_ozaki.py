"""INT8 (Ozaki scheme II) variance engine vs the CPU oracle and the FP64 engine.

Same gate as the FP64 path: posterior mean / variance within 1e-10 relative
(normwise per output vector), through the C ABI.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from gp2d import engine as E  # noqa: E402
from oracle import gp2d_oracle as O  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def tracks(n, seed):
    rng = np.random.default_rng(seed)
    x = np.stack([rng.uniform(0, 60, n), rng.uniform(0, 45, n)], 1)
    y = np.concatenate([np.sin(x[:, 1] / 7), np.cos(x[:, 0] / 9)]) + rng.normal(0, 0.05, 2 * n)
    return x, y


@pytest.mark.parametrize("ntr,m,kind,l", [(100, 700, "df", 5.0), (300, 1500, "mixed", 4.0), (1000, 3000, "cf", 3.0),
                                          (1024, 2048, "df", 5.0), (64, 130, "scalar", 6.0)])
def test_ozaki_matches_oracle(ntr, m, kind, l):
    x, y = tracks(ntr, ntr)
    rng = np.random.default_rng(m)
    xg = np.stack([rng.uniform(-5, 65, m), rng.uniform(-5, 50, m)], 1)
    ratio = 0.5 if kind == "mixed" else 1.0
    ks = E.KernelSpec(kind=kind, l_df=l, l_cf=l * 1.3, ratio=ratio)
    gp = E.fit(ks, x, y, noise=0.0025, variance="ozaki")
    mu, var = E.predict(gp, xg, chunk=1024)
    mo, vo = O.fit_predict(x, y, xg, kind=kind, l_df=l, l_cf=l * 1.3, ratio=ratio, noise=0.0025)
    assert rel(mu.cpu().numpy(), mo) < 1e-10
    assert rel(var.cpu().numpy(), vo) < 1e-10


def test_ozaki_vs_f64_engine_and_golden(golden):
    g = golden("mykernel_divfree_N1024.npz")
    x = np.stack([g["x"], g["y"]], 1)
    y = np.concatenate([g["u"], g["v"]])
    ks = E.KernelSpec(kind="df", l_df=5.0)
    gpo = E.fit(ks, x, y, noise=float(g["noise"]), variance="ozaki")
    gpf = E.fit(ks, x, y, noise=float(g["noise"]))
    mo, vo = (t.cpu().numpy() for t in E.predict(gpo, g["xg"]))
    mf, vf = (t.cpu().numpy() for t in E.predict(gpf, g["xg"]))
    assert rel(vo, g["var"]) < 1e-10 and rel(mo, g["mean"]) < 1e-10
    assert rel(vo, vf) < 1e-11
    # elementwise relative check: the small-variance points (near observations) carry the
    # cancellation kss − ‖W k*‖², so this is the strict form of the 1e-10 gate
    assert np.max(np.abs(vo - vf) / np.abs(vf)) < 1e-10
    assert 1 <= gpo.extra["ozaki"][2] <= E.N.lib().gp2d_ozaki_nmod(gpo.n)


def test_ozaki_sharding_bit_identical():
    from gp2d import data as D
    from gp2d.distributed import assemble_from_shards
    x, y = tracks(500, 9)
    rng = np.random.default_rng(10)
    xg = np.stack([rng.uniform(-5, 65, 3000), rng.uniform(-5, 50, 3000)], 1)
    gp = E.fit(E.KernelSpec(kind="df", l_df=5.0), x, y, noise=0.0025, variance="ozaki")
    m_all, v_all = (t.cpu().numpy() for t in E.predict(gp, xg, chunk=1024))
    shards_m, shards_v = [], []
    for r in range(3):
        lo, hi = D.shard_range(xg.shape[0], 3, r)
        mm, vv = E.predict(gp, xg[lo:hi], chunk=512)
        shards_m.append((lo, hi, mm.cpu().numpy()))
        shards_v.append((lo, hi, vv.cpu().numpy()))
    assert np.array_equal(assemble_from_shards(xg.shape[0], 2, shards_v), v_all)
    assert np.array_equal(assemble_from_shards(xg.shape[0], 2, shards_m), m_all)


def test_ozaki_too_few_moduli_poisons_instead_of_wrapping():
    """A CRT range overflow (too few moduli) must not return plausible numbers: the
    reconstruction kernel flags |V_ij| > 4·sqrt(kss) and the column's variance becomes NaN."""
    x, y = tracks(300, 3)
    rng = np.random.default_rng(4)
    xg = np.stack([rng.uniform(0, 60, 500), rng.uniform(0, 45, 500)], 1)
    gp = E.fit(E.KernelSpec(kind="df", l_df=5.0), x, y, noise=0.0025, variance="ozaki")
    wres, rowscale, nmod, kbits = gp.extra["ozaki"]
    assert nmod >= 12
    mu_ok, var_ok = E.predict(gp, xg)
    assert np.isfinite(var_ok.cpu().numpy()).all()
    gp.extra["ozaki"] = (wres, rowscale, 6, kbits)   # ≈ 47 bits of CRT range for ≈ 94-bit products
    mu, var = E.predict(gp, xg)
    v = var.cpu().numpy()
    assert np.isnan(v).mean() > 0.5
    np.testing.assert_array_equal(mu.cpu().numpy(), mu_ok.cpu().numpy())  # the mean path is separate


# ---------------------------------------------------------------- K* planes ahead of the fit
# gp2d_ozaki_kstar builds the K* residue planes before the fit (they need no α); the predict
# then runs the K* kernel mean-only (K*α in fp64, as inline).  Same 1e-10 gate; the variance
# partials are the same integers as the inline path, so both outputs are bit-identical to it.
def _ahead(ks, x, y, xg, noise, chunk, side=True):
    st = torch.cuda.Stream() if side else None
    planes = E.kstar_planes(ks, x, xg, noise, chunk=chunk, stream=st)
    gp = E.fit(ks, x, y, noise=noise, variance="ozaki")
    pr = E.Predictor(gp, chunk)
    mu, var = pr(xg, planes=planes)
    return gp, planes, mu.cpu().numpy(), var.cpu().numpy()


@pytest.mark.parametrize("ntr,m,kind,l,chunk", [(100, 700, "df", 5.0, 256), (300, 1500, "mixed", 4.0, 1024),
                                                (1000, 3000, "cf", 3.0, 1024), (37, 1, "df", 5.0, 128),
                                                (64, 130, "scalar", 6.0, 8192)])
def test_kstar_ahead_matches_oracle(ntr, m, kind, l, chunk):
    x, y = tracks(ntr, ntr + 1)
    rng = np.random.default_rng(m + 3)
    xg = np.stack([rng.uniform(-5, 65, m), rng.uniform(-5, 50, m)], 1)
    ratio = 0.5 if kind == "mixed" else 1.0
    ks = E.KernelSpec(kind=kind, l_df=l, l_cf=l * 1.3, ratio=ratio)
    gp, planes, mu, var = _ahead(ks, x, y, xg, 0.0025, chunk)
    mo, vo = O.fit_predict(x, y, xg, kind=kind, l_df=l, l_cf=l * 1.3, ratio=ratio, noise=0.0025)
    assert rel(mu, mo) < 1e-10
    assert rel(var, vo) < 1e-10
    mi, vi = (t.cpu().numpy() for t in E.Predictor(gp, chunk)(xg))
    assert np.array_equal(var, vi) and np.array_equal(mu, mi)


@pytest.mark.parametrize("kind,l,noise,jitter", [("df", 5.0, 0.0025, 0.0), ("cf", 2.0, 1e-4, 0.0),
                                                  ("mixed", 8.0, 0.5, 1e-6), ("scalar", 1.0, 0.01, 0.0),
                                                  ("df", 0.7, 1e-6, 0.0)])
def test_nmod_apriori_bounds_data_driven(kind, l, noise, jitter):
    x, y = tracks(700, 5)
    ks = E.KernelSpec(kind=kind, l_df=l, l_cf=l * 1.1, ratio=0.5 if kind == "mixed" else 1.0)
    gp = E.fit(ks, x, y, noise=noise, jitter=jitter, variance="ozaki", guard=False)
    apriori = int(E.N.lib().gp2d_ozaki_nmod_apriori(gp.n, __import__("ctypes").byref(ks.desc()), noise + jitter, 0, 0))
    assert gp.extra["ozaki"][2] <= apriori <= gp.extra["ozaki"][2] + 1
    # at every W precision the accuracy guard can pick: the data-driven count (synchronous
    # prepare) never exceeds the a-priori one the engine uses
    for wb, kb in ((49, 45), (53, 45), (57, 48), (60, 50)):
        E.ozaki_prepare(gp, wbits=wb, kbits=kb)
        ap = int(E.N.lib().gp2d_ozaki_nmod_apriori(gp.n, __import__("ctypes").byref(ks.desc()), noise + jitter, wb, kb))
        assert gp.extra["ozaki"][2] <= ap <= gp.extra["ozaki"][2] + 1, (wb, kb)


def test_kstar_ahead_too_few_moduli_falls_back_inline():
    import dataclasses
    x, y = tracks(300, 11)
    rng = np.random.default_rng(12)
    xg = np.stack([rng.uniform(-5, 65, 900), rng.uniform(-5, 50, 900)], 1)
    ks = E.KernelSpec(kind="df", l_df=5.0)
    planes = E.kstar_planes(ks, x, xg, 0.0025, chunk=512)
    gp = E.fit(ks, x, y, noise=0.0025, variance="ozaki")
    short = dataclasses.replace(planes, nmod=gp.extra["ozaki"][2] - 1)
    pr = E.Predictor(gp, 512)
    mu, var = (t.cpu().numpy() for t in pr(xg, planes=short))
    mi, vi = (t.cpu().numpy() for t in pr(xg))
    assert np.array_equal(mu, mi) and np.array_equal(var, vi)


def test_kstar_ahead_spatiotemporal():
    rng = np.random.default_rng(21)
    n, m = 400, 1000
    x = np.stack([rng.uniform(0, 48, n), rng.uniform(0, 45, n), rng.uniform(0, 60, n)], 1)
    y = np.concatenate([np.sin(x[:, 1] / 7), np.cos(x[:, 2] / 9)]) + rng.normal(0, 0.05, 2 * n)
    xg = np.stack([rng.uniform(0, 48, m), rng.uniform(-5, 50, m), rng.uniform(-5, 65, m)], 1)
    ks = E.KernelSpec(family="vector_st", kind="mixed", l_df=5.0, l_cf=4.0, ratio=0.5, var_t=1.3, l_t=12.0)
    gp, planes, mu, var = _ahead(ks, x, y, xg, 0.0025, 512)
    mi, vi = (t.cpu().numpy() for t in E.Predictor(gp, 512)(xg))
    assert np.array_equal(var, vi) and np.array_equal(mu, mi)


def test_kstar_ahead_bench_size_properties():
    """N_train = 4096 (the bench workload) on a 2-chunk grid: mean and variance are
    bit-identical to the inline path."""
    from gp2d import data as D
    x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
    x = np.stack([x1, x2], 1)
    y = np.concatenate([u, v])
    _, _, xg = D.bbox_grid(x1, x2, 128, pad=5.0)
    ks = E.KernelSpec(kind="df", l_df=5.0)
    gp, planes, mu, var = _ahead(ks, x, y, xg, 0.0025, 8192)
    assert planes.nmod >= gp.extra["ozaki"][2]
    mi, vi = (t.cpu().numpy() for t in E.Predictor(gp, 8192)(xg))
    assert np.array_equal(var, vi) and np.array_equal(mu, mi)
    assert np.all(np.isfinite(var)) and np.all(var > 0)


@pytest.mark.parametrize("kind,l,noise", [("df", 5.0, 0.0025), ("mixed", 3.0, 1e-4), ("cf", 8.0, 0.3)])
def test_async_prepare_matches_data_driven(kind, l, noise):
    """engine.fit prepares the W residue planes with the a-priori moduli count (no host
    round trip); the data-driven preparation gives the same posterior (to the CRT constants'
    rounding when the counts differ) and never more moduli."""
    x, y = tracks(500, 17)
    rng = np.random.default_rng(18)
    xg = np.stack([rng.uniform(-5, 65, 1200), rng.uniform(-5, 50, 1200)], 1)
    ks = E.KernelSpec(kind=kind, l_df=l, l_cf=l * 1.2, ratio=0.5 if kind == "mixed" else 1.0)
    gp = E.fit(ks, x, y, noise=noise, variance="ozaki", guard=False)   # both at the default precision
    n_async = gp.extra["ozaki"][2]
    ma, va = (t.cpu().numpy() for t in E.predict(gp, xg, chunk=512))
    E.ozaki_prepare(gp)   # data-driven count (synchronises)
    n_data = gp.extra["ozaki"][2]
    md, vd = (t.cpu().numpy() for t in E.predict(gp, xg, chunk=512))
    assert n_data <= n_async <= n_data + 1
    if n_async == n_data:
        assert np.array_equal(va, vd) and np.array_equal(ma, md)
    assert rel(va, vd) < 1e-12 and rel(ma, md) < 1e-13
    mo, vo = O.fit_predict(x, y, xg, kind=kind, l_df=l, l_cf=l * 1.2, ratio=ks.ratio, noise=noise)
    assert rel(va, vo) < 1e-10 and rel(ma, mo) < 1e-10


# ---------------------------------------------------------------- zero-slab skipping
# The ozaki engine orders training and grid points along a Morton curve; K* tiles between
# far-apart groups are then exactly zero and the int8 GEMMs skip those K slabs.  Skipping
# must be exact (bit-identical to the dense K loop) and match the oracle.
@pytest.mark.parametrize("kind,l", [("df", 3.0), ("mixed", 4.0)])
def test_zero_slab_skip_is_exact(kind, l):
    rng = np.random.default_rng(31)
    n, m = 1500, 5000
    x = np.stack([rng.uniform(0, 150, n), rng.uniform(0, 120, n)], 1)     # wide domain: ≫ 8ℓ
    y = np.concatenate([np.sin(x[:, 1] / 17), np.cos(x[:, 0] / 23)]) + rng.normal(0, 0.05, 2 * n)
    xg = np.stack([rng.uniform(-5, 155, m), rng.uniform(-5, 125, m)], 1)
    ks = E.KernelSpec(kind=kind, l_df=l, l_cf=l * 1.2, ratio=0.5 if kind == "mixed" else 1.0)
    gp = E.fit(ks, x, y, noise=0.0025, variance="ozaki")
    L = E.N.lib()
    try:
        L.gp2d_ozaki_set_skip(0)
        md, vd = (t.cpu().numpy() for t in E.predict(gp, xg, chunk=1024))
    finally:
        L.gp2d_ozaki_set_skip(1)
    ms, vs = (t.cpu().numpy() for t in E.predict(gp, xg, chunk=1024))
    assert np.array_equal(ms, md) and np.array_equal(vs, vd)
    # the wide domain (≫ 8ℓ) leaves many K* tiles exactly zero: the GEMMs skip a good part of the work
    frac = E.ozaki_executed_fraction(ks, x, xg, 0.0025, chunk=1024)
    assert 0.0 < frac < 0.8
    sub = np.random.default_rng(2).choice(m, 300, replace=False)
    mo, vo = O.fit_predict(x, y, xg[sub], kind=kind, l_df=l, l_cf=l * 1.2, ratio=ks.ratio, noise=0.0025)
    idx = np.concatenate([sub, m + sub])
    assert rel(vs[idx], vo) < 1e-10 and rel(ms[idx], mo) < 1e-10


def test_zero_slab_skip_far_grid_and_planes():
    """A grid block far from every observation: every K slab is skipped (empty list), so the
    variance is exactly the prior kss and the mean exactly 0; the K*-planes-ahead path (block
    flags travel with the planes) gives the same bits."""
    rng = np.random.default_rng(41)
    n = 700
    x = np.stack([rng.uniform(0, 60, n), rng.uniform(0, 45, n)], 1)
    y = np.concatenate([np.sin(x[:, 1] / 7), np.cos(x[:, 0] / 9)]) + rng.normal(0, 0.05, 2 * n)
    near = np.stack([rng.uniform(0, 60, 900), rng.uniform(0, 45, 900)], 1)
    far = np.stack([rng.uniform(900, 960, 700), rng.uniform(900, 945, 700)], 1)
    xg = np.concatenate([near, far])
    ks = E.KernelSpec(kind="df", l_df=5.0)
    gp = E.fit(ks, x, y, noise=0.0025, variance="ozaki")
    mu, var = (t.cpu().numpy() for t in E.predict(gp, xg, chunk=512))
    M = xg.shape[0]
    kss = float(E.N.lib().gp2d_kernel_diag(__import__("ctypes").byref(ks.desc())))
    far_idx = np.concatenate([np.arange(900, M), M + np.arange(900, M)])
    assert np.all(var[far_idx] == kss) and np.all(mu[far_idx] == 0.0)
    _, planes, ma, va = _ahead(ks, x, y, xg, 0.0025, 512)
    assert np.array_equal(ma, mu) and np.array_equal(va, var)
    mo, vo = O.fit_predict(x, y, near[:200], kind="df", l_df=5.0, noise=0.0025)
    idx = np.concatenate([np.arange(200), M + np.arange(200)])
    assert rel(var[idx], vo) < 1e-10 and rel(mu[idx], mo) < 1e-10


def test_morton_training_order_is_consistent():
    """The ozaki fit stores the training points in Morton order (GPFit.perm): x = x_in[perm],
    α follows it, and order-invariant quantities (LML, predictions) match the f64 fit."""
    x, y = tracks(500, 61)
    ks = E.KernelSpec(kind="df", l_df=5.0)
    go = E.fit(ks, x, y, noise=0.0025, variance="ozaki")
    gf = E.fit(ks, x, y, noise=0.0025)
    perm = go.perm.cpu().numpy()
    assert np.array_equal(np.sort(perm), np.arange(500)) and not np.array_equal(perm, np.arange(500))
    assert np.array_equal(go.x.cpu().numpy(), x[perm])
    a_o = go.alpha.cpu().numpy()
    a_f = gf.alpha.cpu().numpy()
    npad = go.n_pad
    for c in range(2):   # α of the reordered fit, component c, back in input order
        back = np.empty(500)
        back[perm] = a_o[c * npad:c * npad + 500]
        assert rel(back, a_f[c * gf.n_pad:c * gf.n_pad + 500]) < 1e-9
    assert abs(E.log_marginal_likelihood(go) - E.log_marginal_likelihood(gf)) < 1e-9 * abs(E.log_marginal_likelihood(gf))


def test_zero_slab_skip_spatiotemporal_exact():
    """3-D (T, Y, X) points: Morton order over all three coordinates; skip on/off bit-identical
    and the oracle gate, with far-in-time grid points exactly at the prior."""
    rng = np.random.default_rng(71)
    n, m = 600, 1500
    x = np.stack([rng.uniform(0, 48, n), rng.uniform(0, 45, n), rng.uniform(0, 60, n)], 1)
    y = np.concatenate([np.sin(x[:, 1] / 7), np.cos(x[:, 2] / 9)]) + rng.normal(0, 0.05, 2 * n)
    xg = np.stack([rng.uniform(0, 48, m), rng.uniform(-5, 50, m), rng.uniform(-5, 65, m)], 1)
    xg[-300:, 0] += 5000.0                       # far in time: K* = 0 through the temporal factor
    ks = E.KernelSpec(family="vector_st", kind="mixed", l_df=5.0, l_cf=4.0, ratio=0.5, var_t=1.3, l_t=12.0)
    gp = E.fit(ks, x, y, noise=0.0025, variance="ozaki")
    L = E.N.lib()
    try:
        L.gp2d_ozaki_set_skip(0)
        md, vd = (t.cpu().numpy() for t in E.predict(gp, xg, chunk=512))
    finally:
        L.gp2d_ozaki_set_skip(1)
    ms, vs = (t.cpu().numpy() for t in E.predict(gp, xg, chunk=512))
    assert np.array_equal(ms, md) and np.array_equal(vs, vd)
    kss = float(L.gp2d_kernel_diag(__import__("ctypes").byref(ks.desc())))
    far = np.concatenate([np.arange(m - 300, m), m + np.arange(m - 300, m)])
    assert np.all(vs[far] == kss) and np.all(ms[far] == 0.0)
    mo, vo = O.st_fit_predict(x, y, xg[:400], kind="mixed", l_df=5.0, l_cf=4.0, ratio=0.5, var_t=1.3, l_t=12.0,
                              noise=0.0025)
    idx = np.concatenate([np.arange(400), m + np.arange(400)])
    assert rel(vs[idx], vo) < 1e-10 and rel(ms[idx], mo) < 1e-10
