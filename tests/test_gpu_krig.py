"""The reference-compatible surface (krig / kern) on the GPU vs golden vectors and the oracle."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

import krig  # noqa: E402
from gp2d import ncio  # noqa: E402
from gp2d import engine as E  # noqa: E402
from gp2d import kern  # noqa: E402
from oracle import gp2d_oracle as O  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def test_laser_recipe_golden(golden):
    """GP_laser.laser posterior (exec'd reference loops) — mean/var within 1e-10."""
    g = golden("laser_mixed_N256.npz")
    # feed the raw (pre-split) observations back in the reference's order
    n = int(g["n_raw"])
    xo = np.empty(n); yo = np.empty(n); uo = np.empty(n); vo = np.empty(n)
    for arr, a, b in ((xo, "xo", "xt"), (yo, "yo", "yt"), (uo, "uo", "ut"), (vo, "vo", "vt")):
        arr[g["samples"]] = g[a]
        arr[g["test"]] = g[b]
    out = krig.laser(xo, yo, uo, vo, l_df=5.0, l_cf=5.0, rate=0.5, noise=0.0025, dx=1.0)
    x, y, uf, vf, _, _, _, _, uvar, vvar, xt, yt, ut, vt, uft, vft = out
    assert np.array_equal(x, g["x"]) and np.array_equal(y, g["y"])
    assert np.array_equal(xt, g["xt"])
    for a, b in ((uf, "uf"), (vf, "vf"), (uvar, "uvar"), (vvar, "vvar"), (uft, "uft"), (vft, "vft")):
        assert rel(a, g[b]) < 1e-10, b


def test_kern_plugin_golden(golden):
    g = golden("gp_scripts_small.npz")
    xa = np.stack([g["x1"], g["x2"]], 1)
    xb = np.stack([g["x1s"], g["x2s"]], 1)
    s = float(g["sigma"])
    assert rel(kern.nonDivK(2, [0, 1], s).K(xa), g["K_1"]) < 1e-13
    assert rel(kern.nonRotK(2, [0, 1], s).K(xb, xa), g["Ks_2"]) < 1e-13
    assert rel(kern.compute_K(g["x1"], g["x2"], s, 0), g["K_0"]) < 1e-13
    assert rel(kern.compute_Ks(g["x1"], g["x2"], g["x1s"], g["x2s"], s, 1), g["Ks_1"]) < 1e-13
    l_df, l_cf, r = g["myK_params"]
    mk = kern.myKernel(2, [0, 1], l_df, l_cf, r)
    assert rel(mk.K(xa), g["myK_mixed_aa"]) < 1e-13
    assert rel(mk.K(xa, xb), g["myK_mixed_ab"]) < 1e-13
    assert rel(kern.vector_K(xa, xb, l_df, l_cf, r), g["myK_mixed_ab"]) < 1e-13
    assert np.allclose(mk.Kdiag(xa), np.diag(g["myK_mixed_aa"]), rtol=1e-14, atol=0)


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_small_posterior_golden(golden, kind):
    g = golden("gp_scripts_small.npz")
    xa = np.stack([g["x1"], g["x2"]], 1)
    xb = np.stack([g["x1s"], g["x2s"]], 1)
    name = {0: "scalar", 1: "df", 2: "cf"}[kind]
    k = krig.Krig(name, l_df=float(g["sigma"]), l_cf=float(g["sigma"]), noise=float(g["noise"])).fit(xa, g["y"])
    mu, var = k.predict(xb)
    M = xb.shape[0]
    assert rel(mu[:, 0], g[f"mean_{kind}"]) < 1e-10
    assert rel(var[:M, 0], g[f"uvar_{kind}"]) < 1e-10
    assert rel(var[M:, 0], g[f"vvar_{kind}"]) < 1e-10


def test_sklearn_config_A_golden(golden):
    """krig.scikit_prior's model on the GPU ARD family vs sklearn 1.7.2 (fixture)."""
    g = golden("sklearn_ard_N128.npz")
    HP = g["HP"]
    spec = E.KernelSpec(family="ard", variances=(HP[0], HP[4]), lengthscales=(tuple(HP[1:4]), tuple(HP[5:8])))
    k = krig.Krig(spec, noise=HP[8], jitter=1e-10, var_mode="sklearn").fit(g["X"], g["u"])
    mu, var = k.predict(g["Xp"])
    assert rel(mu[:, 0], g["mean"]) < 1e-10
    assert rel(np.sqrt(var[:, 0]), g["std"]) < 1e-10


def test_var_modes_and_save_load(tmp_path):
    rng = np.random.default_rng(5)
    x = rng.uniform(0, 30, (150, 2))
    y = rng.normal(0, 0.3, 300)
    xg = rng.uniform(0, 30, (333, 2))
    k = krig.Krig("mixed", l_df=4.0, l_cf=6.0, ratio=0.3, noise=0.01).fit(x, y)
    m0, v0 = k.predict(xg)
    _, v1 = k.predict(xg, var_mode="gpy")
    assert np.allclose(v1 - v0, 0.01, rtol=0, atol=1e-12)
    mo, vo = O.fit_predict(x, y, xg, kind="mixed", l_df=4.0, l_cf=6.0, ratio=0.3, noise=0.01)
    assert rel(m0[:, 0], mo) < 1e-10 and rel(v0[:, 0], vo) < 1e-10
    p = str(tmp_path / "m.npz")
    k.save(p)
    k2 = krig.Krig.load(p)
    m2, v2 = k2.predict(xg)
    assert np.array_equal(m2, m0) and np.array_equal(v2, v0)


def test_kriging_predict_pipeline(tmp_path):
    """kriging → predict → predictTest on synthetic drifters: kernelType 2 (the spatio-temporal
    product Kt × div-free on (T, Y, X), and the spatial kernel with hyper temporal=False) and 1."""
    tr = krig.Tracks.synthetic(n_time=24, n_drifters=40)
    out = str(tmp_path / "model")
    models = krig.kriging(0, 24, sample_step=-2, skip=2, nKernels=1, output=out, kernelType=2, tracks=tr,
                          hyper=dict(var_t=1.5, l_t=4.0))
    k = models["_divFree"]
    assert k.spec.family == "vector_st" and k.spec.input_dim == 3
    f = np.load(out + ".npz")
    assert f["Xo"].shape[1] == 3 and f["obs"].shape[0] == 2 * f["Xo"].shape[0]
    Xp, V, U, VV, UV = krig.predict(out, tlim=[0, 2], ylim=[-5, 40], xlim=[-5, 50], dt=1.0, dx=2.0)
    assert V.shape == U.shape == VV.shape == UV.shape and V.shape[0] == 2
    # same posterior as the oracle with obs=[v; u] on (T, Y, X), first time slice
    pts = Xp[:V.shape[1] * V.shape[2], :]
    mo, vo = O.st_fit_predict(f["Xo"], f["obs"][:, 0], pts, kind="df", l_df=5.0, var_t=1.5, l_t=4.0,
                              noise=0.0025, var_mode="gpy")
    M = pts.shape[0]
    assert rel(V[0].reshape(-1), mo[:M]) < 1e-10 and rel(U[0].reshape(-1), mo[M:]) < 1e-10
    assert rel(VV[0].reshape(-1), vo[:M]) < 1e-10
    # the NetCDF-3 product of krig.py:559-570 (read back through scipy's independent reader)
    from scipy.io import netcdf_file
    with netcdf_file(out + ".nc", "r", mmap=False) as nc:
        assert nc.dimensions["time"] is None and nc.variables["v"].shape == V.shape
        assert np.array_equal(nc.variables["v"][:], V.astype(np.float32))
        assert np.array_equal(nc.variables["uvar"][:], UV.astype(np.float32))
        assert np.array_equal(nc.variables["hyperparam_v"][:], k.param_array.astype(np.float32))
    # purely spatial variant on the (Y, X) columns
    krig.kriging(0, 24, sample_step=-2, skip=2, nKernels=1, output=out + "_xy", kernelType=2, tracks=tr,
                 hyper=dict(temporal=False))
    Xp, V, U, VV, UV = krig.predict(out + "_xy", tlim=[0, 2], ylim=[-5, 40], xlim=[-5, 50], dt=1.0, dx=2.0)
    pts = Xp[:V.shape[1] * V.shape[2], 1:3]
    mo, vo = O.fit_predict(f["Xo"][:, 1:3], f["obs"][:, 0], pts, kind="df", l_df=5.0, noise=0.0025,
                           var_mode="gpy")
    assert rel(V[0].reshape(-1), mo[:M]) < 1e-10 and rel(U[0].reshape(-1), mo[M:]) < 1e-10
    assert rel(VV[0].reshape(-1), vo[:M]) < 1e-10
    V2, U2, VV2, UV2 = krig.predictTest(out)
    assert V2.shape[0] == f["Xt"].shape[0]
    models = krig.kriging(0, 24, sample_step=-2, skip=2, nKernels=2, output=out + "_rbf", kernelType=1, tracks=tr,
                          hyper=dict(variance=0.1, lengthscale=(5.0, 8.0, 8.0), noise=0.001))
    assert set(models) == {"u", "v"}
    Xp, V, U, VV, UV = krig.predict(out + "_rbf", tlim=[0, 2], ylim=[-5, 40], xlim=[-5, 50], dt=1.0, dx=3.0)
    assert np.all(np.isfinite(V)) and np.all(VV > 0)
    # scikit_prior on the pre-existing grid of out_rbf.nc (krig.py:123-141), NetCDF output
    HP = np.array([0.1, 5.0, 8.0, 8.0, 0.001])
    U0, S0 = krig.scikit_prior(out + "_rbf", varname="v", dt=1, HP=HP, xrange=1000.0)
    g = ncio.readNC(out + "_rbf.nc")
    yg, tg, xg = (np.asarray(g[c], dtype=np.float64) for c in ("y", "time", "x"))
    Yg, Tg, Xg = np.meshgrid(yg, tg, xg)
    inc = yg.size * xg.size
    Xq = np.stack([Tg.reshape(-1), Yg.reshape(-1), Xg.reshape(-1)], 1)[inc:2 * inc]
    fm = np.load(out + "_rbf.npz")
    tc = tg[1]
    sel = lambda T: np.where((T[:, 0] >= tc - 6) & (T[:, 0] <= tc + 6))[0]   # tlim = 6, all x
    XT = np.concatenate([fm["Xo"][sel(fm["Xo"])], fm["Xt"][sel(fm["Xt"])]])
    u = np.concatenate([fm["obs"][sel(fm["Xo"]), 0], fm["test_points"][sel(fm["Xt"]), 0]])
    mo, so = O.ard_fit_predict(XT, u, Xq, [0.1], [(5.0, 8.0, 8.0)], 0.001, jitter=1e-10)
    assert rel(U0.reshape(-1), mo) < 1e-10 and rel(S0.reshape(-1), so ** 2) < 1e-10
    outf = out + "_rbf_" + str(np.round(tc, decimals=2)) + "h_scikit_0.nc"
    d = ncio.readNC(outf)
    assert np.array_equal(d["v"], U0.astype(np.float32)) and np.array_equal(d["vvar"], S0.astype(np.float32))
    assert np.array_equal(d["hyperparam_v"], HP.astype(np.float32))


def test_scikit_prior_radar_branch(tmp_path):
    """scikit_prior on an HF-radar grid (krig.py:98-118 + the fit/predict/NetCDF of 146-206):
    the grid comes from a synthetic radar NetCDF written by gp2d.ncio; the posterior is checked
    against the oracle ARD model on the same window and grid (1e-10)."""
    from test_ncio_cpu import _write_radar
    rng = np.random.default_rng(5)
    xc = np.arange(0.0, 12000.0, 2000.0)
    yc = np.arange(0.0, 10000.0, 2000.0)
    radar = str(tmp_path / "radar.nc")
    _write_radar(radar, -88.55, 28.85, xc, yc, 37.5)
    Xr, tg, yg, xg = krig.radar_grid(radar)
    n, m = 150, 40
    Xo = np.stack([tg[0] + rng.uniform(-8, 8, n), rng.uniform(yg[0] - 3, yg[-1] + 3, n),
                   rng.uniform(xg[0] - 3, xg[-1] + 3, n)], 1)
    Xt = np.stack([tg[0] + rng.uniform(-8, 8, m), rng.uniform(yg[0], yg[-1], m), rng.uniform(xg[0], xg[-1], m)], 1)
    obs = np.stack([np.sin(Xo[:, 1] / 4), np.cos(Xo[:, 2] / 5)], 1) + rng.normal(0, 0.05, (n, 2))
    tp = np.stack([np.sin(Xt[:, 1] / 4), np.cos(Xt[:, 2] / 5)], 1)
    f0 = str(tmp_path / "res" / "model")
    os.makedirs(os.path.dirname(f0))
    np.savez(f0 + ".npz", Xo=Xo, Xt=Xt, obs=obs, test_points=tp)
    HP = np.array([0.5, 6.0, 3.0, 4.0, 0.004])
    U, S = krig.scikit_prior(f0, varname="u", radar=radar, HP=HP, xrange=1000.0)
    assert U.shape == (1, yg.size, xg.size)
    sel = lambda T: np.where((T[:, 0] >= tg[0] - 6) & (T[:, 0] <= tg[0] + 6))[0]   # tlim 6, all x
    XT = np.concatenate([Xo[sel(Xo)], Xt[sel(Xt)]])
    u = np.concatenate([obs[sel(Xo), 1], tp[sel(Xt), 1]])
    mo, so = O.ard_fit_predict(XT, u, Xr, [0.5], [(6.0, 3.0, 4.0)], 0.004, jitter=1e-10)
    assert rel(U.reshape(-1), mo) < 1e-10 and rel(S.reshape(-1), so ** 2) < 1e-10
    out = f0 + "_radar_" + str(np.round(tg[0], decimals=2)) + "h_scikit_0.nc"
    d = ncio.readNC(out)
    assert np.array_equal(d["u"], U.astype(np.float32)) and np.array_equal(d["uvar"], S.astype(np.float32))
