"""BASELINE.json configs at their real size through the HIP engine (the bench path).

Fixtures (oracle/make_golden.py, generated from the reference's own code in the build
container; /root/reference is not read here):
  * configs_N4096.npz — the headline (div-free) and config C (mixed ½/½): the bench's seeded
    N_train = 4096 tracks, the full 256 × 256 grid predicted on the GPU, checked at 512 grid
    points (the 256 nearest to an observation + 256 seeded).  `mean`/`var` are the
    reference's GP_laser.py:113-134 recipe (myKernel + np.linalg.inv); `*_refined` is the
    same posterior with an extended-precision refinement step (make_golden._refined_posterior).
  * config_d_rank0.npz — config D's rank-0 shard (N_train = 16384, 32768 of the 512² points).
  * config_e_share.npz — rank 0's share of config E's 64-setting sweep at N_train = 4096.
  * config_b_full.npz — config B at its real workload (div-free, N_train = 1024, the whole
    128 × 128 grid): the reference recipe's mean / variance at all 16,384 points, the refined
    posterior at the 512-point subsample.

Gates (north_star: fp64 posterior mean / variance within 1e-10 relative):
  * normwise: max|a − b| / max|b| ≤ 1e-10 per output vector, against the reference recipe;
  * elementwise variance: max_j |var_j − ref_j| / ref_j ≤ 1e-10 against the refined
    posterior.  The reference's own inv recipe is 1.7e-10 (div-free) / 6.6e-11 (mixed)
    elementwise from the refined one at these points (its rounding is not smaller than the
    gate), so the elementwise gate is taken against the refined values;
  * elementwise mean: |Δmean_j| ≤ 1e-10 · max(|mean_j|, 1e-2 · max|mean|) (the mean crosses
    zero, so a pure ratio is undefined at the crossings).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from gp2d import data as D  # noqa: E402
from gp2d import engine as E  # noqa: E402
from gp2d import hyper as H  # noqa: E402

GATE = 1e-10


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


def elem_var(a, b):
    return float(np.max(np.abs(a - b) / b))


def elem_mean(a, b):
    floor = 1e-2 * np.max(np.abs(b))
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), floor)))


def _at(t, idx, m):
    a = t.cpu().numpy()
    return np.concatenate([a[idx], a[m + idx]])


@pytest.fixture(scope="module")
def n4096(golden):
    g = golden("configs_N4096.npz")
    x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
    assert np.array_equal(x1, g["x"]) and np.array_equal(u, g["u"]) and np.array_equal(v, g["v"])
    _, _, xg = D.bbox_grid(x1, x2, 256, pad=5.0)
    assert np.array_equal(xg[g["idx"]], g["xg"])
    return g, np.stack([x1, x2], 1), np.concatenate([u, v]), xg


@pytest.mark.parametrize("variance", ["ozaki", "f64"])
@pytest.mark.parametrize("name", ["df", "mixed"])
def test_config_n4096_full_grid(n4096, name, variance):
    """Headline (df) and config C (mixed) exactly as bench.py runs them: fit on the device,
    predict all 65,536 grid points in 8192-point chunks (Morton order and zero-slab skipping
    active on the Ozaki engine), then the 512 fixture points."""
    g, x, y, xg = n4096
    rate = float(g[f"{name}_rate"])
    ks = E.KernelSpec(kind=name, l_df=5.0, l_cf=5.0, ratio=rate)
    gp = E.fit(ks, torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda"), noise=0.0025, variance=variance)
    assert (variance == "ozaki") == ("ozaki" in gp.extra)
    mu, var = E.Predictor(gp, 8192)(torch.tensor(xg, device="cuda"))
    m = xg.shape[0]
    idx = g["idx"]
    mu_s, var_s = _at(mu, idx, m), _at(var, idx, m)
    assert np.all(np.isfinite(var.cpu().numpy())) and np.all(var.cpu().numpy() > 0)
    M = idx.size
    for c in (slice(0, M), slice(M, 2 * M)):        # u and v components separately
        assert rel(mu_s[c], g[f"{name}_mean"][c]) < GATE
        assert rel(var_s[c], g[f"{name}_var"][c]) < GATE
    ev = elem_var(var_s, g[f"{name}_var_refined"])
    em = elem_mean(mu_s, g[f"{name}_mean_refined"])
    print(f"{name}/{variance}: var elementwise {ev:.2e}, mean elementwise {em:.2e}, "
          f"var normwise {rel(var_s, g[f'{name}_var']):.2e}")
    assert ev < GATE and em < GATE
    # the nearest-to-observation half is where the cancellation kss − ‖W k*‖² bites
    kss = g[f"{name}_kss"]
    assert np.min(g[f"{name}_var_refined"] / kss) < 1e-2


def test_config_d_rank0_shard(golden):
    """Config D: N_train = 16384 (32768² K_y), rank 0's shard of the 512² grid — the
    per-rank work of the 8-GPU run — on the Ozaki engine, at the fixture's 256 points."""
    g = golden("config_d_rank0.npz")
    x1, x2, u, v = D.synthetic_tracks(16384, seed=2016)
    assert np.allclose([x1.sum(), x2.sum()], g["x_sum"], rtol=0, atol=0)
    _, _, xg_all = D.bbox_grid(x1, x2, 512, pad=5.0)
    lo, hi = D.shard_range(xg_all.shape[0], 8, 0)
    assert (lo, hi) == (0, 32768)
    shard = xg_all[lo:hi]
    assert np.array_equal(shard[g["idx"]], g["xg"])
    ks = E.KernelSpec(kind="mixed", l_df=5.0, l_cf=5.0, ratio=float(g["rate"]))
    gp = E.fit(ks, torch.tensor(np.stack([x1, x2], 1), device="cuda"),
               torch.tensor(np.concatenate([u, v]), device="cuda"), noise=0.0025, variance="ozaki")
    mu, var = E.Predictor(gp, 8192)(torch.tensor(shard, device="cuda"))
    m = shard.shape[0]
    mu_s, var_s = _at(mu, g["idx"], m), _at(var, g["idx"], m)
    del gp
    torch.cuda.empty_cache()
    ev = elem_var(var_s, g["var"])
    print(f"D: mean {rel(mu_s, g['mean']):.2e} var {rel(var_s, g['var']):.2e} var elementwise {ev:.2e}")
    assert rel(mu_s, g["mean"]) < GATE and rel(var_s, g["var"]) < GATE
    assert ev < GATE
    assert elem_mean(mu_s, g["mean"]) < GATE


def test_config_d_distributed_fit_rank0_shard(golden):
    """Config D through the path bench.py's `single_job.distributed_fit` times at every N > 1:
    distributed.fit_distributed (block-cyclic POTRF + TRTRI over 256-column super-blocks) at
    P = 1 on N_train = 16384 (mixed, as D), then rank 0's shard of the 512² grid — against the
    reference fixture with the same normwise and elementwise gates as the engine.fit path
    (/root/reference/krig.py:541-557: one model's large grid, predicted slice by slice)."""
    from gp2d import distributed as GD
    g = golden("config_d_rank0.npz")
    x1, x2, u, v = D.synthetic_tracks(16384, seed=2016)
    assert np.allclose([x1.sum(), x2.sum()], g["x_sum"], rtol=0, atol=0)
    _, _, xg_all = D.bbox_grid(x1, x2, 512, pad=5.0)
    lo, hi = D.shard_range(xg_all.shape[0], 8, 0)
    shard = xg_all[lo:hi]
    ks = E.KernelSpec(kind="mixed", l_df=5.0, l_cf=5.0, ratio=float(g["rate"]))
    gp = GD.fit_distributed(ks, torch.tensor(np.stack([x1, x2], 1), device="cuda"),
                            torch.tensor(np.concatenate([u, v]), device="cuda"), 0.0025, variance="ozaki")
    mu, var = E.Predictor(gp, 8192)(torch.tensor(shard, device="cuda"))
    m = shard.shape[0]
    mu_s, var_s = _at(mu, g["idx"], m), _at(var, g["idx"], m)
    del gp
    torch.cuda.empty_cache()
    ev = elem_var(var_s, g["var"])
    print(f"D (fit_distributed, P = 1): mean {rel(mu_s, g['mean']):.2e} var {rel(var_s, g['var']):.2e} "
          f"var elementwise {ev:.2e}")
    assert rel(mu_s, g["mean"]) < GATE and rel(var_s, g["var"]) < GATE
    assert ev < GATE
    assert elem_mean(mu_s, g["mean"]) < GATE


def test_config_e_sweep_share(golden):
    """Config E: one rank's 8 of the 64 settings at N_train = 4096 through hyper.sweep (the
    call each of the 8 ranks makes): LML of all 8, gradient of 2, against the reference-
    myKernel fixture."""
    g = golden("config_e_share.npz")
    x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
    x, y = np.stack([x1, x2], 1), np.concatenate([u, v])
    settings = [dict(l_df=float(l), noise=float(nz)) for l, nz in zip(g["l_df"], g["noise"])]
    ks = E.KernelSpec(kind="df", l_df=5.0)
    vals, grads = H.sweep(ks, x, y, settings, noise=0.0025, eval_gradient=True)
    assert np.max(np.abs(vals - g["lml"]) / np.abs(g["lml"])) < GATE
    names = list(H.get_params(ks, 0.0025))
    il, inz = names.index("l_df"), names.index("noise")
    for k, gi in enumerate(g["grad_idx"]):
        j = list(g["share"]).index(gi)
        ref = g["grad"][k]
        # ∂/∂ℓ: the fixture's central difference is good to ~1e-8 relative; ∂/∂noise is exact
        assert abs(grads[j, il] - ref[0]) < 1e-6 * abs(ref[0])
        assert abs(grads[j, inz] - ref[1]) < 1e-9 * abs(ref[1])


@pytest.mark.parametrize("variance", ["ozaki", "f64"])
def test_config_b_full_grid(golden, variance):
    """Config B exactly as `bench.py --config B` runs it (df, N_train = 1024, 128² grid, 8192-point
    chunks): normwise per component over ALL 16,384 grid points against the reference recipe,
    elementwise at the 512 subsample points against the refined posterior."""
    g = golden("config_b_full.npz")
    x1, x2, u, v = D.synthetic_tracks(1024, seed=2016)
    assert np.array_equal(g["x_sum"], [x1.sum(), x2.sum()]) and np.array_equal(g["u_sum"], [u.sum(), v.sum()])
    _, _, xg = D.bbox_grid(x1, x2, 128, pad=5.0)
    assert np.array_equal(g["xg_sum"], xg.sum(0))
    ks = E.KernelSpec(kind="df", l_df=5.0)
    gp = E.fit(ks, torch.tensor(np.stack([x1, x2], 1), device="cuda"),
               torch.tensor(np.concatenate([u, v]), device="cuda"), noise=0.0025, variance=variance)
    mu, var = (t.cpu().numpy() for t in E.Predictor(gp, 8192)(torch.tensor(xg, device="cuda")))
    m = xg.shape[0]
    for c in (slice(0, m), slice(m, 2 * m)):
        assert rel(mu[c], g["mean"][c]) < GATE
        assert rel(var[c], g["var"][c]) < GATE
    rows = np.concatenate([g["idx"], m + g["idx"]])
    ev, em = elem_var(var[rows], g["var_refined"]), elem_mean(mu[rows], g["mean_refined"])
    print(f"B/{variance}: var normwise {rel(var, g['var']):.2e}, var elementwise {ev:.2e}, mean elementwise {em:.2e}")
    assert ev < GATE and em < GATE


def test_headline_ozaki_full_grid_elementwise(n4096):
    """The headline's Ozaki variance at EVERY one of the 65,536 grid points (both components),
    elementwise against the FP64-MFMA engine on the same fit inputs (itself 4e-12 from the
    refined posterior at the fixture points): max_j |v_oz − v_f64| / v_f64 ≤ 1e-10; the mean
    (fp64 K*α on both engines, different point orders) elementwise with the mean floor."""
    g, x, y, xg = n4096
    ks = E.KernelSpec(kind="df", l_df=5.0)
    xt, yt, gt = (torch.tensor(a, device="cuda") for a in (x, y, xg))
    out = {}
    for variance in ("ozaki", "f64"):
        gp = E.fit(ks, xt, yt, noise=0.0025, variance=variance)
        out[variance] = [t.cpu().numpy() for t in E.Predictor(gp, 8192)(gt)]
        del gp
    (mo, vo), (mf, vf) = out["ozaki"], out["f64"]
    assert vo.size == 2 * 65536 and np.all(vf > 0)
    ev, em = elem_var(vo, vf), elem_mean(mo, mf)
    print(f"headline full grid, Ozaki vs FP64 engine: var elementwise {ev:.2e}, mean elementwise {em:.2e}")
    assert ev < GATE and em < GATE


@pytest.mark.parametrize("variance", ["ozaki", "f64"])
@pytest.mark.parametrize("name", ["df", "mixed"])
def test_config_n4096_every_grid_point(golden, name, variance):
    """The headline (df) and config C (mixed) through engine.krige_jobs — the job-stream API the
    bench times; its default engine is the guarded int8 Ozaki-II one — at ALL 65,536 grid points
    (both components), normwise per component against the reference's own GP_laser.py:113-134
    recipe (myKernel + np.linalg.inv, K* in chunks) at every point (configs_N4096_full.npz),
    VERDICT r05 item 4."""
    g = golden("configs_N4096_full.npz")
    x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
    assert np.array_equal(g["x_sum"], [x1.sum(), x2.sum()]) and np.array_equal(g["u_sum"], [u.sum(), v.sum()])
    _, _, xg = D.bbox_grid(x1, x2, 256, pad=5.0)
    assert np.array_equal(g["xg_sum"], xg.sum(0))
    rate = float(g[f"{name}_rate"])
    ks = E.KernelSpec(kind=name, l_df=5.0, l_cf=5.0, ratio=rate)
    dev = torch.device("cuda")
    job = (ks, torch.tensor(np.stack([x1, x2], 1), device=dev), torch.tensor(np.concatenate([u, v]), device=dev),
           0.0025, torch.tensor(xg, device=dev))
    stats = {}
    (mu, var), = list(E.krige_jobs([job], variance=variance, stats=stats))
    mu, var = mu.cpu().numpy(), var.cpu().numpy()
    m = xg.shape[0]
    assert var.size == 2 * m and np.all(var > 0)
    errs = []
    for c in (slice(0, m), slice(m, 2 * m)):
        errs += [rel(mu[c], g[f"{name}_mean"][c]), rel(var[c], g[f"{name}_var"][c])]
    print(f"{name}/{variance} every point: normwise mean u/v, var u/v = " + ", ".join(f"{e:.2e}" for e in errs)
          + f"; guard {stats.get('guard')}")
    assert max(errs) < GATE


def test_config_d_every_rank_shard(golden):
    """Config D (mixed, N_train = 16384, 512² grid): the fit on the device (engine.fit, the
    Ozaki engine with its guard), then EACH of the 8 ranks' shards predicted as that rank would
    (data.shard_range), checked at 64 fixture points per shard (config_d_shards.npz: the
    reference's myKernel, a blocked Cholesky)."""
    g = golden("config_d_shards.npz")
    x1, x2, u, v = D.synthetic_tracks(16384, seed=2016)
    assert np.allclose([x1.sum(), x2.sum()], g["x_sum"], rtol=0, atol=0)
    _, _, xg_all = D.bbox_grid(x1, x2, 512, pad=5.0)
    assert np.array_equal(xg_all[g["gidx"]], g["xg"])
    ks = E.KernelSpec(kind="mixed", l_df=5.0, l_cf=5.0, ratio=float(g["rate"]))
    gp = E.fit(ks, torch.tensor(np.stack([x1, x2], 1), device="cuda"),
               torch.tensor(np.concatenate([u, v]), device="cuda"), noise=0.0025, variance="ozaki")
    pred = E.Predictor(gp, 8192)
    gidx = g["gidx"]
    P = 8
    mu_s, var_s = np.empty(2 * gidx.size), np.empty(2 * gidx.size)
    K = gidx.size
    for r in range(P):
        lo, hi = D.shard_range(xg_all.shape[0], P, r)
        mine = np.nonzero((gidx >= lo) & (gidx < hi))[0]
        assert mine.size == 64, r
        mu, var = (t.cpu().numpy() for t in pred(torch.tensor(xg_all[lo:hi], device="cuda")))
        m = hi - lo
        loc = gidx[mine] - lo
        mu_s[mine], mu_s[K + mine] = mu[loc], mu[m + loc]
        var_s[mine], var_s[K + mine] = var[loc], var[m + loc]
    del gp, pred
    torch.cuda.empty_cache()
    ev = elem_var(var_s, g["var"])
    print(f"D all shards: mean {rel(mu_s, g['mean']):.2e} var {rel(var_s, g['var']):.2e} var elementwise {ev:.2e}")
    assert rel(mu_s, g["mean"]) < GATE and rel(var_s, g["var"]) < GATE
    assert ev < GATE
    assert elem_mean(mu_s, g["mean"]) < GATE


def test_config_e_survey_sweep_share(golden):
    """SURVEY §8(d) config E (bench.py --config E): rank 0's 8 of the 64 settings (ℓ_df over
    [1, 10] km at ℓ_cf = 1 km; mixed α = ½, noise 0.0025) at N_train = 4096 through hyper.sweep:
    the LML of all 8 and the full gradient (ℓ_df, ℓ_cf, ratio, noise) of 2, against the
    reference-myKernel fixture (config_e_survey_share.npz)."""
    g = golden("config_e_survey_share.npz")
    x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
    x, y = np.stack([x1, x2], 1), np.concatenate([u, v])
    settings = [dict(l_df=float(a), l_cf=float(b)) for a, b in zip(g["l_df"], g["l_cf"])]
    ks = E.KernelSpec(kind="mixed", l_df=5.0, l_cf=5.0, ratio=float(g["ratio"]))
    vals, grads = H.sweep(ks, x, y, settings, noise=float(g["noise"]), eval_gradient=True)
    print("LML rel err", np.max(np.abs(vals - g["lml"]) / np.abs(g["lml"])))
    assert np.max(np.abs(vals - g["lml"]) / np.abs(g["lml"])) < GATE
    names = list(H.get_params(ks, 0.0025))
    cols = [names.index(k) for k in ("l_df", "l_cf", "ratio", "noise")]
    for k, gi in enumerate(g["grad_idx"]):
        j = list(g["share"]).index(gi)
        ref = g["grad"][k]
        got = grads[j, cols]
        print(f"setting {gi}: grad {got} vs {ref}")
        # ∂/∂ℓ, ∂/∂ratio: the fixture's central differences are good to ~1e-8 relative (of the
        # gradient's scale); ∂/∂noise is exact
        scale = np.max(np.abs(ref[:3]))
        assert np.all(np.abs(got[:3] - ref[:3]) < 1e-6 * scale)
        assert abs(got[3] - ref[3]) < 1e-9 * abs(ref[3])
