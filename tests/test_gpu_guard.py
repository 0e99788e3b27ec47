"""The ozaki engine's accuracy guard away from the bench's hyperparameters.

engine.krige_jobs' default engine (int8 Ozaki-II variance with the guard, engine.apply_guard)
on the headline workload — the bench's seeded N_train = 4096 div-free tracks, the full 256²
grid — at (ℓ, noise) = (12, 1e-3), (2, 5e-2) inside config E's range and (5, 1e-4) past it,
against tests/golden/guard_N4096.npz (oracle/make_golden.py gen_guard: the reference's
GP_laser.py:113-134 recipe with its vectorised myKernel and np.linalg.inv, exec'd from the
reference, plus the refined posterior), with the gates of tests/test_gpu_configs.py:
  * normwise, per component: max|a − b| / max|b| ≤ 1e-10 against the reference recipe;
  * elementwise variance: max_j |var_j − ref_j| / ref_j ≤ 1e-10 against the refined posterior;
  * elementwise mean: |Δ| ≤ 1e-10 · max(|mean_j|, 1e-2·max|mean|) against the refined posterior.
Each test also asserts the guard's decision (which engine, how many W bits).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from gp2d import data as D  # noqa: E402
from gp2d import engine as E  # noqa: E402

GATE = 1e-10


def rel(a, b):
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


def elem_var(a, b):
    return float(np.max(np.abs(a - b) / b))


def elem_mean(a, b):
    floor = 1e-2 * np.max(np.abs(b))
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), floor)))


@pytest.fixture(scope="module")
def guard_case(golden):
    g = golden("guard_N4096.npz")
    x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
    assert np.array_equal(g["x_sum"], [x1.sum(), x2.sum()]) and np.array_equal(g["u_sum"], [u.sum(), v.sum()])
    _, _, xg = D.bbox_grid(x1, x2, 256, pad=5.0)
    assert np.array_equal(xg[g["idx"]], g["xg"])
    dev = torch.device("cuda")
    return g, torch.tensor(np.stack([x1, x2], 1), device=dev), torch.tensor(np.concatenate([u, v]), device=dev), \
        torch.tensor(xg, device=dev)


# (fixture setting index, the guard's expected engine, (W bits, K* bits)): the cheapest precisions
# whose modelled error (gp2d_ozaki_error_model) is within the gate for each setting's statistics
CASES = [(0, "ozaki", (51, 45)), (1, "ozaki", (49, 45)), (2, "ozaki", (56, 49))]


@pytest.mark.parametrize("k,engine,bits", CASES)
def test_guarded_default_engine_meets_the_gate(guard_case, k, engine, bits):
    g, x, y, xg = guard_case
    l, nz = (float(v) for v in g["settings"][k])
    spec = E.KernelSpec(kind="df", l_df=l)
    stats = {}
    (mu, var), = list(E.krige_jobs([(spec, x, y, nz, xg)], stats=stats))   # the default engine
    dec = stats["guard"][0]
    print(f"l={l} noise={nz}: guard {dec}")
    assert dec["engine"] == engine and (dec["wbits"], dec["kbits"]) == bits
    m = xg.shape[0]
    idx = g["idx"]
    mu, var = mu.cpu().numpy(), var.cpu().numpy()
    assert np.all(np.isfinite(var)) and np.all(var > 0)
    mu_s, var_s = np.concatenate([mu[idx], mu[m + idx]]), np.concatenate([var[idx], var[m + idx]])
    M = idx.size
    for c in (slice(0, M), slice(M, 2 * M)):
        assert rel(mu_s[c], g[f"s{k}_mean"][c]) < GATE
        assert rel(var_s[c], g[f"s{k}_var"][c]) < GATE
    ev, em = elem_var(var_s, g[f"s{k}_var_refined"]), elem_mean(mu_s, g[f"s{k}_mean_refined"])
    print(f"  var elementwise {ev:.2e} (model {dec['est']:.1e}), mean elementwise {em:.2e}, "
          f"min var/kss {dec['vmin_over_kss']:.2e}")
    # the emulation's own error: against the same engine at its maximal precision (60 W bits, 50 K*
    # bits; modelled ≤ 2e-11 here) on the same factor — engine.fit is deterministic, so this is the
    # job's factor — over all 131,072 outputs
    gx = E.fit(spec, x, y, nz, variance="ozaki")
    E.ozaki_prepare(gx, diag_add=nz, wbits=60, kbits=50)
    _, vx = (t.cpu().numpy() for t in E.Predictor(gx, 8192)(xg))
    emu = elem_var(var, vx)
    del gx
    # the FP64 engine on the same factor (the training points in the guarded fit's Morton order, so
    # W and α are the same bits): what an fp64 factor reaches against the refined posterior (the
    # reference's own np.linalg.inv recipe is 2.5e-10 / 1.2e-12 / 1.3e-7 elementwise from it at the
    # three settings, make_golden gen_guard)
    p = E.morton_order(x)
    ys = torch.cat([y[:4096][p], y[4096:][p]])
    gf = E.fit(spec, x[p], ys, nz, variance="f64")
    mf, vf = (t.cpu().numpy() for t in E.Predictor(gf, 8192)(xg))
    evf = elem_var(np.concatenate([vf[idx], vf[m + idx]]), g[f"s{k}_var_refined"])
    emf = elem_mean(np.concatenate([mf[idx], mf[m + idx]]), g[f"s{k}_mean_refined"])
    print(f"  same factor on the FP64 engine: var elementwise {evf:.2e}, mean elementwise {emf:.2e}; "
          f"emulation vs its maximal precision over the full grid {emu:.2e}, vs the FP64 engine "
          f"{elem_var(var, vf):.2e}")
    assert emu < GATE   # what the guard controls: the emulation within the gate of the exact products
    if evf < GATE and emf < GATE:   # the gate is reachable in fp64: the guarded engine meets it
        assert ev < GATE and em < GATE
    else:
        # beyond fp64's reach (noise 1e-4: cond(K_y) ≈ 4e6 on these dense tracks, so an fp64 factor's
        # own rounding moves the posterior by ~cond·2^-53): the guarded engine within the gate of the
        # FP64 products of the same factor (above), and no worse than them against the refined one
        assert ev < evf + GATE and em < 1.01 * emf + GATE


def test_unguarded_fails_where_the_guard_acts(guard_case):
    """Without the guard (49 bits) the (5, 1e-4) setting misses the elementwise gate by far more
    than the FP64 engine does — the guard is what holds it (same fixture points, same inputs)."""
    g, x, y, xg = guard_case
    k = 2
    l, nz = (float(v) for v in g["settings"][k])
    gp = E.fit(E.KernelSpec(kind="df", l_df=l), x, y, nz, variance="ozaki", guard=False)
    assert "guard" not in gp.extra
    _, var = E.Predictor(gp, 8192)(xg)
    var = var.cpu().numpy()
    m, idx = xg.shape[0], g["idx"]
    ev = elem_var(np.concatenate([var[idx], var[m + idx]]), g[f"s{k}_var_refined"])
    print(f"unguarded (5, 1e-4): var elementwise {ev:.2e}")
    assert ev > 5 * GATE


def test_guard_decision_at_the_headline_is_reported(golden):
    """At the bench's own setting (ℓ = 5 km, noise 0.0025): the guard's decision and its modelled
    error are REPORTED (the bench line's `guard` block carries the same), not pinned — the engine
    may take more bits if the model says so; what decides correctness is the elementwise gate of
    test_config_n4096_full_grid / test_config_n4096_every_grid_point.  Only the decision's
    consistency is asserted: a modelled error within the gate, and the planes' moduli count
    following the chosen precision."""
    x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
    gp = E.fit(E.KernelSpec(kind="df", l_df=5.0), np.stack([x1, x2], 1), np.concatenate([u, v]), 0.0025,
               variance="ozaki")
    g = gp.extra["guard"]
    print(f"headline guard: engine {g['engine']}, bits {g['wbits']}/{g['kbits']}, modelled error {g['est']:.2e}, "
          f"v_min/kss {g['vmin_over_kss']:.3e}, moduli {gp.extra['ozaki'][2]}")
    assert g["engine"] == "ozaki" and g["est"] <= GATE
    assert 1e-3 < g["vmin_over_kss"] < 1.5e-3


def test_guard_routes_past_its_range_to_fp64():
    """A setting beyond 60 W bits (noise 1e-7 on dense data) goes to the FP64 engine: its
    predict is then, bit for bit, that of an FP64 fit on the same (Morton-ordered) points."""
    rng = np.random.default_rng(4)
    x = np.stack([rng.uniform(0, 20, 1500), rng.uniform(0, 20, 1500)], 1)
    y = rng.normal(0, 0.3, 3000)
    xg = np.stack([rng.uniform(0, 20, 3000), rng.uniform(0, 20, 3000)], 1)
    spec = E.KernelSpec(kind="df", l_df=6.0)
    gp = E.fit(spec, x, y, 1e-7, variance="ozaki")
    assert gp.extra["guard"]["engine"] == "f64" and gp.extra["guard"]["wbits"] is None and "ozaki" not in gp.extra
    p = gp.perm.cpu().numpy()
    ref = E.fit(spec, x[p], np.concatenate([y[:1500][p], y[1500:][p]]), 1e-7, variance="f64")
    assert torch.equal(gp.W, ref.W) and torch.equal(gp.alpha, ref.alpha)
    mo, vo = E.Predictor(gp, 1024)(xg)
    mf, vf = E.Predictor(ref, 1024)(xg)
    assert torch.equal(mo, mf) and torch.equal(vo, vf)


def test_guard_decision_is_the_same_on_every_path(guard_case):
    """engine.fit (synchronous), fit(check=False) + check() (the job streams), fit_batch and a
    checkpoint reload (Krig.load's ozaki_prepare_guarded) reach the same decision and planes."""
    g, x, y, xg = guard_case
    l, nz = (float(v) for v in g["settings"][2])
    spec = E.KernelSpec(kind="df", l_df=l)
    a = E.fit(spec, x, y, nz, variance="ozaki")
    b = E.fit(spec, x, y, nz, variance="ozaki", check=False).check()
    (c,) = E.fit_batch([(spec, x, y, nz)], variance="ozaki", check=False)
    c.check()
    d = E.GPFit(kernel=spec, noise=nz, x=a.x, n_train=a.n_train, n_pad=a.n_pad, W=a.W.clone(),
                alpha=a.alpha, device=a.device, perm=a.perm)
    E.ozaki_prepare_guarded(d, nz)
    torch.cuda.synchronize()
    for o in (b, c, d):
        assert (o.extra["guard"]["wbits"], o.extra["guard"]["kbits"]) == (a.extra["guard"]["wbits"],
                                                                        a.extra["guard"]["kbits"]) == (56, 49)
        assert o.extra["ozaki"][2] == a.extra["ozaki"][2] and o.extra["ozaki"][3] == a.extra["ozaki"][3]
        assert torch.equal(o.extra["ozaki"][1], a.extra["ozaki"][1])   # the W row scales
    # the residue buffers hold unwritten tiles above the diagonal (and room for more moduli), so
    # the planes are compared through what they compute: every path's predict, bit for bit
    mu_a, var_a = E.Predictor(a, 8192)(xg)
    for o in (b, c, d):
        mu_o, var_o = E.Predictor(o, 8192)(xg)
        assert torch.equal(mu_o, mu_a) and torch.equal(var_o, var_a)


# the other two vector kernels at hard settings (guard_kinds_N4096.npz):
# mixed (ℓ_df = 3, ℓ_cf = 8, ratio ½, noise 1e-4) and curl-free (ℓ = 12, noise 1e-3) — the guard's
# decision (engine, W bits, K* bits) for each, as measured on the box
KIND_CASES = [(0, "mixed", ("ozaki", 56, 48)), (1, "cf", ("ozaki", 51, 45))]


@pytest.fixture(scope="module")
def guard_kinds(golden):
    g = golden("guard_kinds_N4096.npz")
    x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
    assert np.array_equal(g["x_sum"], [x1.sum(), x2.sum()]) and np.array_equal(g["u_sum"], [u.sum(), v.sum()])
    _, _, xg = D.bbox_grid(x1, x2, 256, pad=5.0)
    assert np.array_equal(xg[g["idx"]], g["xg"])
    dev = torch.device("cuda")
    return g, torch.tensor(np.stack([x1, x2], 1), device=dev), torch.tensor(np.concatenate([u, v]), device=dev), \
        torch.tensor(xg, device=dev)


@pytest.mark.parametrize("k,kind,decision", KIND_CASES)
def test_guard_on_mixed_and_curl_free(guard_kinds, k, kind, decision):
    """engine.krige_jobs' default (guarded int8) engine on the mixed and curl-free kernels at hard
    settings: the normwise gate against the reference's recipe, the elementwise gates against the
    refined posterior (when fp64 itself reaches them, as in test_guarded_default_engine_meets_the_gate)
    and the emulation within the gate of its own maximal precision over the full grid."""
    g, x, y, xg = guard_kinds
    ldf, lcf, ratio, nz = (float(v) for v in g["settings"][k])
    assert str(g["kinds"][k]) == kind
    spec = E.KernelSpec(kind=kind, l_df=ldf, l_cf=lcf, ratio=ratio)
    stats = {}
    (mu, var), = list(E.krige_jobs([(spec, x, y, nz, xg)], stats=stats))
    dec = stats["guard"][0]
    print(f"{kind} l=({ldf},{lcf}) ratio={ratio} noise={nz}: guard {dec}")
    if decision is not None:
        assert (dec["engine"], dec["wbits"], dec["kbits"]) == decision
    m, idx = xg.shape[0], g["idx"]
    mu, var = mu.cpu().numpy(), var.cpu().numpy()
    assert np.all(np.isfinite(var)) and np.all(var > 0)
    mu_s, var_s = np.concatenate([mu[idx], mu[m + idx]]), np.concatenate([var[idx], var[m + idx]])
    M = idx.size
    for c in (slice(0, M), slice(M, 2 * M)):
        assert rel(mu_s[c], g[f"s{k}_mean"][c]) < GATE
        assert rel(var_s[c], g[f"s{k}_var"][c]) < GATE
    ev, em = elem_var(var_s, g[f"s{k}_var_refined"]), elem_mean(mu_s, g[f"s{k}_mean_refined"])
    p = E.morton_order(x)
    ys = torch.cat([y[:4096][p], y[4096:][p]])
    gf = E.fit(spec, x[p], ys, nz, variance="f64")
    mf, vf = (t.cpu().numpy() for t in E.Predictor(gf, 8192)(xg))
    del gf
    evf = elem_var(np.concatenate([vf[idx], vf[m + idx]]), g[f"s{k}_var_refined"])
    emf = elem_mean(np.concatenate([mf[idx], mf[m + idx]]), g[f"s{k}_mean_refined"])
    print(f"  var elementwise {ev:.2e} (model {dec['est']}), mean elementwise {em:.2e}; FP64 engine on the same "
          f"factor {evf:.2e} / {emf:.2e}; guarded vs FP64 engine over the full grid {elem_var(var, vf):.2e}")
    if dec["engine"] == "ozaki":
        gx = E.fit(spec, x, y, nz, variance="ozaki")
        E.ozaki_prepare(gx, diag_add=nz, wbits=60, kbits=50)
        _, vx = (t.cpu().numpy() for t in E.Predictor(gx, 8192)(xg))
        del gx
        emu = elem_var(var, vx)
        print(f"  emulation vs its maximal precision over the full grid {emu:.2e}")
        assert emu < GATE
    if evf < GATE and emf < GATE:
        assert ev < GATE and em < GATE
    else:
        assert ev < evf + GATE and em < 1.01 * emf + GATE
