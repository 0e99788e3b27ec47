"""engine.krige_jobs — a sweep of independent kriging jobs with job i+1's fit on a side stream
under job i's predict (the pattern bench.py --pipeline times) — must give, job by job, the
same bits as fit() + Predictor() run one job at a time, and raise for a non-SPD job as fit()
does.  The jobs mix sizes (workspace reuse and reallocation), kernel kinds and engines."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from gp2d import engine as E  # noqa: E402


def _job(seed, n, G, kind, noise=0.0025):
    rng = np.random.default_rng(seed)
    x = np.stack([rng.uniform(0, 60, n), rng.uniform(0, 45, n)], 1)
    y = np.concatenate([np.sin(x[:, 1] / 7), np.cos(x[:, 0] / 9)]) + rng.normal(0, 0.05, 2 * n)
    gx, gy = np.linspace(-5, 65, G), np.linspace(-5, 50, G + 3)
    GX, GY = np.meshgrid(gx, gy)
    xg = np.stack([GX.reshape(-1), GY.reshape(-1)], 1)
    spec = E.KernelSpec(kind=kind, l_df=4.0 + seed % 3, l_cf=3.0, ratio=0.5 if kind == "mixed" else 1.0)
    return spec, torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda"), noise, \
        torch.tensor(xg, device="cuda")


JOBS = [(1, 700, 60, "df"), (2, 700, 64, "mixed"), (3, 1500, 50, "df"), (4, 300, 40, "cf"),
        (5, 1500, 72, "mixed"), (6, 1500, 72, "df")]


@pytest.mark.parametrize("variance,ahead,batch,bahead", [
    ("ozaki", 1, None, False), ("f64", 1, None, False), ("ozaki", 2, None, False), ("ozaki", 3, None, False),
    ("ozaki", 0, None, False), ("ozaki", None, None, False), ("ozaki", 0, 1, False), ("ozaki", 0, 2, False),
    ("f64", 0, 3, False), ("ozaki", 0, 2, True), ("ozaki", 0, None, True)])
def test_krige_jobs_bit_identical_to_sequential(variance, ahead, batch, bahead):
    """fits_ahead > 1: consecutive fits in flight together, each drawing its own internal
    factor stream set; fits_ahead = 0: back to back on one stream, the fits of consecutive jobs
    of one matrix order batched (batch_fits; None = auto, 8 here; the mixed sizes of JOBS end
    batches early) — still the bits of one job at a time."""
    jobs = [_job(*j) for j in JOBS]
    got = [(m.clone(), v.clone()) for m, v in E.krige_jobs(jobs, variance=variance, chunk=2048, fits_ahead=ahead,
                                                             batch_fits=batch, batch_ahead=bahead)]
    assert len(got) == len(jobs)
    for (spec, x, y, noise, xg), (m, v) in zip(jobs, got):
        gp = E.fit(spec, x, y, noise, variance=variance)
        rm, rv = E.Predictor(gp, 2048)(xg)
        assert torch.equal(m, rm) and torch.equal(v, rv)


@pytest.mark.parametrize("ahead,bahead", [(0, False), (1, False), (2, False), (0, True)])
def test_krige_jobs_non_spd_raises_at_its_job(ahead, bahead):
    jobs = [_job(1, 500, 40, "df"), _job(2, 500, 40, "df", noise=-100.0), _job(3, 500, 40, "df")]
    gen = E.krige_jobs(jobs, variance="ozaki", chunk=1024, fits_ahead=ahead, batch_fits=2 if bahead else None,
                       batch_ahead=bahead)
    m, v = next(gen)
    assert torch.isfinite(v).all()
    with pytest.raises(np.linalg.LinAlgError):
        next(gen)


def test_krige_jobs_empty():
    assert list(E.krige_jobs([])) == []


@pytest.mark.parametrize("join", [False, True])
def test_fit_join_modes_same_bits_on_a_side_stream(join):
    """fit(join=...) only moves the host wait (gp2d_factor_join): W, α and the predictions are
    the bits of the default synchronous fit, and the mode is restored after the call."""
    spec, x, y, noise, xg = _job(7, 900, 48, "mixed")
    ref = E.fit(spec, x, y, noise, variance="ozaki")
    rm, rv = E.Predictor(ref, 2048)(xg)
    side = E.side_stream(x.device)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        gp = E.fit(spec, x, y, noise, variance="ozaki", check=False, join=join)
        m, v = E.Predictor(gp, 2048)(xg)
    torch.cuda.current_stream().wait_stream(side)
    gp.check()
    torch.cuda.synchronize()
    assert E.N.lib().gp2d_factor_join(-1) == 0
    assert torch.equal(gp.W, ref.W) and torch.equal(gp.alpha, ref.alpha)
    assert torch.equal(m, rm) and torch.equal(v, rv)


def test_factor_sets_deal_fresh_sets_to_a_new_batch():
    """gp2d_factor_sets(k > 1) starts a new batch: streams that drew set 0 at k = 1 (torch's
    pools hand the same streams out again) get distinct sets in the batch, so the batch's
    factorisations overlap instead of queueing on one set."""
    L = E.N.lib()
    spec, x, y, noise, _ = _job(9, 300, 8, "df")
    sides = [E.side_stream(x.device) for _ in range(3)]
    prev = L.gp2d_factor_sets(1)
    try:
        for st in sides:   # every stream first seen at k = 1: set 0
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                E.fit(spec, x, y, noise)
            assert L.gp2d_factor_set_of(st.cuda_stream) == 0
        L.gp2d_factor_sets(2)
        got = []
        for st in sides[1:]:   # a batch of two, in the order krige_jobs / hyper.sweep use them
            with torch.cuda.stream(st):
                E.fit(spec, x, y, noise)
            got.append(L.gp2d_factor_set_of(st.cuda_stream))
        assert sorted(got) == [0, 1], got
    finally:
        L.gp2d_factor_sets(prev)
    torch.cuda.synchronize()


def test_auto_fits_ahead_picks_the_measured_modes():
    """The library's job-shape rule (engine.auto_fits_ahead): config B's small jobs run back to
    back, the headline / C / D shapes pipelined."""
    df, mixed = E.KernelSpec(kind="df"), E.KernelSpec(kind="mixed", ratio=0.5)
    assert E.auto_fits_ahead(df, 1024, 128 * 128) == 0
    assert E.auto_fits_ahead(df, 4096, 256 * 256) == 1
    assert E.auto_fits_ahead(mixed, 4096, 256 * 256) == 1
    assert E.auto_fits_ahead(mixed, 16384, 512 * 512) == 1


def test_predictor_reuses_the_grid_order_only_for_the_same_grid():
    """With reuse_grid (what krige_jobs passes for its job grid) Predictor caches the Morton
    order of a device grid across calls with the same tensor; the bits equal a fresh
    Predictor's, and an in-place change of the grid (its version counter) or another tensor
    recomputes the order.  Without reuse_grid (the default) nothing is cached."""
    spec, x, y, noise, xg = _job(21, 600, 40, "df")
    gp = E.fit(spec, x, y, noise, variance="ozaki")
    pr = E.Predictor(gp, 1024)
    m0, v0 = (t.clone() for t in pr(xg))
    assert pr._grid is None
    m1, v1 = (t.clone() for t in pr(xg, reuse_grid=True))
    m2, v2 = (t.clone() for t in pr(xg, reuse_grid=True))
    assert torch.equal(m1, m2) and torch.equal(v1, v2) and pr._grid[0] is xg
    assert torch.equal(m0, m1) and torch.equal(v0, v1)
    fm, fv = E.Predictor(gp, 1024)(xg.clone())
    assert torch.equal(m1, fm) and torch.equal(v1, fv)
    xg.mul_(0.5)                        # in place: version bump, the cached order is stale
    m3, v3 = pr(xg, reuse_grid=True)
    rm, rv = E.Predictor(gp, 1024)(xg.clone())
    assert torch.equal(m3, rm) and torch.equal(v3, rv)


def test_warm_streams_once_per_device_and_argument_checks():
    """engine.warm_streams binds the predict stream, then the factor streams, to their hardware
    queues once per device (gp2d_factor_warm; DESIGN.md §6 "stream binding"): idempotent, and the
    fits after it are the bits of fits without it (the same kernels on the same streams)."""
    import ctypes
    from gp2d import _native as N
    L = N.lib()
    assert L.gp2d_factor_warm(0, None) < 0 and b"nsets" in L.gp2d_last_error()
    assert L.gp2d_factor_warm(5, None) < 0
    E.warm_streams()
    E.warm_streams(torch.device("cuda", torch.cuda.current_device()))
    assert torch.cuda.current_device() in E._WARM
    assert L.gp2d_factor_warm(1, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0   # sets exist: no-op
    rng = np.random.default_rng(8)
    x = np.stack([rng.uniform(0, 30, 300), rng.uniform(0, 30, 300)], 1)
    y = rng.normal(0, 0.3, 600)
    spec = E.KernelSpec(kind="df", l_df=4.0)
    a = E.fit(spec, x, y, 0.01, variance="ozaki")
    b = E.fit(spec, x, y, 0.01, variance="ozaki")
    assert torch.equal(a.W, b.W) and torch.equal(a.alpha, b.alpha)
