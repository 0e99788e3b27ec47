"""Edge cases of the HIP path (both variance engines) against the CPU oracle: an empty grid,
one training point, ragged training counts (padding to 64 / 128 points), a grid one point
past a chunk boundary, and duplicated observation sites (SPD only through the noise).
Tolerance: 1e-10 relative, normwise per output vector (north_star)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from gp2d import engine as E  # noqa: E402
from oracle import gp2d_oracle as O  # noqa: E402

ENGINES = ["f64", "ozaki"]


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def tracks(n, seed):
    rng = np.random.default_rng(seed)
    x = np.stack([rng.uniform(0, 60, n), rng.uniform(0, 45, n)], 1)
    y = np.concatenate([np.sin(x[:, 1] / 7), np.cos(x[:, 0] / 9)]) + rng.normal(0, 0.05, 2 * n)
    return x, y


def grid(m, seed):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(-5, 65, m), rng.uniform(-5, 50, m)], 1)


@pytest.mark.parametrize("variance", ENGINES)
def test_empty_grid(variance):
    x, y = tracks(50, 1)
    gp = E.fit(E.KernelSpec(kind="df", l_df=5.0), x, y, noise=0.0025, variance=variance)
    mu, var = E.predict(gp, np.zeros((0, 2)))
    assert mu.numel() == 0 and var.numel() == 0


@pytest.mark.parametrize("variance", ENGINES)
@pytest.mark.parametrize("ntr", [1, 63, 65, 129, 257])
def test_ragged_training_counts(variance, ntr):
    x, y = tracks(ntr, ntr)
    xg = grid(300, ntr + 1)
    ks = E.KernelSpec(kind="mixed", l_df=5.0, l_cf=4.0, ratio=0.5)
    gp = E.fit(ks, x, y, noise=0.0025, variance=variance)
    mu, var = (t.cpu().numpy() for t in E.predict(gp, xg))
    mo, vo = O.fit_predict(x, y, xg, kind="mixed", l_df=5.0, l_cf=4.0, ratio=0.5, noise=0.0025)
    assert rel(mu, mo) < 1e-10 and rel(var, vo) < 1e-10


@pytest.mark.parametrize("variance", ENGINES)
def test_grid_one_past_chunk_boundary(variance):
    x, y = tracks(120, 5)
    xg = grid(1025, 6)                     # chunk 1024 → a second chunk with one point
    ks = E.KernelSpec(kind="df", l_df=5.0)
    gp = E.fit(ks, x, y, noise=0.0025, variance=variance)
    mu, var = (t.cpu().numpy() for t in E.predict(gp, xg, chunk=1024))
    mo, vo = O.fit_predict(x, y, xg, kind="df", l_df=5.0, noise=0.0025)
    assert rel(mu, mo) < 1e-10 and rel(var, vo) < 1e-10
    m1, v1 = (t.cpu().numpy() for t in E.predict(gp, xg[-1:], chunk=1024))   # the lone point alone
    assert np.array_equal(m1, mu[[1024, 2049]]) and np.array_equal(v1, var[[1024, 2049]])


@pytest.mark.parametrize("variance", ENGINES)
def test_duplicate_sites(variance):
    x, y = tracks(80, 7)
    x = np.concatenate([x, x[:20]])        # 20 sites observed twice (different noise draws)
    y = np.concatenate([y[:80], y[:20] + 0.01, y[80:], y[80:100] - 0.01])
    xg = grid(400, 8)
    ks = E.KernelSpec(kind="cf", l_cf=6.0)
    gp = E.fit(ks, x, y, noise=0.01, variance=variance)
    mu, var = (t.cpu().numpy() for t in E.predict(gp, xg))
    mo, vo = O.fit_predict(x, y, xg, kind="cf", l_cf=6.0, noise=0.01)
    assert rel(mu, mo) < 1e-10 and rel(var, vo) < 1e-10
