"""The bit-exact host index rows of SURVEY.md §8(a), re-checked on the GPU box.

grids (krig.getGrid, krig.py:648-678), the train/test split with CPython's set order
(GP_laser.py:80-83, krig.py:300-337), the data preparation on simulTracks coordinates
(krig.py:42-86, 300-381) and scikit_prior's observation window (krig.py:146-167) are host
numpy work that feeds the HIP engine.  The CPU suite pins them against the committed
fixtures; this module runs the same product functions against the same fixtures in the
driver's `-m gpu` record (seconds), next to the GPU parity tests that consume their outputs.
"""
import pytest

import test_host_cpu as H

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)


def test_get_grid_bit_exact_on_box(golden):
    H.test_get_grid_bit_exact(golden)


def test_split_indices_bit_exact_on_box(golden):
    H.test_split_indices_bit_exact(golden)


def test_laser_split_and_grid_on_box(golden):
    H.test_laser_split_and_grid(golden)


@pytest.mark.parametrize("case", range(5))
def test_data_prep_bit_exact_on_box(golden, case):
    H.test_data_prep_bit_exact_on_tracks(golden, case)


@pytest.mark.parametrize("case", range(3))
def test_prior_window_bit_exact_on_box(golden, case):
    H.test_prior_window_bit_exact(golden, case)


def test_prepared_tracks_feed_the_engine(golden):
    """The prepared training set of one fixture case goes through the HIP fit + predict: the
    index work's output is what the engine consumes (shapes, component order obs = [v; u])."""
    import numpy as np

    from gp2d import engine as E
    from gp2d import krig as K
    g = golden("prep_tracks.npz")
    tr = K.Tracks(g["time"], g["lat"], g["lon"], g["u"], g["v"])
    st, et, ss, skip, la0, la1, lo0, lo1 = g["c0_args"]
    d = K._prepare(tr, int(st), int(et), (la0, la1), (lo0, lo1), int(ss), int(skip), drop_drifters=(238,))
    X = np.ascontiguousarray(d["X"][:, 1:], dtype=np.float64)   # (Y, X) of the T,Y,X stack
    obs = np.concatenate([d["vo"][:, 0], d["uo"][:, 0]])
    keep = np.arange(min(400, X.shape[0]))
    xs, ys = X[keep], np.concatenate([obs[:X.shape[0]][keep], obs[X.shape[0]:][keep]])
    gp = E.fit(E.KernelSpec(kind="df", l_df=3.0), xs, ys, noise=0.0025, device="cuda:0", variance="ozaki")
    mean, var = E.predict(gp, xs[:64])
    assert mean.shape == (128,) and torch.isfinite(mean).all() and (var >= -1e-12).all()
