"""The ozaki engine's point ordering on the device (csrc/order.hpp, include/gp2d.h
gp2d_morton_sort / gp2d_gather_rows / gp2d_obs_pad / gp2d_status_flip) and the predict's
epilogue scatter (out_order): bit-exact index work against numpy on the same inputs.

The reference never reorders points; the order is the build's own
preprocessing, so the checks are exactness (a stable sort, an exact gather / scatter) and
that predictions come back in the caller's order with the bits of an unordered predict."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from gp2d import _native as N  # noqa: E402
from gp2d import engine as E  # noqa: E402


def _codes(P):
    """Morton codes of the device kernel (gp2d_morton_codes), read back."""
    n, d = P.shape
    bbox = torch.empty(6, dtype=torch.float64, device="cuda")
    code = torch.empty(n, dtype=torch.int64, device="cuda")
    N.check(N.lib().gp2d_morton_codes(E._ptr(P), n, d, E._ptr(bbox), E._ptr(code), E._stream_handle(P.device)),
            "gp2d_morton_codes")
    return code.cpu().numpy()


@pytest.mark.parametrize("n,d,dup", [(1, 2, False), (2, 2, False), (63, 2, True), (4096, 2, False),
                                     (4097, 2, True), (20000, 3, True), (70001, 2, False), (262144, 2, True)])
def test_morton_sort_is_numpy_stable_argsort(n, d, dup):
    """The radix sort's permutation equals numpy's stable argsort of the same codes (ties keep
    the input order), over one and many 4096-key tiles, 2-D (6 digit passes) and 3-D (8)."""
    rng = np.random.default_rng(n + d)
    pts = rng.uniform(-3.0, 70.0, (n, d))
    if dup:   # many equal codes: repeated points
        pts[rng.integers(0, n, n // 2)] = pts[0]
    P = torch.tensor(pts, device="cuda")
    order, Ps = E.morton_sort(P)
    o = order.cpu().numpy()
    ref = np.argsort(_codes(P), kind="stable")
    assert np.array_equal(o, ref)
    assert np.array_equal(Ps.cpu().numpy(), pts[ref])


def test_morton_sort_full_digit_range():
    """Codes that differ only in their top and bottom digits (the bounding-box corners and
    neighbours one grid step apart at 21-bit resolution)."""
    pts = np.array([[0.0, 0.0], [1.0, 1.0], [1.0, 0.0], [0.0, 1.0], [0.5, 0.5],
                    [1.0 / 2097151, 0.0], [0.0, 1.0 / 2097151], [1.0, 1.0], [0.0, 0.0]])
    P = torch.tensor(pts, device="cuda")
    order, _ = E.morton_sort(P)
    assert np.array_equal(order.cpu().numpy(), np.argsort(_codes(P), kind="stable"))


@pytest.mark.parametrize("ntr,npad,bd", [(1, 64, 2), (37, 64, 2), (4096, 4096, 2), (100, 128, 1)])
def test_obs_pad(ntr, npad, bd):
    rng = np.random.default_rng(ntr)
    y = rng.normal(size=bd * ntr)
    perm = rng.permutation(ntr)
    out = E._pad_obs(torch.tensor(y, device="cuda"), ntr, npad, bd, torch.device("cuda"),
                     torch.tensor(perm, device="cuda")).cpu().numpy()
    ref = np.zeros(bd * npad)
    for c in range(bd):
        ref[c * npad:c * npad + ntr] = y[c * ntr:(c + 1) * ntr][perm]
    assert np.array_equal(out, ref)
    out0 = E._pad_obs(y, ntr, npad, bd, torch.device("cuda")).cpu().numpy()   # identity, host input
    ref0 = np.zeros(bd * npad)
    for c in range(bd):
        ref0[c * npad:c * npad + ntr] = y[c * ntr:(c + 1) * ntr]
    assert np.array_equal(out0, ref0)


def test_gather_rows_wide():
    rng = np.random.default_rng(3)
    src = rng.normal(size=(9, 1000))
    order = np.array([8, 0, 3, 3, 7], dtype=np.int64)
    S = torch.tensor(src, device="cuda")
    dst = torch.empty((5, 1000), dtype=torch.float64, device="cuda")
    N.check(N.lib().gp2d_gather_rows(E._ptr(S), E._ptr(torch.tensor(order, device="cuda")), 5, 1000, E._ptr(dst),
                                     E._stream_handle(S.device)), "gp2d_gather_rows")
    assert np.array_equal(dst.cpu().numpy(), src[order])


def test_status_flip_is_an_involution():
    v = np.array([0, 5, 2147483647, -1, 0, 17], dtype=np.int32)
    t = torch.tensor(v, device="cuda")
    L = N.lib()
    N.check(L.gp2d_status_flip(E._ptr(t), t.numel(), E._stream_handle(t.device)), "gp2d_status_flip")
    assert t.cpu().tolist() == [2147483647, 5, 0, -1, 2147483647, 17]
    N.check(L.gp2d_status_flip(E._ptr(t), t.numel(), E._stream_handle(t.device)), "gp2d_status_flip")
    assert np.array_equal(t.cpu().numpy(), v)


def test_potrf_resets_info():
    """gp2d_potrf zeroes the caller's info word itself (the engine allocates it uninitialised)."""
    n = 256
    A = torch.eye(n, dtype=torch.float64, device="cuda") * 2.0
    info = torch.full((1,), 12345, dtype=torch.int32, device="cuda")
    dinv = torch.empty((n // 128, 128, 128), dtype=torch.float64, device="cuda")
    N.check(N.lib().gp2d_potrf(E._ptr(A), n, n, E._ptr(dinv), E._ptr(info), None, 0, E._stream_handle(A.device)),
            "gp2d_potrf")
    assert int(info.item()) == 0


@pytest.mark.parametrize("m", [1, 300, 20000])
def test_predict_scatter_matches_sorted_grid(m):
    """The ozaki predict on a grid it Morton-orders itself (outputs scattered by the epilogue)
    returns, point for point, the bits of a predict on the pre-sorted grid."""
    rng = np.random.default_rng(m)
    x = np.stack([rng.uniform(0, 60, 700), rng.uniform(0, 45, 700)], 1)
    y = rng.normal(0, 0.3, 1400)
    xg = np.stack([rng.uniform(-5, 65, m), rng.uniform(-5, 50, m)], 1)
    gp = E.fit(E.KernelSpec(kind="mixed", l_df=5.0, l_cf=4.0, ratio=0.5), x, y, noise=0.0025, variance="ozaki")
    G = torch.tensor(xg, device="cuda")
    mu, var = (t.cpu().numpy() for t in E.Predictor(gp, 1024)(G))
    order, Gs = E.morton_sort(G)
    o = order.cpu().numpy()
    mu_s, var_s = (t.cpu().numpy() for t in E.Predictor(gp, 1024)(Gs))
    # Gs is already in Morton order, so sorting it again is the identity and no scatter applies
    for c in range(2):
        assert np.array_equal(mu[c * m + o], mu_s[c * m:(c + 1) * m])
        assert np.array_equal(var[c * m + o], var_s[c * m:(c + 1) * m])
