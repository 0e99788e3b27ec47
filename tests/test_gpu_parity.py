"""HIP path vs the CPU oracle on identical seeded inputs (calls through the C ABI).

Tolerances (north_star): fp64 posterior mean / variance within 1e-10 relative,
measured normwise (max |a−b| / max |b|) per output vector; covariance entries
within 1e-13 relative to the matrix max-norm.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from gp2d import engine as E  # noqa: E402
from oracle import gp2d_oracle as O  # noqa: E402


def rel(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def tracks(n, seed=2016):
    rng = np.random.default_rng(seed)
    x = np.stack([rng.uniform(0, 60, n), rng.uniform(0, 45, n)], 1)
    u = np.sin(x[:, 1] / 7) + rng.normal(0, 0.05, n)
    v = np.cos(x[:, 0] / 9) + rng.normal(0, 0.05, n)
    return x, np.concatenate([u, v])


@pytest.mark.parametrize("kind,ratio", [("df", 1.0), ("cf", 0.0), ("mixed", 0.3), ("scalar", 1.0)])
@pytest.mark.parametrize("na,nb", [(1, 1), (37, 100), (130, 64)])
def test_assemble_matches_oracle(kind, ratio, na, nb):
    rng = np.random.default_rng(na * 1000 + nb)
    xa = rng.uniform(0, 10, (na, 2))
    xb = rng.uniform(0, 10, (nb, 2))
    ks = E.KernelSpec(kind=kind, l_df=2.5, l_cf=3.5, ratio=ratio)
    K = E.assemble(ks, xa, xb).cpu().numpy()
    R = O.vector_kernel(xa, xb, kind, 2.5, 3.5, ratio)
    assert K.shape == R.shape
    assert rel(K, R) < 1e-13


def test_assemble_golden_small(golden):
    g = golden("gp_scripts_small.npz")
    xa = np.stack([g["x1"], g["x2"]], 1)
    xb = np.stack([g["x1s"], g["x2s"]], 1)
    for kind, name in ((1, "df"), (2, "cf"), (0, "scalar")):
        ks = E.KernelSpec(kind=name, l_df=float(g["sigma"]), l_cf=float(g["sigma"]))
        assert rel(E.assemble(ks, xa).cpu().numpy(), g[f"K_{kind}"]) < 1e-13
        assert rel(E.assemble(ks, xb, xa).cpu().numpy(), g[f"Ks_{kind}"]) < 1e-13


@pytest.mark.parametrize("ntr,m,kind", [(16, 64, "df"), (100, 300, "mixed"), (256, 1000, "cf"), (700, 2500, "df")])
def test_fit_predict_matches_oracle(ntr, m, kind):
    x, y = tracks(ntr, seed=ntr)
    rng = np.random.default_rng(m)
    xg = np.stack([rng.uniform(-5, 65, m), rng.uniform(-5, 50, m)], 1)
    ks = E.KernelSpec(kind=kind, l_df=5.0, l_cf=4.0, ratio=0.5 if kind == "mixed" else 1.0)
    gp = E.fit(ks, x, y, noise=0.0025)
    mu, var = E.predict(gp, xg, chunk=256)
    mo, vo = O.fit_predict(x, y, xg, kind=kind, l_df=5.0, l_cf=4.0, ratio=ks.ratio, noise=0.0025)
    assert rel(mu.cpu().numpy(), mo) < 1e-10
    assert rel(var.cpu().numpy(), vo) < 1e-10


def test_golden_mykernel_N1024(golden):
    g = golden("mykernel_mixed_N1024.npz")
    x = np.stack([g["x"], g["y"]], 1)
    y = np.concatenate([g["u"], g["v"]])
    ks = E.KernelSpec(kind="mixed", l_df=5.0, l_cf=5.0, ratio=0.5)
    gp = E.fit(ks, x, y, noise=float(g["noise"]))
    mu, var = E.predict(gp, g["xg"])
    assert rel(mu.cpu().numpy(), g["mean"]) < 1e-10
    assert rel(var.cpu().numpy(), g["var"]) < 1e-10


@pytest.mark.parametrize("kind,npts", [("df", 4096), ("mixed", 700), ("cf", 96), ("df", 1)])
def test_assemble_lower_block_triangle(kind, npts):
    """gp2d_assemble(symmetric = 2), the fit's assembly: into a NaN-filled buffer it writes
    exactly K_y's lower triangle (entries (R, C) with C ≤ R), bit for bit the full assembly's
    values there, and leaves every other entry unwritten (still NaN: half the stores at
    n = 8192); gp2d_potrf + gp2d_trtri from that buffer give the bits of the full assembly's
    factor and inverse, so nothing in the factorisation uses the unwritten part.
    npts = 700 pads to 11·64 points (the component boundary inside a 128-block); 1 is a
    single block."""
    import ctypes
    from gp2d import _native as N
    L_ = N.lib()
    x, _ = tracks(npts, seed=npts + 3)
    ks = E.KernelSpec(kind=kind, l_df=5.0, l_cf=4.0, ratio=0.5 if kind == "mixed" else (0.0 if kind == "cf" else 1.0))
    npad = int(L_.gp2d_padded_points(npts))
    n = 2 * npad
    ld = (n + 127) // 128 * 128
    X = torch.tensor(x, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    desc = ks.desc()
    full = torch.full((ld, ld), float("nan"), dtype=torch.float64, device="cuda")
    low = full.clone()
    N.check(L_.gp2d_assemble(P(X), npts, npad, P(X), npts, npad, ctypes.byref(desc), 0.0025, 1, P(full), ld, s), "a1")
    N.check(L_.gp2d_assemble(P(X), npts, npad, P(X), npts, npad, ctypes.byref(desc), 0.0025, 2, P(low), ld, s), "a2")
    F, Lo = full.cpu().numpy()[:n, :n], low.cpu().numpy()[:n, :n]
    R, C = np.indices((n, n))
    keep = C <= R
    assert np.array_equal(Lo[keep], F[keep]) and np.all(np.isfinite(F))
    assert np.all(np.isnan(Lo[~keep]))
    if n >= 8192:   # the stores: ≤ 270 MB at n = 8192
        assert 8 * int(keep.sum()) <= 270e6
    if ld != n:
        return   # gp2d_potrf needs a multiple of 128
    outs = []
    for A in (full, low):
        dinv = torch.empty((n // 128, 128, 128), dtype=torch.float64, device="cuda")
        info = torch.zeros(1, dtype=torch.int32, device="cuda")
        N.check(L_.gp2d_potrf(P(A), n, n, P(dinv), P(info), None, 0, s), "potrf")
        wb = int(L_.gp2d_trtri_workspace(n))
        work = torch.empty(wb // 8 + 1, dtype=torch.float64, device="cuda")
        N.check(L_.gp2d_trtri(P(A), n, n, P(dinv), P(work), wb, s), "trtri")
        torch.cuda.synchronize()
        assert int(info.item()) == 0
        outs.append(A.cpu().numpy())
    assert np.all(np.isfinite(outs[1])) and np.array_equal(outs[0], outs[1])


def _spd(n, seed):
    rng = np.random.default_rng(seed)
    A = rng.normal(size=(n, n))
    return A @ A.T / n + np.eye(n) * 0.5


@pytest.mark.parametrize("n", [128, 384, 1024])
def test_potrf_trtri_potrs_abi(n):
    """gp2d_potrf / gp2d_trtri / gp2d_potrs_inv vs LAPACK on a random SPD matrix."""
    import ctypes
    from gp2d import _native as N
    L_ = N.lib()
    K = _spd(n, n)
    A = torch.tensor(K, device="cuda")
    dinv = torch.empty((n // 128, 128, 128), dtype=torch.float64, device="cuda")
    info = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    N.check(L_.gp2d_potrf(P(A), n, n, P(dinv), P(info), None, 0, s), "potrf")
    assert int(info.item()) == 0
    Lref = np.linalg.cholesky(K)
    Lg = A.cpu().numpy()
    assert np.array_equal(np.triu(Lg, 1), np.zeros_like(Lg))
    assert rel(Lg, Lref) < 1e-13
    wb = int(L_.gp2d_trtri_workspace(n))
    work = torch.empty(wb // 8 + 1, dtype=torch.float64, device="cuda")
    N.check(L_.gp2d_trtri(P(A), n, n, P(dinv), P(work), wb, s), "trtri")
    W = A.cpu().numpy()
    assert rel(W, np.linalg.inv(Lref)) < 1e-12
    y = np.random.default_rng(1).normal(size=n)
    yt = torch.tensor(y, device="cuda")
    al = torch.empty(n, dtype=torch.float64, device="cuda")
    pb = int(L_.gp2d_potrs_workspace(n))
    pw = torch.empty(pb // 8 + 1, dtype=torch.float64, device="cuda")
    N.check(L_.gp2d_potrs_inv(P(A), n, n, P(yt), P(al), P(pw), pb, s), "potrs")
    assert rel(al.cpu().numpy(), np.linalg.solve(K, y)) < 1e-11
    # trtri without the diagonal inverses (stand-alone path)
    A2 = torch.tensor(Lref, device="cuda")
    N.check(L_.gp2d_trtri(P(A2), n, n, None, P(work), wb, s), "trtri(no dinv)")
    assert rel(A2.cpu().numpy(), np.linalg.inv(Lref)) < 1e-12


@pytest.mark.parametrize("n", [128, 384, 1152, 2560, 8192])
def test_potrf_inv_matches_two_calls(n):
    """gp2d_potrf_inv (TRTRI GEMMs overlapped with the factorisation) is bit-identical to
    gp2d_potrf + gp2d_trtri: the same GEMMs on the same operands, only issued earlier.  Sizes
    cover power-of-two and ragged block counts (3, 9, 20 blocks) and the bench's n = 8192."""
    import ctypes
    from gp2d import _native as N
    L_ = N.lib()
    K = _spd(n, n + 1)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    A1 = torch.tensor(K, device="cuda")
    A2 = A1.clone()
    d1 = torch.empty((n // 128, 128, 128), dtype=torch.float64, device="cuda")
    d2 = torch.empty_like(d1)
    i1 = torch.zeros(1, dtype=torch.int32, device="cuda")
    i2 = torch.zeros(1, dtype=torch.int32, device="cuda")
    N.check(L_.gp2d_potrf(P(A1), n, n, P(d1), P(i1), None, 0, s), "potrf")
    wb = int(L_.gp2d_trtri_workspace(n))
    work = torch.empty(wb // 8 + 1, dtype=torch.float64, device="cuda")
    N.check(L_.gp2d_trtri(P(A1), n, n, P(d1), P(work), wb, s), "trtri")
    wb2 = int(L_.gp2d_potrf_inv_workspace(n))
    work2 = torch.full((wb2 // 8 + 1,), float("nan"), dtype=torch.float64, device="cuda")
    N.check(L_.gp2d_potrf_inv(P(A2), n, n, P(d2), P(i2), P(work2), wb2, s), "potrf_inv")
    assert int(i1.item()) == 0 and int(i2.item()) == 0
    assert torch.equal(A1, A2) and torch.equal(d1, d2)
    if n <= 2560:
        assert rel(A2.cpu().numpy(), np.linalg.inv(np.linalg.cholesky(K))) < 1e-12


@pytest.mark.parametrize("variance", ["f64", "ozaki"])
def test_not_positive_definite_raises(variance):
    """Non-SPD K_y → LAPACK-style info → numpy.linalg.LinAlgError (np.linalg.inv / sklearn paths),
    also when the Ozaki preparation runs on the failed factor before `info` is read."""
    x = np.zeros((3, 2))  # three identical points, no noise: singular K
    with pytest.raises(np.linalg.LinAlgError):
        E.fit(E.KernelSpec(kind="df", l_df=1.0), x, np.zeros(6), noise=-1e-3, variance=variance)
    # deferred form (bench.py): fit returns at once, GPFit.check() raises the same error
    gp = E.fit(E.KernelSpec(kind="df", l_df=1.0), x, np.zeros(6), noise=-1e-3, variance=variance, check=False)
    with pytest.raises(np.linalg.LinAlgError):
        gp.check()
    ok = E.fit(E.KernelSpec(kind="df", l_df=1.0), tracks(40, seed=1)[0], tracks(40, seed=1)[1], noise=0.01,
               variance=variance, check=False)
    assert ok.check() is ok and ok.pending is None


def test_sharded_predict_bit_identical():
    """Grid shards (any split) concatenate to the single-launch result bit-for-bit."""
    from gp2d import data as D
    x, y = tracks(300, seed=3)
    rng = np.random.default_rng(4)
    xg = np.stack([rng.uniform(-5, 65, 5000), rng.uniform(-5, 50, 5000)], 1)
    gp = E.fit(E.KernelSpec(kind="mixed", l_df=5.0, l_cf=3.0, ratio=0.4), x, y, noise=0.0025)
    m_all, v_all = (t.cpu().numpy() for t in E.predict(gp, xg, chunk=1024))
    for ws in (2, 3, 8):
        shards_m, shards_v = [], []
        for r in range(ws):
            lo, hi = D.shard_range(xg.shape[0], ws, r)
            mm, vv = E.predict(gp, xg[lo:hi], chunk=512)
            shards_m.append((lo, hi, mm.cpu().numpy()))
            shards_v.append((lo, hi, vv.cpu().numpy()))
        from gp2d.distributed import assemble_from_shards
        assert np.array_equal(assemble_from_shards(xg.shape[0], 2, shards_m), m_all)
        assert np.array_equal(assemble_from_shards(xg.shape[0], 2, shards_v), v_all)


@pytest.mark.parametrize("variance", ["f64", "ozaki"])
def test_jitchol_retry(variance):
    """GPy jitchol semantics (GPy.util.linalg.jitchol; GPy absent here — parity unpinned, the
    published algorithm): a singular K_y (repeated points, no noise) fails without the option;
    with jitchol=5 the fit succeeds with jitter = mean(diag K_y)·1e-6·10^t for the first
    try t that factors, and equals a plain fit with that jitter bit for bit."""
    rng = np.random.default_rng(4)
    x = rng.uniform(0, 20, (60, 2))
    x = np.concatenate([x, x[:5]])   # five repeated points: K is singular
    y = rng.normal(size=2 * x.shape[0])
    ks = E.KernelSpec(kind="df", l_df=3.0)
    with pytest.raises(np.linalg.LinAlgError):
        E.fit(ks, x, y, noise=0.0, variance=variance)
    gp = E.fit(ks, x, y, noise=0.0, variance=variance, jitchol=5)
    jit = gp.extra["jitchol"]
    base = (1.0 / 9.0) * 1e-6                       # mean(diag K_y) = 1/ℓ² for the div-free kernel
    ratios = [jit / (base * 10 ** t) for t in range(5)]
    assert any(abs(r - 1.0) < 1e-12 for r in ratios), jit
    ref = E.fit(ks, x, y, noise=0.0, jitter=jit, variance=variance)
    assert torch.equal(gp.W, ref.W) and torch.equal(gp.alpha, ref.alpha)
    xg = rng.uniform(0, 20, (300, 2))
    a, b = E.predict(gp, xg), E.predict(ref, xg)
    assert torch.equal(a[0], b[0])
    assert torch.equal(a[1], b[1]) or variance == "ozaki"   # (the ozaki CRT may poison both alike: NaN ≠ NaN)
    # a well-posed fit reports no jitter
    assert E.fit(ks, x[:60], y[:120], noise=0.01, variance=variance, jitchol=5).extra["jitchol"] == 0.0


_SCHED_CHILD = r'''
import ctypes, hashlib, json, sys
import numpy as np, torch
sys.path[:0] = sys.argv[2:4]
from gp2d import _native as N
L_ = N.lib()
out = {}
for n in json.loads(sys.argv[1]):
    rng = np.random.default_rng(n)
    X = rng.normal(size=(n, n))
    K = X @ X.T / n + np.eye(n) * 0.5
    A = torch.tensor(K, device="cuda")
    dinv = torch.empty((n // 128, 128, 128), dtype=torch.float64, device="cuda")
    info = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    N.check(L_.gp2d_potrf(P(A), n, n, P(dinv), P(info), None, 0, s), "potrf")
    Lg = A.cpu().numpy()
    Lr = np.linalg.cholesky(K)
    out[n] = dict(info=int(info.item()), upper=float(np.abs(np.triu(Lg, 1)).max()),
                  rel=float(np.abs(Lg - Lr).max() / np.abs(Lr).max()),
                  sha=hashlib.sha256(Lg.tobytes()).hexdigest())
print(json.dumps(out))
'''


def test_potrf_trailing_schedules():
    """Every trailing-update schedule of potrf_impl — pairs (K = 256), four panels (K = 512)
    and four panels with the head/rest split (the large-n default) — against LAPACK at block
    counts 1, 2, 3, 5, 9, 21 (ragged last groups); the split changes no bits (each tile gets
    the same K = 512 sum, only in another launch)."""
    import json
    import subprocess
    import sys
    from conftest import PKG, ROOT
    sizes = [128, 256, 384, 640, 1152, 2688]
    res = {}
    for G, split in [(2, 0), (4, 0), (4, 1)]:
        env = dict(os.environ, GP2D_POTRF_G=str(G), GP2D_POTRF_SPLIT=str(split))
        out = subprocess.run([sys.executable, "-c", _SCHED_CHILD, json.dumps(sizes), ROOT, PKG], env=env,
                             capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stderr[-2000:]
        res[(G, split)] = json.loads(out.stdout.strip().splitlines()[-1])
        for n, r in res[(G, split)].items():
            assert r["info"] == 0 and r["upper"] == 0.0, (G, split, n, r)
            assert r["rel"] < 1e-13, (G, split, n, r)
    for n in map(str, sizes):
        assert res[(4, 0)][n]["sha"] == res[(4, 1)][n]["sha"], n
