"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

TEST INFRASTRUCTURE ONLY — run in the build container (it reads /root/reference,
which does not exist on the GPU box).  The committed .npz files are data: inputs
plus the reference's outputs; no reference source is copied into the repo.

How the reference is run:
  * GP_scripts.py lines 1-142 (myKernel, getMean, getCov, nonDivK, compute_K,
    compute_Ks, sqExp, rbf) are exec'd unmodified from the file text.  The rest of
    that file is Python-2-only (print statement at GP_scripts.py:173).
  * The GP_laser.laser() posterior recipe (GP_laser.py:113-140) and the split
    (GP_laser.py:80-96) are reproduced by calling those exec'd functions with the
    same numpy expressions the script uses.  GP_laser.py itself cannot be imported
    (py2 syntax, geopy/pyproj missing, interp_ALL_2016_2_7.pkl missing).
  * krig.getGrid (krig.py:648-678) is exec'd from the file text with its two
    py2 `print 'here x'` statements replaced by `pass` (no other change).
  * krig.scikit_prior's model (krig.py:174-194) runs on the installed
    scikit-learn (1.7.2; the reference pins no version).
  * simulTracks.pkl supplies realistic drifter coordinates.  It is loaded with a
    restricted unpickler that allows only numpy array reconstruction and the
    laser_class.interpolated_tracks container.

Usage:  python oracle/make_golden.py [--out tests/golden]
"""
from __future__ import annotations

import argparse
import os
import pickle
import time

import numpy as np

REF = "/root/reference"


def load_gp_scripts():
    with open(os.path.join(REF, "GP_scripts.py")) as f:
        lines = f.readlines()
    src = "".join(lines[:142])
    ns: dict = {}
    exec(compile(src, "GP_scripts.py[1:142]", "exec"), ns)
    return ns


def load_get_grid():
    with open(os.path.join(REF, "krig.py")) as f:
        lines = f.readlines()
    body = lines[647:678]  # krig.py:648-678
    fixed = []
    for ln in body:
        if ln.strip().startswith("print "):
            ind = ln[: len(ln) - len(ln.lstrip())]
            fixed.append(ind + "pass\n")
        else:
            fixed.append(ln)
    ns = {"np": np}
    exec(compile("".join(fixed), "krig.py[648:678]", "exec"), ns)
    return ns["getGrid"]


class _Tracks:
    pass


class _RestrictedUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if module == "laser_class" and name == "interpolated_tracks":
            return _Tracks
        if module in ("numpy.core.multiarray", "numpy._core.multiarray") and name in ("_reconstruct", "scalar"):
            import numpy.core.multiarray as m
            return getattr(m, name)
        if module == "numpy" and name in ("ndarray", "dtype"):
            return getattr(np, name)
        raise pickle.UnpicklingError(f"blocked global {module}.{name}")


def load_tracks():
    with open(os.path.join(REF, "simulTracks.pkl"), "rb") as f:
        return _RestrictedUnpickler(f, encoding="latin1").load()


def project_km(lat, lon, lat0=28.69, lon0=-88.28):
    """Signed local equirectangular projection (the reference's geopy/pyproj projections
    are unavailable and simLaser's is unsigned)."""
    R = 6371.0
    x = R * np.cos(np.deg2rad(lat0)) * np.deg2rad(lon - lon0)
    y = R * np.deg2rad(lat - lat0)
    return x, y


def synthetic_tracks(n, seed=2016, box=(60.0, 45.0), amp=1.0, L=15.0, noise_sd=0.05):
    """SURVEY.md §8(d) synthetic inputs (also used by bench.py through gp2d.data)."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(0, box[0], n)
    y = rng.uniform(0, box[1], n)
    x0, y0 = box[0] / 2, box[1] / 2
    psi = amp * np.exp(-((x - x0) ** 2 + (y - y0) ** 2) / L ** 2)
    u = psi * (-2 * (y - y0) / L ** 2)       # u = dψ/dy
    v = -psi * (-2 * (x - x0) / L ** 2)      # v = -dψ/dx
    u = u + rng.normal(0, noise_sd, n)
    v = v + rng.normal(0, noise_sd, n)
    return x, y, u, v


def gen_small(gs, out):
    """compute_K / compute_Ks / getCov / getMean on tiny problems, all three divFree kinds,
    plus the vectorised myKernel (mixed)."""
    rng = np.random.default_rng(7)
    N = 16
    x1 = rng.uniform(0, 3, N)
    x2 = rng.uniform(0, 3, N)
    g = np.linspace(-0.5, 3.5, 8)
    X1s, X2s = np.meshgrid(g, g)
    x1s, x2s = X1s.reshape(-1), X2s.reshape(-1)
    u = rng.normal(0, 1, N)
    v = rng.normal(0, 1, N)
    y = np.concatenate([u, v])[:, None]
    noise = 0.01
    sigma = 0.7
    d = dict(x1=x1, x2=x2, x1s=x1s, x2s=x2s, y=y[:, 0], sigma=sigma, noise=noise)
    for kind in (0, 1, 2):
        K = gs["compute_K"](x1, x2, sigma, kind)
        Ks = gs["compute_Ks"](x1, x2, x1s, x2s, sigma, kind)
        Kss = gs["compute_K"](x1s, x2s, sigma, kind)
        Ky = K + np.identity(K.shape[0]) * noise          # GP_laser.py:114-115
        Ki = np.linalg.inv(Ky)                           # GP_laser.py:118
        Cov = Kss - np.dot(Ks, np.dot(Ki, Ks.T))         # GP_laser.py:129
        M = x1s.size
        f = gs["getMean"](Ks, Ki, y)                     # GP_laser.py:134
        d[f"K_{kind}"] = K
        d[f"Ks_{kind}"] = Ks
        d[f"Kssdiag_{kind}"] = np.diag(Kss)
        d[f"mean_{kind}"] = f
        d[f"uvar_{kind}"] = np.diag(Cov[:M, :M])
        d[f"vvar_{kind}"] = np.diag(Cov[M:, M:])
        if kind != 0:   # divFree=0 broadcasts one scalar into all 4 entries: singular without noise
            ML, _, _ = gs["getCov"](x1, x2, x1s, x2s, sigma, kind)   # noise-free getCov (GP_scripts.py:48-54)
            d[f"getCov_diag_{kind}"] = np.diag(ML)
    # vectorised mixed kernel (GP_scripts.py:6-42)
    xa = np.stack([x1, x2], 1)
    xb = np.stack([x1s, x2s], 1)
    d["myK_mixed_aa"] = gs["myKernel"](xa, xa, 0.7, 1.1, 0.3)
    d["myK_mixed_ab"] = gs["myKernel"](xa, xb, 0.7, 1.1, 0.3)
    d["myK_params"] = np.array([0.7, 1.1, 0.3])
    np.savez_compressed(os.path.join(out, "gp_scripts_small.npz"), **d)


def gen_laser(gs, out):
    """GP_laser.laser() posterior (GP_laser.py:80-140) with the reference's loop kernels,
    on simulTracks coordinates: 384 drifters × 2 time steps, stride-3 split."""
    tr = load_tracks()
    ts = 10
    lat = tr.lat[:384, ts:ts + 2].reshape(-1)
    lon = tr.lon[:384, ts:ts + 2].reshape(-1)
    xo, yo = project_km(lat, lon)
    uo = tr.u[:384, ts:ts + 2].reshape(-1)
    vo = tr.v[:384, ts:ts + 2].reshape(-1)
    xo = xo - xo.min() + 2                                  # GP_laser.py:77-78
    yo = yo - yo.min() + 2
    n_raw = xo.size
    samples = np.arange(0, xo.size, 3)                      # GP_laser.py:81-83 (verbatim)
    test = set(np.arange(xo.size)) - set(samples)
    test = np.array(list(test))
    xt, yt, ut, vt = xo[test], yo[test], uo[test], vo[test]
    xo, yo, uo, vo = xo[samples], yo[samples], uo[samples], vo[samples]
    obs = np.concatenate([uo, vo])
    obs = np.reshape(obs, [obs.size, 1])
    dx = 1.0   # the script uses 0.5; a coarser grid keeps the O(M²) Kss loop tractable
    x = np.arange(np.min([xo.min(), xt.min()]) - 5, np.max([xo.max(), xt.max()]) + 5, dx)
    y = np.arange(np.min([yo.min(), yt.min()]) - 5, np.max([yo.max(), yt.max()]) + 5, dx)
    X, Y = np.meshgrid(x, y)
    Xs = np.reshape(X, [X.size])
    Ys = np.reshape(Y, [Y.size])
    l_df, l_cf, rate, noise = 5.0, 5.0, 0.5, 0.0025
    t0 = time.time()
    K = rate * gs["compute_K"](xo, yo, l_df, 1) + (1 - rate) * gs["compute_K"](xo, yo, l_cf, 2)
    Ko = np.identity(np.size(K, 0)) * noise
    K = K + Ko
    Ki = np.linalg.inv(K)
    Ks = rate * gs["compute_Ks"](xo, yo, Xs, Ys, l_df, 1) + (1 - rate) * gs["compute_Ks"](xo, yo, Xs, Ys, l_cf, 2)
    Kst = rate * gs["compute_Ks"](xo, yo, xt, yt, l_df, 1) + (1 - rate) * gs["compute_Ks"](xo, yo, xt, yt, l_cf, 2)
    Kss = rate * gs["compute_K"](Xs, Ys, l_df, 1) + (1 - rate) * gs["compute_K"](Xs, Ys, l_cf, 2)
    Cov = Kss - np.dot(Ks, np.dot(Ki, Ks.T))
    uvar = np.reshape(np.diag(Cov[:X.size, :X.size]), [y.size, -1])
    vvar = np.reshape(np.diag(Cov[X.size:, X.size:]), [y.size, -1])
    f = gs["getMean"](Ks, Ki, obs)
    uf = np.reshape(f[:f.size // 2], [y.size, -1])
    vf = np.reshape(f[f.size // 2:], [y.size, -1])
    ft = gs["getMean"](Kst, Ki, obs)
    print(f"  laser recipe N={xo.size} M={Xs.size}: {time.time() - t0:.1f}s")
    np.savez_compressed(os.path.join(out, "laser_mixed_N256.npz"),
                        n_raw=n_raw, samples=samples, test=test,
                        xo=xo, yo=yo, uo=uo, vo=vo, xt=xt, yt=yt, ut=ut, vt=vt,
                        x=x, y=y, l_df=l_df, l_cf=l_cf, rate=rate, noise=noise,
                        uf=uf, vf=vf, uvar=uvar, vvar=vvar,
                        uft=ft[:ft.size // 2], vft=ft[ft.size // 2:],
                        K_rowsum=K.sum(1), K_trace=np.trace(K))


def gen_mykernel(gs, out):
    """Vectorised-myKernel posterior (GP_scripts.py:6-46 with the GP_laser.py:113-131 recipe),
    N=1024 synthetic tracks, mixed α=0.5, 32×32 grid."""
    x, y, u, v = synthetic_tracks(1024)
    xa = np.stack([x, y], 1)
    gx = np.linspace(-5, 65, 32)
    gy = np.linspace(-5, 50, 32)
    GX, GY = np.meshgrid(gx, gy)
    xg = np.stack([GX.reshape(-1), GY.reshape(-1)], 1)
    M = xg.shape[0]
    l_df, l_cf, rate, noise = 5.0, 5.0, 0.5, 0.0025
    K = gs["myKernel"](xa, xa, l_df, l_cf, rate)
    K = K + np.identity(K.shape[0]) * noise
    Ki = np.linalg.inv(K)
    Ks = gs["myKernel"](xg, xa, l_df, l_cf, rate)
    obs = np.concatenate([u, v])[:, None]
    f = gs["getMean"](Ks, Ki, obs)
    kssd = np.diag(gs["myKernel"](xg, xg, l_df, l_cf, rate))
    q = np.einsum("ij,ij->i", Ks, Ks @ Ki)
    var = kssd - q
    rows = np.array([0, 1, 511, 1023, 1024, 2047])
    np.savez_compressed(os.path.join(out, "mykernel_mixed_N1024.npz"),
                        x=x, y=y, u=u, v=v, xg=xg, l_df=l_df, l_cf=l_cf, rate=rate, noise=noise,
                        mean=f, var=var, K_rows_idx=rows, K_rows=K[rows], K_rowsum=K.sum(1),
                        Ks_rows=Ks[[0, 5, M, M + 5]])
    # a div-free variant at the same size (the headline kernel)
    K = gs["myKernel"](xa, xa, l_df, l_cf, 1.0) + np.identity(2 * xa.shape[0]) * noise
    Ki = np.linalg.inv(K)
    Ks = gs["myKernel"](xg, xa, l_df, l_cf, 1.0)
    f = gs["getMean"](Ks, Ki, obs)
    var = np.diag(gs["myKernel"](xg, xg, l_df, l_cf, 1.0)) - np.einsum("ij,ij->i", Ks, Ks @ Ki)
    np.savez_compressed(os.path.join(out, "mykernel_divfree_N1024.npz"),
                        x=x, y=y, u=u, v=v, xg=xg, l_df=l_df, noise=noise, mean=f, var=var)


def config_subsample(xa, xg, n_near=256, n_rand=256, seed=5):
    """512 grid indices for the BASELINE-size fixtures: the n_near grid points closest to a
    training point (where var ≪ kss and the cancellation kss − ‖W k*‖² is worst) plus
    n_rand seeded uniform draws from the rest.  Sorted, unique."""
    from scipy.spatial import cKDTree
    d, _ = cKDTree(xa).query(xg)
    near = np.argsort(d, kind="stable")[:n_near]
    rest = np.setdiff1d(np.arange(xg.shape[0]), near)
    rnd = np.random.default_rng(seed).choice(rest, n_rand, replace=False)
    return np.unique(np.concatenate([near, rnd]))


_LD = {}


def _ld_residual_part(cols):
    """rhs[:, cols] − K·z[:, cols] in x87 long double (a worker of _ld_residual)."""
    ld = np.longdouble
    K, rhs, z = _LD["K"], _LD["rhs"], _LD["z"]
    return rhs[:, cols].astype(ld) - K.astype(ld) @ z[:, cols].astype(ld)


def _ld_residual(K, rhs, z, procs=None):
    """The refinement residual rhs − K·z in long double, its columns split over worker processes
    (numpy's long-double matmul has no BLAS: one process takes tens of minutes at n = 8192).
    Every column's arithmetic is the same as in one process."""
    import multiprocessing as mp
    procs = procs or min(8, os.cpu_count() or 1)
    if procs <= 1 or z.shape[1] < 2 * procs:
        _LD.update(K=K, rhs=rhs, z=z)
        return _ld_residual_part(np.arange(z.shape[1]))
    _LD.update(K=K, rhs=rhs, z=z)   # inherited by the forked workers
    chunks = np.array_split(np.arange(z.shape[1]), procs)
    with mp.get_context("fork").Pool(procs) as pool:
        parts = pool.map(_ld_residual_part, chunks)
    _LD.clear()
    return np.concatenate(parts, axis=1)


def _refined_posterior(K, ks, kss, obs):
    """Posterior mean / variance at the fixture points, accurate well past fp64 working
    precision: Cholesky solve of K z = ks, one step of iterative refinement with the residual
    in extended precision (x87 long double), then kss − ks·z and ks·α summed in long
    double.  This is the yardstick for the ELEMENTWISE variance gate, which the reference's
    own np.linalg.inv product cannot serve (its rounding is of the same order)."""
    import scipy.linalg as sla
    ld = np.longdouble
    c = sla.cho_factor(K, lower=True)
    rhs = np.concatenate([ks.T, obs[:, None]], 1)       # (n, 2m + 1)
    z = sla.cho_solve(c, rhs)
    r = _ld_residual(K, rhs, z)
    z = z.astype(ld) + sla.cho_solve(c, r.astype(np.float64)).astype(ld)
    ksl = ks.astype(ld)
    var = kss.astype(ld) - np.einsum("ij,ji->i", ksl, z[:, :-1])
    mean = ksl @ z[:, -1]
    return mean.astype(np.float64), var.astype(np.float64)


def gen_configs(gs, out):
    """BASELINE.json configs at full size: the bench's seeded inputs
    (gp2d.data.synthetic_tracks(4096, seed=2016), bbox_grid(…, 256, pad=5)) through the
    reference's own GP_laser.py:113-134 recipe with its vectorised myKernel
    (GP_scripts.py:6-46) and np.linalg.inv, evaluated at a 512-point grid subsample
    (config_subsample).  Cases: the headline (div-free, α = 1) and config C (mixed, α = ½);
    ℓ_df = ℓ_cf = 5 km, noise 0.0025, as bench.py.  Also stored: the refined posterior
    (_refined_posterior) for the elementwise variance gate."""
    x, y, u, v = synthetic_tracks(4096)
    xa = np.stack([x, y], 1)
    gx = np.linspace(x.min() - 5, x.max() + 5, 256)      # = gp2d.data.bbox_grid(x, y, 256, pad=5)
    gy = np.linspace(y.min() - 5, y.max() + 5, 256)
    GX, GY = np.meshgrid(gx, gy)
    xg_all = np.stack([GX.reshape(-1), GY.reshape(-1)], 1)
    idx = config_subsample(xa, xg_all)
    xg = xg_all[idx]
    m = xg.shape[0]
    obs = np.concatenate([u, v])
    d = dict(x=x, y=y, u=u, v=v, idx=idx, xg=xg, l_df=5.0, l_cf=5.0, noise=0.0025)
    for name, rate in (("df", 1.0), ("mixed", 0.5)):
        t0 = time.time()
        K = gs["myKernel"](xa, xa, 5.0, 5.0, rate)
        K = K + np.identity(K.shape[0]) * 0.0025         # GP_laser.py:114-115
        Ki = np.linalg.inv(K)                            # GP_laser.py:118
        Ks = gs["myKernel"](xg, xa, 5.0, 5.0, rate)      # GP_laser.py:122 (vectorised form)
        f = gs["getMean"](Ks, Ki, obs[:, None])          # GP_laser.py:134
        kss = np.diag(gs["myKernel"](xg, xg, 5.0, 5.0, rate))
        var = kss - np.einsum("ij,ij->i", Ks, Ks @ Ki)   # diag of GP_laser.py:129
        del Ki
        mr, vr = _refined_posterior(K, Ks, kss, obs)
        print(f"  config {name}: N=4096, {m} points, {time.time() - t0:.1f}s; inv recipe vs refined: "
              f"mean {np.max(np.abs(f - mr)) / np.max(np.abs(mr)):.1e}, var elementwise "
              f"{np.max(np.abs(var - vr) / vr):.1e}, min var/kss {np.min(vr / kss):.1e}")
        d[f"{name}_rate"] = rate
        d[f"{name}_mean"] = f
        d[f"{name}_var"] = var
        d[f"{name}_mean_refined"] = mr
        d[f"{name}_var_refined"] = vr
        d[f"{name}_kss"] = kss
        d[f"{name}_K_rowsum"] = K.sum(1)
    np.savez_compressed(os.path.join(out, "configs_N4096.npz"), **d)


def gen_configs_full(gs, out):
    """The headline (div-free, α = 1) and config C (mixed, α = ½) at EVERY point of the 256²
    grid: the bench's seeded N_train = 4096 tracks (gp2d.data.synthetic_tracks(4096, seed=2016),
    bbox_grid(…, 256, pad=5)), ℓ_df = ℓ_cf = 5 km, noise 0.0025, through the reference's own
    GP_laser.py:113-134 recipe — vectorised myKernel (GP_scripts.py:6-46) and np.linalg.inv —
    with K* taken in 4096-point chunks (one 131,072 × 8192 K* would need 8.6 GB).  Mean and
    variance of all 2 × 65,536 outputs per case."""
    x, y, u, v = synthetic_tracks(4096)
    xa = np.stack([x, y], 1)
    gx = np.linspace(x.min() - 5, x.max() + 5, 256)      # = gp2d.data.bbox_grid(x, y, 256, pad=5)
    gy = np.linspace(y.min() - 5, y.max() + 5, 256)
    GX, GY = np.meshgrid(gx, gy)
    xg = np.stack([GX.reshape(-1), GY.reshape(-1)], 1)
    M = xg.shape[0]
    obs = np.concatenate([u, v])[:, None]
    d = dict(x_sum=np.array([x.sum(), y.sum()]), u_sum=np.array([u.sum(), v.sum()]), xg_sum=xg.sum(0))
    c = 4096
    for name, rate in (("df", 1.0), ("mixed", 0.5)):
        t0 = time.time()
        K = gs["myKernel"](xa, xa, 5.0, 5.0, rate)
        K = K + np.identity(K.shape[0]) * 0.0025         # GP_laser.py:114-115
        Ki = np.linalg.inv(K)                            # GP_laser.py:118
        d0 = np.diag(gs["myKernel"](xg[:2], xg[:2], 5.0, 5.0, rate))   # the diagonal is constant (r = 0)
        assert np.all(d0 == d0[0])
        mean, var = np.empty(2 * M), np.empty(2 * M)
        for r0 in range(0, M, c):
            Ks = gs["myKernel"](xg[r0:r0 + c], xa, 5.0, 5.0, rate)   # rows [u(chunk); v(chunk)]
            f = np.ravel(gs["getMean"](Ks, Ki, obs))                 # GP_laser.py:134
            q = d0[0] - np.einsum("ij,ij->i", Ks, Ks @ Ki)            # diag of GP_laser.py:129
            mean[r0:r0 + c], mean[M + r0:M + r0 + c] = f[:c], f[c:]
            var[r0:r0 + c], var[M + r0:M + r0 + c] = q[:c], q[c:]
        print(f"  full grid {name}: N=4096, {M} points, {time.time() - t0:.1f}s, min var {var.min():.2e}")
        d[f"{name}_rate"] = rate
        d[f"{name}_mean"] = mean
        d[f"{name}_var"] = var
    np.savez_compressed(os.path.join(out, "configs_N4096_full.npz"), **d)


GUARD_KIND_SETTINGS = (("mixed", 3.0, 8.0, 0.5, 1e-4), ("cf", 12.0, 12.0, 0.0, 1e-3))


def gen_guard_kinds(gs, out):
    """The accuracy guard's yardstick on the other two vector kernels: the
    bench's seeded N_train = 4096 tracks and 256² bbox grid at the 512-point config_subsample,
    mixed (ℓ_df = 3, ℓ_cf = 8, ratio ½, noise 1e-4) and curl-free (ℓ = 12, noise 1e-3), through
    the reference's GP_laser.py:113-134 recipe (vectorised myKernel, np.linalg.inv) plus the
    refined posterior (_refined_posterior)."""
    x, y, u, v = synthetic_tracks(4096)
    xa = np.stack([x, y], 1)
    gx = np.linspace(x.min() - 5, x.max() + 5, 256)
    gy = np.linspace(y.min() - 5, y.max() + 5, 256)
    GX, GY = np.meshgrid(gx, gy)
    xg_all = np.stack([GX.reshape(-1), GY.reshape(-1)], 1)
    idx = config_subsample(xa, xg_all)
    xg = xg_all[idx]
    obs = np.concatenate([u, v])
    d = dict(x_sum=np.array([x.sum(), y.sum()]), u_sum=np.array([u.sum(), v.sum()]), idx=idx, xg=xg,
             settings=np.array([[ldf, lcf, r, nz] for _, ldf, lcf, r, nz in GUARD_KIND_SETTINGS]),
             kinds=np.array([k for k, *_ in GUARD_KIND_SETTINGS]))
    for k, (kind, ldf, lcf, rate, nz) in enumerate(GUARD_KIND_SETTINGS):
        t0 = time.time()
        K = gs["myKernel"](xa, xa, ldf, lcf, rate)
        K = K + np.identity(K.shape[0]) * nz              # GP_laser.py:114-115
        Ki = np.linalg.inv(K)                            # GP_laser.py:118
        Ks = gs["myKernel"](xg, xa, ldf, lcf, rate)      # GP_laser.py:122 (vectorised form)
        f = np.ravel(gs["getMean"](Ks, Ki, obs[:, None]))   # GP_laser.py:134
        kss = np.diag(gs["myKernel"](xg, xg, ldf, lcf, rate))
        var = kss - np.einsum("ij,ij->i", Ks, Ks @ Ki)   # diag of GP_laser.py:129
        del Ki
        mr, vr = _refined_posterior(K, Ks, kss, obs)
        print(f"  guard {kind} l=({ldf},{lcf}) ratio={rate} noise={nz}: {time.time() - t0:.1f}s; inv recipe vs "
              f"refined: var elementwise {np.max(np.abs(var - vr) / vr):.1e}, normwise "
              f"{np.max(np.abs(var - vr)) / np.max(vr):.1e}; min var/kss {np.min(vr / kss):.1e}")
        d[f"s{k}_mean"], d[f"s{k}_var"] = f, var
        d[f"s{k}_mean_refined"], d[f"s{k}_var_refined"] = mr, vr
        d[f"s{k}_kss"] = kss
    np.savez_compressed(os.path.join(out, "guard_kinds_N4096.npz"), **d)


GUARD_SETTINGS = ((12.0, 1e-3), (2.0, 5e-2), (5.0, 1e-4))   # (ℓ, noise): VERDICT r04 "next" item 1


def gen_guard(gs, out):
    """The headline workload (div-free, the bench's seeded N_train = 4096 tracks, the 256² bbox
    grid at the 512-point config_subsample) at hyperparameters away from the bench's ℓ = 5 km,
    noise 0.0025 — GUARD_SETTINGS, inside config E's range (ℓ ∈ [2, 12] km, noise ∈ [1e-3, 5e-2],
    bench.py) and one step past it (noise 1e-4): the reference's GP_laser.py:113-134 recipe with
    its vectorised myKernel and np.linalg.inv, plus the refined posterior (_refined_posterior).
    The yardstick for the ozaki engine's accuracy guard (tests/test_gpu_guard.py)."""
    x, y, u, v = synthetic_tracks(4096)
    xa = np.stack([x, y], 1)
    gx = np.linspace(x.min() - 5, x.max() + 5, 256)      # = gp2d.data.bbox_grid(x, y, 256, pad=5)
    gy = np.linspace(y.min() - 5, y.max() + 5, 256)
    GX, GY = np.meshgrid(gx, gy)
    xg_all = np.stack([GX.reshape(-1), GY.reshape(-1)], 1)
    idx = config_subsample(xa, xg_all)
    xg = xg_all[idx]
    obs = np.concatenate([u, v])
    d = dict(x_sum=np.array([x.sum(), y.sum()]), u_sum=np.array([u.sum(), v.sum()]), idx=idx, xg=xg,
             settings=np.array(GUARD_SETTINGS))
    for k, (l, nz) in enumerate(GUARD_SETTINGS):
        t0 = time.time()
        K = gs["myKernel"](xa, xa, l, l, 1.0)
        K = K + np.identity(K.shape[0]) * nz              # GP_laser.py:114-115
        Ki = np.linalg.inv(K)                            # GP_laser.py:118
        Ks = gs["myKernel"](xg, xa, l, l, 1.0)           # GP_laser.py:122 (vectorised form)
        f = np.ravel(gs["getMean"](Ks, Ki, obs[:, None]))   # GP_laser.py:134
        kss = np.diag(gs["myKernel"](xg, xg, l, l, 1.0))
        var = kss - np.einsum("ij,ij->i", Ks, Ks @ Ki)   # diag of GP_laser.py:129
        del Ki
        mr, vr = _refined_posterior(K, Ks, kss, obs)
        print(f"  guard l={l} noise={nz}: {time.time() - t0:.1f}s; inv recipe vs refined: var elementwise "
              f"{np.max(np.abs(var - vr) / vr):.1e}, normwise {np.max(np.abs(var - vr)) / np.max(vr):.1e}, "
              f"mean {np.max(np.abs(f - mr)) / np.max(np.abs(mr)):.1e}; min var/kss {np.min(vr / kss):.1e}")
        d[f"s{k}_mean"], d[f"s{k}_var"] = f, var
        d[f"s{k}_mean_refined"], d[f"s{k}_var_refined"] = mr, vr
        d[f"s{k}_kss"] = kss
    np.savez_compressed(os.path.join(out, "guard_N4096.npz"), **d)


def gen_config_b(gs, out):
    """BASELINE config B at its real workload: div-free (α = 1, ℓ = 5 km, noise 0.0025),
    N_train = 1024 bench tracks (gp2d.data.synthetic_tracks(1024, seed=2016)), the whole
    128 × 128 bbox grid (bbox_grid(…, 128, pad=5)) through the reference's GP_laser.py:113-134
    recipe with its vectorised myKernel and np.linalg.inv — mean and variance at ALL 16,384
    points — plus the refined posterior (_refined_posterior) at the 512-point subsample for the
    elementwise gate."""
    x, y, u, v = synthetic_tracks(1024)
    xa = np.stack([x, y], 1)
    gx = np.linspace(x.min() - 5, x.max() + 5, 128)      # = gp2d.data.bbox_grid(x, y, 128, pad=5)
    gy = np.linspace(y.min() - 5, y.max() + 5, 128)
    GX, GY = np.meshgrid(gx, gy)
    xg = np.stack([GX.reshape(-1), GY.reshape(-1)], 1)
    obs = np.concatenate([u, v])
    t0 = time.time()
    K = gs["myKernel"](xa, xa, 5.0, 5.0, 1.0)
    K = K + np.identity(K.shape[0]) * 0.0025             # GP_laser.py:114-115
    Ki = np.linalg.inv(K)                                # GP_laser.py:118
    Ks = gs["myKernel"](xg, xa, 5.0, 5.0, 1.0)           # GP_laser.py:122 (vectorised form)
    f = np.ravel(gs["getMean"](Ks, Ki, obs[:, None]))    # GP_laser.py:134
    d0 = np.diag(gs["myKernel"](xg[:2], xg[:2], 5.0, 5.0, 1.0))   # the diagonal is constant (r = 0)
    assert np.all(d0 == d0[0])
    kss = np.full(2 * xg.shape[0], d0[0])
    var = kss - np.einsum("ij,ij->i", Ks, Ks @ Ki)       # diag of GP_laser.py:129
    idx = config_subsample(xa, xg)
    M = xg.shape[0]
    rows = np.concatenate([idx, M + idx])
    mr, vr = _refined_posterior(K, Ks[rows], kss[rows], obs)
    print(f"  config B: N=1024, {M} points, {time.time() - t0:.1f}s; inv recipe vs refined at {idx.size}: "
          f"var elementwise {np.max(np.abs(var[rows] - vr) / vr):.1e}")
    np.savez_compressed(os.path.join(out, "config_b_full.npz"), x_sum=np.array([x.sum(), y.sum()]),
                        u_sum=np.array([u.sum(), v.sum()]), xg_sum=xg.sum(0), mean=f, var=var, idx=idx,
                        mean_refined=mr, var_refined=vr)


def gen_config_d(gs, out):
    """BASELINE config D on rank 0's shard: mixed (α = ½, ℓ = 5), N_train = 16384 (a 32768²
    K), the 512 × 512 bbox grid cut into 8 shards (gp2d.data.shard_range) — rank 0 holds the
    first 32768 points.  K is built from the reference's myKernel (GP_scripts.py:6-42) in
    row chunks (one call on 16384² pairs would need ~40 GB of temporaries); at this size the
    fixture factors K_y by Cholesky (scipy) instead of np.linalg.inv, and evaluates the
    posterior at 256 points of the shard (128 nearest to a training point + 128 seeded)."""
    import scipy.linalg as sla
    N, rate = 16384, 0.5
    x, y, u, v = synthetic_tracks(N)
    xa = np.stack([x, y], 1)
    gx = np.linspace(x.min() - 5, x.max() + 5, 512)
    gy = np.linspace(y.min() - 5, y.max() + 5, 512)
    GX, GY = np.meshgrid(gx, gy)
    xg_all = np.stack([GX.reshape(-1), GY.reshape(-1)], 1)
    shard = xg_all[:32768]                                # shard_range(262144, 8, 0) = [0, 32768)
    idx = config_subsample(xa, shard, 128, 128)
    xg = shard[idx]
    t0 = time.time()
    K = np.empty((2 * N, 2 * N))
    c = 1024
    for r0 in range(0, N, c):
        blk = gs["myKernel"](xa[r0:r0 + c], xa, 5.0, 5.0, rate)   # rows [u(r0:r0+c); v(r0:r0+c)]
        K[r0:r0 + c] = blk[:c]
        K[N + r0:N + r0 + c] = blk[c:]
        del blk
    K[np.diag_indices(2 * N)] += 0.0025
    rowsum = K.sum(1)
    Ks = gs["myKernel"](xg, xa, 5.0, 5.0, rate)
    kss = np.diag(gs["myKernel"](xg, xg, 5.0, 5.0, rate))
    obs = np.concatenate([u, v])
    # scipy's and numpy's Cholesky both segfault at n = 32768 in this container (OpenBLAS), so
    # the factor is blocked here (4096-wide blocks, LAPACK on the blocks).  Only the forward
    # solve is needed: with Z = L⁻¹[Ksᵀ, y], var = kss − ‖Z_j‖² and
    # mean = Z_jᵀ Z_y.
    bs = 4096
    L = K                                                 # blocked right-looking Cholesky in place
    for k0 in range(0, 2 * N, bs):
        k1 = k0 + bs
        L[k0:k1, k0:k1] = np.linalg.cholesky(L[k0:k1, k0:k1])
        if k1 < 2 * N:
            L[k1:, k0:k1] = sla.solve_triangular(L[k0:k1, k0:k1], L[k1:, k0:k1].T, lower=True,
                                                 check_finite=False).T
            for j0 in range(k1, 2 * N, bs):
                L[j0:, j0:j0 + bs] -= L[j0:, k0:k1] @ L[j0:j0 + bs, k0:k1].T
    B = np.concatenate([Ks.T, obs[:, None]], 1)
    Z = np.empty_like(B)
    for i0 in range(0, 2 * N, bs):
        r = B[i0:i0 + bs] - L[i0:i0 + bs, :i0] @ Z[:i0]
        Z[i0:i0 + bs] = sla.solve_triangular(L[i0:i0 + bs, i0:i0 + bs], r, lower=True, check_finite=False)
    mean = Z[:, :-1].T @ Z[:, -1]     # (blocked forward substitution above, 4096-row blocks)
    var = kss - np.einsum("ij,ij->j", Z[:, :-1], Z[:, :-1])
    print(f"  config D rank-0 shard: N={N}, {xg.shape[0]} points, {time.time() - t0:.1f}s, "
          f"min var/kss {np.min(var / kss):.1e}")
    np.savez_compressed(os.path.join(out, "config_d_rank0.npz"), idx=idx, xg=xg, rate=rate, l=5.0, noise=0.0025,
                        mean=mean, var=var, kss=kss, K_rowsum=rowsum, x_sum=np.array([x.sum(), y.sum()]))


def gen_config_d_shards(gs, out):
    """Config D at EVERY rank's shard: as gen_config_d — mixed (α = ½,
    ℓ = 5, noise 0.0025), N_train = 16384 (a 32768² K from the reference's myKernel in row
    chunks), the 512² bbox grid cut into 8 shards (gp2d.data.shard_range) — with 64 points
    from EACH shard (32 nearest to a training point + 32 seeded, config_subsample), 512 in all.
    Blocked Cholesky (LAPACK on 4096-wide blocks) and forward substitution as gen_config_d."""
    import scipy.linalg as sla
    N, rate, P = 16384, 0.5, 8
    x, y, u, v = synthetic_tracks(N)
    xa = np.stack([x, y], 1)
    gx = np.linspace(x.min() - 5, x.max() + 5, 512)
    gy = np.linspace(y.min() - 5, y.max() + 5, 512)
    GX, GY = np.meshgrid(gx, gy)
    xg_all = np.stack([GX.reshape(-1), GY.reshape(-1)], 1)
    Mall = xg_all.shape[0]
    sel = []
    for r in range(P):                                    # shard_range(262144, 8, r) (align 64)
        lo, hi = r * Mall // P, (r + 1) * Mall // P
        sel.append(lo + config_subsample(xa, xg_all[lo:hi], 32, 32, seed=5 + r))
    gidx = np.concatenate(sel)
    xg = xg_all[gidx]
    t0 = time.time()
    K = np.empty((2 * N, 2 * N))
    c = 1024
    for r0 in range(0, N, c):
        blk = gs["myKernel"](xa[r0:r0 + c], xa, 5.0, 5.0, rate)   # rows [u(r0:r0+c); v(r0:r0+c)]
        K[r0:r0 + c] = blk[:c]
        K[N + r0:N + r0 + c] = blk[c:]
        del blk
    K[np.diag_indices(2 * N)] += 0.0025
    Ks = gs["myKernel"](xg, xa, 5.0, 5.0, rate)
    kss = np.diag(gs["myKernel"](xg, xg, 5.0, 5.0, rate))
    obs = np.concatenate([u, v])
    bs = 4096
    L = K
    for k0 in range(0, 2 * N, bs):
        k1 = k0 + bs
        L[k0:k1, k0:k1] = np.linalg.cholesky(L[k0:k1, k0:k1])
        if k1 < 2 * N:
            L[k1:, k0:k1] = sla.solve_triangular(L[k0:k1, k0:k1], L[k1:, k0:k1].T, lower=True,
                                                 check_finite=False).T
            for j0 in range(k1, 2 * N, bs):
                L[j0:, j0:j0 + bs] -= L[j0:, k0:k1] @ L[j0:j0 + bs, k0:k1].T
    B = np.concatenate([Ks.T, obs[:, None]], 1)
    Z = np.empty_like(B)
    for i0 in range(0, 2 * N, bs):
        r = B[i0:i0 + bs] - L[i0:i0 + bs, :i0] @ Z[:i0]
        Z[i0:i0 + bs] = sla.solve_triangular(L[i0:i0 + bs, i0:i0 + bs], r, lower=True, check_finite=False)
    mean = Z[:, :-1].T @ Z[:, -1]
    var = kss - np.einsum("ij,ij->j", Z[:, :-1], Z[:, :-1])
    print(f"  config D all shards: N={N}, {xg.shape[0]} points, {time.time() - t0:.1f}s, "
          f"min var/kss {np.min(var / kss):.1e}")
    np.savez_compressed(os.path.join(out, "config_d_shards.npz"), gidx=gidx, xg=xg, rate=rate, l=5.0, noise=0.0025,
                        mean=mean, var=var, kss=kss, x_sum=np.array([x.sum(), y.sum()]))


def config_e_survey_settings():
    """SURVEY.md §8(d)'s config E: 8 ℓ_df × 8 ℓ_cf on a log grid over [1, 10] km, mixed kernel
    with α = ½, noise 0.0025 (ℓ_df-major order)."""
    g = np.geomspace(1.0, 10.0, 8)
    return [dict(l_df=float(a), l_cf=float(b)) for a in g for b in g]


def gen_config_e_survey(gs, out):
    """SURVEY §8(d) config E, rank 0's share of the 64 settings over 8 GPUs
    (settings 0, 8, …, 56; setting i = (ℓ_df[i // 8], ℓ_cf[i % 8]), so rank 0 holds ℓ_cf = 1 km
    at every ℓ_df — the grid's short end) at N_train = 4096 (seeded tracks),
    mixed α = ½, noise 0.0025: the LML of each, with K from the reference's myKernel
    (GP_scripts.py:6-42) and a Cholesky factor; for two of them the gradient in (ℓ_df, ℓ_cf,
    ratio) by a 4-point central difference of that LML and ∂/∂noise = ½(αᵀα − tr K_y⁻¹) exactly
    (the reference's analytic gradient, myKernel.py:59-106, is not a derivative)."""
    import scipy.linalg as sla
    x, y, u, v = synthetic_tracks(4096)
    xa = np.stack([x, y], 1)
    obs = np.concatenate([u, v])
    S = config_e_survey_settings()
    share = list(range(0, 64, 8))

    def lml(p, want=False):
        K = gs["myKernel"](xa, xa, p[0], p[1], p[2])
        K[np.diag_indices_from(K)] += p[3]
        L = np.linalg.cholesky(K)
        a = sla.cho_solve((L, True), obs)
        val = -0.5 * obs @ a - np.sum(np.log(np.diag(L))) - 0.5 * obs.size * np.log(2 * np.pi)
        return (val, L, a) if want else val

    t0 = time.time()
    vals = np.array([lml([S[i]["l_df"], S[i]["l_cf"], 0.5, 0.0025]) for i in share])
    grads = []
    gidx = [share[2], share[5]]
    for i in gidx:
        p = [S[i]["l_df"], S[i]["l_cf"], 0.5, 0.0025]
        g = []
        for j in range(3):
            h = 1e-4 * (p[j] if j < 2 else 1.0)
            f = []
            for t in (-2, -1, 1, 2):
                q = list(p)
                q[j] += t * h
                f.append(lml(q))
            g.append((f[0] - 8 * f[1] + 8 * f[2] - f[3]) / (12 * h))
        _, L, a = lml(p, want=True)
        Li = sla.solve_triangular(L, np.identity(L.shape[0]), lower=True)
        g.append(0.5 * (a @ a - np.sum(Li * Li)))
        grads.append(g)
    print(f"  config E (SURVEY grid) share: 8 settings x N=4096, {time.time() - t0:.1f}s")
    np.savez_compressed(os.path.join(out, "config_e_survey_share.npz"), share=np.array(share),
                        l_df=np.array([S[i]["l_df"] for i in share]), l_cf=np.array([S[i]["l_cf"] for i in share]),
                        ratio=0.5, noise=0.0025, lml=vals, grad_idx=np.array(gidx), grad=np.array(grads))


def config_e_settings():
    """BASELINE config E's 64 hyperparameter settings: ℓ_df on 8 log-spaced values in
    [2, 12] km × noise σ² on 8 log-spaced values in [1e-3, 5e-2] (div-free kernel)."""
    return [dict(l_df=float(l), noise=float(nz)) for l in np.geomspace(2.0, 12.0, 8)
            for nz in np.geomspace(1e-3, 5e-2, 8)]


def gen_config_e(gs, out):
    """BASELINE config E, rank 0's share of the 64-setting sweep over 8 GPUs (settings 0, 8,
    …, 56 — gp2d.hyper.sweep deals them round-robin) at N_train = 4096 (seeded tracks): the
    log marginal likelihood of each, with K from the reference's myKernel (GP_scripts.py:6-42)
    and a Cholesky factor; for two of them also the gradient in (ℓ_df, noise): ∂/∂ℓ_df by a
    4-point central difference of that LML, ∂/∂noise = ½(αᵀα − tr K_y⁻¹) exactly."""
    import scipy.linalg as sla
    x, y, u, v = synthetic_tracks(4096)
    xa = np.stack([x, y], 1)
    obs = np.concatenate([u, v])
    S = config_e_settings()
    share = list(range(0, 64, 8))

    def lml(l, nz, want=False):
        K = gs["myKernel"](xa, xa, l, l, 1.0)
        K[np.diag_indices_from(K)] += nz
        L = np.linalg.cholesky(K)
        a = sla.cho_solve((L, True), obs)
        val = -0.5 * obs @ a - np.sum(np.log(np.diag(L))) - 0.5 * obs.size * np.log(2 * np.pi)
        return (val, L, a) if want else val

    t0 = time.time()
    vals = np.array([lml(S[i]["l_df"], S[i]["noise"]) for i in share])
    grads = []
    gidx = [share[2], share[5]]
    for i in gidx:
        l, nz = S[i]["l_df"], S[i]["noise"]
        h = 1e-4 * l
        f = [lml(l + t * h, nz) for t in (-2, -1, 1, 2)]
        gl = (f[0] - 8 * f[1] + 8 * f[2] - f[3]) / (12 * h)
        _, L, a = lml(l, nz, want=True)
        Li = sla.solve_triangular(L, np.identity(L.shape[0]), lower=True)
        gn = 0.5 * (a @ a - np.sum(Li * Li))
        grads.append([gl, gn])
    print(f"  config E share: 8 settings x N=4096, {time.time() - t0:.1f}s")
    np.savez_compressed(os.path.join(out, "config_e_share.npz"), share=np.array(share),
                        l_df=np.array([S[i]["l_df"] for i in share]), noise=np.array([S[i]["noise"] for i in share]),
                        lml=vals, grad_idx=np.array(gidx), grad=np.array(grads))


def gen_sklearn(out):
    """Config A: krig.scikit_prior's model (krig.py:174-194) on 3-D (T,Y,X) inputs, N=128,
    32×32 grid at one time slice."""
    from sklearn.gaussian_process import GaussianProcessRegressor, kernels
    rng = np.random.default_rng(11)
    N = 128
    X = np.stack([rng.uniform(0, 6, N), rng.uniform(0, 20, N), rng.uniform(-5, 15, N)], 1)
    u = np.sin(X[:, 1] / 4) * np.cos(X[:, 2] / 5) + 0.1 * X[:, 0] / 6 + rng.normal(0, 0.05, N)
    HP = np.array([0.8, 3.0, 4.0, 5.0, 0.2, 10.0, 1.5, 2.0, 0.004])   # var1,lt,ly,lx,var2,lt,ly,lx,noise
    k = HP[0] * kernels.RBF(length_scale=[HP[1], HP[2], HP[3]])
    k = k + HP[4] * kernels.RBF(length_scale=[HP[5], HP[6], HP[7]])
    k = k + kernels.WhiteKernel(noise_level=HP[-1])
    model = GaussianProcessRegressor(kernel=k, optimizer=None)
    model.fit(X, u[:, None])
    yg = np.linspace(1, 15, 32)
    xg = np.linspace(-5, 15, 32)
    Yg, Tg, Xg = np.meshgrid(yg, np.array([3.0]), xg)
    Xp = np.concatenate([Tg.reshape(-1, 1), Yg.reshape(-1, 1), Xg.reshape(-1, 1)], 1)
    U, Ustd = model.predict(Xp, return_std=True)
    np.savez_compressed(os.path.join(out, "sklearn_ard_N128.npz"), X=X, u=u, HP=HP, Xp=Xp,
                        mean=np.asarray(U).reshape(-1), std=np.asarray(Ustd).reshape(-1))


def gen_lml(gs, out):
    """Log marginal likelihood + gradient fixtures.

    vector kernels: K from the reference's own myKernel (GP_scripts.py:6-42) at N=300
    synthetic tracks; LML by Cholesky; the gradient by a 4-point central difference of that
    LML in each hyperparameter (l_df, l_cf, rate) — the reference's analytic gradient
    (myKernel.py:59-105) is not a derivative — and ∂/∂noise exactly.
    ARD: scikit-learn's log_marginal_likelihood(theta, eval_gradient=True) for the
    krig.scikit_prior model (krig.py:174-180) at N=128, gradient mapped from log-space."""
    import scipy.linalg as sla
    from sklearn.gaussian_process import GaussianProcessRegressor, kernels
    x, y, u, v = synthetic_tracks(300, seed=7)
    xa = np.stack([x, y], 1)
    obs = np.concatenate([u, v])
    d = dict(x=x, y=y, u=u, v=v)

    def lml(p):
        K = gs["myKernel"](xa, xa, p[0], p[1], p[2]) + np.identity(2 * xa.shape[0]) * p[3]
        L = np.linalg.cholesky(K)
        a = sla.cho_solve((L, True), obs)
        return -0.5 * obs @ a - np.sum(np.log(np.diag(L))) - 0.5 * obs.size * np.log(2 * np.pi), L, a

    cases = [("df", [4.0, 5.0, 1.0, 0.0025]), ("cf", [5.0, 3.5, 0.0, 0.0025]),
             ("mixed", [6.0, 4.0, 0.4, 0.01])]
    for name, p in cases:
        val, L, a = lml(p)
        g = np.zeros(4)
        for i in range(3):
            if (name == "df" and i != 0) or (name == "cf" and i != 1):
                continue
            h = 1e-4 * (p[i] if i < 2 else 1.0)
            f = []
            for t in (-2, -1, 1, 2):
                q = list(p)
                q[i] += t * h
                f.append(lml(q)[0])
            g[i] = (f[0] - 8 * f[1] + 8 * f[2] - f[3]) / (12 * h)
        Ki = sla.cho_solve((L, True), np.identity(L.shape[0]))
        g[3] = 0.5 * (a @ a - np.trace(Ki))
        d[f"{name}_params"] = np.array(p)
        d[f"{name}_lml"] = np.array(val)
        d[f"{name}_grad"] = g
    np.savez_compressed(os.path.join(out, "lml_vector_N300.npz"), **d)

    rng = np.random.default_rng(12)
    N = 128
    X = np.stack([rng.uniform(0, 6, N), rng.uniform(0, 20, N), rng.uniform(-5, 15, N)], 1)
    uu = np.sin(X[:, 1] / 4) * np.cos(X[:, 2] / 5) + 0.1 * X[:, 0] / 6 + rng.normal(0, 0.05, N)
    e = dict(X=X, u=uu)
    for T, HP in ((1, np.array([0.8, 3.0, 4.0, 5.0, 0.004])),
                  (2, np.array([0.8, 3.0, 4.0, 5.0, 0.2, 10.0, 1.5, 2.0, 0.004]))):
        k = HP[0] * kernels.RBF(length_scale=list(HP[1:4]))
        if T == 2:
            k = k + HP[4] * kernels.RBF(length_scale=list(HP[5:8]))
        k = k + kernels.WhiteKernel(noise_level=HP[-1])
        model = GaussianProcessRegressor(kernel=k, optimizer=None).fit(X, uu)
        val, glog = model.log_marginal_likelihood(model.kernel_.theta, eval_gradient=True)
        e[f"T{T}_HP"] = HP
        e[f"T{T}_lml"] = np.array(val)
        e[f"T{T}_grad"] = np.asarray(glog) / HP   # ∂/∂x = ∂/∂log x ÷ x
    np.savez_compressed(os.path.join(out, "lml_sklearn_ard_N128.npz"), **e)


def gen_st(gs, out):
    """Spatio-temporal product kernel: Kt(var_t, l_t) × vector kernel on
    (T, Y, X), the GPy product of scratch.py:506-508.  The spatial factor is the reference's own
    myKernel (GP_scripts.py:6-42) on (Y, X); the temporal factor is the GPy RBF of Kt.K
    (myKernel.py:347-355) = var·exp(−Δt²/2ℓ²), evaluated by scikit-learn's RBF (GPy is absent).
    N=150 tracks over 6 days, 2 time slices × 10×10 grid; posterior by the GP_laser.py:113-131
    recipe (np.linalg.inv)."""
    from sklearn.gaussian_process import kernels
    rng = np.random.default_rng(31)
    N = 150
    t = rng.uniform(0, 6, N)
    yy = rng.uniform(0, 45, N)
    xx = rng.uniform(0, 60, N)
    v = np.cos(xx / 9) + 0.1 * t + rng.normal(0, 0.05, N)
    u = np.sin(yy / 7) - 0.05 * t + rng.normal(0, 0.05, N)
    obs = np.concatenate([v, u])        # components follow (Y, X): [v; u] (krig.py:390)
    gy, gx = np.meshgrid(np.linspace(0, 45, 10), np.linspace(0, 60, 10), indexing="ij")
    G = np.concatenate([np.stack([np.full(100, tt), gy.reshape(-1), gx.reshape(-1)], 1) for tt in (2.0, 4.5)])
    d = dict(t=t, y=yy, x=xx, obs=obs, G=G)
    for name, (ldf, lcf, rate, var_t, l_t, noise) in (("df", (5.0, 5.0, 1.0, 5.0, 1.0, 0.0025)),
                                                     ("mixed", (6.0, 4.0, 0.4, 2.0, 1.5, 0.01))):
        def K_st(A, B):
            C = var_t * kernels.RBF(length_scale=l_t)(A[:, :1], B[:, :1])
            S = gs["myKernel"](A[:, 1:], B[:, 1:], ldf, lcf, rate)
            return S * np.block([[C, C], [C, C]])
        X = np.stack([t, yy, xx], 1)
        K = K_st(X, X) + np.identity(2 * N) * noise
        Ki = np.linalg.inv(K)
        Ks = K_st(G, X)
        f = gs["getMean"](Ks, Ki, obs[:, None])
        kss = np.diag(K_st(G, G))
        var = kss - np.einsum("ij,ij->i", Ks, Ks @ Ki)
        d[f"{name}_params"] = np.array([ldf, lcf, rate, var_t, l_t, noise])
        d[f"{name}_K_rows"] = K[[0, 1, N, 2 * N - 1]]
        d[f"{name}_mean"] = np.asarray(f).reshape(-1)
        d[f"{name}_var"] = var
    np.savez_compressed(os.path.join(out, "st_product_N150.npz"), **d)


def gen_prep(out):
    """Data-prep parity on real tracks: the reference's own getData
    (krig.py:50-65 + its return expression, krig.py:77) and kriging selection block
    (krig.py:274-381: boundData, projection, split, NaN filter, T,Y,X stacking) exec'd from
    the file text (py2 `print` lines → `pass`), on simulTracks.pkl coordinates (transposed
    to time × drifter, 12 steps × 240 drifters, with NaN tails injected so the filters act).
    pyproj is absent: NAD83 is the build's documented stand-in (krig.nad83, restated here).
    The outputs are large, so the fixture keeps SHA-256 digests of their bytes (bit-exact
    check) plus shapes and a few rows."""
    import hashlib
    with open(os.path.join(REF, "krig.py")) as f:
        lines = f.readlines()

    def block(a, b, indent):
        out = []
        for ln in lines[a - 1:b]:
            body = ln[indent:] if ln[:indent].strip() == "" else ln.lstrip()
            if body.lstrip().startswith("print "):
                out.append(body[:len(body) - len(body.lstrip())] + "pass\n")
            else:
                out.append(body)
        return "".join(out)

    getdata_body = block(50, 65, 6)                    # NaN-ing of drifter 238 … order[::-1]
    ret = lines[76].strip()                            # krig.py:77
    assert ret.startswith("return ")
    ret = ret[len("return "):]
    bound_src = block(79, 86, 0)                       # def boundData(...)
    krig_body = block(274, 381, 3)                     # getData call … obst = …
    tr = load_tracks()
    rng = np.random.default_rng(41)
    T, D = 12, 240
    lat = np.array(tr.lat[:D, :T].T)
    lon = np.array(tr.lon[:D, :T].T)
    u = np.array(tr.u[:D, :T].T)
    v = np.array(tr.v[:D, :T].T)
    for c in rng.choice(D, 30, replace=False):         # drifters that stop reporting
        k = int(rng.integers(1, T))
        lat[k:, c] = np.nan
        lon[k:, c] = np.nan
    time = np.array(tr.time[:T])

    class TR:
        pass

    R = 6371000.0
    lat0, lon0 = 28.8, -88.6

    def NAD83(lo, la):                                 # = krig.nad83
        return (R * np.cos(np.deg2rad(lat0)) * np.deg2rad(np.asarray(lo, dtype=np.float64)),
                R * np.deg2rad(np.asarray(la, dtype=np.float64)))

    def getData(st, et, laser=1):
        t = TR()
        t.lat, t.lon, t.u, t.v, t.time = lat.copy(), lon.copy(), u.copy(), v.copy(), time.copy()
        ns = {"np": np, "tr": t, "st": st, "et": et}
        exec(compile(getdata_body, "krig.py[50:65]", "exec"), ns)
        return eval(ret, ns)

    bns = {"np": np}
    exec(compile(bound_src, "krig.py[79:86]", "exec"), bns)
    x_ori, y_ori = NAD83(lon0, lat0)
    d = dict(time=time, lat=lat, lon=lon, u=u, v=v)
    cases = [dict(st=0, et=12, sample_step=5, skip=1, lalim=[0, 0], lolim=[0, 0]),
             dict(st=0, et=12, sample_step=-2, skip=1, lalim=[0, 0], lolim=[0, 0]),
             dict(st=1, et=11, sample_step=-3, skip=3, lalim=[0, 0], lolim=[0, 0]),
             dict(st=0, et=12, sample_step=-1, skip=2, lalim=[0, 0],
                  lolim=[float(np.nanpercentile(lon[0], 20)), float(np.nanpercentile(lon[0], 80))]),
             dict(st=2, et=12, sample_step=4, skip=1, lolim=[0, 0],
                  lalim=[float(np.nanpercentile(lat[0], 10)), float(np.nanpercentile(lat[0], 70))])]
    names = ("X", "LL_o", "obs", "Xt", "LL_t", "obst")
    for i, c in enumerate(cases):
        ns = {"np": np, "getData": getData, "boundData": bns["boundData"], "NAD83": NAD83, "x_ori": x_ori, "output": "m",
              "y_ori": y_ori, "laser": 1, **c}
        exec(compile(krig_body, "krig.py[274:381]", "exec"), ns)
        d[f"c{i}_args"] = np.array([c["st"], c["et"], c["sample_step"], c["skip"], *c["lalim"], *c["lolim"]],
                                   dtype=np.float64)
        for nm in names:
            a = np.ascontiguousarray(ns[nm], dtype=np.float64)
            d[f"c{i}_{nm}_shape"] = np.array(a.shape)
            d[f"c{i}_{nm}_sha256"] = np.frombuffer(hashlib.sha256(a.tobytes()).digest(), dtype=np.uint8)
            d[f"c{i}_{nm}_rows"] = a[[0, -1]] if a.shape[0] else a
    d["ncases"] = np.array(len(cases))
    np.savez_compressed(os.path.join(out, "prep_tracks.npz"), **d)


def gen_prior_window(out):
    """scikit_prior's observation window (krig.py:146-157 and the component choice at
    krig.py:164-167), exec'd from the file text on seeded (T, Y, X) observation / test arrays,
    for several windows."""
    with open(os.path.join(REF, "krig.py")) as f:
        lines = f.readlines()
    sel = "".join(("pass\n" if ln.strip().startswith("print ") else ln[3:]) for ln in lines[145:157])  # 146-157
    comp = "".join(ln[3:] for ln in lines[163:167])          # krig.py:164-167
    d = {}
    rng = np.random.default_rng(9)
    Xo = np.stack([rng.uniform(0, 6, 400), rng.uniform(-20, 20, 400), rng.uniform(-30, 30, 400)], 1)
    Xt = np.stack([rng.uniform(0, 6, 300), rng.uniform(-20, 20, 300), rng.uniform(-30, 30, 300)], 1)
    obs = rng.normal(size=(400, 2))
    obst = rng.normal(size=(300, 2))
    fm = {"Xo": Xo, "Xt": Xt, "obs": obs, "test_points": obst}
    d.update(Xo=Xo, Xt=Xt, obs=obs, test_points=obst)
    cases = [(3.0, 6, [-10.0, 10.0], 3, "v"), (1.0, 2, [0.0, 25.0], 0, "u"), (5.5, 1, [-40.0, 40.0], 10, "v")]
    for i, (tc, tlim, xlim, xrange, varname) in enumerate(cases):
        ns = {"np": np, "fm": fm, "tcenter": np.array([tc]), "tlim": tlim, "xlim": xlim, "xrange": xrange,
              "varname": varname}
        exec(compile(sel, "krig.py[146:157]", "exec"), ns)
        exec(compile(comp, "krig.py[164:167]", "exec"), ns)
        d[f"c{i}_args"] = np.array([tc, tlim, xlim[0], xlim[1], xrange, 1.0 if varname == "u" else 0.0])
        d[f"c{i}_XT"] = np.concatenate([ns["Xo"], ns["Xt"]], axis=0)
        d[f"c{i}_u"] = ns["u"][:, 0]
    d["ncases"] = np.array(len(cases))
    np.savez_compressed(os.path.join(out, "prior_window.npz"), **d)


def gen_indices(out):
    """Split index arrays, verbatim reference expression (GP_laser.py:81-83, krig.py:335-337)."""
    sizes = list(range(30, 40)) + list(range(128, 140)) + [257, 1000, 1031, 3000, 12288]
    d = {}
    for step in (2, 3, 5):
        for n in sizes:
            samples = np.arange(0, n, step)
            test = set(np.arange(n)) - set(samples)
            test = np.array(list(test))
            d[f"test_{step}_{n}"] = test.astype(np.int64)
    d["sizes"] = np.array(sizes)
    np.savez_compressed(os.path.join(out, "split_indices.npz"), **d)


def gen_grids(out):
    getGrid = load_get_grid()
    rng = np.random.default_rng(3)
    d = {}
    cases = [
        dict(to=rng.uniform(0, 6, 50), yo=rng.uniform(0, 20, 50), xo=rng.uniform(-5, 15, 50), dt=1.0, dx=0.7, xL=40, yL=40),
        dict(to=rng.uniform(0, 3, 40), yo=rng.uniform(-30, 30, 40), xo=rng.uniform(0, 70, 40), dt=0.5, dx=1.3, xL=40, yL=40),
        dict(to=np.array([12.0, 13.0]), ylim_case=True, yo=np.array([1.0, 15.0]), xo=np.array([-5.0, 15.0]), dt=1.0, dx=0.5, xL=40, yL=40),
    ]
    for i, c in enumerate(cases):
        c.pop("ylim_case", None)
        X, tg, yg, xg = getGrid(c["to"], c["yo"], c["xo"], c["dt"], c["dx"], c["xL"], c["yL"])
        for k, v in c.items():
            d[f"c{i}_{k}"] = np.asarray(v)
        d[f"c{i}_X"], d[f"c{i}_tg"], d[f"c{i}_yg"], d[f"c{i}_xg"] = X, tg, yg, xg
    d["ncases"] = np.array(len(cases))
    np.savez_compressed(os.path.join(out, "grids.npz"), **d)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    gs = load_gp_scripts()
    jobs = dict(small=lambda: gen_small(gs, a.out), laser=lambda: gen_laser(gs, a.out),
                mykernel=lambda: gen_mykernel(gs, a.out), sklearn=lambda: gen_sklearn(a.out),
                indices=lambda: gen_indices(a.out), grids=lambda: gen_grids(a.out),
                lml=lambda: gen_lml(gs, a.out), st=lambda: gen_st(gs, a.out),
                prep=lambda: gen_prep(a.out), window=lambda: gen_prior_window(a.out),
                configs=lambda: gen_configs(gs, a.out), config_b=lambda: gen_config_b(gs, a.out),
                config_d=lambda: gen_config_d(gs, a.out),
                config_e=lambda: gen_config_e(gs, a.out), guard=lambda: gen_guard(gs, a.out),
                configs_full=lambda: gen_configs_full(gs, a.out), guard_kinds=lambda: gen_guard_kinds(gs, a.out),
                config_d_shards=lambda: gen_config_d_shards(gs, a.out),
                config_e_survey=lambda: gen_config_e_survey(gs, a.out))
    for name, fn in jobs.items():
        if a.only and name not in a.only.split(","):
            continue
        t = time.time()
        fn()
        print(f"{name}: {time.time() - t:.1f}s")


if __name__ == "__main__":
    main()
