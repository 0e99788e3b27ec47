"""The reference's ``krig`` module surface, backed by the MI355X engine.

Reference: krig.py (module functions), runKrig.py / runPredict.py (drivers),
GP_laser.py:16-142 (the explicit-numpy posterior).  ``Krig`` is the stateful
fit/predict object the north_star names (`krig.Krig`); the module functions
keep the reference's names, argument meaning and error behaviour.

Differences forced by the environment (documented in DESIGN.md):
  * data files (Filtered_2016_2_7.pkl, .mat outputs, GPy pickles) do not exist:
    functions take a track container (``Tracks``) or ``.npz`` paths; model files
    are ``.npz`` (inputs + hyperparameters, optionally the factor);
  * pyproj / NAD83 is absent: ``project`` is a signed local equirectangular
    projection in km about (lat0, lon0);
  * NetCDF: krig.predict writes filename+'.nc' (CDF-2, printNCFiles layout) through
    ``gp2d.ncio`` (netCDF4 is absent; a self-contained classic-format writer), plus the
    ``.npz`` of the same arrays;
  * hyperparameter optimisation (GPy optimize / optimize_restarts) runs on the GPU
    (``gp2d.hyper``: HIP LML + exact gradient, scipy L-BFGS-B on the host);
  * kernelType 2/3/4 use the spatio-temporal product Kt(var_t, l_t) × div-free /
    curl-free / mixed kernel on (T, Y, X) (engine family 'vector_st', the form of
    scratch.py:506-508) — the reference's myKernel2 (var, lt, ly, lx) is missing from
    the reference itself (krig.py:9), so ly = lx = ℓ here;
    hyper={'temporal': False} gives the purely spatial kernel on (Y, X).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from datetime import datetime, timedelta

import numpy as np
import torch

from . import data as D
from . import engine as E
from . import hyper as H
from . import ncio as NC

lat0 = 28.8
lon0 = -88.6

KERNEL_NAMES = {"df": "df", "divfree": "df", "div-free": "df", 1: "df",
                "cf": "cf", "curlfree": "cf", "curl-free": "cf", 2: "cf",
                "mixed": "mixed", "combined": "mixed", 3: "mixed",
                "scalar": "scalar", "isotropic": "scalar", 0: "scalar"}


def nad83(lon, lat):
    """Stand-in for the reference's NAD83 / EPSG:3452 projection (krig.py:19; pyproj is absent):
    a signed equirectangular projection in metres, scaled at lat0."""
    R = 6371000.0
    x = R * np.cos(np.deg2rad(lat0)) * np.deg2rad(np.asarray(lon, dtype=np.float64))
    y = R * np.deg2rad(np.asarray(lat, dtype=np.float64))
    return x, y


x_ori, y_ori = nad83(lon0, lat0)   # krig.py:20


def project(lon, lat):
    """Track coordinates to km about (lat0, lon0), with the reference's arithmetic
    (krig.py:291-298): (NAD83(lon, lat) − origin) / 1000."""
    x, y = nad83(lon, lat)
    return (x - x_ori) / 1000.0, (y - y_ori) / 1000.0


def _to_numpy(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


# =============================================================================== Krig
class Krig:
    """Stateful GP kriging object: ``Krig(...).fit(X, obs).predict(Xg)``.

    kernel: 'df' (divergence-free, GP_scripts divFree=1), 'cf' (curl-free, 2),
    'mixed' (ratio·df + (1−ratio)·cf, GP_laser.py:113), 'scalar' (divFree=0),
    a ``kern.myKernel``/``nonDivK``/``nonRotK`` instance, or an ``engine.KernelSpec``
    (incl. family='ard' for the sklearn model of krig.scikit_prior).
    var_mode: 'latent' (GP_laser.py:128-131), 'gpy' (+noise, GPy model.predict),
    'sklearn' (+noise, clipped at 0, _gpr.py:473-485).
    variance: 'f64' (default) — the FP64-MFMA engine, FP64 arithmetic throughout as in the
    reference; 'ozaki' (opt-in, vector kernels) — the int8 Ozaki-II emulation of the same FP64
    product, held to the 1e-10 gate by its calibrated accuracy guard (engine.apply_guard: more
    W bits, or FP64 past its range).  The job-stream API (engine.krige_jobs) and bench.py use
    'ozaki'; the drop-in object keeps the reference's arithmetic unless asked.
    """

    def __init__(self, kernel="df", l_df: float = 5.0, l_cf: float = 5.0, ratio: float = None,
                 noise: float = 0.0025, jitter: float = 0.0, var_mode: str = "latent", device=None,
                 chunk: int = 8192, variance: str = "f64", jitchol: int = 0):
        self.spec = self._make_spec(kernel, l_df, l_cf, ratio)
        self.jitchol = int(jitchol)   # GPy jitchol retries on a non-PD K_y (engine.fit)
        if variance == "ozaki" and not self.spec.is_vector:
            raise ValueError("the ozaki variance engine supports the vector kernels only")
        if variance not in E.VARIANCE_ENGINES:
            raise ValueError(f"variance must be one of {E.VARIANCE_ENGINES}")
        self.variance = variance
        self.noise = float(noise)
        self.jitter = float(jitter)
        self.var_mode = var_mode
        self.device = device
        self.chunk = int(chunk)
        self.gp = None
        self._pred = None
        self._X = None
        self._y = None

    @staticmethod
    def _make_spec(kernel, l_df, l_cf, ratio):
        if isinstance(kernel, E.KernelSpec):
            return kernel
        if hasattr(kernel, "_spec"):
            return kernel._spec()
        kind = KERNEL_NAMES[kernel.lower() if isinstance(kernel, str) else kernel]
        if ratio is None:
            ratio = 0.5 if kind == "mixed" else (0.0 if kind == "cf" else 1.0)
        return E.KernelSpec(kind=kind, l_df=float(l_df), l_cf=float(l_cf), ratio=float(ratio))

    # ------------------------------------------------------------------ fit
    def fit(self, X, obs):
        """X: (N, dim) inputs; obs: (2N,) = [u; v] (or (N, 2) columns u, v) for the
        vector kernels, (N,) for the scalar ARD family."""
        X = np.asarray(X, dtype=np.float64) if not isinstance(X, torch.Tensor) else X
        bd = self.spec.block_dim
        y = obs if isinstance(obs, torch.Tensor) else np.asarray(obs, dtype=np.float64)
        if bd == 2 and not isinstance(y, torch.Tensor) and y.ndim == 2 and y.shape[1] == 2:
            y = np.concatenate([y[:, 0], y[:, 1]])
        self.gp = E.fit(self.spec, X, y, self.noise, jitter=self.jitter, device=self.device,
                        variance=self.variance, jitchol=self.jitchol)
        self._pred = E.Predictor(self.gp, self.chunk)
        self._X, self._y = X, y
        return self

    def _check(self):
        if self.gp is None:
            raise RuntimeError("Krig.fit must be called before predict")

    # ------------------------------------------------------------------ predict
    def predict_device(self, Xg, var_mode=None, compute_var=True):
        """Posterior mean and variance as device tensors ([u..., v...] for vector kernels)."""
        self._check()
        return self._pred(Xg, var_mode=var_mode or self.var_mode, compute_var=compute_var)

    def predict(self, Xg, var_mode=None, compute_var=True):
        """(mean, var) numpy arrays of shape (bd·M, 1), as GPy's model.predict returns
        (krig.py:543-544; f[:M] = u, f[M:] = v, GP_plots.py:768-771)."""
        mu, var = self.predict_device(Xg, var_mode=var_mode, compute_var=compute_var)
        mu = _to_numpy(mu)[:, None]
        return mu, (_to_numpy(var)[:, None] if compute_var else None)

    def predict_grid(self, x, y, var_mode=None):
        """GP_laser.py:107-136 on the grid meshgrid(x, y): returns uf, vf, uvar, vvar,
        each reshaped to [y.size, x.size]."""
        X, Y = np.meshgrid(x, y)
        pts = np.stack([X.reshape(-1), Y.reshape(-1)], 1)
        mu, var = self.predict_device(pts, var_mode=var_mode)
        mu, var = _to_numpy(mu), _to_numpy(var)
        M = pts.shape[0]
        shp = [np.size(y), -1]
        return (mu[:M].reshape(shp), mu[M:].reshape(shp), var[:M].reshape(shp), var[M:].reshape(shp))

    # ------------------------------------------------------------------ hyperparameters
    def log_likelihood(self, eval_gradient: bool = False):
        """GPy model.log_likelihood() / sklearn log_marginal_likelihood() of the current fit;
        with eval_gradient also ∂/∂θ in param_array order (engine.param_names)."""
        self._check()
        return E.log_marginal_likelihood(self.gp, eval_gradient=eval_gradient)

    def _apply(self, res: "H.OptResult"):
        self.spec, self.noise = res.kernel, float(res.noise)
        self.fit(self._X, self._y)
        return res

    def optimize(self, fix=(), messages: bool = False, maxiter: int = 200):
        """GPy model.optimize (laser_io_methods.py:496): L-BFGS-B on the LML, refit at the optimum."""
        self._check()
        return self._apply(H.optimize(self.spec, self._X, self._y, self.noise, fix=fix, jitter=self.jitter,
                                      device=self.device, maxiter=maxiter, messages=messages))

    def optimize_restarts(self, num_restarts: int = 10, fix=(), seed: int = 0, messages: bool = False,
                          maxiter: int = 200):
        """GPy model.optimize_restarts (krig.py:450): best of num_restarts L-BFGS-B runs."""
        self._check()
        return self._apply(H.optimize_restarts(self.spec, self._X, self._y, self.noise, num_restarts=num_restarts,
                                               fix=fix, jitter=self.jitter, device=self.device, seed=seed,
                                               maxiter=maxiter, messages=messages))

    # ------------------------------------------------------------------ state
    @property
    def param_array(self):
        s = self.spec
        if s.family == "ard":
            hp = []
            for v, ls in zip(s.variances, s.lengthscales):
                hp += [v, *ls]
            return np.array(hp + [self.noise])
        if s.family == "vector_st":
            return np.array([s.l_df, s.l_cf, s.ratio, s.var_t, s.l_t, self.noise])
        return np.array([s.l_df, s.l_cf, s.ratio, self.noise])

    def save(self, path: str, with_factor: bool = False):
        """Checkpoint: inputs, observations, hyperparameters (and optionally W = L⁻¹, α),
        the analogue of model.pickle (krig.py:412)."""
        self._check()
        s = self.spec
        d = dict(X=_to_numpy(self._X), y=_to_numpy(self._y), family=s.family, kind=str(s.kind), l_df=s.l_df,
                 l_cf=s.l_cf, ratio=s.ratio, variances=np.asarray(s.variances, dtype=np.float64),
                 lengthscales=np.asarray(s.lengthscales, dtype=np.float64), var_t=s.var_t, l_t=s.l_t,
                 noise=self.noise, jitter=self.jitter, jitchol=self.jitchol,
                 jitchol_used=float(self.gp.extra.get("jitchol", 0.0)),
                 var_mode=self.var_mode, variance=self.variance, chunk=self.chunk)
        if with_factor:
            d["W"] = _to_numpy(self.gp.W)
            d["alpha"] = _to_numpy(self.gp.alpha)
            if self.gp.perm is not None:   # W and α follow the training points in X[perm] order
                d["perm"] = _to_numpy(self.gp.perm)
        np.savez(path, **d)

    @classmethod
    def load(cls, path: str, device=None, refit: bool = True):
        """Restore a checkpoint written by save(): GPy.load / pickle.load of a fitted model
        (krig.py:478-483).  A checkpoint with the factor (save(with_factor=True)) is restored
        without refitting — W, α and the training order go back to the device as saved, so
        predictions are bit-identical to the saved model's; without it the model is refitted
        from the stored inputs (refit=False then returns an unfitted model)."""
        z = np.load(path, allow_pickle=False)
        fam = str(z["family"])
        if fam == "ard":
            spec = E.KernelSpec(family="ard", variances=tuple(z["variances"].tolist()),
                                lengthscales=tuple(tuple(r) for r in z["lengthscales"].tolist()))
        else:
            st = dict(var_t=float(z["var_t"]), l_t=float(z["l_t"])) if "var_t" in z.files else {}
            spec = E.KernelSpec(family=fam, kind=str(z["kind"]), l_df=float(z["l_df"]), l_cf=float(z["l_cf"]),
                                ratio=float(z["ratio"]), **st)
        extra = {}
        if "variance" in z.files:   # older checkpoints carry none: they were written by the f64 engine
            extra = dict(variance=str(z["variance"]), chunk=int(z["chunk"]))
        if "jitchol" in z.files:
            extra["jitchol"] = int(z["jitchol"])
        k = cls(spec, noise=float(z["noise"]), jitter=float(z["jitter"]), var_mode=str(z["var_mode"]),
                device=device, **extra)
        if "W" in z.files:
            used = float(z["jitchol_used"]) if "jitchol_used" in z.files else 0.0
            k._restore(z["X"], z["y"], z["W"], z["alpha"], z["perm"] if "perm" in z.files else None, used)
        elif refit:
            k.fit(z["X"], z["y"])
        return k

    def _restore(self, X, y, W, alpha, perm, jitchol_used: float = 0.0):
        """Rebuild the device fit from a saved factor (no assembly, no factorisation).
        `jitchol_used` is the jitter a jitchol retry added to the saved factor's K_y diagonal:
        the Ozaki residue planes take the a-priori moduli count from the diagonal the factor was
        built with (noise + jitter + that jitter), exactly as fit() did."""
        dev = E._require_device(self.device)
        spec = self.spec
        bd, d = spec.block_dim, spec.input_dim
        Xd = torch.as_tensor(np.ascontiguousarray(np.asarray(X, dtype=np.float64).reshape(-1, d)), device=dev)
        ntr = Xd.shape[0]
        npad, n = E.fit_layout(spec, ntr, self.variance)
        if W.shape != (n, n) or alpha.shape != (n,):
            raise ValueError(f"saved factor has shape {W.shape}, the fit layout needs ({n}, {n})")
        pm = None
        if perm is not None:
            pm = torch.as_tensor(np.asarray(perm, dtype=np.int64), device=dev)
            Xs = torch.empty_like(Xd)
            E.N.check(E.N.lib().gp2d_gather_rows(E._ptr(Xd), E._ptr(pm), ntr, Xd.shape[1], E._ptr(Xs),
                                                 E._stream_handle(dev)), "gp2d_gather_rows")
            Xd = Xs
        Y = E._pad_obs(y, ntr, npad, bd, dev, pm)
        gp = E.GPFit(kernel=spec, noise=self.noise, x=Xd, n_train=ntr, n_pad=npad,
                     W=torch.as_tensor(np.ascontiguousarray(W), device=dev),
                     alpha=torch.as_tensor(np.ascontiguousarray(alpha), device=dev), device=dev, y=Y, perm=pm)
        gp.extra["jitchol"] = float(jitchol_used)
        if self.variance == "ozaki":
            E.ozaki_prepare_guarded(gp, float(self.noise + (self.jitter + jitchol_used)))
        self.gp = gp
        self._pred = E.Predictor(gp, self.chunk)
        self._X, self._y = X, y
        return self


# ===================================================================== module functions
def rmse(ys, y):
    """krig.rmse (krig.py:641-645)."""
    error = np.reshape(np.asarray(ys) - np.asarray(y), [-1])
    return np.sqrt(np.mean(np.square(error)))


def getGrid(to, yo, xo, dt=0.5, dx=0.5, xL=40, yL=40):
    """krig.getGrid (krig.py:648-678) — bit-exact (tests/golden/grids.npz)."""
    return D.get_grid(to, yo, xo, dt, dx, xL, yL)


def boundData(var, varlim, lat, lon, v, u):
    """krig.boundData (krig.py:79-86)."""
    return D.bound_data(var, varlim, lat, lon, v, u)


@dataclass
class Tracks:
    """Drifter track container (the fields of laser_class.interpolated_tracks used by
    krig.getData, krig.py:42-77): time (T,), lat/lon/u/v (T, D)."""
    time: np.ndarray
    lat: np.ndarray
    lon: np.ndarray
    u: np.ndarray
    v: np.ndarray

    @classmethod
    def load(cls, path: str) -> "Tracks":
        z = np.load(path, allow_pickle=False)
        return cls(z["time"], z["lat"], z["lon"], z["u"], z["v"])

    @classmethod
    def synthetic(cls, n_time: int = 96, n_drifters: int = 64, seed: int = 2016) -> "Tracks":
        """Drifters advected through the div-free Gaussian eddy of data.synthetic_tracks."""
        rng = np.random.default_rng(seed)
        x = rng.uniform(0, 60, n_drifters)
        y = rng.uniform(0, 45, n_drifters)
        dt_h = 0.25
        X = np.empty((n_time, n_drifters))
        Y = np.empty((n_time, n_drifters))
        U = np.empty((n_time, n_drifters))
        V = np.empty((n_time, n_drifters))
        for t in range(n_time):
            psi = np.exp(-((x - 30) ** 2 + (y - 22.5) ** 2) / 15.0 ** 2)
            u = psi * (-2 * (y - 22.5) / 15.0 ** 2) + rng.normal(0, 0.02, n_drifters)
            v = -psi * (-2 * (x - 30) / 15.0 ** 2) + rng.normal(0, 0.02, n_drifters)
            X[t], Y[t], U[t], V[t] = x, y, u, v
            x = x + u * 3.6 * dt_h
            y = y + v * 3.6 * dt_h
        R = 6371.0
        lat = lat0 + np.rad2deg(Y / R)
        lon = lon0 + np.rad2deg(X / (R * np.cos(np.deg2rad(lat0))))
        return cls(np.arange(n_time) * dt_h * 3600.0, lat, lon, U, V)


def getData(st, et, tracks: Tracks, drop_drifters=()):
    """krig.getData (krig.py:42-77) on a track container: time in hours from the first
    sample, columns ordered by decreasing number of valid points.  drop_drifters are set to
    NaN first — the reference hard-codes drifter 238 of Filtered_2016_2_7.pkl (krig.py:46-52);
    pass (238,) for that file.  The caller's container is not modified."""
    lat, lon, u, v = (np.array(a, dtype=np.float64) for a in (tracks.lat, tracks.lon, tracks.u, tracks.v))
    for c in drop_drifters:
        lat[:, c] = np.nan
        lon[:, c] = np.nan
        u[:, c] = np.nan
        v[:, c] = np.nan
    time_h = (tracks.time[st:et] - tracks.time[0]) / 3600.0
    latt = lat[st:et, :]
    lont = lon[st:et, :]
    uob = u[st:et, :]
    vob = v[st:et, :]
    valid = np.array([np.size(np.where((~np.isnan(lont[:, i])) & (~np.isnan(latt[:, i])))[0])
                      for i in range(latt.shape[1])])
    order = np.squeeze(valid.argsort(axis=0))[::-1]
    return time_h, latt[:, order], lont[:, order], vob[:, order], uob[:, order], valid[order]


def _prepare(tracks, st, et, lalim, lolim, sample_step, skip, drop_drifters=()):
    """Data selection of krig.kriging (krig.py:274-381): bounds, projection, split,
    NaN filter, T,Y,X stacking.  Returns dict of observation / test arrays.
    Bit-exact with the reference's code on the same tracks (tests/golden/prep_tracks.npz)."""
    time_h, latt, lont, vob, uob, _ = getData(st, et, tracks, drop_drifters)
    if lolim[1] > lolim[0]:
        latt, lont, vob, uob = boundData(lont, lolim, latt, lont, vob, uob)
    if lalim[1] > lalim[0]:
        latt, lont, vob, uob = boundData(latt, lalim, latt, lont, vob, uob)
    xob, yob = nad83(lont, latt)
    tob = np.repeat(time_h[:, None], latt.shape[1], axis=1)
    yob[np.where(np.isnan(lont))] = np.nan
    xob[np.where(np.isnan(lont))] = np.nan
    xob = (xob - x_ori) / 1000.0
    yob = (yob - y_ori) / 1000.0
    if (sample_step < 0) or (skip > 1):
        samples, testt, testd = D.drifter_split(tob.shape[0], tob.shape[1], sample_step, skip)

        def pick(a):
            return np.reshape(a[samples, ::skip], [-1, 1]), np.reshape(a[testt[:, None], testd], [-1, 1])
    else:
        samples, test = D.split_indices(xob.size, sample_step)

        def pick(a):
            return np.reshape(a, [-1])[samples, None], np.reshape(a, [-1])[test, None]
    (to, tt), (yo, yt), (xo, xt) = pick(tob), pick(yob), pick(xob)
    (lat_o, lat_t), (lon_o, lon_t) = pick(latt), pick(lont)
    (uo, ut), (vo, vt) = pick(uob), pick(vob)
    vo_mask = np.where((~np.isnan(xo)) & (~np.isnan(yo)))
    vt_mask = np.where((~np.isnan(xt)) & (~np.isnan(yt)))
    o = [a[vo_mask][:, None] for a in (to, yo, xo, lat_o, lon_o, uo, vo)]
    t = [a[vt_mask][:, None] for a in (tt, yt, xt, lat_t, lon_t, ut, vt)]
    return dict(X=np.concatenate([o[0], o[1], o[2]], 1), LL_o=np.concatenate([o[0], o[3], o[4]], 1),
                uo=o[5], vo=o[6], Xt=np.concatenate([t[0], t[1], t[2]], 1),
                LL_t=np.concatenate([t[0], t[3], t[4]], 1), ut=t[5], vt=t[6])


def kriging(st, et, lalim=(0, 0), lolim=(0, 0), sample_step=5, skip=5, nKernels=1, output="rbfModel",
            pkg="gp2d", kernelType=1, laser=1, tracks: Tracks = None, hyper: dict = None, device=None,
            drop_drifters=()):
    """krig.kriging (krig.py:259-418): build the GP model(s) for a drifter data window.

    kernelType 1: scalar ARD RBF on (T, Y, X), one model per component (v, u);
    2 / 3 / 4: Kt(var_t, l_t) × div-free / curl-free / mixed vector kernel on (T, Y, X) with
    obs = [v; u] (krig.py:392-404; hyper 'temporal': False → spatial kernel on (Y, X)).  nKernels > 1 sums nKernels identical ARD terms (krig.py:405-407;
    ≤ 2 supported).  Hyperparameters come from `hyper` (no optimisation here).
    Writes output+'.npz' (the .mat of krig.py:417) and the model files; returns the models.
    """
    if tracks is None:
        raise ValueError("tracks= is required (the reference's Filtered_2016_2_7.pkl is not available)")
    t0 = time.time()
    h = dict(l_df=5.0, l_cf=5.0, ratio=None, noise=0.0025, variance=1.0, lengthscale=(1.0, 1.0, 1.0),
             var_t=1.0, l_t=1.0, temporal=True)
    h.update(hyper or {})
    d = _prepare(tracks, st, et, lalim, lolim, sample_step, skip, drop_drifters)
    X, Xt = d["X"], d["Xt"]
    models = {}
    if kernelType == 1:
        nk = min(int(nKernels), 2)
        spec = E.KernelSpec(family="ard", variances=tuple([h["variance"]] * nk),
                            lengthscales=tuple([tuple(h["lengthscale"])] * nk))
        for name, obs in (("v", d["vo"]), ("u", d["uo"])):
            k = Krig(spec, noise=h["noise"], var_mode="gpy", device=device).fit(X, obs[:, 0])
            k.save(output + f"_{name}.npz")
            models[name] = k
        obs_all = np.concatenate([d["vo"], d["uo"]], 1)
        obst = np.concatenate([d["vt"], d["ut"]], 1)
    else:
        kind = {2: "df", 3: "cf", 4: "mixed"}[int(kernelType)]
        obs_all = np.concatenate([d["vo"], d["uo"]], 0)
        obst = np.concatenate([d["vt"], d["ut"]], 0)
        ratio = h["ratio"] if h["ratio"] is not None else {"df": 1.0, "cf": 0.0, "mixed": 0.5}[kind]
        if h["temporal"]:
            spec = E.KernelSpec(family="vector_st", kind=kind, l_df=h["l_df"], l_cf=h["l_cf"], ratio=ratio,
                                var_t=h["var_t"], l_t=h["l_t"])
            k = Krig(spec, noise=h["noise"], var_mode="gpy", device=device).fit(X, obs_all[:, 0])
        else:
            k = Krig(kind, l_df=h["l_df"], l_cf=h["l_cf"], ratio=ratio, noise=h["noise"], var_mode="gpy",
                     device=device).fit(X[:, 1:3], obs_all[:, 0])
        tag = {2: "_divFree", 3: "_curlFree", 4: "_combined"}[int(kernelType)]
        k.save(output + tag + ".npz")
        models[tag] = k
    np.savez(output + ".npz", Xo=X, obs=obs_all, Xt=Xt, LL_o=d["LL_o"], LL_t=d["LL_t"], test_points=obst,
             kernelType=kernelType)
    print("End of script, time : " + str(time.time() - t0))
    return models


def runRestarts(fname, nres=10, nKernels=2, device=None, seed=0):
    """krig.runRestarts (krig.py:430-468): load a saved model, optimize_restarts its
    hyperparameters (nres runs), save it back and print old : new values.  Model files are
    .npz (Krig.save) instead of GPy pickles; the restart history is kept in the model file
    (the reference's fname_dict.pkl workaround, krig.py:439-457, is not needed)."""
    t0 = time.time()
    filename = fname if fname.endswith(".npz") else fname + ".npz"
    model = Krig.load(filename, device=device)
    hyp_old = model.param_array.copy()
    res = model.optimize_restarts(num_restarts=nres, seed=seed)
    hyp = model.param_array
    model.save(filename)
    print("Optimized Hyperparameters =================================================")
    names = E.param_names(model.spec)
    for nm, a, b in zip(names, hyp_old, hyp):
        print(f"{nm} = {a}   :   {b}")
    print("===========================================================================")
    print("End of script, time : " + str(time.time() - t0))
    return res


def _vec_cols(model, X):
    """(T, Y, X) rows for the spatio-temporal kernel, (Y, X) for the spatial one."""
    return X if model.spec.input_dim == 3 else X[:, 1:3]


def predict(filename, tlim=(0, 0), ylim=(0, 0), xlim=(0, 0), dt=0.5, dx=0.5, xL=40, yL=40, Simul=0,
            device=None):
    """krig.predict (krig.py:471-574): grid posterior per time slice for the u and v
    models saved by kriging(); writes filename+'.nc' (krig.py:559-570) and filename+'_pred.npz', returns
    (Xp, V, U, VVar, UVar) reshaped [tp, yp, xp]."""
    t0 = time.time()
    f = np.load(filename + ".npz", allow_pickle=False)
    kt = int(f["kernelType"]) if "kernelType" in f.files else 1
    if (ylim[0] == ylim[1]) and (xlim[0] == xlim[1]):
        Xo = f["Xo"]
        Xp, tp, yp, xp = getGrid(Xo[:, 0], Xo[:, 1], Xo[:, 2])
    else:
        Xp, tp, yp, xp = getGrid(tlim, ylim, xlim, dt, dx, xL, yL)
    inc = yp.size * xp.size
    V, U, VV, UV = [], [], [], []
    if kt == 1:
        mv = Krig.load(filename + "_v.npz", device=device)
        mu_ = Krig.load(filename + "_u.npz", device=device)
    else:
        tag = {2: "_divFree", 3: "_curlFree", 4: "_combined"}[kt]
        mvec = Krig.load(filename + tag + ".npz", device=device)
    for i in range(tp.size):                         # krig.py:541-557
        Xp2 = Xp[i * inc:(i + 1) * inc, :]
        if kt == 1:
            v2, vv2 = mv.predict(Xp2)
            u2, uv2 = mu_.predict(Xp2)
        else:
            f2, fv2 = mvec.predict(_vec_cols(mvec, Xp2))
            v2, u2 = f2[:inc], f2[inc:]
            vv2, uv2 = fv2[:inc], fv2[inc:]
        V.append(v2)
        U.append(u2)
        VV.append(vv2)
        UV.append(uv2)
    shp = [tp.size, yp.size, xp.size]
    V, U, VV, UV = (np.reshape(np.concatenate(a, 0), shp) for a in (V, U, VV, UV))
    np.savez(filename + "_pred.npz", time=tp, y=yp, x=xp, v=V, u=U, vvar=VV, uvar=UV)
    # NetCDF-3 product, krig.py:559-570 (createNC + writeNC of v, u, vvar, uvar, hyperparams)
    hyp_v = (mv if kt == 1 else mvec).param_array
    hyp_u = (mu_ if kt == 1 else mvec).param_array
    NC.write_prediction(filename + ".nc", tp, yp, xp, V, U, VV, UV, hyp_v, hyp_u)
    print("End of script, time : " + str(time.time() - t0))
    return Xp, V, U, VV, UV


def predictTest(filename, device=None):
    """krig.predictTest (krig.py:578-616): predict at the held-out test points in 10
    chunks (step = Nt // 10, the py2 integer division of krig.py:593)."""
    f = np.load(filename + ".npz", allow_pickle=False)
    Xt = f["Xt"]
    obst = f["test_points"]
    kt = int(f["kernelType"]) if "kernelType" in f.files else 1
    Nt = Xt.shape[0]
    step = max(Nt // 10, 1)
    if kt == 1:
        mv = Krig.load(filename + "_v.npz", device=device)
        mu_ = Krig.load(filename + "_u.npz", device=device)
    else:
        tag = {2: "_divFree", 3: "_curlFree", 4: "_combined"}[kt]
        mvec = Krig.load(filename + tag + ".npz", device=device)
    V, U, VV, UV = [], [], [], []
    for i in range(0, Nt, step):
        Xt2 = Xt[i:i + step, :] if i + step < Nt else Xt[i:, :]
        if kt == 1:
            v2, vv2 = mv.predict(Xt2)
            u2, uv2 = mu_.predict(Xt2)
        else:
            m = Xt2.shape[0]
            f2, fv2 = mvec.predict(_vec_cols(mvec, Xt2))
            v2, u2, vv2, uv2 = f2[:m], f2[m:], fv2[:m], fv2[m:]
        V.append(v2)
        U.append(u2)
        VV.append(vv2)
        UV.append(uv2)
    V, U, VV, UV = (np.concatenate(a, 0) for a in (V, U, VV, UV))
    np.savez(filename + "_test.npz", Xt=Xt, Vp=V, VpVar=VV, Up=U, UpVar=UV, test_points=obst)
    return V, U, VV, UV


def _prior_window(fm, tcenter, tlim, xlim, xrange, varname):
    """scikit_prior's observation window (krig.py:146-167): observation and test points within
    ±tlim of tcenter and within xrange of the x window, stacked [obs; test], and the chosen
    velocity component.  Bit-exact with the reference (tests/golden/prior_window.npz); a
    window holding a single point stays 2-D here (the reference's squeeze() would make it 1-D)."""
    to, tt = fm["Xo"][:, 0], fm["Xt"][:, 0]
    xo, xt = fm["Xo"][:, 2], fm["Xt"][:, 2]
    ito = np.where((to >= tcenter - tlim) & (to <= tcenter + tlim) & (xo >= xlim[0] - xrange) & (xo <= xlim[1] + xrange))
    itt = np.where((tt >= tcenter - tlim) & (tt <= tcenter + tlim) & (xt >= xlim[0] - xrange) & (xt <= xlim[1] + xrange))
    Xo = fm["Xo"][ito, :].squeeze(0)
    Xt = fm["Xt"][itt, :].squeeze(0)
    XT = np.concatenate([Xo, Xt], axis=0)
    obs = fm["obs"][ito, :].squeeze(0)
    obst = fm["test_points"][itt, :].squeeze(0)
    col = 1 if varname == "u" else 0
    return XT, np.concatenate([obs[:, col], obst[:, col]])


RADAR_T0 = datetime(2016, 1, 1)             # radar time origin (days), krig.py:110
RADAR_T0D = datetime(2016, 2, 7, 2, 15)     # first time of Filtered_2016_2_7.pkl, krig.py:111


def radar_grid(radar):
    """The HF-radar grid branch of scikit_prior (krig.py:98-118): the radar NetCDF's image
    origin (imageOriginPosition = lon, lat) projected and shifted to the drifter frame in km,
    plus its xCoords / yCoords (m); the first radar time, counted in days from 2016-01-01,
    becomes hours since the drifter data's first time.  Returns (X (M, 3) in T, Y, X order,
    tcenter, yg, xg) with the meshgrid(yg, tg, xg) flattening of krig.py:114-118.
    Reference quirk: that branch never sets `tcenter`, which krig.py:143 then reads (NameError);
    the build takes the radar time tg as the window centre, the evident intent."""
    R = NC.readNC(radar)
    lon_r, lat_r = (float(v) for v in np.asarray(R["imageOriginPosition"], dtype=np.float64).reshape(-1)[:2])
    x0, y0 = nad83(lon_r, lat_r)
    x0 = (x0 - x_ori) / 1000.0
    y0 = (y0 - y_ori) / 1000.0
    xg = x0 + np.asarray(R["xCoords"], dtype=np.float64) / 1000.0
    yg = y0 + np.asarray(R["yCoords"], dtype=np.float64) / 1000.0
    tr = np.asarray(R["time"], dtype=np.float64).reshape(-1)
    tg = np.array([(RADAR_T0 + timedelta(float(tr[0])) - RADAR_T0D).total_seconds() / 3600])
    Yg, Tg, Xg = np.meshgrid(yg, tg, xg)
    X = np.concatenate([Tg.reshape(-1, 1), Yg.reshape(-1, 1), Xg.reshape(-1, 1)], axis=1)
    return X, tg, yg, xg


def scikit_prior(filename0, varname="v", dt=0, tlim=6, radar="", xlim=(0, 0), ylim=(0, 0), dx=0, ind=0, xrange=3,
                 HP=None, device=None):
    """krig.scikit_prior (krig.py:88-207): fixed-hyperparameter scalar GP
    HP0·RBF([lt,ly,lx]) (+ HP4·RBF) + White(noise) on the windowed observations,
    predicted on a radar NetCDF's grid (radar=path, radar_grid, krig.py:98-118), at time dt
    on the getGrid window (xlim/ylim given) or on the grid of a pre-existing
    filename0+'.nc' (krig.py:123-141).  Model inputs come from
    filename0+'.npz' (written by kriging); HP = [var1, lt, ly, lx, (var2, lt, ly, lx,) noise]
    (the GPy param_array the reference loads at krig.py:159-161).
    Writes <filename>_<t>h_scikit_<ind>.nc (createNC if absent, then varname, varname+'var',
    hyperparam_<varname>, krig.py:197-206) and returns (U, Ustd²) reshaped [1, yg, xg]."""
    fm = np.load(filename0 + ".npz", allow_pickle=False)
    if HP is None:
        raise ValueError("HP (hyperparameters) is required: the reference reads them from a GPy pickle")
    HP = np.asarray(HP, dtype=np.float64)
    if radar:                                                         # krig.py:98-118
        X, tcenter, yg, xg = radar_grid(radar)
        filename = filename0 + "_radar"
    elif (xlim[1] > xlim[0]) and (ylim[1] > ylim[0]):
        X, tcenter, yg, xg = getGrid([dt, dt + 1], ylim, xlim, 1, dx)   # krig.py:121
        filename = filename0 + "_cyc"
    else:                                                             # krig.py:123-141
        g = NC.readNC(filename0 + ".nc")
        xg, yg, tg = (np.asarray(g[k], dtype=np.float64) for k in ("x", "y", "time"))
        it = int(dt)
        tcenter = np.array([tg[it]])
        Yg, Tg, Xg = np.meshgrid(yg, tg, xg)
        X = np.concatenate([Tg.reshape(-1, 1), Yg.reshape(-1, 1), Xg.reshape(-1, 1)], 1)
        filename = filename0
        inc = yg.size * xg.size
        X = X[inc * it:inc * it + inc, :]
    filename = filename + "_" + str(np.round(tcenter[0], decimals=2)) + "h_scikit_"
    outFile = filename + str(ind) + ".nc"
    XT, u = _prior_window(fm, tcenter, tlim, xlim, xrange, varname)
    N = HP.size - 1
    variances = [HP[0]]
    lengths = [tuple(HP[1:4])]
    if N > 5:
        variances.append(HP[4])
        lengths.append(tuple(HP[5:8]))
    spec = E.KernelSpec(family="ard", variances=tuple(variances), lengthscales=tuple(lengths))
    # sklearn: WhiteKernel adds noise to K_y and to the predictive diagonal; fit adds alpha=1e-10
    k = Krig(spec, noise=HP[-1], jitter=1e-10, var_mode="sklearn", device=device).fit(XT, u)
    Um, Uvar = k.predict(X)
    U = np.reshape(Um, [tcenter.size, yg.size, xg.size])
    Ustd2 = np.reshape(Uvar, [tcenter.size, yg.size, xg.size])
    if not os.path.isfile(outFile):
        NC.createNC(outFile, tcenter, yg, xg, HP)
    with NC.openNC(outFile, "a") as fi:
        NC.writeNC(fi, varname, U)
        NC.writeNC(fi, varname + "var", Ustd2)
        NC.writeNC(fi, "hyperparam_" + varname, HP)
    return U, Ustd2


def laser(xo, yo, uo, vo, l_df=5, l_cf=5, rate=0.5, noise=0.0025, nsamples=1, dx=0.5, device=None):
    """GP_laser.laser (GP_laser.py:16-142) from projected observations (the pickle /
    pyproj loading of GP_laser.py:26-78 is data plumbing outside the hot path):
    stride-3 split, grid over obs ∪ test ± 5 km, mixed kernel rate·K_df + (1−rate)·K_cf
    + noise·I, posterior mean / variance on the grid and mean at the test points.
    Returns (x, y, uf, vf, xo, yo, uo, vo, uvar, vvar, xt, yt, ut, vt, uft, vft)."""
    xo, yo, uo, vo = (np.asarray(a, dtype=np.float64).reshape(-1) for a in (xo, yo, uo, vo))
    if nsamples > 0:
        samples, test = D.split_indices(xo.size, 3)
        xt, yt, ut, vt = xo[test], yo[test], uo[test], vo[test]
        xo, yo, uo, vo = xo[samples], yo[samples], uo[samples], vo[samples]
    else:
        xt = yt = ut = vt = np.array([0.0])
    x, y, Xs, Ys = D.laser_grid(xo, yo, xt, yt, dx=dx)
    k = Krig("mixed", l_df=l_df, l_cf=l_cf, ratio=rate, noise=noise, device=device)
    k.fit(np.stack([xo, yo], 1), np.concatenate([uo, vo]))
    uf, vf, uvar, vvar = k.predict_grid(x, y)
    ft, _ = k.predict(np.stack([xt, yt], 1), compute_var=False)
    ft = ft[:, 0]
    return x, y, uf, vf, xo, yo, uo, vo, uvar, vvar, xt, yt, ut, vt, ft[:ft.size // 2], ft[ft.size // 2:]
