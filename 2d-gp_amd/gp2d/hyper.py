"""Hyperparameter fitting on the GPU.

Replaces GPy's model.optimize / optimize_restarts (krig.py:430-468 runRestarts;
GP_plots.py:673-765; laser_io_methods.py:496-676) and sklearn's internal
L-BFGS-B restarts (_gpr.py:298-333).  Every objective evaluation is one HIP fit
(assemble → POTRF → TRTRI → α) plus gp2d_lml / gp2d_lml_grad; only the optimiser
state (a handful of scalars) lives on the host.

Free parameters are optimised in an unconstrained space, as GPy does through its
constraints (myKernel.py:19-21): length scales, variances and the noise variance
through log (GPy: constrain_positive), the div-free weight `ratio` through the
logistic map (GPy: constrain_bounded(0, 1)).  Restarts draw the starting point
uniformly within ±`spread` of the current point in that space (GPy's randomize()
draws from the parameters' priors; the reference sets none, so the spread is ours).

Config E (64 hyperparameter settings × N=4096, BASELINE.json) is `sweep`: the
settings are dealt round-robin to ranks (one GP per GPU at a time), each rank
evaluates its own, and one all-reduce of a zero-padded vector assembles the
results — every entry has exactly one non-zero contributor, so the result is
bit-identical for any world size.
"""
from __future__ import annotations

import collections

import dataclasses
import math
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.distributed as dist

from . import comm as C
from . import engine as E

_BAD = 1e25  # objective for a non-positive-definite K_y (rejected by the line search)


def free_names(kernel: E.KernelSpec, fix=()) -> tuple:
    """Names (engine.param_names order) of the parameters the optimiser moves."""
    if kernel.is_vector:
        used = {"df": ("l_df",), "scalar": ("l_df",), "cf": ("l_cf",),
                "mixed": ("l_df", "l_cf", "ratio")}[_kind_name(kernel.kind)]
        if kernel.family == "vector_st":
            used = used + ("var_t", "l_t")
        names = used + ("noise",)
    else:
        names = E.param_names(kernel)
    return tuple(n for n in names if n not in set(fix))


def _kind_name(kind):
    return {0: "scalar", 1: "df", 2: "cf", 3: "mixed"}.get(kind, kind)


def get_params(kernel: E.KernelSpec, noise: float) -> dict:
    names = E.param_names(kernel)
    if kernel.family == "vector2d":
        vals = (kernel.l_df, kernel.l_cf, kernel.ratio, noise)
    elif kernel.family == "vector_st":
        vals = (kernel.l_df, kernel.l_cf, kernel.ratio, kernel.var_t, kernel.l_t, noise)
    else:
        vals = []
        for v, ls in zip(kernel.variances, kernel.lengthscales):
            vals += [v, *ls]
        vals.append(noise)
    return dict(zip(names, (float(v) for v in vals)))


def set_params(kernel: E.KernelSpec, params: dict):
    """(KernelSpec, noise) with `params` (a get_params-style dict) applied."""
    if kernel.family == "vector2d":
        k = dataclasses.replace(kernel, l_df=params["l_df"], l_cf=params["l_cf"], ratio=params["ratio"])
        return k, params["noise"]
    if kernel.family == "vector_st":
        k = dataclasses.replace(kernel, l_df=params["l_df"], l_cf=params["l_cf"], ratio=params["ratio"],
                                var_t=params["var_t"], l_t=params["l_t"])
        return k, params["noise"]
    var, ls = [], []
    for t, l in enumerate(kernel.lengthscales):
        var.append(params[f"variance_{t}"])
        ls.append(tuple(params[f"lengthscale_{t}_{d}"] for d in range(len(l))))
    return dataclasses.replace(kernel, variances=tuple(var), lengthscales=tuple(ls)), params["noise"]


def _to_free(name, v):
    if name == "ratio":
        v = min(max(v, 1e-12), 1 - 1e-12)
        return math.log(v / (1 - v))
    return math.log(v)


def _from_free(name, z):
    if name == "ratio":
        return 1.0 / (1.0 + math.exp(-z))
    return math.exp(z)


def _dfree(name, v):
    """d(value)/d(free coordinate)."""
    return v * (1 - v) if name == "ratio" else v


@dataclass
class OptResult:
    kernel: E.KernelSpec
    noise: float
    lml: float
    nit: int = 0
    nfev: int = 0
    success: bool = True
    message: str = ""
    runs: list = field(default_factory=list)   # per-restart (params dict, lml), GPy optimization_runs


class Objective:
    """−LML and its gradient in the free coordinates, one HIP fit per evaluation."""

    def __init__(self, kernel, x, y, noise, names, jitter=0.0, device=None):
        self.kernel, self.noise = kernel, float(noise)
        self.x, self.y = x, y
        self.names = tuple(names)
        self.jitter = float(jitter)
        self.device = device
        self.base = get_params(kernel, noise)
        self.order = E.param_names(kernel)
        self.nfev = 0

    def params(self, z) -> dict:
        p = dict(self.base)
        for n, zi in zip(self.names, z):
            p[n] = _from_free(n, float(zi))
        return p

    def __call__(self, z):
        self.nfev += 1
        p = self.params(z)
        k, noise = set_params(self.kernel, p)
        try:
            gp = E.fit(k, self.x, self.y, noise, jitter=self.jitter, device=self.device)
        except np.linalg.LinAlgError:
            return _BAD, np.zeros(len(z))
        val, g = E.log_marginal_likelihood(gp, eval_gradient=True)
        del gp
        gd = dict(zip(self.order, g))
        gz = np.array([gd[n] * _dfree(n, p[n]) for n in self.names])
        if not np.isfinite(val) or not np.all(np.isfinite(gz)):
            return _BAD, np.zeros(len(z))
        return -val, -gz


def optimize(kernel: E.KernelSpec, x, y, noise: float, fix=(), jitter: float = 0.0, device=None,
             maxiter: int = 200, start: dict = None, messages: bool = False) -> OptResult:
    """Maximise the LML over the free hyperparameters with L-BFGS-B (GPy model.optimize,
    krig.py:450 / laser_io_methods.py:496).  `fix` names parameters to hold (GPy
    constrain_fixed, GP_plots.py:761-762)."""
    from scipy.optimize import minimize
    names = free_names(kernel, fix)
    obj = Objective(kernel, x, y, noise, names, jitter=jitter, device=device)
    p0 = dict(obj.base)
    if start:
        p0.update(start)
    z0 = np.array([_to_free(n, p0[n]) for n in names])
    if len(names) == 0:
        val = -obj(z0)[0]
        return OptResult(kernel, float(noise), val, nfev=1)
    res = minimize(obj, z0, jac=True, method="L-BFGS-B", options=dict(maxiter=maxiter, disp=bool(messages)))
    p = obj.params(res.x)
    k, nz = set_params(kernel, p)
    return OptResult(k, nz, float(-res.fun), nit=int(res.nit), nfev=obj.nfev, success=bool(res.success),
                     message=str(res.message))


def optimize_restarts(kernel: E.KernelSpec, x, y, noise: float, num_restarts: int = 10, fix=(),
                      jitter: float = 0.0, device=None, seed: int = 0, spread: float = 1.0,
                      maxiter: int = 200, messages: bool = False) -> OptResult:
    """GPy model.optimize_restarts (krig.py:450): the first run starts at the current
    hyperparameters, the others at random points within ±spread (free coordinates);
    the best run is returned, all runs are listed in .runs."""
    rng = np.random.default_rng(seed)
    names = free_names(kernel, fix)
    base = get_params(kernel, noise)
    best = None
    runs = []
    for r in range(max(1, int(num_restarts))):
        start = None
        if r > 0:
            start = {n: _from_free(n, _to_free(n, base[n]) + rng.uniform(-spread, spread)) for n in names}
        res = optimize(kernel, x, y, noise, fix=fix, jitter=jitter, device=device, maxiter=maxiter, start=start,
                       messages=messages)
        runs.append((get_params(res.kernel, res.noise), res.lml))
        if best is None or res.lml > best.lml:
            best = res
    best.runs = runs
    return best


def sweep(kernel: E.KernelSpec, x, y, settings, noise: float = None, jitter: float = 0.0, device=None,
          eval_gradient: bool = False, concurrent: int | None = None, batch: int | None = None):
    """LML (and gradient) for each hyperparameter setting (a list of get_params-style dicts,
    missing keys taken from kernel/noise) — BASELINE config E.  Under torch.distributed the
    settings are dealt round-robin over ranks and the results all-reduced (bit-identical to
    one rank).  Returns (lml[S], grad[S, P] or None); a non-PD setting gives -inf.

    concurrent = c > 1: the settings' fit + LML (+ gradient) are queued on c streams with no
    host round trip for the results (engine.fit(check=False), engine.lml_device), read back 2c
    settings behind; each fit joins its chain on the host (fit(join=True)), so setting i's LML
    and gradient run under setting i+1's factorisation (config E: 60.8–61.2 vs 58.3–59.2
    settings/s at c = 1; without the join, 41.9).  Same kernels, same bits as c = 1.
    concurrent = None (default): auto_concurrent() — 2 when there is a gradient to overlap and
    this rank holds at least two settings, else 1.
    batch = b > 1: the settings are fitted b at a time in one batched factorisation
    (engine.fit_batch: the fit's latency-bound diagonal chain paid once per b settings), then
    each setting's LML (+ gradient) runs on the filled chip; same bits as b = 1.  batch = None
    (default): auto_batch() — used instead of `concurrent` when it applies."""
    ws, rank = (dist.get_world_size(), dist.get_rank()) if dist.is_available() and dist.is_initialized() else (1, 0)
    base = get_params(kernel, noise if noise is not None else 0.0)
    S = len(settings)
    P = len(base)
    vals = np.zeros(S)
    grads = np.zeros((S, P))
    mine = list(range(rank, S, ws))
    bsz = auto_batch(kernel, x, len(mine), concurrent) if batch is None else max(1, int(batch))
    c = auto_concurrent(len(mine), eval_gradient) if concurrent is None else max(1, int(concurrent))
    if bsz > 1:
        _sweep_batched(kernel, x, y, settings, base, mine, jitter, device, eval_gradient, bsz, vals, grads)
    elif c == 1:
        for i in mine:
            p = dict(base)
            p.update(settings[i])
            k, nz = set_params(kernel, p)
            try:
                gp = E.fit(k, x, y, nz, jitter=jitter, device=device)
            except np.linalg.LinAlgError:
                vals[i] = -np.inf
                continue
            if eval_gradient:
                vals[i], grads[i] = E.log_marginal_likelihood(gp, eval_gradient=True)
            else:
                vals[i] = E.log_marginal_likelihood(gp)
            del gp
    else:
        dev = E._require_device(device)
        main = torch.cuda.current_stream(dev)
        streams = [E.side_stream(dev) for _ in range(c)]
        inflight = collections.deque()

        def drain(limit):
            while len(inflight) > limit:
                i, gp, out, g, ev = inflight.popleft()
                ev.synchronize()
                try:
                    gp.check()
                except np.linalg.LinAlgError:
                    vals[i] = -np.inf
                    continue
                vals[i] = float(out.item())
                if g is not None:
                    grads[i] = g.cpu().numpy()

        prev_sets = E.N.lib().gp2d_factor_sets(c)   # one internal factor stream set per stream
        try:
            _sweep_concurrent(kernel, x, y, settings, base, mine, jitter, dev, eval_gradient, streams, main,
                              inflight, drain)
            drain(0)
        finally:   # any exception (GP2DError, KeyboardInterrupt, ...) restores the process-wide setting
            E.N.lib().gp2d_factor_sets(prev_sets)
    if ws > 1:
        vals, grads = allreduce_disjoint(vals, grads, device)
    return vals, (grads if eval_gradient else None)


BATCH_MAX = 16              # config E (64 settings, N_train = 4096): 8 / 12 / 16 / 32 / 64 per batch
BATCH_MAX_BYTES = 32 << 30   # 90.1 / 90.8 / 92.3 / 93.0 / 92.7 settings/s (profiles/r04_ebatch_ab.jsonl);
                             # factor + TRTRI workspace of one batch


def auto_batch(kernel: E.KernelSpec, x, n_settings: int, concurrent=None) -> int:
    """hyper.sweep's default batch: up to BATCH_MAX settings per batched factorisation when the
    caller did not ask for concurrent streams, there are at least two settings and the batch's
    matrices (n² doubles each, plus the TRTRI's quarter-size workspace) fit BATCH_MAX_BYTES."""
    if concurrent is not None or n_settings < 2:
        return 1
    npad, n = E.fit_layout(kernel, E._point_count(x, kernel.input_dim))
    return max(1, min(BATCH_MAX, n_settings, BATCH_MAX_BYTES // E.fit_problem_bytes(n)))


def _sweep_batched(kernel, x, y, settings, base, mine, jitter, device, eval_gradient, bsz, vals, grads):
    dev = E._require_device(device)
    for g0 in range(0, len(mine), bsz):
        group = mine[g0:g0 + bsz]
        problems = []
        for i in group:
            p = dict(base)
            p.update(settings[i])
            k, nz = set_params(kernel, p)
            problems.append((k, x, y, nz))
        # joined on the host (the chain runs with no wait pending on this stream, cf. fit(join))
        fits = E.fit_batch(problems, jitter=jitter, device=dev, check=False, join=True)
        outs = [E.lml_device(gp, eval_gradient) for gp in fits]
        for i, gp, (out, g) in zip(group, fits, outs):
            try:
                gp.check()
            except np.linalg.LinAlgError:
                vals[i] = -np.inf
                continue
            vals[i] = float(out.item())
            if g is not None:
                grads[i] = g.cpu().numpy()
        del fits, outs


def auto_concurrent(n_settings: int, eval_gradient: bool) -> int:
    """hyper.sweep's default stream count: two streams overlap setting i's K_y⁻¹ + gradient
    contractions (≈ 3.4 ms at N = 4096) with setting i+1's fit chain (config E: 60.6–61.2 vs
    58.3–59.9 settings/s, profiles/r03_ring_depth_E_B_ab.txt); the LML alone (0.045 ms) has
    nothing to overlap, and a single setting has no next one."""
    return 2 if (eval_gradient and n_settings >= 2) else 1


def _sweep_concurrent(kernel, x, y, settings, base, mine, jitter, dev, eval_gradient, streams, main, inflight,
                      drain):
    c = len(streams)
    for j, i in enumerate(mine):
        p = dict(base)
        p.update(settings[i])
        k, nz = set_params(kernel, p)
        st = streams[j % c]
        st.wait_stream(main)
        with torch.cuda.stream(st):
            # joined on the host: the chain never runs with this stream's wait pending
            # beside it (≈ 40 % slower); what overlaps is the previous
            # setting's LML + gradient under this setting's chain
            gp = E.fit(k, x, y, nz, jitter=jitter, device=dev, check=False, join=True)
            out, g = E.lml_device(gp, eval_gradient)
            ev = torch.cuda.Event()
            ev.record(st)
        inflight.append((i, gp, out, g, ev))
        drain(2 * c)


def allreduce_disjoint(vals: np.ndarray, grads: np.ndarray, device=None):
    """Combine per-rank results whose non-zero entries are disjoint (sum of x and exact zeros:
    bit-exact).  -inf entries travel as a separate mask."""
    bad = np.isneginf(vals)
    v = np.where(bad, 0.0, vals)
    if torch.cuda.is_available() and dist.get_backend() == "nccl":   # RCCL reduces device tensors only
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    else:
        dev = "cpu"
    buf = torch.as_tensor(np.concatenate([v, bad.astype(np.float64), grads.reshape(-1)]), device=dev)
    C.all_reduce(buf, "sum")
    out = buf.cpu().numpy()
    S = vals.size
    v, bad = out[:S], out[S:2 * S] > 0
    return np.where(bad, -np.inf, v), out[2 * S:].reshape(grads.shape)
