"""Device-resident GP engine: fit (assemble → POTRF → TRTRI → α) and predict.

Host orchestration over the C ABI of libgp2d.so.  torch-ROCm tensors are used
only as device-memory containers and for the current HIP stream; every FLOP runs
in the hand-written HIP kernels.

Reference call sites replaced:
  * GP_laser.laser  GP_laser.py:113-140  (K, +noise·I, inv, Ks, mean, var)
  * GPy GPRegression fit / model.predict  krig.py:411, :543-544
  * sklearn GaussianProcessRegressor fit / predict(return_std)  krig.py:182-194
"""
from __future__ import annotations

import collections
import os
import ctypes
import itertools
import math
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _native as N

NB = 128


def _stream_handle(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


def _require_device(device=None) -> torch.device:
    if not torch.cuda.is_available():
        raise N.NativeLibraryError("gp2d needs a HIP device (torch.cuda.is_available() is False); "
                                   "there is no CPU fallback")
    N.lib()
    dev = torch.device(device if device is not None else "cuda")
    warm_streams(dev)
    return dev


_WARM = set()


def warm_streams(device=None):
    """Bind the current (predict) stream and then the library's internal factorisation streams
    to their hardware queues, once per device (gp2d_factor_warm).  HIP binds a stream to a queue
    at its first command; a job stream ran 53.1–53.9 ms per headline job with the predict stream,
    the factor streams and the side streams first used in that order, and 56.4–56.7 ms in the
    other orders measured (tools/probe_first_fit.py, DESIGN.md §6 "bench state").  Every device
    entry point of the engine calls it (through _require_device) before it touches a stream of
    its own; a caller that uses its own side streams before any gp2d call should call it first."""
    dev = torch.device(device if device is not None else "cuda")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx in _WARM:
        return
    with torch.cuda.device(idx):
        N.check(N.lib().gp2d_factor_warm(1, ctypes.c_void_p(torch.cuda.current_stream(idx).cuda_stream)),
                "gp2d_factor_warm")
    _WARM.add(idx)


def morton_sort(P: torch.Tensor):
    """(order, P[order]) for device points (N, d), d ∈ {2, 3}: the Z-order (Morton) curve of
    their bounding box (21 bits per coordinate), sorted by a stable device radix sort and
    gathered on the device (gp2d_morton_sort; equal codes keep their input order, so the
    permutation is deterministic).  The ozaki engine orders training and grid points this way so
    that 64 consecutive training points and 256 consecutive grid points are spatially compact:
    K* tiles of far-apart groups are then exactly zero and the int8 GEMMs skip them
    (csrc/ozaki.hpp, ozaki_slab_list_kernel).  Other shapes: (None, P) — no reordering."""
    n, d = P.shape
    if n < 1 or d not in (2, 3):
        return None, P
    P = P.contiguous()
    L = N.lib()
    wb = int(L.gp2d_morton_sort_workspace(n))
    work = torch.empty(wb, dtype=torch.uint8, device=P.device)
    order = torch.empty(n, dtype=torch.int64, device=P.device)
    out = torch.empty_like(P)
    N.check(L.gp2d_morton_sort(_ptr(P), n, d, _ptr(out), _ptr(order), _ptr(work), wb, _stream_handle(P.device)),
            "gp2d_morton_sort")
    return order, out


def morton_order(P: torch.Tensor) -> torch.Tensor:
    """The permutation of morton_sort (sorted point j is P[order[j]])."""
    order, _ = morton_sort(P)
    if order is None:
        raise ValueError("morton_order: points must be (N, 2) or (N, 3) with N ≥ 1")
    return order


def side_stream(device=None) -> torch.cuda.Stream:
    """A stream for work that has to overlap the current (predict) stream — a job's fit, a
    broadcast, concurrent settings.  Taken from torch's HIGH-priority pool: HIP maps streams
    onto at most GPU_MAX_HW_QUEUES hardware queues per priority level (4 on the box), and two
    streams that share a queue run in order, so a side stream on the current stream's queue
    overlaps nothing.  torch's normal-priority pool streams can land there (tools/probe_queues.py (git f1195df):
    pool streams 6 and 10 of 12 did, profiles/r03_queue_aliasing.json); the high-priority pool is
    a different set of queues."""
    return torch.cuda.Stream(device, priority=-1)


class MaskedStream:
    """A HIP stream restricted to the CUs of mask bits [first, first + count)
    (gp2d_stream_create_cumask; bit i lies in XCD i mod 8), usable as a torch stream
    (`.stream`, a torch.cuda.ExternalStream); destroyed with the object."""

    def __init__(self, first: int, count: int, device=None):
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            N.check(N.lib().gp2d_stream_create_cumask(int(first), int(count), ctypes.byref(h)),
                    "gp2d_stream_create_cumask")
        self.handle = h
        self.stream = torch.cuda.ExternalStream(h.value, device=dev)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                torch.cuda.synchronize(self.stream.device)
                N.lib().gp2d_stream_destroy(h)
            except Exception:   # noqa: BLE001 — interpreter shutdown
                pass
            self.handle = None


def _as_points(x, dim: int, device) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        t = x.to(device=device, dtype=torch.float64)
    else:
        t = torch.as_tensor(np.ascontiguousarray(np.asarray(x, dtype=np.float64)), device=device)
    return t.reshape(-1, dim).contiguous()


@dataclass
class KernelSpec:
    """Hyperparameters of the covariance function.

    family 'vector2d' (the reference's div-free / curl-free SE kernels):
        kind 'df' | 'cf' | 'mixed' | 'scalar' (divFree 1 | 2 | mixed | 0),
        l_df, l_cf, ratio  (myKernel.py:13-22; GP_laser.py:16 `l_df, l_cf, rate`)
    family 'ard' (the sklearn model of krig.scikit_prior, krig.py:174-180):
        variances (1-2 terms), lengthscales (per term, 1-3 dims)
    family 'vector_st' (SURVEY.md §8f item 2): the spatio-temporal product
        Kt(var_t, l_t) × (the vector2d kernel of `kind`) on (T, Y, X) points — GPy
        `Kt(...) * nonDivK(2, [1, 2], ℓ)` (scratch.py:506-508; Kt myKernel.py:337-363),
        standing in for the reference's missing myKernel2 (krig.py:397-404)
    """
    family: str = "vector2d"
    kind: str = "df"
    l_df: float = 5.0
    l_cf: float = 5.0
    ratio: float = 1.0
    variances: tuple = ()
    lengthscales: tuple = ()
    var_t: float = 1.0
    l_t: float = 1.0

    _KINDS = {"scalar": N.KIND_SCALAR, "df": N.KIND_DIVFREE, "cf": N.KIND_CURLFREE, "mixed": N.KIND_MIXED,
              0: N.KIND_SCALAR, 1: N.KIND_DIVFREE, 2: N.KIND_CURLFREE, 3: N.KIND_MIXED}

    def desc(self) -> N.KernelDesc:
        if self.family == "vector2d":
            return N.vector_kernel_desc(self._KINDS[self.kind], self.l_df, self.l_cf, self.ratio)
        if self.family == "ard":
            return N.ard_kernel_desc(self.variances, self.lengthscales)
        if self.family == "vector_st":
            return N.vector_st_kernel_desc(self._KINDS[self.kind], self.l_df, self.l_cf, self.ratio, self.var_t,
                                           self.l_t)
        raise ValueError(f"unknown kernel family {self.family!r}")

    @property
    def is_vector(self) -> bool:
        return self.family in ("vector2d", "vector_st")

    @property
    def block_dim(self) -> int:
        return 2 if self.is_vector else 1

    @property
    def input_dim(self) -> int:
        if self.family == "vector2d":
            return 2
        return 3 if self.family == "vector_st" else len(self.lengthscales[0])

    def kdiag(self) -> float:
        return float(N.lib().gp2d_kernel_diag(ctypes.byref(self.desc())))


def padded_points(n: int) -> int:
    return int(N.lib().gp2d_padded_points(int(n)))


def assemble(kernel: KernelSpec, xa, xb=None, diag_add: float = 0.0, device=None) -> torch.Tensor:
    """Covariance matrix K(xa, xb) on the device, exactly as the reference lays it out
    ((bd·Na) × (bd·Nb) component-major; no padding in the returned tensor)."""
    dev = _require_device(device)
    d = kernel.input_dim
    bd = kernel.block_dim
    A = _as_points(xa, d, dev)
    sym = xb is None
    B = A if sym else _as_points(xb, d, dev)
    na, nb = A.shape[0], B.shape[0]
    nap, nbp = padded_points(na), padded_points(nb)
    out = torch.empty((bd * nap, bd * nbp), dtype=torch.float64, device=dev)
    desc = kernel.desc()
    N.check(N.lib().gp2d_assemble(_ptr(A), na, nap, _ptr(B), nb, nbp, ctypes.byref(desc), float(diag_add),
                                  int(sym), _ptr(out), out.shape[1], _stream_handle(dev)), "gp2d_assemble")
    if bd == 1:
        return out[:na, :nb]
    idx_r = torch.cat([torch.arange(na, device=dev), nap + torch.arange(na, device=dev)])
    idx_c = torch.cat([torch.arange(nb, device=dev), nbp + torch.arange(nb, device=dev)])
    return out.index_select(0, idx_r).index_select(1, idx_c)


@dataclass
class GPFit:
    """A fitted GP resident in HBM: W = L⁻¹ (n×n), α = K_y⁻¹y, training points."""
    kernel: KernelSpec
    noise: float
    x: torch.Tensor          # (N, dim) device
    n_train: int
    n_pad: int               # padded point count
    W: torch.Tensor          # (n, n) lower-triangular inverse Cholesky factor
    alpha: torch.Tensor      # (n,)
    device: torch.device
    info: int = 0
    extra: dict = field(default_factory=dict)
    y: torch.Tensor = None   # (n,) padded observations (LML)
    perm: torch.Tensor = None  # ozaki engine: x = x_input[perm] (Morton order; α, W follow x)
    pending: tuple = None      # fit(check=False): (pinned status copy, its event, prepare error)
    n_mat: int = 0             # matrix order when W is None (a job stream's receiving rank keeps
    #                            only the INT8 planes, distributed.broadcast_fit)

    def check(self) -> "GPFit":
        """Raise what fit(check=False) deferred: LinAlgError for a non-SPD K_y (waits only
        for the factor's status word, not for later work on the stream), then apply the ozaki
        engine's accuracy guard (apply_guard) with the statistics that travel in the same word.
        Call it before the fit's predict is queued: the guard may re-prepare the planes."""
        if self.pending is not None:
            host, ev, err = self.pending
            self.pending = None
            ev.synchronize()
            inf = int(host.view(torch.int32)[0].item())
            vmin, wmax = float(host[1].item()), float(host[2].item())
            _PINNED_STATUS.append(host)
            _raise_fit_errors(inf, err)
            apply_guard(self, vmin, wmax)
        return self

    def record_stream(self, stream) -> "GPFit":
        """Mark the fit's device tensors as in use on `stream` — for a fit made on one stream
        and predicted on another: the caching allocator then keeps their memory until the
        work queued on `stream` when they are freed has finished."""
        oz = self.extra.get("ozaki", ())
        for t in (self.x, self.W, self.alpha, self.y, self.perm, *oz[:2]):
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(stream)
        return self

    @property
    def n(self) -> int:
        return self.W.shape[0] if self.W is not None else self.n_mat

    def ready_on(self, stream) -> "GPFit":
        """Make `stream` wait for the work the accuracy guard queued in check() (re-prepared
        planes, or W unpacked for the FP64 engine), if any."""
        g = self.extra.get("guard")
        ev = g.pop("event", None) if g else None
        if ev is not None:
            stream.wait_event(ev)
        return self


def _pad_obs(y, n_train: int, n_pad: int, bd: int, device, perm: torch.Tensor | None = None) -> torch.Tensor:
    """The fit's observation vector [u(n_pad), v(n_pad)] with zeros for the padded points, in the
    order of perm (sorted point i is input point perm[i]) — gp2d_obs_pad on the device."""
    if isinstance(y, torch.Tensor):
        yt = y.to(device=device, dtype=torch.float64).reshape(-1)
    else:
        yt = torch.as_tensor(np.asarray(y, dtype=np.float64).reshape(-1), device=device)
    if yt.numel() != bd * n_train:
        raise ValueError(f"observation vector has {yt.numel()} entries, expected {bd * n_train}")
    yt = yt.contiguous()
    out = torch.empty(bd * n_pad, dtype=torch.float64, device=device)
    N.check(N.lib().gp2d_obs_pad(_ptr(yt), n_train, n_pad, bd, None if perm is None else _ptr(perm), _ptr(out),
                                 _stream_handle(device)), "gp2d_obs_pad")
    return out


VARIANCE_ENGINES = ("f64", "ozaki")
ASSEMBLE_LOWER = 2   # gp2d_assemble's symmetric mode: K_y's lower block triangle only

# fit: the two-call gp2d_potrf + gp2d_trtri sequence, or gp2d_potrf_inv (the left half of the
# inverse and the top-level T = L21·W11 issued under the second half of the factorisation).
# Bit-identical results; measured a wash at N = 4096 (the concurrent GEMMs slow the POTRF
# critical path by what they save: 13.5 ms either way), so off by default.
FUSED_INVERSE = False


def fit_layout(kernel: KernelSpec, n_train: int, variance: str = "f64"):
    """(padded point count, matrix order n) of a fit: points padded to 64, n a multiple of
    128 (of 256 for the ozaki engine, whose int8 GEMM tiles are 256 wide)."""
    bd = kernel.block_dim
    npad = padded_points(n_train)
    n = bd * npad
    if n % NB:  # scalar (ARD) family: the matrix order itself must be a multiple of 128
        npad = (npad + NB - 1) // NB * NB
        n = bd * npad
    if variance == "ozaki" and n % 256:
        npad = (npad + 127) // 128 * 128
        n = bd * npad
    return npad, n


# pinned 3-double status slots for fit(check=False) (see status_block), reused after
# GPFit.check(), so the steady state allocates no pinned memory
_PINNED_STATUS: list = []


def status_block(device) -> tuple:
    """A fit's device status word: 3 doubles — [0] holds the LAPACK-style info as an int32 in its
    low bytes (gp2d_potrf writes it there through the returned int32 view), [1:3] the accuracy
    guard's statistics (gp2d_ozaki_guard: min latent variance at the observations, max |W|;
    NaN when the fit ran no guard — apply_guard then keeps the default precision, so a receiving
    rank never acts on stale bytes).  One copy to the host (or one broadcast) carries all of it."""
    st = torch.empty(3, dtype=torch.float64, device=device)
    return st, st.view(torch.int32)[0:1]


def _raise_fit_errors(inf: int, err):
    if inf < 0:   # a status word from the job stream: the fit raised on its owner's host
        if err is not None:
            raise err
        raise RuntimeError("the fit failed on the rank that owned it (see that rank's error)")
    if inf != 0:
        raise np.linalg.LinAlgError(
            f"K_y is not positive definite (leading minor of order {inf}); "
            "increase the noise / jitter (cf. sklearn _gpr.py:350-358)")
    if err is not None:
        raise err


def pending_status(status: torch.Tensor, err=None) -> tuple:
    """A GPFit.pending triple for a device status block (status_block; info < 0: failed on
    another rank): copied to pinned host memory after the work queued so far on the current
    stream, checked by GPFit.check()."""
    host = _PINNED_STATUS.pop() if _PINNED_STATUS else torch.empty(3, dtype=torch.float64, pin_memory=True)
    host.copy_(status, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(status.device))
    return host, ev, err


# The accuracy the guard holds the int8 variance to: north_star's fp64 posterior gate (1e-10
# relative), elementwise.
GUARD_TARGET = 1e-10
OZAKI_DEFAULT_BITS = (49, 45)   # (W, K*) integer bits: csrc/ozaki.hpp OZ_PW, OZ_PB
OZAKI_MAX_BITS = (60, 50)       # OZ_PW_MAX, OZ_PB_MAX
# fit(guard=None) default; GP2D_GUARD=0 turns the guard off (dev A/Bs only, tools/runs)
GUARD_DEFAULT = os.environ.get("GP2D_GUARD", "1") != "0"


def _guard_stats(W: torch.Tensor, n: int, ntr: int, npad: int, diag_add: float, status: torch.Tensor, dev):
    """gp2d_ozaki_guard into status[1:3] (status_block) on the current stream."""
    L = N.lib()
    wb = int(L.gp2d_ozaki_guard_workspace(n))
    work = torch.empty(wb, dtype=torch.uint8, device=dev)
    N.check(L.gp2d_ozaki_guard(_ptr(W), n, W.stride(0), ntr, npad, float(diag_add),
                               ctypes.c_void_p(status.data_ptr() + 8), _ptr(work), wb, _stream_handle(dev)),
            "gp2d_ozaki_guard")


def apply_guard(gp: GPFit, vmin: float, wmax: float) -> GPFit:
    """The ozaki engine's accuracy guard, once the fit's statistics are on the
    host: the variance's elementwise error grows as the posterior variance falls against kss,
    ≈ A·2^(49 − wbits)·X^1.5 + B·2^(45 − kbits)·X with X = kss / v_min (gp2d_ozaki_error_model;
    v_min: the smallest latent posterior variance at the observations, exact from W).  The cheapest
    W / K* precisions (wbits 49..60, kbits 45..50) that keep the model within GUARD_TARGET are
    taken — the planes re-prepared on the fit's stream when that is more than the defaults — or,
    past them, the fit switches to the FP64 engine.  The decision is in gp.extra['guard']:
    engine, wbits, kbits, vmin_over_kss, wmax, est."""
    g = gp.extra.get("guard")
    if not g or not g.get("pending"):
        return gp
    if math.isnan(vmin):   # the owner's fit ran no guard (status_block's sentinel): default precision
        g.pop("stream", None)
        gp.extra.pop("packed", None)
        g.update(pending=False, engine="ozaki", wbits=OZAKI_DEFAULT_BITS[0], kbits=OZAKI_DEFAULT_BITS[1],
                 vmin_over_kss=None, wmax=None, est=None)
        return gp
    L = N.lib()
    kss = gp.kernel.kdiag()
    wb, kb = ctypes.c_int(0), ctypes.c_int(0)
    ok = int(L.gp2d_ozaki_guard_bits(kss, vmin, GUARD_TARGET, ctypes.byref(wb), ctypes.byref(kb)))
    g.update(pending=False, vmin_over_kss=vmin / kss, wmax=wmax)
    stream = g.pop("stream", None) or torch.cuda.current_stream(gp.device)
    packed = gp.extra.pop("packed", None)
    if ok <= 0:   # beyond the emulation's range (or a non-positive v_min): exact FP64 products
        g.update(engine="f64", wbits=None, kbits=None,
                 est=float(L.gp2d_ozaki_error_model(kss, vmin, OZAKI_MAX_BITS[0], OZAKI_MAX_BITS[1])))
        gp.extra.pop("ozaki", None)
        if gp.W is None:   # a receiving rank kept only the packed payload
            with torch.cuda.stream(stream):
                W = torch.zeros((gp.n, gp.n), dtype=torch.float64, device=gp.device)
                N.check(L.gp2d_pack_lower(_ptr(W), gp.n, gp.n, _ptr(packed), 1, _stream_handle(gp.device)),
                        "gp2d_pack_lower")
                g["event"] = torch.cuda.Event()
                g["event"].record(stream)
            gp.W = W
        return gp
    wbits, kbits = wb.value, kb.value
    g.update(engine="ozaki", wbits=wbits, kbits=kbits, est=float(L.gp2d_ozaki_error_model(kss, vmin, wbits, kbits)))
    if (wbits, kbits) != OZAKI_DEFAULT_BITS:
        with torch.cuda.stream(stream):
            ozaki_prepare(gp, diag_add=g["diag_add"], wbits=wbits, kbits=kbits, packed=packed)
            gp.extra.pop("packed", None)
            g["event"] = torch.cuda.Event()
            g["event"].record(stream)
    return gp


def ozaki_prepare_guarded(gp: GPFit, diag_add: float, guard: bool = True) -> GPFit:
    """The ozaki engine's planes for a fit whose W is already final (a loaded checkpoint, the
    distributed factor): the accuracy guard's statistics read synchronously, then the planes at
    the guard's precision (or none: the FP64 engine) — apply_guard without the deferred path."""
    if not guard:
        return ozaki_prepare(gp, diag_add=float(diag_add))
    status, _ = status_block(gp.device)
    _guard_stats(gp.W, gp.n, gp.n_train, gp.n_pad, diag_add, status, gp.device)
    host = status.cpu()
    gp.extra["guard"] = dict(pending=True, diag_add=float(diag_add), stream=torch.cuda.current_stream(gp.device))
    apply_guard(gp, float(host[1]), float(host[2]))
    if "ozaki" not in gp.extra and gp.extra["guard"]["engine"] == "ozaki":
        ozaki_prepare(gp, diag_add=float(diag_add))
    return gp.ready_on(torch.cuda.current_stream(gp.device))


def fit(kernel: KernelSpec, x, y, noise: float, jitter: float = 0.0, device=None, variance: str = "f64",
        check: bool = True, jitchol: int = 0, join: bool | None = None, guard: bool | None = None) -> GPFit:
    """K_y = K(x,x) + (noise+jitter)·I → L = chol(K_y) → W = L⁻¹ → α = Wᵀ W y.

    jitchol = k > 0: GPy's jitchol retry (GPy.util.linalg.jitchol, maxtries = k; GPy is not
    installed here, so this follows its published algorithm and is parity-unpinned): if K_y is
    not positive definite, refit with an extra diagonal jitter of mean(diag K_y)·1e-6, ten times
    larger on each further try, up to k tries, then raise LinAlgError.  The jitter that succeeded
    is gp.extra['jitchol'] (0.0 when the first factorisation did).  Implies check=True.

    variance: 'f64'   — predictive variance by the FP64-MFMA contraction;
              'ozaki' — the same contraction emulated exactly on the INT8 matrix cores
                        (Ozaki scheme II, csrc/ozaki.hpp); vector2d family only.
    guard (ozaki): hold the emulated variance to GUARD_TARGET whatever the hyperparameters
    (apply_guard: more W bits, or the FP64 engine); False keeps the default 49 bits.
    Raises numpy.linalg.LinAlgError if K_y is not positive definite (the
    reference's np.linalg.inv / GPy jitchol / sklearn error paths).  check=False returns
    without waiting for the factor (no host sync); the error is raised by GPFit.check().

    join (default: = check): the host waits for the factorisation's chain before it enqueues
    the rest of the fit (gp2d_factor_join), so the current stream holds no wait pending beside
    the chain — a pending wait on some of torch's streams slows the chain by up to 40 %
    (DESIGN.md §6).  It costs nothing when the caller blocks on the result anyway; join=False
    keeps a check=False fit fully asynchronous, join=True blocks one that has nothing to
    overlap (a job stream's first fit).
    """
    if jitchol:
        try:
            gp = fit(kernel, x, y, noise, jitter=jitter, device=device, variance=variance)
            gp.extra["jitchol"] = 0.0
            return gp
        except np.linalg.LinAlgError:
            diag = float(N.lib().gp2d_kernel_diag(ctypes.byref(kernel.desc()))) + noise + jitter
            if not diag > 0.0:
                raise np.linalg.LinAlgError("not pd: non-positive diagonal elements") from None
            jit = diag * 1e-6
            for _ in range(int(jitchol)):
                if not np.isfinite(jit):
                    break
                try:
                    gp = fit(kernel, x, y, noise, jitter=jitter + jit, device=device, variance=variance)
                    gp.extra["jitchol"] = jit
                    return gp
                except np.linalg.LinAlgError:
                    jit *= 10.0
            raise np.linalg.LinAlgError("not positive definite, even with jitter.") from None
    if variance not in VARIANCE_ENGINES:
        raise ValueError(f"variance must be one of {VARIANCE_ENGINES}")
    if variance == "ozaki" and not kernel.is_vector:
        raise ValueError("the ozaki variance engine supports the vector families only")
    dev = _require_device(device)
    L = N.lib()
    d, bd = kernel.input_dim, kernel.block_dim
    X = _as_points(x, d, dev)
    ntr = X.shape[0]
    if ntr < 1:
        raise ValueError("need at least one training point")
    npad, n = fit_layout(kernel, ntr, variance)
    if variance == "ozaki" and n >= 131072:
        # the int8 GEMM epilogue's biased sums stay below 2^32 only for K = n < 2^17
        raise ValueError(f"the ozaki variance engine supports n < 131072 (N_train < 65536); got n = {n}: "
                         "use variance='f64'")
    perm = None
    if variance == "ozaki" and ntr > 1:   # Morton order: exact-zero K* slabs cluster (skipped)
        perm, X = morton_sort(X)
    s = _stream_handle(dev)
    desc = kernel.desc()
    A = torch.empty((n, n), dtype=torch.float64, device=dev)
    # the vector families: K_y's lower block triangle only (symmetric = 2), all gp2d_potrf reads
    N.check(L.gp2d_assemble(_ptr(X), ntr, npad, _ptr(X), ntr, npad, ctypes.byref(desc), float(noise + jitter),
                            ASSEMBLE_LOWER if kernel.is_vector else 1, _ptr(A), n, s), "gp2d_assemble")
    dinv = torch.empty((n // NB, NB, NB), dtype=torch.float64, device=dev)
    status, info = status_block(dev)   # gp2d_potrf resets info
    prev_join = L.gp2d_factor_join(1 if (check if join is None else join) else 0)
    try:
        if FUSED_INVERSE:   # factor and inverse in one call, the TRTRI GEMMs overlapped with POTRF
            wbytes = int(L.gp2d_potrf_inv_workspace(n))
            work = torch.empty(wbytes // 8 + 1, dtype=torch.float64, device=dev)
            N.check(L.gp2d_potrf_inv(_ptr(A), n, n, _ptr(dinv), _ptr(info), _ptr(work), wbytes, s),
                    "gp2d_potrf_inv")
        else:
            N.check(L.gp2d_potrf(_ptr(A), n, n, _ptr(dinv), _ptr(info), None, 0, s), "gp2d_potrf")
    finally:
        L.gp2d_factor_join(prev_join)
    if not FUSED_INVERSE:
        wbytes = int(L.gp2d_trtri_workspace(n))
        work = torch.empty(wbytes // 8 + 1, dtype=torch.float64, device=dev)
        N.check(L.gp2d_trtri(_ptr(A), n, n, _ptr(dinv), _ptr(work), wbytes, s), "gp2d_trtri")
    del work, dinv
    guard = (GUARD_DEFAULT if guard is None else guard) and variance == "ozaki"
    if guard:   # the guard's statistics from W, into the status word beside info
        _guard_stats(A, n, ntr, npad, noise + jitter, status, dev)
    else:       # "no guard ran": a receiving rank of the job stream keeps the default precision
        status[1:].fill_(float("nan"))
    pend = None
    if not check:
        # α (and the ozaki preparation) are enqueued before the status is read (one host sync per
        # fit); a failed factor raises in GPFit.check(), which also applies the guard
        pend = pending_status(status)
    Y = _pad_obs(y, ntr, npad, bd, dev, perm)
    alpha = torch.empty(n, dtype=torch.float64, device=dev)
    pbytes = int(L.gp2d_potrs_workspace(n))
    pwork = torch.empty(pbytes // 8 + 1, dtype=torch.float64, device=dev)
    N.check(L.gp2d_potrs_inv(_ptr(A), n, n, _ptr(Y), _ptr(alpha), _ptr(pwork), pbytes, s), "gp2d_potrs_inv")
    gp = GPFit(kernel=kernel, noise=float(noise), x=X, n_train=ntr, n_pad=npad, W=A, alpha=alpha, device=dev,
               y=Y, perm=perm)
    gp.extra["status_dev"] = status   # info + guard statistics on the device (the job stream broadcasts it)
    del pwork
    err = None
    if variance == "ozaki":
        # enqueued before the status is read, with the a-priori moduli count at the default
        # precision: the fit's only host round trip is the status read below
        if guard:
            gp.extra["guard"] = dict(pending=True, diag_add=float(noise + jitter),
                                     stream=torch.cuda.current_stream(dev))
        try:
            ozaki_prepare(gp, diag_add=float(noise + jitter))
        except N.GP2DError as e:   # a failed factor (NaN rows) makes prepare fail too: info decides
            err = e
    if not check:
        gp.pending = (pend[0], pend[1], err)
        return gp
    host = status.cpu()
    _raise_fit_errors(int(host.view(torch.int32)[0].item()), err)
    apply_guard(gp, float(host[1]), float(host[2]))
    return gp


def fit_batch(problems, variance: str = "f64", jitter: float = 0.0, device=None, check: bool = True,
              join: bool | None = None, guard: bool | None = None) -> list:
    """Fit several GPs of one size together: `problems` is a sequence of (kernel, x, y, noise)
    whose matrices K_y share the order n (a hyperparameter sweep's settings over one training
    set, or a job stream's next jobs with equal point counts).  Their K_y are factored and
    inverted in ONE chain (gp2d_potrf_batched + gp2d_trtri_batched: every launch carries every
    problem), so the latency-bound diagonal chain of a fit is paid once per
    batch instead of once per fit; each problem's W, α (and INT8 residue planes) are those of
    engine.fit on it alone, bit for bit.  Returns one GPFit per problem (W views into one
    (B, n, n) tensor).  check=True raises LinAlgError for the first non-PD problem (the index
    is in the message); check=False defers it to each GPFit.check().  join, guard as in fit()."""
    if variance not in VARIANCE_ENGINES:
        raise ValueError(f"variance must be one of {VARIANCE_ENGINES}")
    probs = list(problems)
    if not probs:
        return []
    if len(probs) > 64:
        raise ValueError("fit_batch: at most 64 problems per batch")
    dev = _require_device(device)
    L = N.lib()
    s = _stream_handle(dev)
    prep = []
    for kernel, x, y, noise in probs:
        if variance == "ozaki" and not kernel.is_vector:
            raise ValueError("the ozaki variance engine supports the vector families only")
        X = _as_points(x, kernel.input_dim, dev)
        ntr = X.shape[0]
        if ntr < 1:
            raise ValueError("need at least one training point")
        ny = y.numel() if isinstance(y, torch.Tensor) else np.asarray(y).size
        if ny != kernel.block_dim * ntr:   # every problem's shape is checked before any GPU work
            raise ValueError(f"problem {len(prep)}: observation vector has {ny} entries, "
                             f"expected {kernel.block_dim * ntr}")
        npad, n = fit_layout(kernel, ntr, variance)
        perm = None
        if variance == "ozaki" and ntr > 1:
            perm, X = morton_sort(X)
        prep.append((kernel, X, y, float(noise), ntr, npad, n, perm))
    n = prep[0][6]
    if any(p[6] != n for p in prep):
        raise ValueError("fit_batch: every problem must have the same matrix order n")
    if variance == "ozaki" and n >= 131072:
        raise ValueError("the ozaki variance engine supports n < 131072")
    B = len(prep)
    A = torch.empty((B, n, n), dtype=torch.float64, device=dev)
    for b, (kernel, X, _, noise, ntr, npad, _, _) in enumerate(prep):
        N.check(L.gp2d_assemble(_ptr(X), ntr, npad, _ptr(X), ntr, npad, ctypes.byref(kernel.desc()),
                                float(noise + jitter), ASSEMBLE_LOWER if kernel.is_vector else 1, _ptr(A[b]), n, s),
                "gp2d_assemble")
    dinv = torch.empty((B, n // NB, NB, NB), dtype=torch.float64, device=dev)
    info = torch.empty(B, dtype=torch.int32, device=dev)   # gp2d_potrf_batched resets them
    prev_join = L.gp2d_factor_join(1 if (check if join is None else join) else 0)
    try:
        N.check(L.gp2d_potrf_batched(_ptr(A), n, n, n * n, B, _ptr(dinv), _ptr(info), s), "gp2d_potrf_batched")
    finally:
        L.gp2d_factor_join(prev_join)
    wbytes = int(L.gp2d_trtri_batched_workspace(n, B))
    work = torch.empty(wbytes // 8 + 1, dtype=torch.float64, device=dev)
    N.check(L.gp2d_trtri_batched(_ptr(A), n, n, n * n, B, _ptr(dinv), _ptr(work), wbytes, s), "gp2d_trtri_batched")
    del work, dinv
    pbytes = int(L.gp2d_potrs_workspace(n))
    pwork = torch.empty(pbytes // 8 + 1, dtype=torch.float64, device=dev)
    guard = (GUARD_DEFAULT if guard is None else guard) and variance == "ozaki"
    statuses = torch.empty((B, 3), dtype=torch.float64, device=dev)   # status_block per problem
    fits, errs = [], []
    for b, (kernel, X, y, noise, ntr, npad, _, perm) in enumerate(prep):
        statuses[b].view(torch.int32)[0:1].copy_(info[b:b + 1])        # a 4-byte device copy
        if guard:
            _guard_stats(A[b], n, ntr, npad, noise + jitter, statuses[b], dev)
        else:
            statuses[b, 1:].fill_(float("nan"))
        bd = kernel.block_dim
        Y = _pad_obs(y, ntr, npad, bd, dev, perm)
        alpha = torch.empty(n, dtype=torch.float64, device=dev)
        W = A[b]
        N.check(L.gp2d_potrs_inv(_ptr(W), n, n, _ptr(Y), _ptr(alpha), _ptr(pwork), pbytes, s), "gp2d_potrs_inv")
        gp = GPFit(kernel=kernel, noise=noise, x=X, n_train=ntr, n_pad=npad, W=W, alpha=alpha, device=dev, y=Y,
                   perm=perm)
        gp.extra["status_dev"] = statuses[b]
        err = None
        if variance == "ozaki":
            if guard:
                gp.extra["guard"] = dict(pending=True, diag_add=float(noise + jitter),
                                         stream=torch.cuda.current_stream(dev))
            try:
                ozaki_prepare(gp, diag_add=float(noise + jitter))
            except N.GP2DError as e:
                err = e
        if not check:
            gp.pending = pending_status(statuses[b], err)
        fits.append(gp)
        errs.append(err)
    del pwork
    if check:
        host = statuses.cpu()
        for b, err in enumerate(errs):
            try:
                _raise_fit_errors(int(host[b].view(torch.int32)[0].item()), err)
            except np.linalg.LinAlgError as e:
                raise np.linalg.LinAlgError(f"problem {b}: {e}") from None
        for b, gp in enumerate(fits):
            apply_guard(gp, float(host[b, 1]), float(host[b, 2]))
    return fits


def ozaki_prepare(gp: GPFit, diag_add: float | None = None, packed: torch.Tensor | None = None,
                  wbits: int = 0, kbits: int = 0) -> GPFit:
    """Residue planes of W for the INT8 variance engine (once per fit).  With `diag_add`
    (the noise + jitter of K_y's diagonal) the moduli count is the a-priori bound and nothing
    synchronises (gp2d_ozaki_prepare_async); without it, the data-driven count of the
    factor's row bounds (one device → host read).  packed: W as the factor broadcast's packed
    lower block triangle (gp2d_ozaki_prepare_packed, needs diag_add) — gp.W may then be None.
    wbits / kbits: integer bits per W row and of K* (0 = the defaults 49 / 45; the accuracy guard's
    choice, apply_guard).  gp.extra['ozaki'] = (residue planes, row scales, moduli count, kbits)."""
    L = N.lib()
    n = gp.n
    desc = gp.kernel.desc()
    # the planes this fit will use: the a-priori count is known before the call (the async and
    # packed preparations use exactly it); the data-driven one only after (the worst case)
    nm = int(L.gp2d_ozaki_nmod_apriori(n, ctypes.byref(desc), float(diag_add), int(wbits), int(kbits))) \
        if diag_add is not None else 0
    wbytes = nm * n * n if nm > 0 else int(L.gp2d_ozaki_wres_bytes(n))
    wres = torch.empty(wbytes, dtype=torch.int8, device=gp.device)
    rowscale = torch.empty(n, dtype=torch.float64, device=gp.device)
    nmod = ctypes.c_int(0)
    if packed is not None:
        if diag_add is None:
            raise ValueError("ozaki_prepare from the packed factor needs diag_add (the a-priori moduli count)")
        N.check(L.gp2d_ozaki_prepare_packed(_ptr(packed), n, ctypes.byref(desc), float(diag_add), int(wbits),
                                            int(kbits), _ptr(wres), _ptr(rowscale), ctypes.byref(nmod),
                                            _stream_handle(gp.device)), "gp2d_ozaki_prepare_packed")
    elif diag_add is not None:
        N.check(L.gp2d_ozaki_prepare_async(_ptr(gp.W), n, n, ctypes.byref(desc), float(diag_add), int(wbits),
                                           int(kbits), _ptr(wres), _ptr(rowscale), ctypes.byref(nmod),
                                           _stream_handle(gp.device)), "gp2d_ozaki_prepare_async")
    else:
        N.check(L.gp2d_ozaki_prepare(_ptr(gp.W), n, n, ctypes.byref(desc), int(wbits), int(kbits), _ptr(wres),
                                     _ptr(rowscale),
                                     ctypes.byref(nmod), _stream_handle(gp.device)), "gp2d_ozaki_prepare")
    gp.extra["ozaki"] = (wres, rowscale, int(nmod.value), int(kbits))
    if packed is not None:
        gp.extra["packed"] = packed   # kept until the guard has decided (it may need more bits, or W)
    return gp


@dataclass
class KstarPlanes:
    """INT8 residue planes of K*ᵀ for a whole grid (every chunk), generated ahead of the fit:
    they depend on the training points, the grid and the kernel only (not on α), so they can
    run on a side stream while the fit runs (gp2d_ozaki_kstar)."""
    kernel: KernelSpec
    x: torch.Tensor
    m: int
    n: int
    n_pad: int
    chunk: int
    nmod: int
    bres: torch.Tensor
    event: torch.cuda.Event
    xg: torch.Tensor = None     # the grid in plane order (Morton)
    order: torch.Tensor = None  # plane row j ↔ input grid point order[j]


def kstar_planes(kernel: KernelSpec, x, xg, noise: float, jitter: float = 0.0, chunk: int = 8192, stream=None,
                 out: KstarPlanes | None = None, device=None) -> KstarPlanes:
    """Launch the K* residue planes of grid `xg` against training points `x` on `stream`
    (default: the current stream) after the current stream's pending work; returns at once.
    The moduli count is gp2d_ozaki_nmod_apriori's bound for K_y,ii = kdiag + noise + jitter,
    which covers any fit of these hyperparameters.  `out` reuses a previous buffer."""
    if not kernel.is_vector:
        raise ValueError("K* planes are an ozaki-engine feature (vector families)")
    dev = _require_device(device)
    L = N.lib()
    d = kernel.input_dim
    X = _as_points(x, d, dev)
    if X.shape[0] > 1:
        X = morton_sort(X)[1]                     # the order fit() gives the training points
    order, G = morton_sort(_as_points(xg, d, dev))
    ntr, m = X.shape[0], G.shape[0]
    npad, n = fit_layout(kernel, ntr, "ozaki")
    chunk = max(128, (int(chunk) + 127) // 128 * 128)
    desc = kernel.desc()
    nmod = int(L.gp2d_ozaki_nmod_apriori(n, ctypes.byref(desc), float(noise + jitter), 0, 0))
    if nmod <= 0:
        N.check(-1, "gp2d_ozaki_nmod_apriori")
    nbytes = int(L.gp2d_ozaki_kstar_bytes(n, m, chunk, nmod))
    bres = out.bres if (out is not None and out.bres.numel() >= nbytes) else \
        torch.empty(max(nbytes, 1), dtype=torch.int8, device=dev)
    main = torch.cuda.current_stream(dev)
    st = stream if stream is not None else main
    if st is not main:
        st.wait_stream(main)   # the points (and a reused buffer's last reader) are ordered before
    N.check(L.gp2d_ozaki_kstar(_ptr(X), ntr, npad, _ptr(G), m, ctypes.byref(desc), nmod, 0, chunk, _ptr(bres),
                               bres.numel(), ctypes.c_void_p(st.cuda_stream)), "gp2d_ozaki_kstar")
    if st is not main:
        # the caching allocator must not hand these blocks to main-stream work (the fit)
        # while the side stream still reads / writes them
        for t in (X, G, bres):
            t.record_stream(st)
    ev = torch.cuda.Event()
    ev.record(st)
    return KstarPlanes(kernel=kernel, x=X, m=m, n=n, n_pad=npad, chunk=chunk, nmod=nmod, bres=bres, event=ev,
                       xg=G, order=order)


def ozaki_executed_fraction(kernel: KernelSpec, x, xg, noise: float, jitter: float = 0.0, chunk: int = 8192,
                            device=None) -> float:
    """Measurement helper (bench.py): the fraction of the dense int8 GEMM work (W lower-
    triangular, every K slab) the zero-slab skipping executes for this training set and grid —
    read from the K* block flags gp2d_ozaki_kstar stores after each chunk's planes, with the
    slab-list rules of ozaki_slab_list_kernel / igemm_nt_mod_kernel."""
    pl = kstar_planes(kernel, x, xg, noise, jitter, chunk, device=device)
    pl.event.synchronize()
    n, ntb, m, ch = pl.n, pl.n_pad // 64, pl.m, pl.chunk
    cpm = (ch + 255) // 256 * 256
    planes = pl.nmod * n * 2 * cpm
    stride = planes + ((cpm // 64) * ntb + 255) // 256 * 256
    nbi = n // 256
    ke_slabs = 4 * np.arange(1, nbi + 1)          # a_lower: row block bi reads slabs < 4(bi+1)
    executed = dense = 0
    for ci, c0 in enumerate(range(0, m, ch)):
        cp = (min(ch, m - c0) + 255) // 256 * 256
        off = ci * stride + planes
        f = pl.bres[off:off + (cp // 64) * ntb].view(torch.uint8).cpu().numpy().reshape(cp // 256, 4, ntb)
        kept = np.concatenate([f.any(1)] * 2, axis=1)            # (grid tile, slab): u then v blocks
        cum = np.cumsum(kept, axis=1)[:, ke_slabs - 1]           # listed slabs below each row block's end
        run = np.where((cum > 0) & (cum < 3), ke_slabs[None, :], cum)   # 1–2 slabs run dense
        executed += 2 * int(run.sum())                           # u rows and v rows of each tile
        dense += 2 * (cp // 256) * int(ke_slabs.sum())
    return executed / dense if dense else 1.0


_VAR_MODES = {"latent": N.VAR_LATENT, "gpy": N.VAR_NOISY, "noisy": N.VAR_NOISY, "sklearn": N.VAR_CLIPPED,
              "clipped": N.VAR_CLIPPED}


class Predictor:
    """Reusable predict workspace for one GPFit (chunked over the grid)."""

    def __init__(self, gp: GPFit, chunk: int = 8192):
        self.gp = gp
        bd = gp.kernel.block_dim
        self.ozaki = "ozaki" in gp.extra
        unit = 128 if (bd == 1 or self.ozaki) else 64
        self.chunk = max(unit, (int(chunk) + unit - 1) // unit * unit)
        self.wnmod = 0   # the moduli count the ozaki workspace is sized for (grows on demand)
        if self.ozaki:
            self._ozaki_workspace(gp.extra["ozaki"][2])
        else:
            self.wbytes = int(N.lib().gp2d_predict_workspace(gp.n, self.chunk, bd))
            self.work = torch.empty(self.wbytes // 8 + 1, dtype=torch.float64, device=gp.device)
        self._grid = None   # (the caller's grid tensor, its version, Morton order, the grid in that order)

    def _ozaki_workspace(self, nmod: int):
        """Size the ozaki workspace for a fit with `nmod` moduli (its layout follows nmod): the
        accuracy guard may give later fits more, and a worst-case buffer would hold 1.5× the bytes
        at n = 32,768 for nothing."""
        if nmod > self.wnmod:
            self.wbytes = int(N.lib().gp2d_predict_ozaki_workspace_nmod(self.gp.n, self.chunk, int(nmod)))
            if self.wbytes <= 0:
                raise N.GP2DError(f"no ozaki workspace for {nmod} moduli at n = {self.gp.n}")
            if self.wnmod:   # a grown workspace: the old one may still be read by queued predicts
                torch.cuda.synchronize(self.gp.device)
            self.work = None
            self.work = torch.empty(self.wbytes // 8 + 1, dtype=torch.float64, device=self.gp.device)
            self.wnmod = int(nmod)

    def _grid_order(self, xg, G: torch.Tensor, reuse: bool):
        """Morton order of the grid and the grid in that order.  reuse=True (a job stream predicting
        one device grid job after job — the reference's per-window krig.predict on one grid): for the
        same tensor, at the same address and unmodified by version-tracked ops since (its version
        counter), the order of the previous call is reused — the tensor is held, so its memory cannot
        be handed to another grid.  Writes that bypass the version counter (DLPack aliases, raw
        data_ptr kernels) are not seen: callers that modify a grid that way must not ask for reuse."""
        c = self._grid
        st = torch.cuda.current_stream(G.device)
        if reuse and isinstance(xg, torch.Tensor) and c is not None and c[0] is xg and c[1] == xg._version \
                and c[5] == xg.data_ptr() and c[3].shape == G.shape and c[4] == st:   # made on this stream
            return c[2], c[3]
        order, Gs = morton_sort(G)
        self._grid = (xg, xg._version, order, Gs, st, xg.data_ptr()) \
            if reuse and isinstance(xg, torch.Tensor) and xg.is_cuda else None
        return order, Gs

    def fits(self, gp: GPFit) -> bool:
        """True if this workspace serves `gp` as is: same matrix order, engine and block size
        (the FP64 workspace and the chunk rounding depend on the block size)."""
        return (self.gp.n == gp.n and self.ozaki == ("ozaki" in gp.extra)
                and self.gp.kernel.block_dim == gp.kernel.block_dim)

    def __call__(self, xg, var_mode: str = "latent", compute_var: bool = True, out=None,
                 planes: KstarPlanes | None = None, reuse_grid: bool = False):
        """planes: K* residue planes of this same grid from kstar_planes() (ozaki engine):
        the variance GEMMs read them and the K* kernel runs mean-only (same results as without).
        reuse_grid: the grid is the one of the previous call, unmodified (_grid_order)."""
        gp = self.gp
        L = N.lib()
        d, bd = gp.kernel.input_dim, gp.kernel.block_dim
        G = _as_points(xg, d, gp.device)
        m = G.shape[0]
        if out is None:
            mean = torch.empty(bd * m, dtype=torch.float64, device=gp.device)
            var = torch.empty(bd * m, dtype=torch.float64, device=gp.device)
        else:
            mean, var = out
        desc = gp.kernel.desc()
        if self.ozaki and "ozaki" in gp.extra:
            wres, rowscale, nmod, kbits = gp.extra["ozaki"]
            self._ozaki_workspace(nmod)
            use_planes = planes is not None and compute_var
            if use_planes and (planes.m != m or planes.n != gp.n or planes.chunk != self.chunk):
                raise ValueError("K* planes were made for another grid, fit layout or chunk size")
            # the variance runs on the grid in Morton order (zero K* tiles cluster and are
            # skipped); every output point is independent of the others, so reordering
            # changes no bits — the epilogue stores each result at its input position
            order, Gs = None, G
            if compute_var and m > 1:
                if use_planes:
                    order, Gs = planes.order, planes.xg
                else:
                    order, Gs = self._grid_order(xg, G, reuse_grid)
            po = None if order is None else _ptr(order)
            rc = -3
            if use_planes:
                s = torch.cuda.current_stream(gp.device)
                s.wait_event(planes.event)
                rc = L.gp2d_predict_ozaki_planes(_ptr(wres), _ptr(rowscale), nmod, kbits, gp.n, _ptr(gp.alpha),
                                                 _ptr(gp.x), gp.n_train, gp.n_pad, _ptr(Gs), m, ctypes.byref(desc),
                                                 _VAR_MODES[var_mode], float(gp.noise), _ptr(planes.bres),
                                                 planes.nmod, 0, _ptr(mean), _ptr(var), po, self.chunk, _ptr(self.work),
                                                 self.wbytes, ctypes.c_void_p(s.cuda_stream))
                if rc != -3:   # −3: the fit needs more moduli than the planes carry → inline K*
                    N.check(rc, "gp2d_predict_ozaki_planes")
            if rc == -3:
                N.check(L.gp2d_predict_ozaki(_ptr(wres), _ptr(rowscale), nmod, kbits, gp.n, _ptr(gp.alpha), _ptr(gp.x),
                                             gp.n_train, gp.n_pad, _ptr(Gs), m, ctypes.byref(desc),
                                             _VAR_MODES[var_mode], float(gp.noise), int(bool(compute_var)),
                                             _ptr(mean), _ptr(var), po, self.chunk, _ptr(self.work), self.wbytes,
                                             _stream_handle(gp.device)), "gp2d_predict_ozaki")
            return mean, (var if compute_var else None)
        N.check(L.gp2d_predict(_ptr(gp.W), gp.n, gp.n, _ptr(gp.alpha), _ptr(gp.x), gp.n_train, gp.n_pad,
                               _ptr(G), m, ctypes.byref(desc), _VAR_MODES[var_mode], float(gp.noise),
                               int(bool(compute_var)), _ptr(mean), _ptr(var), self.chunk, _ptr(self.work),
                               self.wbytes, _stream_handle(gp.device)), "gp2d_predict")
        return mean, (var if compute_var else None)


def predict(gp: GPFit, xg, var_mode: str = "latent", compute_var: bool = True, chunk: int = 8192):
    return Predictor(gp, chunk)(xg, var_mode=var_mode, compute_var=compute_var)


def note_guard(stats: dict | None, gp: GPFit):
    """Record a checked fit's accuracy-guard decision in a job stream's `stats` (stats['guard'],
    one dict per job in job order: engine, wbits, kbits, vmin_over_kss, wmax, est)."""
    if stats is not None:
        g = gp.extra.get("guard")
        stats.setdefault("guard", []).append(
            {k: v for k, v in g.items() if k in ("engine", "wbits", "kbits", "vmin_over_kss", "wmax", "est")}
            if g else None)


def note_fit_issued(stats: dict | None):
    """Count a fit enqueued by a job stream (krige_jobs / krige_jobs_sharded) with its host
    time stamp — bench.py checks that every timed job's fit is issued inside its clock."""
    if stats is not None:
        stats["fits_issued"] = stats.get("fits_issued", 0) + 1
        stats.setdefault("fit_issue_times", []).append(time.perf_counter())


def krige_jobs(jobs, variance: str = "ozaki", chunk: int = 8192, var_mode: str = "latent",
               compute_var: bool = True, jitter: float = 0.0, device=None, stats: dict | None = None,
               fits_ahead: int | None = None, batch_fits: int | None = None,
               batch_ahead: bool | None = None):
    """Independent kriging jobs (kernel, x, y, noise, xg), one after another — the reference's
    runKrig.py:1-40 sweep (one GP_laser / krig.kriging fit + grid predict per setting or
    time window) run in one process.  Yields (mean, var) per job, in order, on the current
    stream; results are bit-identical to fit() + Predictor() called per job.

    Job i+1's fit is queued on a side stream as soon as job i's predict is, so the factor
    (latency-bound, a few hundred workgroups) runs on the CUs the predict's GEMMs leave idle
    (bench.py --pipeline).  The fit of job i+1 waits for the work queued on the
    current stream before it (so input tensors made there are ready); a non-SPD K_y of job i
    raises numpy.linalg.LinAlgError when job i is yielded, as fit() would.  The predict
    workspace is reused while consecutive jobs have the same padded size.  Nothing is read
    ahead before the first next(): a fresh generator's first fit is issued by that call (the
    bench times its jobs on a fresh generator for this reason).  `stats` counts the fits issued.

    fits_ahead = k > 1: up to k fits in flight on k side streams, each queued before the
    predict stream waits for the job ahead of it, so consecutive fits also overlap each other
    (gp2d_potrf draws a separate internal stream set per call).  fits_ahead = 0: each job's fit
    and predict strictly one after the other on the current stream — the fastest form for small
    jobs whose latency-bound fit outlasts their predict (config B: a fit beside a predict runs
    ≈ 2.4× longer).  fits_ahead = None (default): auto_fits_ahead() on the first
    job's shape — 1 where its predict outlasts its fit enough to hide it, else 0.

    batch_fits = b > 1 (with fits_ahead = 0): the next b jobs of one matrix order are fitted
    together (engine.fit_batch: one batched factorisation, the fit's latency-bound chain paid
    once per b jobs), then predicted one by one; same bits.  batch_fits = None (default):
    auto_fit_batch() for the back-to-back form, 1 otherwise.  batch_ahead=True: batch g+1's fit
    on a side stream under batch g's predicts; None (default): auto_batch_ahead() on the first
    job's shape."""
    dev = _require_device(device)
    main = torch.cuda.current_stream(dev)
    it = iter(jobs)
    if fits_ahead is None:
        first = next(it, None)
        if first is None:
            return
        it = itertools.chain([first], it)
        kernel, x, _, _, xg = first
        fits_ahead = auto_fits_ahead(kernel, _point_count(x, kernel.input_dim),
                                     _point_count(xg, kernel.input_dim), variance, compute_var)
    if int(fits_ahead) <= 0:
        if batch_fits is None or batch_ahead is None:
            first = next(it, None)
            if first is None:
                return
            it = itertools.chain([first], it)
            kernel, x, xg = first[0], first[1], first[4]
            ntr = _point_count(x, kernel.input_dim)
            if batch_fits is None:
                batch_fits = auto_fit_batch(kernel, ntr, variance)
            if batch_ahead is None:
                batch_ahead = auto_batch_ahead(kernel, ntr, _point_count(xg, kernel.input_dim), int(batch_fits),
                                               variance, compute_var)
        if int(batch_fits) > 1:
            yield from _krige_jobs_batched(it, int(batch_fits), variance, chunk, var_mode, compute_var, jitter, dev,
                                           stats, ahead=bool(batch_ahead))
        else:
            yield from _krige_jobs_serial(it, variance, chunk, var_mode, compute_var, jitter, dev, stats)
        return
    k = max(1, int(fits_ahead))
    sides = [side_stream(dev) for _ in range(k)]
    prev_sets = N.lib().gp2d_factor_sets(k) if k > 1 else None   # one internal factor set per side stream
    issued = [0]

    def queue_fit(job):
        kernel, x, y, noise, _ = job
        side = sides[issued[0] % k]
        # one fit in flight: the first has no predict to overlap, so it joins on the host (no
        # wait left pending on the side stream beside its chain, fit(join=...))
        join = k == 1 and issued[0] == 0
        issued[0] += 1
        side.wait_stream(main)
        note_fit_issued(stats)
        with torch.cuda.stream(side):
            return side, fit(kernel, x, y, noise, jitter=jitter, device=dev, variance=variance, check=False,
                             join=join)

    queue = collections.deque()   # (job, side stream, gp) with the fit queued

    def fill(limit):
        while len(queue) < limit:
            job = next(it, None)
            if job is None:
                return
            queue.append((job, *queue_fit(job)))

    try:
        fill(1)
        pred = None
        while queue:
            if k > 1:
                fill(k)   # before the predict stream waits for the head job's fit
            job, side, gp = queue.popleft()
            # this job's status (LinAlgError, the accuracy guard — which may re-prepare the
            # planes on `side`) before its predict is queued; the host waits for this fit only,
            # which ran under the previous job's predict, so the GPU never waits for the host
            with torch.cuda.stream(side):
                gp.check()
            note_guard(stats, gp)
            main.wait_stream(side)
            gp.record_stream(main)
            if k == 1:
                fill(1)   # the next job's fit, under this job's predict
            if pred is None or not pred.fits(gp):
                pred = Predictor(gp, chunk)
            pred.gp = gp
            out = pred(job[4], var_mode=var_mode, compute_var=compute_var, reuse_grid=True)
            yield out
    finally:
        if prev_sets is not None:
            N.lib().gp2d_factor_sets(prev_sets)


def _point_count(x, dim: int) -> int:
    if isinstance(x, torch.Tensor):
        return x.numel() // dim
    return int(np.size(x)) // dim


# job-shape model of auto_fits_ahead, fitted to the one-GPU measurements of DESIGN.md §6
# (profiles/r03_problem_sizes.txt, r03_ring_depth_E_B_ab.txt): a job's predict takes ≈ 1 ms +
# 48 ms · (M / 65,536) · (N / 4096)² on the Ozaki engine (×2.5 on FP64), its fit ≈ 0.061 ms ·
# (n / 128)^1.3 (2.24 ms at n = 2048, 13.6 ms at n = 8192), and a fit beside a predict runs
# ≈ 2.4× longer than alone (its dependent chain is dispatched behind the predict's GEMMs)
_PRED_MS_REF, _FIT_MS_COEF, _FIT_MS_EXP, _FIT_STRETCH = 48.0, 0.061, 1.3, 2.4


def _predict_ms_model(kernel: KernelSpec, n: int, m_grid: int, variance: str, compute_var: bool) -> float:
    scale = (m_grid / 65536.0) * (n / (2.0 * 4096)) ** 2 * (kernel.block_dim / 2.0)
    p = (1.0 + _PRED_MS_REF * scale) * (1.0 if variance == "ozaki" else 2.5)
    return 1.0 + 0.1 * (p - 1.0) if not compute_var else p


def auto_batch_ahead(kernel: KernelSpec, n_train: int, m_grid: int, b: int, variance: str = "ozaki",
                     compute_var: bool = True) -> bool:
    """krige_jobs' default for batched back-to-back jobs: batch g+1's fit under batch g's
    predicts when the batch's predicts outlast its stretched fit by the model of auto_fits_ahead,
    with the batched fit ≈ max(f·(1 + 0.15·(b − 1)), b·(2n³/3) / 46 TF/s) (chain-bound small
    batches, FLOP-bound large ones; profiles/r04_fit_batch.jsonl).  Config B (b = 8): 8.8e6 vs
    7.8e6 points/s back to back; with b = 4, 7.1e6 (profiles/r04_batch_ahead_ab.txt)."""
    if b <= 1:
        return False
    _, n = fit_layout(kernel, max(1, int(n_train)), variance)
    f1 = _FIT_MS_COEF * (n / NB) ** _FIT_MS_EXP
    fb = max(f1 * (1.0 + 0.15 * (b - 1)), b * (2.0 * n ** 3 / 3.0) / 46e9)
    return b * _predict_ms_model(kernel, n, m_grid, variance, compute_var) > (_FIT_STRETCH - 1.0) * fb


def auto_fits_ahead(kernel: KernelSpec, n_train: int, m_grid: int, variance: str = "ozaki",
                    compute_var: bool = True) -> int:
    """krige_jobs' default fits in flight for jobs of this shape: 1 (job i+1's fit under job
    i's predict) when that is faster by the model above, else 0 (each job's fit and predict back
    to back).  A pipelined job takes max(p, 2.4·f) + the fit's displaced GEMM work (≈ 0.1·p),
    a serial one f + p, so the overlap pays when p > 1.4·f.  Measured: config B (N = 1024, 128²
    grid) 4.19e6 points/s back to back vs 2.8–3.3e6 with one fit in flight; the headline
    (N = 4096, 256²) 55.7 vs 61.3 ms per job with one."""
    _, n = fit_layout(kernel, max(1, int(n_train)), variance)
    p = _predict_ms_model(kernel, n, m_grid, variance, compute_var)
    f = _FIT_MS_COEF * (n / NB) ** _FIT_MS_EXP
    return 1 if p > (_FIT_STRETCH - 1.0) * f else 0


FIT_BATCH_MAX = 8
FIT_BATCH_MAX_SMALL = 16        # matrix order ≤ FIT_BATCH_SMALL_N: the chain-bound sizes
FIT_BATCH_SMALL_N = 2048
FIT_BATCH_MAX_BYTES = 16 << 30   # two batches in flight (batch_ahead: g predicted, g+1 fitted)


def fit_problem_bytes(n: int) -> int:
    """Device bytes one problem of a batched fit holds: its n×n matrix (W in place) and its share
    of the TRTRI workspace ((n/2 + NB)² doubles) — the estimate of auto_fit_batch and
    hyper.auto_batch."""
    return 8 * (n * n + (n // 2 + NB) ** 2)


def auto_fit_batch(kernel: KernelSpec, n_train: int, variance: str = "ozaki") -> int:
    """krige_jobs' default batch for back-to-back jobs: up to FIT_BATCH_MAX fits per batched
    factorisation (FIT_BATCH_MAX_SMALL for matrix orders ≤ FIT_BATCH_SMALL_N, whose fit is the
    diagonal chain's latency) while TWO batches' matrices (batch_ahead keeps the predicted batch
    and the next one alive) stay below FIT_BATCH_MAX_BYTES.
    Measured (profiles/r04_fit_batch.jsonl): N_train = 1024, 1/2/4/8 fits in 2.27 / 2.56 / 3.20 /
    4.67 ms (2.28 ms each alone); 4096: 8 fits in 64 ms (13.4 each).  Config B's job stream
    (N_train = 1024, profiles/r04_bfit16_ab.jsonl): 8.33–8.38e6 points/s with 8 fits per batch,
    9.39–9.46e6 with 16, 9.24–9.27e6 with 32."""
    _, n = fit_layout(kernel, max(1, int(n_train)), variance)
    cap = FIT_BATCH_MAX_SMALL if n <= FIT_BATCH_SMALL_N else FIT_BATCH_MAX
    return max(1, min(cap, FIT_BATCH_MAX_BYTES // (2 * fit_problem_bytes(n))))


def _job_groups(jobs, b, variance):
    """Consecutive jobs in groups of up to b with one matrix order (a job of another order starts
    the next group)."""
    group, n0 = [], None
    for job in jobs:
        n1 = fit_layout(job[0], _point_count(job[1], job[0].input_dim), variance)[1]
        if group and (n1 != n0 or len(group) == b):
            yield group
            group = []
        group.append(job)
        n0 = n1
    if group:
        yield group


def _krige_jobs_batched(jobs, b, variance, chunk, var_mode, compute_var, jitter, dev, stats, ahead=False):
    """Jobs with their fits in batches of up to b jobs of one matrix order (engine.fit_batch),
    predicted one by one.  ahead=False: each batch's fit, then its predicts, on the current
    stream.  ahead=True: batch g+1's fit on a side stream under batch g's predicts (queued after
    batch g's first predict); the first batch, with nothing to overlap, joins on the host."""
    main = torch.cuda.current_stream(dev)
    side = side_stream(dev) if ahead else None
    groups = _job_groups(jobs, b, variance)

    def issue(group, first):
        for _ in group:
            note_fit_issued(stats)
        probs = [(k, x, y, nz) for k, x, y, nz, _ in group]
        if side is None:
            return fit_batch(probs, variance=variance, jitter=jitter, device=dev, check=False)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            return fit_batch(probs, variance=variance, jitter=jitter, device=dev, check=False, join=first)

    pred = None
    group = next(groups, None)
    fits = issue(group, True) if group else None
    while group:
        if side is not None:
            main.wait_stream(side)
            for gp in fits:
                gp.record_stream(main)
        nxt, nfits = None, None
        # status + accuracy guard of EVERY fit of the batch before the next batch's fit is queued
        # on `side`: a guard that re-prepares planes then queues that work ahead of the next
        # batch's factorisation, not behind it (the batch's fits end together, so checking them
        # all now waits no longer than checking the first); an error raises at its own job
        errs = []
        for gp in fits:
            try:
                with torch.cuda.stream(side if side is not None else main):
                    gp.check()
                errs.append(None)
            except Exception as e:   # noqa: BLE001 — re-raised when its job is reached
                errs.append(e)
        for q, (job, gp) in enumerate(zip(group, fits)):
            if errs[q] is not None:
                raise errs[q]
            note_guard(stats, gp)
            if side is not None:
                gp.ready_on(main)   # only the guard's own work: `side` may carry the next batch's fit
                gp.record_stream(main)
            if pred is None or not pred.fits(gp):
                pred = Predictor(gp, chunk)
            pred.gp = gp
            out = pred(job[4], var_mode=var_mode, compute_var=compute_var, reuse_grid=True)
            if q == 0 and side is not None:   # the next batch's fit under this batch's predicts
                nxt = next(groups, None)
                nfits = issue(nxt, False) if nxt else None
            yield out
        if side is None:
            nxt = next(groups, None)
            nfits = issue(nxt, False) if nxt else None
        group, fits = nxt, nfits


def _krige_jobs_serial(jobs, variance, chunk, var_mode, compute_var, jitter, dev, stats):
    pred = None
    for job in jobs:
        kernel, x, y, noise, xg = job
        note_fit_issued(stats)
        gp = fit(kernel, x, y, noise, jitter=jitter, device=dev, variance=variance, check=False)
        gp.check()   # status + accuracy guard before the predict
        note_guard(stats, gp)
        if pred is None or not pred.fits(gp):
            pred = Predictor(gp, chunk)
        pred.gp = gp
        out = pred(xg, var_mode=var_mode, compute_var=compute_var, reuse_grid=True)
        yield out


# ------------------------------------------------------------------ hyperparameters
def param_names(kernel: KernelSpec) -> tuple:
    """Gradient / parameter order of log_marginal_likelihood: vector2d (l_df, l_cf, ratio, noise);
    vector_st (l_df, l_cf, ratio, var_t, l_t, noise); ARD per term (variance, lengthscale_0..D−1),
    then noise (GPy param_array order, krig.py:459-466)."""
    if kernel.family == "vector2d":
        return ("l_df", "l_cf", "ratio", "noise")
    if kernel.family == "vector_st":
        return ("l_df", "l_cf", "ratio", "var_t", "l_t", "noise")
    names = []
    for t, ls in enumerate(kernel.lengthscales):
        names += [f"variance_{t}"] + [f"lengthscale_{t}_{d}" for d in range(len(ls))]
    return tuple(names + ["noise"])


def log_marginal_likelihood(gp: GPFit, eval_gradient: bool = False):
    """log p(y | X, θ) of a fit, and optionally ∂/∂θ in natural units (param_names order).

    Replaces the objective of GPy model.optimize (krig.py:450; GP_plots.py:673-765) and
    sklearn log_marginal_likelihood(theta, eval_gradient=True) (_gpr.py:584-650); the
    gradient is the exact one (the reference's myKernel.update_gradients_full is not,
    SURVEY.md §0.2).  Both run in HIP kernels (gp2d_lml, gp2d_lml_grad)."""
    out, g = lml_device(gp, eval_gradient)
    if not eval_gradient:
        return float(out.item())
    return float(out.item()), g.cpu().numpy()


def lml_device(gp: GPFit, eval_gradient: bool = False):
    """log_marginal_likelihood without a host round trip: (lml, grad or None) as device tensors,
    queued on the current stream (hyper.sweep overlaps settings this way)."""
    if gp.y is None:
        raise ValueError("this fit carries no observations (it was not made by engine.fit)")
    L = N.lib()
    s = _stream_handle(gp.device)
    bd = gp.kernel.block_dim
    out = torch.empty(1, dtype=torch.float64, device=gp.device)
    N.check(L.gp2d_lml(_ptr(gp.W), gp.n, gp.n, _ptr(gp.alpha), _ptr(gp.y), bd * gp.n_train, _ptr(out), s),
            "gp2d_lml")
    if not eval_gradient:
        return out, None
    desc = gp.kernel.desc()
    ng = int(L.gp2d_lml_grad_count(ctypes.byref(desc)))
    wbytes = int(L.gp2d_lml_grad_workspace(gp.n))
    work = torch.empty(wbytes // 8 + 1, dtype=torch.float64, device=gp.device)
    g = torch.empty(ng, dtype=torch.float64, device=gp.device)
    N.check(L.gp2d_lml_grad(_ptr(gp.W), gp.n, gp.n, _ptr(gp.alpha), _ptr(gp.x), gp.n_train, gp.n_pad,
                            ctypes.byref(desc), _ptr(g), _ptr(work), wbytes, s), "gp2d_lml_grad")
    return out, g


def kernel_grad(kernel: KernelSpec, xa, dL_dK, xb=None, device=None) -> np.ndarray:
    """Σ dL_dK ⊙ ∂K(xa, xb)/∂θ for θ = param_names(kernel) without the noise — the contraction
    GPy's Kern.update_gradients_full performs (myKernel.py:59-105; the exact derivative, not the
    reference's formula).  dL_dK: (bd·Na, bd·Nb) in the reference's component-major layout."""
    dev = _require_device(device)
    L = N.lib()
    d = kernel.input_dim
    A = _as_points(xa, d, dev)
    B = A if xb is None else _as_points(xb, d, dev)
    G = dL_dK.to(device=dev, dtype=torch.float64) if isinstance(dL_dK, torch.Tensor) else \
        torch.as_tensor(np.ascontiguousarray(np.asarray(dL_dK, dtype=np.float64)), device=dev)
    G = G.contiguous()
    bd = kernel.block_dim
    if tuple(G.shape) != (bd * A.shape[0], bd * B.shape[0]):
        raise ValueError(f"dL_dK has shape {tuple(G.shape)}, expected {(bd * A.shape[0], bd * B.shape[0])}")
    desc = kernel.desc()
    ng = int(L.gp2d_kernel_grad_count(ctypes.byref(desc)))
    wbytes = int(L.gp2d_kernel_grad_workspace(A.shape[0], B.shape[0]))
    work = torch.empty(wbytes // 8 + 1, dtype=torch.float64, device=dev)
    g = torch.empty(ng, dtype=torch.float64, device=dev)
    N.check(L.gp2d_kernel_grad(_ptr(A), A.shape[0], _ptr(B), B.shape[0], ctypes.byref(desc), _ptr(G), G.shape[1],
                               _ptr(g), _ptr(work), wbytes, _stream_handle(dev)), "gp2d_kernel_grad")
    return g.cpu().numpy()


# ------------------------------------------------------------------ dense helpers
def _as_matrix(a, device) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        t = a.to(device=device, dtype=torch.float64)
    else:
        t = torch.as_tensor(np.ascontiguousarray(np.asarray(a, dtype=np.float64)), device=device)
    return t.reshape(t.shape[0], -1) if t.dim() != 2 else t


def _padded(t: torch.Tensor, rows: int, cols: int) -> torch.Tensor:
    if tuple(t.shape) == (rows, cols) and t.is_contiguous():
        return t
    out = torch.zeros((rows, cols), dtype=torch.float64, device=t.device)
    out[:t.shape[0], :t.shape[1]] = t
    return out


def _up(v: int, m: int) -> int:
    return max(m, (v + m - 1) // m * m)


def gemm(A, B, transb: bool = False, alpha: float = 1.0, C=None, beta: float = 0.0, device=None) -> torch.Tensor:
    """alpha·A·op(B) + beta·C on the FP64 MFMA GEMM core (gp2d_gemm); op(B) = Bᵀ if transb.
    Operands of any shape are zero-padded to the kernel's 128/128/16 tiles (the padding adds
    exact zeros to every sum).  The dense product of GP_scripts.getMean / getCov."""
    dev = _require_device(device)
    A = _as_matrix(A, dev)
    B = _as_matrix(B, dev)
    m, k = A.shape
    n = B.shape[0] if transb else B.shape[1]
    if (B.shape[1] if transb else B.shape[0]) != k:
        raise ValueError(f"gemm: inner dimensions differ ({tuple(A.shape)} x {tuple(B.shape)}, transb={transb})")
    mp, np_, kp = _up(m, NB), _up(n, NB), _up(k, 16)
    Ap = _padded(A, mp, kp)
    Bp = _padded(B, np_, kp) if transb else _padded(B, kp, np_)
    Cp = torch.zeros((mp, np_), dtype=torch.float64, device=dev)
    if C is not None and beta != 0.0:
        Cp[:m, :n] = _as_matrix(C, dev)
    N.check(N.lib().gp2d_gemm(int(bool(transb)), mp, np_, kp, float(alpha), _ptr(Ap), kp, _ptr(Bp), Bp.shape[1],
                              float(beta), _ptr(Cp), np_, _stream_handle(dev)), "gp2d_gemm")
    return Cp[:m, :n]


def spd_inverse(K, device=None, return_factor: bool = False):
    """K⁻¹ of a symmetric positive-definite matrix through the engine's factor:
    L = chol(K) (gp2d_potrf), W = L⁻¹ (gp2d_trtri), K⁻¹ = WᵀW (gp2d_transpose + gp2d_gemm).
    Stands in for np.linalg.inv(K) (GP_scripts.py:50, GP_laser.py:118) on the matrices those
    call sites build; raises numpy.linalg.LinAlgError when K is not positive definite (where
    np.linalg.inv raises only for an exactly singular K).  K is padded to a multiple of 128
    with an identity block, which the block-diagonal inverse leaves decoupled."""
    dev = _require_device(device)
    K = _as_matrix(K, dev)
    n0 = K.shape[0]
    if K.shape[1] != n0:
        raise ValueError("spd_inverse: K must be square")
    L = N.lib()
    n = _up(n0, NB)
    A = torch.eye(n, dtype=torch.float64, device=dev)
    A[:n0, :n0] = K
    s = _stream_handle(dev)
    dinv = torch.empty((n // NB, NB, NB), dtype=torch.float64, device=dev)
    info = torch.empty(1, dtype=torch.int32, device=dev)
    N.check(L.gp2d_potrf(_ptr(A), n, n, _ptr(dinv), _ptr(info), None, 0, s), "gp2d_potrf")
    wbytes = int(L.gp2d_trtri_workspace(n))
    work = torch.empty(wbytes // 8 + 1, dtype=torch.float64, device=dev)
    N.check(L.gp2d_trtri(_ptr(A), n, n, _ptr(dinv), _ptr(work), wbytes, s), "gp2d_trtri")
    _raise_fit_errors(int(info.item()), None)
    Wt = torch.empty((n, n), dtype=torch.float64, device=dev)
    N.check(L.gp2d_transpose(_ptr(A), n, n, _ptr(Wt), s), "gp2d_transpose")
    Ki = torch.empty((n, n), dtype=torch.float64, device=dev)
    N.check(L.gp2d_gemm(1, n, n, n, 1.0, _ptr(Wt), n, _ptr(Wt), n, 0.0, _ptr(Ki), n, s), "gp2d_gemm")
    Ki = Ki[:n0, :n0]
    return (Ki, A[:n0, :n0]) if return_factor else Ki


def timing_enable(on: bool = True):
    N.lib().gp2d_timing_enable(int(bool(on)))


def timing_read():
    ms = ctypes.c_double()
    cnt = ctypes.c_int64()
    fl = ctypes.c_double()
    N.check(N.lib().gp2d_timing_read(ctypes.byref(ms), ctypes.byref(cnt), ctypes.byref(fl)), "gp2d_timing_read")
    return ms.value, cnt.value, fl.value
