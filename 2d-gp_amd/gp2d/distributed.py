"""Multi-GPU grid sharding: one process per GPU, fit once,
broadcast the inverse Cholesky factor over RCCL (xGMI), predict disjoint,
tile-aligned grid shards, gather in rank order.

Grid points are independent given (X_train, W = L⁻¹, α, hyperparameters), and
every per-point reduction in the predict kernels has a fixed order that does not
depend on shard boundaries, so the concatenated result is bit-identical to the
single-GPU result.
"""
from __future__ import annotations

import collections

import numpy as np
import torch
import torch.distributed as dist

from . import data as D
from . import engine as E


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def broadcast_fit(gp: E.GPFit | None, spec: E.KernelSpec, noise: float, x, device, src: int = 0,
                  error: Exception | None = None) -> E.GPFit:
    """Broadcast W, α and the training points from `src` to every rank (RCCL
    ncclBroadcast under the 'nccl' backend).  Ranks other than `src` pass gp=None.
    If the fit failed on `src` (`error`, e.g. a non-positive-definite K_y) the status word of
    the metadata broadcast carries it and EVERY rank raises (numpy.linalg.LinAlgError for a
    failed factor) instead of waiting for a factor that never comes."""
    ws, rank = world()
    if ws == 1:
        if error is not None:
            raise error
        return gp
    meta = torch.zeros(4, dtype=torch.int64, device=device)
    if rank == src:
        if error is None:
            meta[0], meta[1], meta[2] = gp.n, gp.n_train, gp.n_pad
        else:
            meta[3] = 1 if isinstance(error, np.linalg.LinAlgError) else 2
    dist.broadcast(meta, src)
    n, ntr, npad, status = (int(v) for v in meta.tolist())
    if status != 0:
        if rank == src:
            raise error
        if status == 1:
            raise np.linalg.LinAlgError(f"the fit on rank {src} failed: K_y is not positive definite")
        raise RuntimeError(f"the fit on rank {src} failed")
    blocks = packed_blocks(n)
    packed = torch.empty(blocks[-1][2], dtype=torch.float64, device=device)
    if rank != src:
        W = torch.zeros((n, n), dtype=torch.float64, device=device)
        alpha = torch.empty(n, dtype=torch.float64, device=device)
        X = torch.empty((ntr, spec.input_dim), dtype=torch.float64, device=device)
    else:
        W, X, alpha = gp.W, gp.x, gp.alpha
        for r0, c1, off in blocks[:-1]:
            packed[off:off + PACK_ROWS * c1].view(PACK_ROWS, c1).copy_(W[r0:r0 + PACK_ROWS, :c1])
    # W = L⁻¹ is lower-triangular: only the row blocks' [0, end of their diagonal block)
    # columns travel (≈ half of n² doubles)
    dist.broadcast(packed, src)
    dist.broadcast(alpha, src)
    dist.broadcast(X, src)
    if rank == src:
        return gp
    for r0, c1, off in blocks[:-1]:
        W[r0:r0 + PACK_ROWS, :c1].copy_(packed[off:off + PACK_ROWS * c1].view(PACK_ROWS, c1))
    return E.GPFit(kernel=spec, noise=float(noise), x=X, n_train=ntr, n_pad=npad, W=W, alpha=alpha,
                   device=torch.device(device))


PACK_ROWS = 128   # the matrix order is a multiple of 128 (engine.fit_layout)


def packed_blocks(n: int):
    """Row-block packing of a lower-triangular n×n matrix: [(first row, columns kept,
    offset)] per 128-row block (columns up to the end of its diagonal block), then a final
    (n, 0, total length) sentinel."""
    out, off = [], 0
    for r0 in range(0, n, PACK_ROWS):
        c1 = min(n, r0 + PACK_ROWS)
        out.append((r0, c1, off))
        off += PACK_ROWS * c1
    out.append((n, 0, off))
    return out


def fit_sharded(spec: E.KernelSpec, x, y, noise: float, device, mode: str = "bcast", jitter: float = 0.0,
                variance: str = "f64", check: bool = True):
    """mode 'bcast': rank 0 fits, factor broadcast over RCCL; 'replicate': every rank
    fits redundantly (no communication).  With variance='ozaki' every rank derives its
    INT8 residue planes from the broadcast factor locally (no extra traffic).  check=False as
    in engine.fit (replicate mode; in bcast mode rank 0 checks before broadcasting)."""
    ws, rank = world()
    if ws == 1 or mode == "replicate":
        return E.fit(spec, x, y, noise, jitter=jitter, device=device, variance=variance, check=check)
    gp, err = None, None
    if rank == 0:
        try:
            gp = E.fit(spec, x, y, noise, jitter=jitter, device=device, variance=variance)
        except Exception as e:   # noqa: BLE001 — re-raised on every rank by broadcast_fit
            err = e
    gp = broadcast_fit(gp, spec, noise, x, device, error=err)
    if variance == "ozaki" and "ozaki" not in gp.extra:
        E.ozaki_prepare(gp, diag_add=float(noise + jitter))   # a-priori moduli count: no host sync
    return gp


def krige_jobs_sharded(jobs, variance: str = "ozaki", chunk: int = 8192, var_mode: str = "latent",
                       compute_var: bool = True, jitter: float = 0.0, device=None, align: int = 64,
                       stats: dict | None = None):
    """A stream of independent kriging jobs (kernel, x, y, noise, xg) — the reference's
    runKrig.py sweep / per-window krig.kriging calls — spread over all ranks: job j is FITTED
    by rank j mod world only (round robin, on a side stream, up to one job per rank ahead),
    its factor W = L⁻¹, α and training points are broadcast from that rank (broadcast_fit,
    RCCL under the 'nccl' backend), and EVERY rank predicts its tile-aligned shard of job j's
    grid (predict_shard).  Yields (lo, hi, mean, var) per job, in job order, on every rank;
    the shards are bit-identical to one process's fit + predict (fixed-order reductions).

    Per job a rank does 1/world of a fit plus 1/world of the predict, so for a stream of jobs
    the fit — the serial part of a one-job multi-GPU predict — is divided like the grid
    (DESIGN.md §5).  Every rank must pass the same job sequence (x, y are read on the owner
    only); a non-SPD K_y raises numpy.linalg.LinAlgError on every rank at that job.  Nothing is
    read ahead before the first next(); `stats` counts the fits this rank issues (with their
    host time stamps, engine.note_fit_issued)."""
    ws, rank = world()
    dev = E._require_device(device)
    if ws == 1:   # one rank: the single-GPU pipelined form (the next fit under this predict)
        seen = collections.deque()

        def feed():
            for job in jobs:
                seen.append(job)
                yield job
        for mean, var in E.krige_jobs(feed(), variance=variance, chunk=chunk, var_mode=var_mode,
                                      compute_var=compute_var, jitter=jitter, device=dev, stats=stats):
            xg = seen.popleft()[4]
            yield 0, int(xg.shape[0]), mean, var
        return
    main = torch.cuda.current_stream(dev)
    fit_stream = torch.cuda.Stream(dev)
    comm = torch.cuda.Stream(dev)   # broadcasts + the receivers' int8 preparation
    it = iter(jobs)
    window = collections.deque()   # (index, job) read ahead
    own = {}                       # index → (gp, error, event) of this rank's fits in flight
    count = 0

    def refill():
        nonlocal count
        while len(window) < ws + 1:
            job = next(it, None)
            if job is None:
                break
            window.append((count, job))
            count += 1
        for idx, job in window:   # this rank's fits among the jobs read ahead
            if idx % ws == rank and idx not in own:
                spec, x, y, noise, _ = job
                fit_stream.wait_stream(main)
                E.note_fit_issued(stats)
                gp, err = None, None
                with torch.cuda.stream(fit_stream):
                    try:
                        gp = E.fit(spec, x, y, noise, jitter=jitter, device=dev, variance=variance, check=False)
                    except Exception as e:   # noqa: BLE001 — travels in broadcast_fit's status word
                        err = e
                    ev = torch.cuda.Event()
                    ev.record(fit_stream)
                own[idx] = (gp, err, ev)

    def receive(idx, job):
        """Job idx's factor from its owner, on the comm stream: (gp, ready event) or the
        exception every rank raises for it (kept until the job's turn)."""
        spec, x, _, noise, _ = job
        owner = idx % ws
        gp, err = None, None
        if owner == rank:
            gp, err, ev = own.pop(idx)
            if gp is not None:
                comm.wait_event(ev)
                gp.record_stream(comm)
                try:
                    gp.check()
                except Exception as e:   # noqa: BLE001
                    gp, err = None, e
        try:
            with torch.cuda.stream(comm):
                gp = broadcast_fit(gp, spec, noise, x, dev, src=owner, error=err)
                if variance == "ozaki" and "ozaki" not in gp.extra:
                    E.ozaki_prepare(gp, diag_add=float(noise + jitter))   # a-priori moduli count
                ready = torch.cuda.Event()
                ready.record(comm)
        except Exception as e:   # noqa: BLE001
            return e
        return gp, ready

    refill()
    if not window:
        return
    cur = receive(*window[0])
    pred = None
    while window:
        idx, (spec, x, y, noise, xg) = window.popleft()
        if isinstance(cur, Exception):
            raise cur
        gp, ready = cur
        main.wait_event(ready)
        gp.record_stream(main)
        if pred is None or not pred.fits(gp):
            pred = E.Predictor(gp, chunk)
        pred.gp = gp
        out = predict_shard(pred, E._as_points(xg, spec.input_dim, dev), var_mode=var_mode,
                            compute_var=compute_var, align=align)
        refill()
        # the next job's factor travels (host may wait for its owner) while this predict runs
        cur = receive(*window[0]) if window else None
        yield out


def predict_shard(pred: E.Predictor, xg_all, var_mode: str = "latent", compute_var: bool = True, align: int = 64):
    """Predict this rank's contiguous shard of the flattened grid; returns
    (lo, hi, mean, var) with mean/var in the [u..., v...] layout of the shard."""
    ws, rank = world()
    m = int(xg_all.shape[0])
    lo, hi = D.shard_range(m, ws, rank, align)
    mean, var = pred(xg_all[lo:hi], var_mode=var_mode, compute_var=compute_var)
    return lo, hi, mean, var


def gather_shards(m: int, bd: int, lo: int, hi: int, mean, var, device, align: int = 64):
    """All-gather the shards and reassemble the full [u(M)..., v(M)...] vectors in rank order.
    `align` must be the one predict_shard used (checked against this rank's (lo, hi))."""
    ws, rank = world()
    if ws == 1:
        return mean, var
    ranges = [D.shard_range(m, ws, r, align) for r in range(ws)]
    if ranges[rank] != (lo, hi):
        raise ValueError(f"gather_shards: rank {rank} holds [{lo}, {hi}) but align={align} gives "
                         f"{ranges[rank]}; pass predict_shard's align")
    maxlen = max(b - a for a, b in ranges)
    outs = []
    for t in (mean, var):
        buf = torch.zeros(bd * maxlen, dtype=torch.float64, device=device)
        k = hi - lo
        for c in range(bd):
            buf[c * maxlen:c * maxlen + k] = t[c * k:(c + 1) * k]
        parts = [torch.empty_like(buf) for _ in range(ws)]
        dist.all_gather(parts, buf)
        full = torch.empty(bd * m, dtype=torch.float64, device=device)
        for (a, b), p in zip(ranges, parts):
            k = b - a
            for c in range(bd):
                full[c * m + a:c * m + b] = p[c * maxlen:c * maxlen + k]
        outs.append(full)
    return outs[0], outs[1]


def shard_layout(m: int, bd: int, world_size: int):
    """Host-side description of the shards (used by tests): list of (lo, hi)."""
    return [D.shard_range(m, world_size, r) for r in range(world_size)]


def assemble_from_shards(m: int, bd: int, shards):
    """Concatenate per-rank [u..., v...] shard vectors into the global layout (numpy)."""
    full = np.empty(bd * m)
    for lo, hi, vec in shards:
        k = hi - lo
        for c in range(bd):
            full[c * m + lo:c * m + hi] = vec[c * k:(c + 1) * k]
    return full
