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
import ctypes
import os
import time

import numpy as np
import torch
import torch.distributed as dist

from . import comm as C
from . import data as D
from . import engine as E


# GP2D_FORCE_COLLECTIVES=1 (tests only): run the multi-rank code paths (broadcasts, all-gathers,
# round-robin fits) even at world size 1 — the real RCCL calls on a one-GPU box
FORCE_COLLECTIVES = os.environ.get("GP2D_FORCE_COLLECTIVES") == "1"
# GP2D_RECV_UNPACK=1 (measurement only): receivers of a job stream rebuild the full n×n W and
# prepare from it (the round-4 path) instead of preparing the int8 planes from the packed payload
RECV_UNPACK = os.environ.get("GP2D_RECV_UNPACK") == "1"


def _solo(ws: int) -> bool:
    return ws == 1 and not (FORCE_COLLECTIVES and dist.is_available() and dist.is_initialized())


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def broadcast_fit(gp: E.GPFit | None, spec: E.KernelSpec, noise: float, x, device, src: int = 0,
                  error: Exception | None = None, layout: tuple | None = None,
                  planes_only: float | None = None, comm: dict | None = None) -> E.GPFit:
    """Broadcast W, α and the training points from `src` to every rank (RCCL
    ncclBroadcast under the 'nccl' backend).  Ranks other than `src` pass gp=None.

    layout=None: a metadata broadcast first carries the sizes, a status word and the owner's
    accuracy-guard decision (engine.apply_guard), read on the host (one round trip); if the fit
    failed on `src` (`error`, e.g. a non-positive-definite K_y) EVERY rank raises here
    (numpy.linalg.LinAlgError for a failed factor) instead of waiting for a factor that never comes.

    layout=(n, n_train, n_pad) (the job stream, where every rank knows the job's sizes): no host
    round trip at all — the owner's status block (engine.status_block: POTRF `info`, or −1 for an
    error raised on the host, and the guard's statistics) travels on the device beside the factor
    and the returned fit carries it as pending: GPFit.check() raises on every rank, and applies
    the same guard decision on every rank, before the job's predict is queued.

    planes_only=diag_add (the receiver of a job stream that predicts with the ozaki engine): the
    receiving ranks build their INT8 residue planes straight from the packed payload
    (gp2d_ozaki_prepare_packed) and keep no n×n W (the returned fit has W = None) — no zero-fill
    and no unpack of an n×n matrix per job.
    comm (optional dict): bytes this rank sends / receives and the collectives' HIP-event times
    are appended under 'bcast' (collect with comm_summary)."""
    ws, rank = world()
    if _solo(ws):
        if error is not None:
            raise error
        return gp
    dev = torch.device(device)
    status = None
    wbits = kbits = None   # the owner's guard decision (layout=None): wbits −1 = FP64 engine
    if layout is None:
        if rank == src:
            g = (gp.extra.get("guard") or {}) if gp is not None else {}
            wb = -1 if g.get("engine") == "f64" else int(g.get("wbits") or 0)
            kb = int(g.get("kbits") or 0)
            st = 0 if error is None else (1 if isinstance(error, np.linalg.LinAlgError) else 2)
            vals = [gp.n, gp.n_train, gp.n_pad, st, wb, kb] if error is None else [0, 0, 0, st, 0, 0]
            meta = torch.tensor(vals, dtype=torch.int64).to(dev)
        else:
            meta = torch.empty(6, dtype=torch.int64, device=dev)
        C.broadcast(meta, src)
        n, ntr, npad, st, wbits, kbits = (int(v) for v in meta.tolist())
        if st != 0:
            if rank == src:
                raise error
            if st == 1:
                raise np.linalg.LinAlgError(f"the fit on rank {src} failed: K_y is not positive definite")
            raise RuntimeError(f"the fit on rank {src} failed")
    else:
        n, ntr, npad = (int(v) for v in layout)
        prep_err = gp.pending[2] if (gp is not None and gp.pending is not None) else None
        if rank == src and error is None and gp is not None and prep_err is None:
            status = gp.extra["status_dev"]   # broadcast in place (the owner's pending read is its own)
        elif rank == src:
            # an error raised on the owner's host, or one its fit deferred to check() (a failed
            # int8 preparation): status −1, so the receivers raise at this job too
            status = torch.tensor([0.0, 0.0, 0.0], dtype=torch.float64)
            status.view(torch.int32)[0] = -1
            status = status.to(dev)
        else:
            status = torch.empty(3, dtype=torch.float64, device=dev)
        C.broadcast(status, src)
    packed = torch.empty(_packed_len(n), dtype=torch.float64, device=dev)
    owner_ok = rank == src and gp is not None and error is None
    if owner_ok:
        X, alpha = gp.x, gp.alpha
        _pack_lower(gp.W, n, packed, unpack=False)
    elif rank == src:   # a failed fit: the receivers still expect the payload (and raise on its status)
        alpha = torch.zeros(n, dtype=torch.float64, device=dev)
        X = torch.zeros((ntr, spec.input_dim), dtype=torch.float64, device=dev)
        packed.zero_()
    else:               # overwritten by the broadcasts
        alpha = torch.empty(n, dtype=torch.float64, device=dev)
        X = torch.empty((ntr, spec.input_dim), dtype=torch.float64, device=dev)
    # W = L⁻¹ is lower-triangular: only the row blocks' [0, end of their diagonal block)
    # columns travel (≈ half of n² doubles)
    with _timed(comm, "bcast", rank == src, 8 * (packed.numel() + alpha.numel() + X.numel()), ws, device=dev):
        C.broadcast(packed, src)
        C.broadcast(alpha, src)
        C.broadcast(X, src)
    if owner_ok:
        out = gp
    elif planes_only is not None and spec.is_vector and packed.is_cuda and not RECV_UNPACK:
        with _timed(comm, "recv_prepare", False, 0, ws, recv=0, device=dev):
            out = E.GPFit(kernel=spec, noise=float(noise), x=X, n_train=ntr, n_pad=npad, W=None, alpha=alpha,
                          device=dev, n_mat=n)
            E.ozaki_prepare(out, diag_add=float(planes_only), packed=packed)
        # the owner's guard statistics arrive in the status block: check() applies the same rule
        out.extra["guard"] = dict(pending=True, diag_add=float(planes_only),
                                  stream=torch.cuda.current_stream(dev))
    else:
        with _timed(comm, "recv_prepare", False, 0, ws, recv=0, device=dev):
            W = torch.zeros((n, n), dtype=torch.float64, device=dev)   # the strict upper part stays 0
            _pack_lower(W, n, packed, unpack=True)
            out = E.GPFit(kernel=spec, noise=float(noise), x=X, n_train=ntr, n_pad=npad, W=W, alpha=alpha, device=dev)
            if planes_only is not None and RECV_UNPACK:   # the round-4 receive path (measurement only)
                E.ozaki_prepare(out, diag_add=float(planes_only))
                out.extra["guard"] = dict(pending=True, diag_add=float(planes_only),
                                          stream=torch.cuda.current_stream(dev))
        if wbits is not None and wbits != 0:   # the owner's guard decision, applied as is
            out.extra["guard"] = dict(pending=False, engine="f64" if wbits < 0 else "ozaki",
                                      wbits=None if wbits < 0 else wbits, kbits=None if wbits < 0 else kbits)
    if status is not None and out is not gp:   # the owner's own fit keeps its pending status read
        out.pending = E.pending_status(status, error if rank == src else None)
    return out


class _timed:
    """Context manager around one collective (or a group of them) for the N > 1 bench line's
    `comm` block: HIP events on the current stream for device tensors (the collective's stream
    is ordered with it both ways by torch.distributed), host wall time otherwise (the gloo CPU
    tests).  Appends (start, end, bytes sent, bytes received) to comm[key]; comm=None records
    nothing.  Bytes are the payload this rank puts in / takes out of the collective: the root of
    a broadcast sends it once and the others receive it; an all-gather sends this rank's part and
    receives the other ranks' parts (the transport's own fan-out is RCCL's)."""

    def __init__(self, comm: dict | None, key: str, sends: bool, nbytes: int, ws: int, recv: int | None = None,
                 device=None):
        self.comm, self.key = comm, key
        self.sent = int(nbytes) if sends else 0
        self.recv = int(recv) if recv is not None else (0 if sends else int(nbytes))
        dev = torch.device(device) if device is not None else None
        self.dev = dev if (dev is not None and dev.type == "cuda") else None

    def __enter__(self):
        if self.comm is None:
            return self
        if self.dev is not None:
            self.t0 = torch.cuda.Event(enable_timing=True)
            self.t0.record(torch.cuda.current_stream(self.dev))
        else:
            self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.comm is None or exc[0] is not None:
            return False
        if self.dev is not None:
            t1 = torch.cuda.Event(enable_timing=True)
            t1.record(torch.cuda.current_stream(self.dev))
        else:
            t1 = time.perf_counter()
        self.comm.setdefault(self.key, []).append((self.t0, t1, self.sent, self.recv))
        return False


def comm_summary(comm: dict | None) -> dict:
    """{key: {calls, ms, bytes_sent, bytes_recv}} from a comm dict filled by the collectives
    (waits for their end events); the dict is emptied."""
    out = {}
    for key, recs in (comm or {}).items():
        ms = 0.0
        for t0, t1, _, _ in recs:
            if isinstance(t0, float):
                ms += 1e3 * (t1 - t0)
            else:
                t1.synchronize()
                ms += t0.elapsed_time(t1)
        out[key] = dict(calls=len(recs), ms=ms, bytes_sent=sum(r[2] for r in recs),
                        bytes_recv=sum(r[3] for r in recs))
    if comm is not None:
        comm.clear()
    return out


def _packed_len(n: int) -> int:
    return packed_blocks(n)[-1][2]


def _pack_lower(W: torch.Tensor, n: int, packed: torch.Tensor, unpack: bool):
    """W's lower block triangle ↔ the packed payload: one gp2d_pack_lower launch on a device
    tensor; CPU tensors (the gloo CPU tests of the communication logic) are copied block by
    block."""
    if W.is_cuda:
        E.N.check(E.N.lib().gp2d_pack_lower(E._ptr(W), n, W.stride(0), E._ptr(packed), int(unpack),
                                            E._stream_handle(W.device)), "gp2d_pack_lower")
        return
    for r0, c1, off in packed_blocks(n)[:-1]:
        blk = packed[off:off + PACK_ROWS * c1].view(PACK_ROWS, c1)
        if unpack:
            W[r0:r0 + PACK_ROWS, :c1].copy_(blk)
        else:
            blk.copy_(W[r0:r0 + PACK_ROWS, :c1])


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
    if _solo(ws) or mode == "replicate":
        return E.fit(spec, x, y, noise, jitter=jitter, device=device, variance=variance, check=check)
    gp, err = None, None
    if rank == 0:
        try:
            gp = E.fit(spec, x, y, noise, jitter=jitter, device=device, variance=variance)
        except Exception as e:   # noqa: BLE001 — re-raised on every rank by broadcast_fit
            err = e
    gp = broadcast_fit(gp, spec, noise, x, device, error=err)
    g = gp.extra.get("guard") or {}
    if variance == "ozaki" and "ozaki" not in gp.extra and g.get("engine") != "f64":
        # a-priori moduli count (no host sync), at the owner's guard precision
        E.ozaki_prepare(gp, diag_add=float(noise + jitter), wbits=int(g.get("wbits") or 0),
                        kbits=int(g.get("kbits") or 0))
    return gp


def super_block() -> int:
    """Super-block width of the distributed factor (csrc/dfact.hpp DF_SB, gp2d_dfact_sb)."""
    return int(E.N.lib().gp2d_dfact_sb())


def dfact_layout(spec: E.KernelSpec, n_train: int):
    """(padded point count, matrix order n) of a distributed fit: engine.fit's ozaki layout with
    n rounded up to a multiple of the super-block (the padded points add identity rows)."""
    sb = super_block()
    npad, n = E.fit_layout(spec, n_train, "ozaki")
    bd = spec.block_dim
    step = max(1, sb // bd)
    npad = (npad + step - 1) // step * step
    return npad, bd * npad


def _owned_blocks(nsb: int, ws: int, r: int):
    return list(range(r, nsb, ws))


def fit_distributed(spec: E.KernelSpec, x, y, noise: float, device=None, variance: str = "ozaki",
                    jitter: float = 0.0, lookahead: bool = True, stats: dict | None = None,
                    emulate: tuple | None = None, comm: dict | None = None) -> E.GPFit:
    """ONE job's fit spread over all ranks (the config-D single job: /root/reference/krig.py:541-557
    predicts one model's large grid): every rank assembles K_y, then a 1-D block-cyclic POTRF
    fused with the right-looking TRTRI (include/gp2d.h gp2d_dfact_*) — rank s mod P factors
    super-column s (512 wide), broadcasts the panel [L_ss⁻¹; L21] (torch.distributed: RCCL under
    'nccl'), and every rank applies it to its own K_y columns (POTRF trailing update) and to its
    own W = L⁻¹ columns (TRTRI step).  The owned W columns are then all-gathered (lower parts only,
    ≈ n²/2 doubles in all), so every rank ends with the full W, α and the ozaki residue planes,
    ready to predict its grid shard (predict_shard).

    Per rank: 1/P of the POTRF's and the TRTRI's GEMM flops, one panel receive per step
    (n²/2 doubles in all) and the all-gather.  The next owner updates its next super-column with
    the panel first and factors it while the rest of the step's GEMMs run (look-ahead), so the
    chain of diagonal factorisations is not serialised behind the trailing updates.

    Every element's arithmetic is the same for any world size, so P ranks return the bits of one
    (tests/test_gpu_distributed.py); a non-SPD K_y raises numpy.linalg.LinAlgError on every rank.
    `stats` (optional dict) receives host-side timestamps of the phases.

    emulate=(P, r) (measurement only, tools/probe_dfit.py; one process, no process group): run
    rank r's share of a P-rank factorisation — its panels, updates and inverse steps, no
    broadcast (the panels it did not factor hold stale data) and no all-gather; the returned
    factor is NOT W.

    comm (optional dict): per-collective bytes and HIP-event times — 'panel_bcast' (one per step),
    'w_allgather', 'alpha_allgather' (comm_summary)."""
    ws, rank = world()
    if emulate is not None:
        if ws != 1:
            raise ValueError("emulate is for one process without a process group")
        ws, rank = int(emulate[0]), int(emulate[1])
    dev = E._require_device(device)
    if variance not in E.VARIANCE_ENGINES:
        raise ValueError(f"variance must be one of {E.VARIANCE_ENGINES}")
    if variance == "ozaki" and not spec.is_vector:
        raise ValueError("the ozaki variance engine supports the vector families only")
    L = E.N.lib()
    d, bd = spec.input_dim, spec.block_dim
    X = E._as_points(x, d, dev)
    ntr = X.shape[0]
    if ntr < 1:
        raise ValueError("need at least one training point")
    npad, n = dfact_layout(spec, ntr)   # n a multiple of the super-block
    SB = super_block()
    if variance == "ozaki" and n >= 131072:
        raise ValueError(f"the ozaki variance engine supports n < 131072; got n = {n}")
    perm = None
    if variance == "ozaki" and ntr > 1:
        perm, X = E.morton_sort(X)
    main = torch.cuda.current_stream(dev)
    sh = E._stream_handle(dev)
    P = E._ptr
    desc = spec.desc()
    nsb = n // SB
    multi = emulate is not None or not _solo(ws)
    mine = _owned_blocks(nsb, ws, rank)
    A = torch.empty((n, n), dtype=torch.float64, device=dev)
    if multi and spec.is_vector:
        # a rank reads and writes only its own super-columns: assemble just those (each 256-column
        # half lies inside one component), the same arithmetic as the full symmetric assembly
        for t in mine:
            for c0 in (t * SB, t * SB + SB // 2):
                E.N.check(L.gp2d_assemble_cols(P(X), ntr, npad, ctypes.byref(desc), float(noise + jitter), P(A), n,
                                               c0, SB // 2, sh), "gp2d_assemble_cols")
    else:
        E.N.check(L.gp2d_assemble(P(X), ntr, npad, P(X), ntr, npad, ctypes.byref(desc), float(noise + jitter), 1,
                                  P(A), n, sh), "gp2d_assemble")
    pdoubles = int(L.gp2d_dfact_panel_doubles(n))
    panels = [torch.empty(pdoubles, dtype=torch.float64, device=dev) for _ in range(2)]
    wbytes = int(L.gp2d_dfact_workspace(n))
    work = torch.empty(wbytes // 8 + 1, dtype=torch.float64, device=dev)
    info = torch.zeros(1, dtype=torch.int32, device=dev)   # the owners' panels only ever raise it
    cstream = E.side_stream(dev)
    t0 = time.perf_counter()

    factored = {}   # s → event after the owner's gp2d_dfact_panel(s) (main or crit stream)
    done = {}       # s → events after step s's last reads of its panel buffer (main, inv)
    # lookahead: the owners' chain of panel factorisations on `crit`, and the TRTRI steps (W
    # columns ≤ s) on `inv` beside the POTRF trailing updates (K_y columns > s) on main — the
    # regions are disjoint, and the TRTRI step's small D_s product no longer idles the chip
    crit = E.side_stream(dev) if lookahead else main
    inv = E.side_stream(dev) if lookahead else main

    def wait_done(st, s):
        for ev in done.get(s, ()):
            st.wait_event(ev)

    def factor(s, st):   # owner of s: panel s into its buffer, on stream st
        with torch.cuda.stream(st):
            E.N.check(L.gp2d_dfact_panel(P(A), n, n, s, P(panels[s % 2]), P(info), P(work), wbytes,
                                         E._stream_handle(dev)), "gp2d_dfact_panel")
            ev = torch.cuda.Event()
            ev.record(st)
        factored[s] = ev

    if rank == 0:
        factor(0, main)
    for s in range(nsb):
        owner = s % ws
        buf = panels[s % 2]
        rows = n - s * SB
        if not _solo(ws) and emulate is None:
            # the buffer's previous user (step s − 2) is done; the owner's panel s is written —
            # the broadcast does not wait for the rest of step s − 1 (it overlaps it)
            if s >= 2:
                wait_done(cstream, s - 2)
                done.pop(s - 2)
            if owner == rank:
                cstream.wait_event(factored.pop(s))
            with torch.cuda.stream(cstream), _timed(comm, "panel_bcast", owner == rank, 8 * rows * SB, ws, device=dev):
                C.broadcast(buf[:rows * SB], owner)
            main.wait_stream(cstream)
        elif s in factored:   # one rank: the panel was factored on the chain stream
            main.wait_event(factored.pop(s))
        nxt = s + 1
        rest_lo = nxt
        if lookahead and nxt < nsb and nxt % ws == rank:
            # look-ahead: bring super-column s+1 up to date with panel s, then factor it on the
            # chain stream while the rest of step s (trailing update, TRTRI step) runs on main
            E.N.check(L.gp2d_dfact_update(P(A), n, n, s, P(buf), ws, rank, nxt, nxt + 1, sh), "gp2d_dfact_update")
            ev = torch.cuda.Event()
            ev.record(main)
            crit.wait_event(ev)
            wait_done(crit, nxt - 2)   # its panel buffer was last read by step nxt − 2
            factor(nxt, crit)
            rest_lo = nxt + 1
        if inv is not main:   # the TRTRI step needs panel s (and the owner's factor of it) only
            ev = torch.cuda.Event()
            ev.record(main)
            inv.wait_event(ev)
        E.N.check(L.gp2d_dfact_update(P(A), n, n, s, P(buf), ws, rank, rest_lo, nsb, sh), "gp2d_dfact_update")
        if not lookahead and nxt < nsb and nxt % ws == rank:
            factor(nxt, main)
        with torch.cuda.stream(inv):
            E.N.check(L.gp2d_dfact_invstep(P(A), n, n, s, P(buf), ws, rank, P(work), wbytes, E._stream_handle(dev)),
                      "gp2d_dfact_invstep")
        evs = []
        for st in ([main, inv] if inv is not main else [main]):
            ev = torch.cuda.Event()
            ev.record(st)
            evs.append(ev)
        done[s] = evs
    main.wait_stream(crit)   # the chain's last panel (and its info word) before the gather
    main.wait_stream(inv)
    del panels, work
    t1 = time.perf_counter()
    if not _solo(ws) and emulate is None:
        _allgather_w_columns(A, n, ws, rank, dev, comm)
        allreduce_first_failure(info)
    if multi:
        # W = L⁻¹ is zero above each super-block's diagonal block: the owned columns were reset
        # to the identity block column (zeros above), the gathered ones carry stale K_y there
        for t in range(nsb):
            if t % ws != rank and t > 0:
                A[:t * SB, t * SB:(t + 1) * SB].zero_()
    t2 = time.perf_counter()
    Y = E._pad_obs(y, ntr, npad, bd, dev, perm)
    alpha = _alpha_owned(A, n, Y, ws, rank, nsb, SB, dev, collective=not _solo(ws) and emulate is None, comm=comm)
    gp = E.GPFit(kernel=spec, noise=float(noise), x=X, n_train=ntr, n_pad=npad, W=A, alpha=alpha, device=dev,
                 y=Y, perm=perm)
    if emulate is not None:
        return gp
    E._raise_fit_errors(int(info.item()), None)
    if variance == "ozaki":   # every rank holds the whole W: each applies the guard itself (same bits)
        E.ozaki_prepare_guarded(gp, float(noise + jitter))
    if stats is not None:
        stats.update(host_factor_s=t1 - t0, host_gather_s=t2 - t1)
    return gp


def _alpha_owned(A: torch.Tensor, n: int, Y: torch.Tensor, ws: int, rank: int, nsb: int, SB: int, dev,
                 collective: bool, comm: dict | None = None) -> torch.Tensor:
    """α = Wᵀ(W y) from this rank's super-columns only (gp2d_dfact_zpart / _zsum / _alpha_blocks):
    z = Σ_t W[:, t]·y[t] over the super-columns in t order (each rank's partials gathered), then
    α[t] = W[:, t]ᵀ·z for the owned t, gathered.  Every piece is computed from one super-column
    in a fixed order, so any world size gives the bits of one rank; each rank reads 1/P of W
    twice instead of all of it."""
    L = E.N.lib()
    P, sh = E._ptr, E._stream_handle(dev)
    mine = _owned_blocks(nsb, ws, rank) if (collective or ws > 1) else list(range(nsb))
    cap = (nsb + ws - 1) // ws if (collective or ws > 1) else nsb
    dt = ws if (collective or ws > 1) else 1
    zp = torch.zeros((cap, n), dtype=torch.float64, device=dev)
    if mine:
        E.N.check(L.gp2d_dfact_zpart(P(A), n, n, mine[0], dt, len(mine), P(Y), P(zp), sh), "gp2d_dfact_zpart")
    if collective:
        allz = torch.empty((ws, cap, n), dtype=torch.float64, device=dev)
        with _timed(comm, "alpha_allgather", True, 8 * zp.numel(), ws, recv=8 * zp.numel() * (ws - 1), device=dev):
            _all_gather(allz, zp, ws)
        order = _cyclic_order(nsb, ws, cap, dev)
        parts = torch.empty((nsb, n), dtype=torch.float64, device=dev)
        E.N.check(L.gp2d_gather_rows(P(allz), P(order), nsb, n, P(parts), sh), "gp2d_gather_rows")
    elif ws > 1:   # emulate: this rank's partials only (the emulated factor is not W either)
        parts = zp[:len(mine)].contiguous()
    else:
        parts = zp
    z = torch.empty(n, dtype=torch.float64, device=dev)
    E.N.check(L.gp2d_dfact_zsum(P(parts), parts.shape[0], n, P(z), sh), "gp2d_dfact_zsum")
    ab = torch.zeros((cap, SB), dtype=torch.float64, device=dev)
    if mine:
        wb = int(L.gp2d_dfact_alpha_workspace(n, len(mine)))
        work = torch.empty(wb // 8 + 1, dtype=torch.float64, device=dev)
        E.N.check(L.gp2d_dfact_alpha_blocks(P(A), n, n, mine[0], dt, len(mine), P(z), P(ab), P(work), wb, sh),
                  "gp2d_dfact_alpha_blocks")
    if not collective:
        if ws > 1:
            return torch.zeros(n, dtype=torch.float64, device=dev)
        return ab.reshape(-1)[:n].contiguous()
    alla = torch.empty((ws, cap, SB), dtype=torch.float64, device=dev)
    with _timed(comm, "alpha_allgather", True, 8 * ab.numel(), ws, recv=8 * ab.numel() * (ws - 1), device=dev):
        _all_gather(alla, ab, ws)
    alpha = torch.empty(nsb * SB, dtype=torch.float64, device=dev)
    E.N.check(L.gp2d_gather_rows(P(alla), P(_cyclic_order(nsb, ws, cap, dev)), nsb, SB, P(alpha), sh),
              "gp2d_gather_rows")
    return alpha


def _cyclic_order(nsb: int, ws: int, cap: int, dev) -> torch.Tensor:
    """Row of the all-gathered (rank, slot) buffer that holds super-column t, for t < nsb (rank
    t mod ws, its slot t div ws) — the block-cyclic deal back in column order."""
    return torch.as_tensor(np.array([(t % ws) * cap + t // ws for t in range(nsb)], dtype=np.int64), device=dev)


def _all_gather(out: torch.Tensor, t: torch.Tensor, ws: int):
    C.all_gather_into(out, t, ws)


def allreduce_first_failure(info: torch.Tensor) -> torch.Tensor:
    """All-reduce LAPACK-style info words (0 = success, k > 0 = leading minor k not positive)
    to the FIRST failing minor over the ranks, in place.  A non-SPD panel's NaNs spread into
    later panels that other ranks own, so a MAX would report the last failure and the message
    would change with the world size; 0 → INT32_MAX, MIN, back gives the one-rank answer."""
    if info.is_cuda:
        flip = lambda: E.N.check(E.N.lib().gp2d_status_flip(E._ptr(info), info.numel(),   # noqa: E731
                                                            E._stream_handle(info.device)), "gp2d_status_flip")
    else:   # the gloo CPU tests of the communication logic
        big = torch.iinfo(torch.int32).max

        def flip():
            z, b = info == 0, info == big
            info[z] = big
            info[b] = 0
    flip()                                 # 0 ↔ INT32_MAX, so MIN finds the first failure
    C.all_reduce(info, "min")
    flip()
    return info


def _allgather_w_columns(A: torch.Tensor, n: int, ws: int, rank: int, dev, comm: dict | None = None):
    """Every rank's W super-columns to every rank: super-column t travels as its rows
    [SB·t, n) (the part below the diagonal block's top; W is zero above it)."""
    L = E.N.lib()
    SB = super_block()
    P, sh = E._ptr, E._stream_handle(dev)
    nsb = n // SB
    sizes = [sum((n - t * SB) * SB for t in _owned_blocks(nsb, ws, r)) for r in range(ws)]
    cap = max(sizes)
    send = torch.empty(cap, dtype=torch.float64, device=dev)
    off = 0
    for t in _owned_blocks(nsb, ws, rank):
        rows = n - t * SB
        E.N.check(L.gp2d_copy2d(P(send[off:]), SB, P(A[t * SB:, t * SB:]), n, rows, SB, sh), "gp2d_copy2d")
        off += rows * SB
    recv = torch.empty(ws * cap, dtype=torch.float64, device=dev)
    with _timed(comm, "w_allgather", True, 8 * sizes[rank], ws, recv=8 * (sum(sizes) - sizes[rank]), device=dev):
        C.all_gather_into(recv, send, ws)
    for r in range(ws):
        if r == rank:
            continue
        off = r * cap
        for t in _owned_blocks(nsb, ws, r):
            rows = n - t * SB
            E.N.check(L.gp2d_copy2d(P(A[t * SB:, t * SB:]), n, P(recv[off:]), SB, rows, SB, sh), "gp2d_copy2d")
            off += rows * SB


def krige_jobs_sharded(jobs, variance: str = "ozaki", chunk: int = 8192, var_mode: str = "latent",
                       compute_var: bool = True, jitter: float = 0.0, device=None, align: int = 64,
                       stats: dict | None = None, comm: dict | None = None):
    """A stream of independent kriging jobs (kernel, x, y, noise, xg) — the reference's
    runKrig.py sweep / per-window krig.kriging calls — spread over all ranks: job j is FITTED
    by rank j mod world only (round robin, on a side stream, up to one job per rank ahead),
    its factor W = L⁻¹, α and training points are broadcast from that rank (broadcast_fit,
    RCCL under the 'nccl' backend), and EVERY rank predicts its tile-aligned shard of job j's
    grid (predict_shard).  Yields (lo, hi, mean, var) per job, in job order, on every rank;
    the shards are bit-identical to one process's fit + predict (fixed-order reductions).

    Per job a rank does 1/world of a fit plus 1/world of the predict, so for a stream of jobs
    the fit — the serial part of a one-job multi-GPU predict — is divided like the grid
    (DESIGN.md §5).  Every rank must pass the same job sequence: x with the job's point count
    on every rank (its size sizes the broadcast), while the values of x and y are read on the
    owner only; x may be a tensor, an array or a nested list.  A non-SPD K_y raises
    numpy.linalg.LinAlgError on every rank at that job.  Nothing is
    read ahead before the first next(); `stats` counts the fits this rank issues (with their
    host time stamps, engine.note_fit_issued); `comm` collects the factor broadcasts' bytes and
    HIP-event times (comm_summary).  A receiving rank of the ozaki engine keeps only the INT8
    planes of a job's factor (broadcast_fit planes_only)."""
    ws, rank = world()
    dev = E._require_device(device)
    if _solo(ws):   # one rank: the single-GPU pipelined form (the next fit under this predict)
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
    fit_stream = E.side_stream(dev)
    comm_stream = E.side_stream(dev)   # broadcasts + the receivers' int8 preparation
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
        """Job idx's factor from its owner, on the comm stream: (gp, ready event); the fit's
        status travels on the device (gp.check() raises on every rank when the job is yielded),
        so no rank waits on the host for another rank's fit."""
        spec, x, _, noise, _ = job
        owner = idx % ws
        gp, err = None, None
        if owner == rank:
            gp, err, ev = own.pop(idx)
            if gp is not None:
                comm_stream.wait_event(ev)
                gp.record_stream(comm_stream)   # its status word is the factor's info (the owner's
                #                                 own check() also raises a preparation error)
            else:
                comm_stream.wait_stream(main)
        ntr = E._point_count(x, spec.input_dim)   # every rank passes x with the job's point count
        npad, n = E.fit_layout(spec, ntr, variance)
        with torch.cuda.stream(comm_stream):
            gp = broadcast_fit(gp, spec, noise, x, dev, src=owner, error=err, layout=(n, ntr, npad),
                               planes_only=float(noise + jitter) if variance == "ozaki" else None, comm=comm)
            if variance == "ozaki" and "ozaki" not in gp.extra:
                E.ozaki_prepare(gp, diag_add=float(noise + jitter))   # a-priori moduli count
            ready = torch.cuda.Event()
            ready.record(comm_stream)
        return gp, ready

    refill()
    if not window:
        return
    cur = receive(*window[0])
    pred = None
    while window:
        idx, (spec, x, y, noise, xg) = window.popleft()
        gp, ready = cur
        # this job's status (broadcast with its factor): raises on every rank, and applies the
        # owner's accuracy-guard statistics on every rank (the same decision everywhere) before
        # the predict is queued; the broadcast ran under the previous job's predict
        gp.check()
        E.note_guard(stats, gp)
        main.wait_event(ready)
        gp.ready_on(main)
        gp.record_stream(main)
        if pred is None or not pred.fits(gp):
            pred = E.Predictor(gp, chunk)
        pred.gp = gp
        out = predict_shard(pred, E._as_points(xg, spec.input_dim, dev), var_mode=var_mode,
                            compute_var=compute_var, align=align)
        refill()
        # the next job's factor travels while this predict runs
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
    if _solo(ws):
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
        allp = torch.empty(ws * buf.numel(), dtype=buf.dtype, device=buf.device)
        C.all_gather_into(allp, buf, ws)
        parts = allp.view(ws, -1).unbind(0)
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
