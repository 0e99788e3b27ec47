"""The library's own RCCL communicator (include/gp2d.h gp2d_comm_*).

The multi-GPU data path — a job's packed factor W = L⁻¹ + α + training points
(distributed.broadcast_fit), the distributed factor's panels, its W column and α all-gathers,
its status all-reduce and a sweep's result all-reduce — goes through RCCL calls the library
makes itself (gp2d_bcast / gp2d_allgather / gp2d_allreduce / gp2d_sendrecv) on a communicator
it creates (gp2d_comm_init), on the caller's current HIP stream: no torch.distributed
collective and no extra stream hop on the data path.  torch.distributed stays for the host
rendezvous only: its TCP store carries the 128-byte ncclUniqueId from rank 0 to the others,
and its gloo backend runs the CPU / shared-card rehearsals (RCCL refuses two ranks on one
device), for which every function here falls back to the torch.distributed collective.

The reference is single-process; its parallelism is the job array (runKrig.py:7,14-17) and the
per-slice predict (krig.py:541-557).
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from . import _native as N

_COMMS: dict = {}   # (world size, rank, device index) → Communicator
_SEQ = [0]          # communicators created so far (the store key of the next one)


class Communicator:
    """An RCCL communicator of `ws` ranks made by the library (collective: every rank of the
    default process group constructs it, in the same order)."""

    def __init__(self, ws: int, rank: int, device: torch.device, store=None):
        L = N.lib()
        self.ws, self.rank, self.device = int(ws), int(rank), torch.device(device)
        nbytes = int(L.gp2d_comm_id_bytes())
        key = f"gp2d_comm/{_SEQ[0]}"
        _SEQ[0] += 1
        if store is None:
            store = dist.distributed_c10d._get_default_store()
        if self.rank == 0:
            uid = ctypes.create_string_buffer(nbytes)
            N.check(L.gp2d_comm_unique_id(uid), "gp2d_comm_unique_id")
            store.set(key, uid.raw)
        raw = store.get(key)   # blocks until rank 0 has published it
        uid = ctypes.create_string_buffer(bytes(raw), nbytes)
        h = ctypes.c_void_p()
        N.check(L.gp2d_comm_init(ctypes.byref(h), self.ws, uid, self.rank, self.device.index or 0), "gp2d_comm_init")
        self.handle = h
        self.calls = {}   # collective → calls made through this communicator (tests, the bench line)
        n, r = ctypes.c_int(), ctypes.c_int()
        N.check(L.gp2d_comm_size(h, ctypes.byref(n), ctypes.byref(r)), "gp2d_comm_size")
        if (n.value, r.value) != (self.ws, self.rank):
            raise RuntimeError(f"gp2d communicator reports ({n.value}, {r.value}), expected ({self.ws}, {self.rank})")

    def _count(self, what: str):
        self.calls[what] = self.calls.get(what, 0) + 1

    def _stream(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        return ctypes.c_void_p(s.cuda_stream)

    def broadcast(self, t: torch.Tensor, root: int, stream=None):
        """In place, from `root`, on the current stream (gp2d_bcast)."""
        _dense(t)
        self._count("broadcast")
        N.check(N.lib().gp2d_bcast(ctypes.c_void_p(t.data_ptr()), t.numel() * t.element_size(), int(root),
                                   self.handle, self._stream(stream)), "gp2d_bcast")

    def all_gather_into(self, out: torch.Tensor, t: torch.Tensor, stream=None):
        """out = the ranks' `t` in rank order (gp2d_allgather); out holds ws·t.numel() elements."""
        _dense(t)
        _dense(out)
        nb = t.numel() * t.element_size()
        if out.numel() * out.element_size() != self.ws * nb:
            raise ValueError("all_gather_into: out must hold world_size times the input")
        self._count("all_gather")
        N.check(N.lib().gp2d_allgather(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(out.data_ptr()), nb,
                                       self.handle, self._stream(stream)), "gp2d_allgather")

    def all_reduce(self, t: torch.Tensor, op: str = "sum", stream=None):
        """In place over the ranks; int32 / float64, op 'sum' | 'max' | 'min' (gp2d_allreduce)."""
        _dense(t)
        dt = {torch.int32: N.COMM_INT32, torch.float64: N.COMM_FLOAT64}.get(t.dtype)
        if dt is None:
            raise TypeError(f"all_reduce: int32 or float64 only, got {t.dtype}")
        o = {"sum": N.COMM_SUM, "max": N.COMM_MAX, "min": N.COMM_MIN}[op]
        self._count("all_reduce")
        N.check(N.lib().gp2d_allreduce(ctypes.c_void_p(t.data_ptr()), t.numel(), dt, o, self.handle,
                                       self._stream(stream)), "gp2d_allreduce")

    def sendrecv(self, send: torch.Tensor | None, send_peer: int, recv: torch.Tensor | None, recv_peer: int,
                 stream=None):
        """One grouped send (→ send_peer) + receive (← recv_peer) of the same byte count
        (gp2d_sendrecv); a rank may name itself."""
        ref = send if send is not None else recv
        nb = ref.numel() * ref.element_size()
        for t in (send, recv):
            if t is not None:
                _dense(t)
                if t.numel() * t.element_size() != nb:
                    raise ValueError("sendrecv: send and recv must have the same byte count")
        self._count("sendrecv")
        N.check(N.lib().gp2d_sendrecv(None if send is None else ctypes.c_void_p(send.data_ptr()), int(send_peer),
                                      None if recv is None else ctypes.c_void_p(recv.data_ptr()), int(recv_peer),
                                      nb, self.handle, self._stream(stream)), "gp2d_sendrecv")

    def destroy(self):
        if self.handle:
            N.check(N.lib().gp2d_comm_destroy(self.handle), "gp2d_comm_destroy")
            self.handle = None


def _dense(t: torch.Tensor):
    if not (t.is_cuda and t.is_contiguous()):
        raise ValueError("the library's RCCL calls take contiguous device tensors")


def get(device=None) -> Communicator | None:
    """The library communicator over the default process group's ranks on `device`, created on
    first use (collective), when the group runs on RCCL ('nccl' backend) and the device is a HIP
    device; None otherwise (gloo rehearsals: callers use torch.distributed)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_backend() != "nccl":
        return None
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.type != "cuda":
        return None
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    key = (dist.get_world_size(), dist.get_rank(), dev.index)
    c = _COMMS.get(key)
    if c is None:
        c = Communicator(key[0], key[1], dev)
        _COMMS[key] = c
    return c


def shutdown():
    """Destroy the library's communicators (call before dist.destroy_process_group)."""
    for c in list(_COMMS.values()):
        c.destroy()
    _COMMS.clear()


# --------------------------------------------------------------- the data path's collectives
# Device tensors on an RCCL process group go through the library's communicator on the current
# stream; anything else (gloo, CPU tensors) through torch.distributed.

def broadcast(t: torch.Tensor, src: int):
    c = get(t.device) if t.is_cuda else None
    if c is None:
        dist.broadcast(t, src)
    else:
        c.broadcast(t, src)


def all_gather_into(out: torch.Tensor, t: torch.Tensor, ws: int):
    """out (ws × t's elements, rank order) = every rank's t."""
    c = get(t.device) if t.is_cuda else None
    if c is not None:
        c.all_gather_into(out, t)
    elif dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, t)
    else:   # gloo (the CPU / shared-card rehearsals)
        dist.all_gather(list(out.reshape(ws, -1).unbind(0)), t.reshape(-1))


def all_reduce(t: torch.Tensor, op: str = "sum"):
    c = get(t.device) if t.is_cuda else None
    if c is None:
        dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op])
    else:
        c.all_reduce(t, op)
