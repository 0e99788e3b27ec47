"""One rank's share of the N-GPU round-robin job stream, emulated on ONE GPU (dev tool; VERDICT r05
item 1: S(8) ≥ 6 had no measurement, not even a one-GPU proxy).

distributed.krige_jobs_sharded runs UNCHANGED as rank r of P: it fits the jobs j ≡ r (mod P) on its
fit stream (a full fit, under the predict), predicts its 1/P tile-aligned shard of EVERY job's
256² grid, and receives the other P − 1 of every P jobs' factors.  Only the transport is
emulated: a broadcast this rank receives is a grouped RCCL send/recv to itself (gp2d_sendrecv on
the library's one-rank communicator — RCCL's copy kernel moves the real payload bytes on the comm
stream, under the predict) from a payload captured from a real fit of the same job (packed
W = L⁻¹, α, the Morton-ordered points, the status block with the guard's statistics); the
receiver then prepares its int8 planes from the packed payload as in the product.  A broadcast this
rank sends is a no-op (the root's buffer is already in place).  What the emulation cannot show is
the xGMI transfer's own duration (RCCL's ring broadcast holds its copy kernels' CUs for the
transfer; here the copy runs at HBM speed) — bounded separately from the measured copy cost.

The N-GPU job rate this implies is (grid points per job) / (this rank's ms per job): every rank
does the same share, and the stream never waits for a transfer it has a job to overlap with.
One JSON line per (P, r, transport).
usage: python tools/probe_rank_share.py [--jobs 48] [--P 1,2,4,8] [--ranks first,last]"""
import argparse
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gp2d import comm as C  # noqa: E402
from gp2d import data as D  # noqa: E402
from gp2d import distributed as GD  # noqa: E402
from gp2d import engine as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--jobs", type=int, default=48)
ap.add_argument("--P", default="1,2,4,8")
ap.add_argument("--ranks", default="first,last", help="first,last or all")
ap.add_argument("--transport", default="rccl,none")
ap.add_argument("--warm", type=int, default=0, help="warm jobs before each timed stream (default 2·P)")
ap.add_argument("--copy-repeat", type=int, default=1,
                help="RCCL copies per received payload (stretches the copy kernel's residency toward an "
                     "xGMI transfer's duration: 10 ≈ 4 ms per job)")
a = ap.parse_args()

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
E.warm_streams(dev)   # as bench.py: the predict and factor streams bound before RCCL's first use
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29563", rank=0, world_size=1, device_id=dev)
comm = C.get(dev)

x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
xt = torch.tensor(np.stack([x1, x2], 1), device=dev)
yt = torch.tensor(np.concatenate([u, v]), device=dev)
xg = torch.tensor(D.bbox_grid(x1, x2, 256, pad=5.0)[2], device=dev)
spec = E.KernelSpec(kind="df", l_df=5.0)
noise = 0.0025
job = (spec, xt, yt, noise, xg)
m = xg.shape[0]

# the payload a receiving rank gets for this job: from a real fit (the job stream's settings)
gp = E.fit(spec, xt, yt, noise, variance="ozaki", check=False)
gp.check()
n = gp.n
packed = torch.empty(GD._packed_len(n), dtype=torch.float64, device=dev)
GD._pack_lower(gp.W, n, packed, unpack=False)
payload = {}
for t in (packed, gp.alpha, gp.x, gp.extra["status_dev"]):
    payload[(tuple(t.shape), t.dtype)] = t.contiguous().clone()
torch.cuda.synchronize()
del gp

state = {"P": 1, "r": 0, "transport": "rccl", "bytes": 0}
real_world = GD.world


def fake_world():
    return state["P"], state["r"]


def fake_broadcast(t, src):
    if src == state["r"]:
        return                                  # this rank's own factor: nothing arrives
    s = payload[(tuple(t.shape), t.dtype)]
    state["bytes"] += t.numel() * t.element_size()
    if state["transport"] == "rccl":
        for _ in range(a.copy_repeat if t.numel() > 1 << 20 else 1):
            comm.sendrecv(s, 0, t, 0)            # RCCL's copy kernel on the current (comm) stream
    else:
        t.copy_(s)                              # a plain device copy (the transport's cost removed)


GD.world = fake_world
C.broadcast = fake_broadcast


def run(P, r, transport, jobs):
    state.update(P=P, r=r, transport=transport, bytes=0)
    for _ in GD.krige_jobs_sharded(itertools.repeat(job, max(a.warm, 2 * P)), chunk=8192):   # every owner twice
        pass
    torch.cuda.synchronize()
    stats = {}
    state["bytes"] = 0
    t0 = time.perf_counter()
    for _ in GD.krige_jobs_sharded(itertools.repeat(job, jobs), chunk=8192, stats=stats):
        pass
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ms = 1e3 * dt / jobs
    out = {"P": P, "rank": r, "transport": transport if P > 1 else "none (one rank)", "jobs": jobs,
           "copy_repeat": a.copy_repeat,
           "ms_per_job": ms, "implied_points_per_s": m / (ms * 1e-3), "fits_issued": stats.get("fits_issued", 0),
           "received_mb_per_job": state["bytes"] / jobs / 1e6,
           "shard_points": int(np.diff(D.shard_range(m, P, r))[0])}
    print(json.dumps(out), flush=True)
    return out


for P in [int(p) for p in a.P.split(",")]:
    if a.ranks == "all":
        ranks = list(range(P))
    else:
        ranks = sorted({(0 if w == "first" else P - 1 if w == "last" else int(w)) % P for w in a.ranks.split(",")})
    for r in ranks:
        for transport in (a.transport.split(",") if P > 1 else ["none"]):
            run(P, r, transport, a.jobs)
torch.cuda.synchronize()
GD.world = real_world
C.shutdown()
dist.destroy_process_group()
