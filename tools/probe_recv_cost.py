"""What a received factor costs a running predict, on ONE GPU (dev tool).

At N > 1 every rank receives most jobs' packed factor (268 MB at the headline, 7/8 of the jobs
at N = 8) while its int8 predict GEMMs run.  RCCL moves it with its own copy kernels, which need
CU slots the GEMM (one workgroup per CU, 464 of 512 VGPRs) also wants.  Proxy: a one-rank RCCL
communicator made by the library (gp2d/comm.py), and once per job a grouped ncclSend + ncclRecv
of MB megabytes to itself (gp2d_sendrecv: RCCL's copy kernel) on a third stream, under the
headline job stream (engine.krige_jobs, df, N_train = 4096, 256² grid).  Variants:
  base      — the job stream alone;
  copy      — plus the per-job copy on a high-priority side stream (as the comm stream of
              distributed.krige_jobs_sharded);
  mask<R>   — the predict stream restricted to all CUs but R (R/8 per XCD), no copy;
  maskcopy<R> — the same, with the copy on a stream restricted to those R CUs.
Per variant: points/s, ms per job, the int8 GEMM's average launch (HIP events on its stream), the
copy's HIP-event ms per job and rate.  One JSON line per variant.
usage: python tools/probe_recv_cost.py [--jobs 40] [--mb 235] [--mask 16,32] [--order A,B,...]"""
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
from gp2d import engine as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--jobs", type=int, default=40)
ap.add_argument("--mb", type=float, default=235.0)
ap.add_argument("--mask", default="16,32")
ap.add_argument("--order", default=None, help="comma list of variants (default: base,copy,mask*,maskcopy*,base)")
a = ap.parse_args()

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29561", rank=0, world_size=1, device_id=dev)
comm = C.get(dev)
ncu = torch.cuda.get_device_properties(dev).multi_processor_count

x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
xt = torch.tensor(np.stack([x1, x2], 1), device=dev)
yt = torch.tensor(np.concatenate([u, v]), device=dev)
xg = torch.tensor(D.bbox_grid(x1, x2, 256, pad=5.0)[2], device=dev)
spec = E.KernelSpec(kind="df", l_df=5.0)
job = (spec, xt, yt, 0.0025, xg)
m = xg.shape[0]
nbytes = int(a.mb * 1e6) // 16 * 16
src = torch.ones(nbytes // 8, dtype=torch.float64, device=dev)
dst = torch.empty_like(src)
masks = [int(r) for r in a.mask.split(",") if r]
# every variant uses the SAME streams: the job stream's fit side stream (krige_jobs draws one from
# torch's high-priority pool per call, and which pool stream it gets moves its hardware queue —
# tools/probe_stream_pick.py) and the copy's stream are drawn once here
copy_side = E.side_stream(dev)
fit_side = E.side_stream(dev)
E.side_stream = lambda device=None, _s=fit_side: _s


def run(variant, jobs):
    copy = variant == "copy" or variant.startswith("maskcopy")
    R = int(variant[len("maskcopy"):]) if variant.startswith("maskcopy") else (
        int(variant[len("mask"):]) if variant.startswith("mask") else 0)
    keep = []
    if R:
        ps = E.MaskedStream(0, ncu - R, dev)
        keep.append(ps)
        pstream = ps.stream
    else:
        pstream = torch.cuda.current_stream(dev)
    if copy and R:
        cs = E.MaskedStream(ncu - R, R, dev)
        keep.append(cs)
        cstream = cs.stream
    else:
        cstream = copy_side
    evs = []
    with torch.cuda.stream(pstream):
        for _ in E.krige_jobs(itertools.repeat(job, 2), variance="ozaki"):   # warm
            pass
        torch.cuda.synchronize()
        E.timing_enable(True)
        E.timing_read()
        t0 = time.perf_counter()
        for i, _ in enumerate(E.krige_jobs(itertools.repeat(job, jobs), variance="ozaki")):
            if copy:
                if len(evs) >= 2:
                    evs[-2][1].synchronize()   # at most two copies queued
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(cstream)
                comm.sendrecv(src, 0, dst, 0, stream=cstream)
                e1.record(cstream)
                evs.append((e0, e1))
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        kms, kl, _ = E.timing_read()
        E.timing_enable(False)
    copy_ms = [e0.elapsed_time(e1) for e0, e1 in evs]
    out = {"variant": variant, "jobs": jobs, "points_per_s": m * jobs / (t1 - t0), "ms_per_job": 1e3 * (t1 - t0) / jobs,
           "igemm_avg_launch_ms": kms / kl / 12 if kl else None, "masked_cus": R, "cus": ncu,
           "copy_mb": nbytes / 1e6 if copy else 0, "copy_ms_mean": float(np.mean(copy_ms)) if copy_ms else None,
           "copy_gbs": nbytes / 1e9 / (np.mean(copy_ms) * 1e-3) if copy_ms else None}
    print(json.dumps(out), flush=True)
    del keep
    return out


order = a.order.split(",") if a.order else (["base", "copy"] + [f"mask{r}" for r in masks] +
                                            [f"maskcopy{r}" for r in masks] + ["base", "copy"])
for vname in order:
    run(vname, a.jobs)
torch.cuda.synchronize()
C.shutdown()
dist.destroy_process_group()
