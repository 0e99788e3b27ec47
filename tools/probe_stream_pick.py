"""Which of torch's high-priority pool streams the job stream's fit lands on, and what it costs
(dev tool).  engine.krige_jobs draws its fit side stream from torch's pool (32 high-priority
streams per device, dealt round robin); HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues
per priority level (4 on the box), and streams that share a queue run in order.  For k = 0..7:
draw k pool streams (kept alive), then time a fresh krige_jobs stream of the headline job (df,
N_train = 4096, 256² grid) — its side stream is pool stream (drawn so far) mod 32.  One JSON line
per run, two passes.
usage: python tools/probe_stream_pick.py [jobs]"""
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gp2d import data as D  # noqa: E402
from gp2d import engine as E  # noqa: E402

JOBS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
xt = torch.tensor(np.stack([x1, x2], 1), device=dev)
yt = torch.tensor(np.concatenate([u, v]), device=dev)
xg = torch.tensor(D.bbox_grid(x1, x2, 256, pad=5.0)[2], device=dev)
job = (E.KernelSpec(kind="df", l_df=5.0), xt, yt, 0.0025, xg)
m = xg.shape[0]
drawn = [0]
real_side = E.side_stream
handles = []


def counted(device=None):
    drawn[0] += 1
    s = real_side(device)
    handles.append(s.cuda_stream)
    return s


E.side_stream = counted
keep = []
for _ in E.krige_jobs(itertools.repeat(job, 2), variance="ozaki"):   # warm (draws one)
    pass
torch.cuda.synchronize()
for rep in range(2):
    for k in range(8):
        for _ in range(k):
            keep.append(counted(dev))
        idx = drawn[0]
        t0 = time.perf_counter()
        for _ in E.krige_jobs(itertools.repeat(job, JOBS), variance="ozaki"):
            pass
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"pass": rep, "extra_drawn": k, "pool_index": idx % 32, "pool_index_mod4": idx % 4,
                          "stream": hex(handles[idx]), "ms_per_job": 1e3 * dt / JOBS, "points_per_s": m * JOBS / dt}),
              flush=True)
