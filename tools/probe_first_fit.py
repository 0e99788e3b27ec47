"""Which first action of a process puts engine.krige_jobs in its fast state (dev tool, r06).

bench.py's job stream runs 53 ms per headline job when ONE unpipelined fit + predict ran before
it in the process, 56.5 ms when the first fit of the process comes from krige_jobs itself
(`tools/runs/r06_benchstate2.sh`); the state is sticky for the process.  Run once per first action
(a fresh process each), then time 40 jobs of a fresh krige_jobs stream:
  none        — krige_jobs straight away;
  fit_nocheck — engine.fit(check=False) on the current (null) stream, then check() (bench.py's
                unpipelined job), no predict;
  fit_check   — engine.fit(check=True) on the current stream;
  fit_side    — engine.fit(check=False) issued from a side stream (krige_jobs' first fit);
  job         — bench.py's unpipelined job: fit(check=False), check(), Predictor, predict;
  potrf_tiny  — one gp2d_potrf of a 128×128 identity from the current stream (the library's
                internal factor streams are created there);
  pool_then_potrf — a kernel on one of torch's high-priority pool streams first, then the raw
                gp2d_potrf (no engine call: nothing warms the factor streams before the pool
                stream's first use).
The engine's own entry points warm the factor streams first (engine.warm_streams) since round 6,
so `none` and `fit_side` measure that fix.
usage: python tools/probe_first_fit.py ACTION [jobs]"""
import ctypes
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

ACTION = sys.argv[1]
JOBS = int(sys.argv[2]) if len(sys.argv) > 2 else 40
dev = torch.device("cuda", 0)
x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
xt = torch.tensor(np.stack([x1, x2], 1), device=dev)
yt = torch.tensor(np.concatenate([u, v]), device=dev)
xg = torch.tensor(D.bbox_grid(x1, x2, 256, pad=5.0)[2], device=dev)
spec = E.KernelSpec(kind="df", l_df=5.0)
job = (spec, xt, yt, 0.0025, xg)
m = xg.shape[0]
torch.cuda.synchronize()
if ACTION == "fit_nocheck":
    E.fit(spec, xt, yt, 0.0025, variance="ozaki", check=False).check()
elif ACTION == "fit_check":
    E.fit(spec, xt, yt, 0.0025, variance="ozaki")
elif ACTION == "fit_side":
    s = E.side_stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        gp = E.fit(spec, xt, yt, 0.0025, variance="ozaki", check=False)
    gp.check()
elif ACTION == "job":
    gp = E.fit(spec, xt, yt, 0.0025, variance="ozaki", check=False)
    gp.check()
    gp.ready_on(torch.cuda.current_stream(dev))
    E.Predictor(gp, 8192)(xg)
elif ACTION == "potrf_tiny":
    L = E.N.lib()
    A = torch.eye(128, dtype=torch.float64, device=dev)
    dinv = torch.empty((1, 128, 128), dtype=torch.float64, device=dev)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    E.N.check(L.gp2d_potrf(E._ptr(A), 128, 128, E._ptr(dinv), E._ptr(info), None, 0,
                           E._stream_handle(dev)), "gp2d_potrf")
elif ACTION == "pool_then_potrf":
    s = torch.cuda.Stream(dev, priority=-1)
    with torch.cuda.stream(s):
        torch.ones(16, device=dev).add_(1)
    torch.cuda.synchronize()
    L = E.N.lib()
    A = torch.eye(128, dtype=torch.float64, device=dev)
    dinv = torch.empty((1, 128, 128), dtype=torch.float64, device=dev)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    E.N.check(L.gp2d_potrf(E._ptr(A), 128, 128, E._ptr(dinv), E._ptr(info), None, 0,
                           E._stream_handle(dev)), "gp2d_potrf")
elif ACTION != "none":
    sys.exit(f"unknown action {ACTION}")
torch.cuda.synchronize()
for _ in E.krige_jobs(itertools.repeat(job, 2), variance="ozaki"):
    pass
torch.cuda.synchronize()
E.timing_enable(True)
E.timing_read()
t0 = time.perf_counter()
for _ in E.krige_jobs(itertools.repeat(job, JOBS), variance="ozaki"):
    pass
torch.cuda.synchronize()
dt = time.perf_counter() - t0
kms, kl, _ = E.timing_read()
print(json.dumps({"first_action": ACTION, "jobs": JOBS, "ms_per_job": 1e3 * dt / JOBS, "points_per_s": m * JOBS / dt,
                  "igemm_avg_launch_ms": kms / kl / 12 if kl else None}), flush=True)
