"""Why bench.py's timed job stream runs faster after its unpipelined phase (dev tool, r06).

tools/runs/r06_benchstate.sh: the default bench 53.0 ms per job, the same without its 20
unpipelined jobs 56.2 ms (24 pipelined warmup jobs do not replace them).  Each case below times a
fresh engine.krige_jobs stream of the headline job (df, N_train = 4096, 256² grid) after a
different preamble, in one process:
  bare      — nothing before (2 warm jobs);
  predictor — a separate Predictor has predicted the grid once and stays alive (as bench.py's
              pred_cache["p"] does through the timed region);
  ballast   — a plain 4 GB device tensor allocated and kept instead;
  freed     — the predictor / ballast released and the allocator cache emptied;
  unpiped   — 20 fit + predict jobs strictly one after another first (bench.py's reference phase).
One JSON line per case: ms per job and the int8 GEMM's average launch (HIP events).
usage: python tools/probe_alloc_state.py [jobs] [order]"""
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

JOBS = int(sys.argv[1]) if len(sys.argv) > 1 else 40
ORDER = (sys.argv[2] if len(sys.argv) > 2 else "bare,predictor,freed,ballast,freed,unpiped,bare").split(",")
dev = torch.device("cuda", 0)
x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
xt = torch.tensor(np.stack([x1, x2], 1), device=dev)
yt = torch.tensor(np.concatenate([u, v]), device=dev)
xg = torch.tensor(D.bbox_grid(x1, x2, 256, pad=5.0)[2], device=dev)
spec = E.KernelSpec(kind="df", l_df=5.0)
job = (spec, xt, yt, 0.0025, xg)
m = xg.shape[0]
held = []


def stream(k):
    for _ in E.krige_jobs(itertools.repeat(job, k), variance="ozaki"):
        pass


for case in ORDER:
    if case == "predictor":
        gp = E.fit(spec, xt, yt, 0.0025, variance="ozaki")
        pr = E.Predictor(gp, 8192)
        pr(xg)
        held.append(pr)
    elif case == "ballast":
        held.append(torch.empty(4 << 30, dtype=torch.uint8, device=dev))
    elif case == "freed":
        held.clear()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    elif case == "unpiped":
        pr = None
        for _ in range(20):
            gp = E.fit(spec, xt, yt, 0.0025, variance="ozaki")
            pr = E.Predictor(gp, 8192) if pr is None or not pr.fits(gp) else pr
            pr.gp = gp
            pr(xg)
        held.append(pr)
    stream(2)
    torch.cuda.synchronize()
    E.timing_enable(True)
    E.timing_read()
    t0 = time.perf_counter()
    stream(JOBS)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kms, kl, _ = E.timing_read()
    E.timing_enable(False)
    print(json.dumps({"case": case, "jobs": JOBS, "ms_per_job": 1e3 * dt / JOBS, "points_per_s": m * JOBS / dt,
                      "igemm_avg_launch_ms": kms / kl / 12 if kl else None,
                      "allocated_gb": torch.cuda.memory_allocated(dev) / 2**30,
                      "reserved_gb": torch.cuda.memory_reserved(dev) / 2**30}), flush=True)
