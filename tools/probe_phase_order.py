"""Phase-order probe (dev tool): synchronous fit + predict jobs on the
current stream before and after an engine.krige_jobs stream in the same process, with the
fit's host join (fit(check=True) default, gp2d_factor_join) and without it (join=False, the
round-2 behaviour).  usage: python tools/probe_phase_order.py [N_train] [grid]"""
import itertools
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gp2d import data as D  # noqa: E402
from gp2d import engine as E  # noqa: E402

NTR = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
G = int(sys.argv[2]) if len(sys.argv) > 2 else 256
x1, x2, u, v = D.synthetic_tracks(NTR, seed=2016)
xt = torch.tensor(np.stack([x1, x2], 1), device="cuda")
yt = torch.tensor(np.concatenate([u, v]), device="cuda")
xg = torch.tensor(D.bbox_grid(x1, x2, G, pad=5.0)[2], device="cuda")
spec = E.KernelSpec(kind="df", l_df=5.0)
pred = [None]


def sync_jobs(k, join):
    """k jobs as a Krig.fit + predict user runs them: fit(check=True), predict, read back."""
    ts = []
    for _ in range(k):
        t = time.perf_counter()
        gp = E.fit(spec, xt, yt, 0.0025, variance="ozaki", join=join)
        if pred[0] is None or not pred[0].fits(gp):
            pred[0] = E.Predictor(gp, 8192)
        pred[0].gp = gp
        m, var = pred[0](xg)
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t))
    return np.mean(ts[1:]), np.min(ts)


def phase(name, k, join):
    mean, mn = sync_jobs(k, join)
    print(f"  {name:48s} {mean:7.2f} ms per job (min {mn:.2f})", flush=True)


print(f"N_train {NTR}, grid {G}^2")
phase("before krige_jobs, host join (default)", 6, None)
phase("before krige_jobs, no host join", 6, False)
t = time.perf_counter()
for _ in E.krige_jobs(itertools.repeat((spec, xt, yt, 0.0025, xg), 12), variance="ozaki"):
    pass
torch.cuda.synchronize()
print(f"  krige_jobs, 12 jobs: {1e3 * (time.perf_counter() - t) / 12:.2f} ms per job", flush=True)
phase("after krige_jobs, no host join (round 2)", 6, False)
phase("after krige_jobs, host join (default)", 6, None)
phase("after krige_jobs, no host join (again)", 6, False)
