"""Job-stream timeline probe (dev tool): config B (df, N_train = 1024, 128² grid) through
engine.krige_jobs, with host time stamps of each fit enqueue, predict enqueue and check, and GPU
completion times of each fit (event on its side stream) and predict (event on the main stream),
relative to one base event.  usage: python tools/probe_jobs_b.py [fits_ahead] [pipeline]"""
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

ahead = int(sys.argv[1]) if len(sys.argv) > 1 else 1
NTR, G = 1024, 128
x1, x2, u, v = D.synthetic_tracks(NTR, seed=2016)
xt = torch.tensor(np.stack([x1, x2], 1), device="cuda")
yt = torch.tensor(np.concatenate([u, v]), device="cuda")
xg = torch.tensor(D.bbox_grid(x1, x2, G, pad=5.0)[2], device="cuda")
spec = E.KernelSpec(kind="df", l_df=5.0)
job = (spec, xt, yt, 0.0025, xg)
for _ in E.krige_jobs(itertools.repeat(job, 5), fits_ahead=ahead):
    pass
torch.cuda.synchronize()

log = []
orig_fit, orig_call, orig_check = E.fit, E.Predictor.__call__, E.GPFit.check
base = torch.cuda.Event(enable_timing=True)


def fit(*a, **k):
    t = time.perf_counter()
    gp = orig_fit(*a, **k)
    ev = torch.cuda.Event(enable_timing=True)
    ev.record(torch.cuda.current_stream())
    log.append(("fit", t, time.perf_counter(), ev))
    return gp


def call(self, *a, **k):
    t = time.perf_counter()
    out = orig_call(self, *a, **k)
    ev = torch.cuda.Event(enable_timing=True)
    ev.record(torch.cuda.current_stream())
    log.append(("pred", t, time.perf_counter(), ev))
    return out


def check(self):
    t = time.perf_counter()
    r = orig_check(self)
    log.append(("check", t, time.perf_counter(), None))
    return r


E.fit, E.Predictor.__call__, E.GPFit.check = fit, call, check
ms0 = torch.cuda.memory_stats()
base.record()
t0 = time.perf_counter()
for _ in E.krige_jobs(itertools.repeat(job, 12), fits_ahead=ahead):
    pass
torch.cuda.synchronize()
t1 = time.perf_counter()
ms1 = torch.cuda.memory_stats()
print(f"fits_ahead {ahead}: {1e3 * (t1 - t0) / 12:.2f} ms per job; alloc retries "
      f"{ms1.get('num_alloc_retries', 0) - ms0.get('num_alloc_retries', 0)}, device allocs "
      f"{ms1.get('num_device_alloc', 0) - ms0.get('num_device_alloc', 0)}, device frees "
      f"{ms1.get('num_device_free', 0) - ms0.get('num_device_free', 0)}")
for kind, a, b, ev in log[:24]:
    gpu = f"gpu done {base.elapsed_time(ev):8.2f}" if ev is not None else ""
    print(f"  {kind:5s} host {1e3 * (a - t0):8.2f} .. {1e3 * (b - t0):8.2f}  {gpu}")
