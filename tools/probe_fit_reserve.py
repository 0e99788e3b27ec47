"""The fit's critical path on reserved CUs (dev tool, r06): gp2d_factor_reserve(R) before the
first fit confines the factor chain (crit, aux) to R CUs and the trailing SYRK / inverse (bulk,
inv) to the rest; R = 0 is the product default.  Times a lone fit at N_train = 1024 / 4096 (median
of 8) and a 24-job headline job stream (krige_jobs) in the same process.
With FUSED = 1 the fit runs gp2d_potrf_inv (engine.FUSED_INVERSE: the left half of the inverse
and T = L21·W11 on `inv` under the second half of the factorisation); STREAM = 0 skips the job
stream.
usage: python tools/probe_fit_reserve.py R [FUSED] [STREAM]"""
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

R = int(sys.argv[1])
FUSED = int(sys.argv[2]) if len(sys.argv) > 2 else 0
STREAM = int(sys.argv[3]) if len(sys.argv) > 3 else 1
E.FUSED_INVERSE = bool(FUSED)
dev = torch.device("cuda", 0)
prev = E.N.lib().gp2d_factor_reserve(R)
assert prev >= 0, E.N.lib().gp2d_last_error()
out = {"reserve_cus": R, "fused_inverse": FUSED}
for ntr in (1024, 4096):
    E.warm_streams(dev)
    x1, x2, u, v = D.synthetic_tracks(ntr, seed=2016)
    X = torch.tensor(np.stack([x1, x2], 1), device=dev)
    y = torch.tensor(np.concatenate([u, v]), device=dev)
    spec = E.KernelSpec(kind="df", l_df=5.0)
    E.fit(spec, X, y, 0.0025, variance="ozaki")
    ts = []
    for _ in range(8):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        E.fit(spec, X, y, 0.0025, variance="ozaki")
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t0))
    out[f"fit_{ntr}_ms"] = float(np.median(ts))
if not STREAM:
    print(json.dumps(out), flush=True)
    sys.exit(0)
xg = torch.tensor(D.bbox_grid(x1, x2, 256, pad=5.0)[2], device=dev)
job = (spec, X, y, 0.0025, xg)
for _ in E.krige_jobs(itertools.repeat(job, 2)):
    pass
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in E.krige_jobs(itertools.repeat(job, 24)):
    pass
torch.cuda.synchronize()
out["stream_ms_per_job"] = 1e3 * (time.perf_counter() - t0) / 24
print(json.dumps(out), flush=True)
