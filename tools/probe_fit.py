"""Fit-stage probe (dev tool): seeded div-free fit (Ozaki prepare included), inputs resident
on the device; fused factor+inverse (gp2d_potrf_inv) vs the two-call potrf + trtri.
usage: python tools/probe_fit.py [N_train ...]"""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gp2d import data as D  # noqa: E402
from gp2d import engine as E  # noqa: E402

for ntr in [int(a) for a in sys.argv[1:]] or [4096]:
    x1, x2, u, v = D.synthetic_tracks(ntr, seed=2016)
    x = torch.tensor(np.stack([x1, x2], 1), device="cuda")
    y = torch.tensor(np.concatenate([u, v]), device="cuda")
    ks = E.KernelSpec(kind="df", l_df=5.0)
    reps = 6 if ntr <= 4096 else 3
    for fused in (True, False, True):
        E.FUSED_INVERSE = fused
        ts = []
        for r in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gp = E.fit(ks, x, y, noise=0.0025, variance="ozaki")
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            del gp
        print(f"fit N={ntr} fused={fused}: median {1e3 * np.median(ts[1:]):.2f} ms "
              f"(min {1e3 * min(ts[1:]):.2f})", flush=True)
