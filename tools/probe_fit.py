"""Fit-stage probe (dev tool): N=4096 div-free, Ozaki prepare included; run under
rocprofv3 --kernel-trace --stats for the per-kernel split of the fit."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np, torch
from gp2d import engine as E
ntr = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
rng = np.random.default_rng(2016)
x = np.stack([rng.uniform(0, 60, ntr), rng.uniform(0, 45, ntr)], 1)
y = rng.normal(0, 0.3, 2 * ntr)
ks = E.KernelSpec(kind="df", l_df=5.0)
for r in range(4):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    gp = E.fit(ks, x, y, noise=0.0025, variance="ozaki")
    torch.cuda.synchronize()
    print(f"fit N={ntr}: {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
