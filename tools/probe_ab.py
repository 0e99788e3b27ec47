"""Interleaved A/B of the bench step in ONE process (dev tool): async (a-priori moduli)
vs data-driven (synchronising) Ozaki preparation.  usage: python tools/probe_ab.py [rounds]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np, torch
from gp2d import data as D, engine as E

x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
xt = torch.tensor(np.stack([x1, x2], 1), device="cuda")
yt = torch.tensor(np.concatenate([u, v]), device="cuda")
_, _, xg = D.bbox_grid(x1, x2, 256, pad=5.0)
xg = torch.tensor(xg, device="cuda")
ks = E.KernelSpec(kind="df", l_df=5.0)
orig = E.ozaki_prepare
arms = {"async": orig, "sync": lambda gp, diag_add=None: orig(gp)}
pred = {}
mean = torch.empty(2 * xg.shape[0], dtype=torch.float64, device="cuda")
var = torch.empty_like(mean)


def step():
    gp = E.fit(ks, xt, yt, noise=0.0025, variance="ozaki")
    p = pred.get("p")
    if p is None:
        p = pred["p"] = E.Predictor(gp, 8192)
    p.gp = gp
    p(xg, out=(mean, var))


res = {k: [] for k in arms}
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
for r in range(rounds):
    for name, fn in arms.items():
        E.ozaki_prepare = fn
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        res[name].append(1e3 * (time.perf_counter() - t0) / 3)
for name, v in res.items():
    print(f"{name}: median {np.median(v):.2f} ms  min {np.min(v):.2f}  all {np.round(v, 2).tolist()}")
