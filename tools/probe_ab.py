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


def morton(p, bits=16):
    q = ((p - p.min(0)) / (p.max(0) - p.min(0) + 1e-9) * (2 ** bits - 1)).astype(np.uint64)
    code = np.zeros(len(p), np.uint64)
    for b in range(bits):
        code |= ((q[:, 0] >> np.uint64(b)) & np.uint64(1)) << np.uint64(2 * b)
        code |= ((q[:, 1] >> np.uint64(b)) & np.uint64(1)) << np.uint64(2 * b + 1)
    return code


X = np.stack([x1, x2], 1)
perm = np.argsort(morton(X), kind="stable")
xs = torch.tensor(X[perm], device="cuda")
ys = torch.tensor(np.concatenate([u[perm], v[perm]]), device="cuda")
G = xg.cpu().numpy().reshape(256, 256, 2)
patch = torch.tensor(G.reshape(16, 16, 16, 16, 2).transpose(0, 2, 1, 3, 4).reshape(-1, 2).copy(), device="cuda")
inputs = {"plain": (xt, yt, xg), "sorted": (xs, ys, xg), "sorted+patch": (xs, ys, patch)}
arms = {k: orig for k in inputs}
pred = {}
mean = torch.empty(2 * xg.shape[0], dtype=torch.float64, device="cuda")
var = torch.empty_like(mean)


cur = {"k": "plain"}


def step():
    a, b, g = inputs[cur["k"]]
    gp = E.fit(ks, a, b, noise=0.0025, variance="ozaki")
    p = pred.get("p")
    if p is None:
        p = pred["p"] = E.Predictor(gp, 8192)
    p.gp = gp
    p(g, out=(mean, var))


res = {k: [] for k in arms}
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
for r in range(rounds):
    for name, fn in arms.items():
        cur["k"] = name
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        res[name].append(1e3 * (time.perf_counter() - t0) / 3)
for name, v in res.items():
    print(f"{name}: median {np.median(v):.2f} ms  min {np.min(v):.2f}  all {np.round(v, 2).tolist()}")
