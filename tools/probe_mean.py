"""Mean accuracy of the K*-planes-ahead path (planes made before the fit) against the
inline mean (K*α in fp64) and the CPU oracle, at the bench sizes (dev tool).
usage: python tools/probe_mean.py [H] [C] [D]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np, torch
from gp2d import engine as E
from gp2d import data as D
from oracle import gp2d_oracle as O
CFG = {"H": ("df", 1.0, 4096, 256, 1), "C": ("mixed", 0.5, 4096, 256, 1), "D": ("mixed", 0.5, 16384, 512, 8)}


def rel(a, b): return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


for name in [a for a in sys.argv[1:]] or ["H", "C"]:
    kind, ratio, ntr, g, world = CFG[name]
    x1, x2, u, w = D.synthetic_tracks(ntr, seed=2016)
    x = np.stack([x1, x2], 1); y = np.concatenate([u, w])
    _, _, xg_all = D.bbox_grid(x1, x2, g, pad=5.0)
    lo, hi = D.shard_range(xg_all.shape[0], world, 0)
    xg = xg_all[lo:hi]
    ks = E.KernelSpec(kind=kind, l_df=5.0, l_cf=5.0, ratio=ratio)
    planes = E.kstar_planes(ks, x, xg, 0.0025)
    gp = E.fit(ks, x, y, 0.0025, variance="ozaki")
    pr = E.Predictor(gp)
    ma, va = (t.cpu().numpy() for t in pr(xg, planes=planes))
    mi, vi = (t.cpu().numpy() for t in pr(xg))
    m = xg.shape[0]
    sub = np.random.default_rng(0).choice(m, 256, replace=False)
    mr, vr = O.fit_predict(x, y, xg[sub], kind=kind, l_df=5.0, l_cf=5.0, ratio=ratio, noise=0.0025)
    idx = np.concatenate([sub, m + sub])
    print(f"{name} N={ntr} nmod {gp.extra['ozaki'][2]}/{planes.nmod}: planes-mean vs inline {rel(ma, mi):.2e} "
          f"(elementwise max |d|/max|m| over grid); vs oracle: planes {rel(ma[idx], mr):.2e} inline {rel(mi[idx], mr):.2e}; "
          f"var planes==inline {np.array_equal(va, vi)}; var vs oracle {rel(va[idx], vr):.2e}", flush=True)
    del planes, gp, pr
    torch.cuda.empty_cache()
