"""Accuracy margin of the Ozaki variance engine at bench scale (dev tool):
ozaki vs f64 engine on the full grid, both vs the CPU oracle on a subset."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np, torch
from gp2d import engine as E
from gp2d import data as D
from oracle import gp2d_oracle as O
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
for kind, ratio in (("df", 1.0), ("mixed", 0.5)):
    x1, x2, u, w = D.synthetic_tracks(N)
    x = np.stack([x1, x2], 1); y = np.concatenate([u, w])
    _, _, xg = D.bbox_grid(x1, x2, 256)
    ks = E.KernelSpec(kind=kind, l_df=5.0, l_cf=5.0, ratio=ratio)
    go = E.fit(ks, x, y, 0.0025, variance="ozaki"); gf = E.fit(ks, x, y, 0.0025)
    mo, vo = (t.cpu().numpy() for t in E.predict(go, xg)); mf, vf = (t.cpu().numpy() for t in E.predict(gf, xg))
    sub = np.random.default_rng(0).choice(xg.shape[0], 256, replace=False)
    t0 = time.time()
    mr, vr = O.fit_predict(x, y, xg[sub], kind=kind, l_df=5.0, l_cf=5.0, ratio=ratio, noise=0.0025)
    M = xg.shape[0]; idx = np.concatenate([sub, M + sub])
    def rel(a, b): return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))
    print(f"N={N} {kind}: var ozaki-vs-f64 normwise {rel(vo, vf):.2e} elementwise {np.max(np.abs(vo-vf)/np.abs(vf)):.2e}; "
          f"vs oracle: ozaki {rel(vo[idx], vr):.2e} (elementwise {np.max(np.abs(vo[idx]-vr)/np.abs(vr)):.2e}) "
          f"f64 {rel(vf[idx], vr):.2e}; nmod {go.extra['ozaki'][2]}; mean vs oracle {rel(mo[idx], mr):.2e}; "
          f"var range [{vf.min():.2e},{vf.max():.2e}] ({time.time()-t0:.0f}s oracle)", flush=True)
