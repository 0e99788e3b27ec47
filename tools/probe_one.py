"""One N=4096 fit + predict (dev tool for PMC collection)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np, torch
from gp2d import engine as E
from gp2d import data as D
v = sys.argv[1] if len(sys.argv) > 1 else "ozaki"
x1, x2, u, w = D.synthetic_tracks(4096)
_, _, xg = D.bbox_grid(x1, x2, 128)
gp = E.fit(E.KernelSpec(kind="df", l_df=5.0), np.stack([x1, x2], 1), np.concatenate([u, w]), 0.0025, variance=v)
mu, var = E.predict(gp, xg, chunk=8192)
torch.cuda.synchronize()
print("done", float(var.sum()))
