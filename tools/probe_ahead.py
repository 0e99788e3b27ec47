"""Probe: K*-ahead (planes) path vs inline ozaki path at the bench size (dev tool)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np, torch
from gp2d import data as D, engine as E

x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
x = np.stack([x1, x2], 1); y = np.concatenate([u, v])
_, _, xg = D.bbox_grid(x1, x2, 128, pad=5.0)
ks = E.KernelSpec(kind="df", l_df=5.0)
for side in (False, True):
    st = torch.cuda.Stream() if side else None
    planes = E.kstar_planes(ks, x, xg, 0.0025, chunk=8192, stream=st)
    gp = E.fit(ks, x, y, noise=0.0025, variance="ozaki")
    torch.cuda.synchronize()
    mu, var = (t.cpu().numpy() for t in E.Predictor(gp, 8192)(xg, planes=planes))
    mi, vi = (t.cpu().numpy() for t in E.Predictor(gp, 8192)(xg))
    mi2, vi2 = (t.cpu().numpy() for t in E.Predictor(gp, 8192)(xg))
    d = np.abs(var - vi)
    print("side", side, "nmod planes", planes.nmod, "fit", gp.extra["ozaki"][2])
    print("  var diff: n=%d max=%.3e rel=%.3e  inline-vs-inline n=%d" % ((d > 0).sum(), d.max(), (d / np.abs(vi)).max(), (vi != vi2).sum()))
    idx = np.nonzero(d)[0]
    print("  first diff idx", idx[:10], "per-chunk counts", np.bincount((idx % 16384) // 8192, minlength=2) if len(idx) else None)
    print("  mean rel", np.abs(mu - mi).max() / np.abs(mi).max())
