"""Ozaki accuracy away from the bench's hyperparameters (dev tool).

For each (ℓ, noise) setting at N_train = 4096 (bench tracks, df kernel, full 256² grid):
the Ozaki engine's variance against the FP64 engine's, elementwise over all 131,072 outputs,
and the fit statistics a conditioning rule could read (max |W|, the latent variance at the
training points σ² − σ⁴·(K_y⁻¹)_ii from W's column norms, the moduli count).
Usage: GP2D_LIB=... python tools/probe_guard.py [l:noise ...]"""
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

settings = [tuple(float(v) for v in a.split(":")) for a in sys.argv[1:]] or \
    [(5.0, 0.0025), (12.0, 1e-3), (2.0, 5e-2), (5.0, 1e-4)]
x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
x = torch.tensor(np.stack([x1, x2], 1), device="cuda")
y = torch.tensor(np.concatenate([u, v]), device="cuda")
_, _, xg = D.bbox_grid(x1, x2, 256, pad=5.0)
g = torch.tensor(xg, device="cuda")
lib = os.path.basename(os.environ.get("GP2D_LIB", "libgp2d.so"))
for l, nz in settings:
    ks = E.KernelSpec(kind="df", l_df=l)
    kss = ks.kdiag()
    t0 = time.time()
    go = E.fit(ks, x, y, nz, variance="ozaki")
    mo, vo = E.predict(go, g)
    W = go.W
    wmax = float(W.abs().max())
    rowmax = W.abs().amax(1)
    cinv = (W * W).sum(0)                           # diag K_y⁻¹ (Morton order, padded tail = 1)
    ntr, npad = go.n_train, go.n_pad
    ci = torch.cat([cinv[:ntr], cinv[npad:npad + ntr]])
    vtrain = nz - nz * nz * ci                     # latent posterior variance at the training points
    nmod = go.extra["ozaki"][2]
    del go, W
    gf = E.fit(ks, x, y, nz, variance="f64")
    mf, vf = E.predict(gf, g)
    del gf
    vo, vf, mo, mf = (t.cpu().numpy() for t in (vo, vf, mo, mf))
    rel = np.abs(vo - vf) / vf
    j = int(np.argmax(rel))
    mfl = 1e-2 * np.max(np.abs(mf))
    rec = dict(lib=lib, l=l, noise=nz, kss=kss, nmod=nmod, var_elem=float(rel.max()),
               var_elem_p999=float(np.quantile(rel, 0.999)), var_norm=float(np.max(np.abs(vo - vf)) / np.max(vf)),
               mean_elem=float(np.max(np.abs(mo - mf) / np.maximum(np.abs(mf), mfl))),
               min_var_over_kss=float(vf.min() / kss), var_over_kss_at_worst=float(vf[j] / kss),
               wmax=wmax, wmax_sq_kss=wmax * wmax * kss, rowmax_median=float(rowmax.median()),
               vtrain_min_over_kss=float(vtrain.min()) / kss, cinv_max=float(ci.max()),
               neg_var=int((vo <= 0).sum()), nan=int(np.isnan(vo).sum()), s=round(time.time() - t0, 1))
    print(json.dumps(rec), flush=True)
