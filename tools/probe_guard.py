"""Calibration of the ozaki accuracy guard (dev tool).

For each (ℓ, noise) setting at N_train = 4096 (bench tracks, df kernel, full 256² grid) and each
(W bits, K* bits): the int8 variance elementwise over all 131,072 outputs against the same
engine at its maximal precision (60 W bits, 50 K* bits — the yardstick of the emulation error:
its own modelled error is ≤ 2e-11 at these settings) and against the FP64 engine on the same
factor (the training points in the ozaki fit's Morton order, so W and α are the same bits; the
FP64 products carry their own rounding, ≈ 8e-15·kss/v_min elementwise, which floors that column),
beside the guard's statistics, its model (gp2d_ozaki_error_model) and decision
(gp2d_ozaki_guard_bits).
Usage: python tools/probe_guard.py [l:noise ...]  (JSON lines on stdout)"""
import ctypes
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

# a setting: l:noise (div-free) or kind:l:noise (kind df | cf | mixed; mixed: l_cf = l, ratio 0.5)
settings = [tuple(a.split(":")) for a in sys.argv[1:]] or \
    [(5.0, 0.0025), (12.0, 1e-3), (2.0, 5e-2), (5.0, 1e-4), (5.0, 5e-4), (8.0, 0.0025), (12.0, 0.0025), (3.0, 1e-3),
     (2.0, 1e-4)]
BITS = [(49, 45), (50, 45), (52, 45), (56, 45), (49, 47), (49, 48), (51, 46), (53, 47), (53, 48), (56, 48), (58, 50)]
x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
x = torch.tensor(np.stack([x1, x2], 1), device="cuda")
y = torch.tensor(np.concatenate([u, v]), device="cuda")
_, _, xg = D.bbox_grid(x1, x2, 256, pad=5.0)
g = torch.tensor(xg, device="cuda")
L = E.N.lib()
for st in settings:
    kind, l, nz = ("df", *st) if len(st) == 2 else st
    l, nz = float(l), float(nz)
    ks = E.KernelSpec(kind=kind, l_df=l, l_cf=l, ratio=0.5 if kind == "mixed" else 1.0)
    kss = ks.kdiag()
    t0 = time.time()
    go = E.fit(ks, x, y, nz, variance="ozaki")           # guarded: its statistics and decision
    dec = {k: go.extra["guard"][k] for k in ("engine", "wbits", "kbits", "vmin_over_kss", "wmax", "est")}
    p = go.perm
    gf = E.fit(ks, x[p], torch.cat([y[:4096][p], y[4096:][p]]), nz, variance="f64")
    assert torch.equal(gf.W, go.W)
    mf, vf = (t.cpu().numpy() for t in E.predict(gf, g))
    del gf
    vmin = dec["vmin_over_kss"] * kss
    E.ozaki_prepare(go, diag_add=nz, wbits=60, kbits=50)
    mx, vx = (t.cpu().numpy() for t in E.predict(go, g))
    fl = np.abs(vx - vf) / vf
    print(json.dumps(dict(kind=kind, l=l, noise=nz, kss=kss, wbits=60, kbits=50, ref="f64", var_elem=float(fl.max()),
                          model=float(L.gp2d_ozaki_error_model(kss, vmin, 60, 50)), guard=dec)), flush=True)
    for wb, kb in BITS:
        E.ozaki_prepare(go, diag_add=nz, wbits=wb, kbits=kb)
        mo, vo = (t.cpu().numpy() for t in E.predict(go, g))
        rel = np.abs(vo - vx) / vx
        rec = dict(kind=kind, l=l, noise=nz, kss=kss, wbits=wb, kbits=kb, nmod=go.extra["ozaki"][2], ref="max",
                   var_elem=float(rel.max()), var_elem_p999=float(np.quantile(rel, 0.999)),
                   var_elem_f64=float(np.max(np.abs(vo - vf) / vf)),
                   mean_elem=float(np.max(np.abs(mo - mf) / np.maximum(np.abs(mf), 1e-2 * np.abs(mf).max()))),
                   model=float(L.gp2d_ozaki_error_model(kss, vmin, wb, kb)), guard=dec,
                   min_var_over_kss=float(vf.min() / kss), s=round(time.time() - t0, 1))
        print(json.dumps(rec), flush=True)
    del go
    torch.cuda.empty_cache()
