"""POTRF trailing-update schedules (gp2d.hip potrf_schedule): time engine.fit and gp2d_potrf
alone at the given sizes under the schedule in the environment (GP2D_POTRF_G = 2 | 4,
GP2D_POTRF_SPLIT = 0 | 1; unset = the library's choice by n).  One JSON line per size.

    GP2D_POTRF_G=4 GP2D_POTRF_SPLIT=1 python tools/probe_potrf_sched.py --sizes 4096,16384
"""
import argparse
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,16384")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = E.N.lib()
    P = E._ptr
    for ntr in (int(s) for s in a.sizes.split(",")):
        x1, x2, u, v = D.synthetic_tracks(ntr, seed=2016)
        xt = torch.tensor(np.stack([x1, x2], 1), device=dev)
        yt = torch.tensor(np.concatenate([u, v]), device=dev)
        kind = "df" if ntr <= 4096 else "mixed"
        spec = E.KernelSpec(kind=kind, l_df=5.0, l_cf=5.0, ratio=1.0 if kind == "df" else 0.5)
        reps = a.reps if ntr <= 8192 else 2
        E.fit(spec, xt, yt, 0.0025, device=dev, variance="ozaki")
        torch.cuda.synchronize()
        fits = []
        for _ in range(reps):
            t = time.perf_counter()
            gp = E.fit(spec, xt, yt, 0.0025, device=dev, variance="ozaki")
            torch.cuda.synchronize()
            fits.append(1e3 * (time.perf_counter() - t))
        n = gp.n
        W = gp.W
        del gp
        npad = n // 2
        K = torch.empty((n, n), dtype=torch.float64, device=dev)
        X = xt[E.morton_order(xt)].contiguous()
        desc = spec.desc()
        sh = E._stream_handle(dev)
        E.N.check(L.gp2d_assemble(P(X), ntr, npad, P(X), ntr, npad, ctypes.byref(desc), 0.0025, 1, P(K), n, sh),
                  "assemble")
        A = torch.empty_like(K)
        dinv = torch.empty((n // 128, 128, 128), dtype=torch.float64, device=dev)
        info = torch.zeros(1, dtype=torch.int32, device=dev)
        pot = []
        for _ in range(reps):
            A.copy_(K)
            torch.cuda.synchronize()
            t = time.perf_counter()
            E.N.check(L.gp2d_potrf(P(A), n, n, P(dinv), P(info), None, 0, sh), "potrf")
            torch.cuda.synchronize()
            pot.append(1e3 * (time.perf_counter() - t))
        # the factor's residual against K on a row sample: ‖L Lᵀ − K‖ / ‖K‖
        rows = torch.arange(0, n, max(1, n // 256), device=dev)
        Ls = A[rows]
        res = float(torch.linalg.norm(Ls @ A.T - K[rows]) / torch.linalg.norm(K[rows]))
        print(json.dumps({"n_train": ntr, "n": n, "G": os.environ.get("GP2D_POTRF_G", "auto"),
                          "split": os.environ.get("GP2D_POTRF_SPLIT", "auto"), "info": int(info.item()),
                          "fit_ms": sorted(fits), "potrf_ms": sorted(pot), "factor_residual": res,
                          "W_norm": float(torch.linalg.norm(W))}), flush=True)
        del A, K, W, dinv
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
