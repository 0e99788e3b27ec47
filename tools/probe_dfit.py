"""Distributed-factor probe (one process): fit_distributed at world size 1 — the same kernels
and step sequence a rank runs at P = 1 — against engine.fit, at the headline (N = 4096) and
config D (N = 16384) sizes; per size the fit time of each and the relative difference of W.

    python tools/probe_dfit.py [--sizes 4096,16384] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gp2d import data as D  # noqa: E402
from gp2d import distributed as GD  # noqa: E402
from gp2d import engine as E  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t) / reps, out


def chain_ms(spec, xt, dev):
    """Σ over steps of (update of super-column s+1 by panel s, then gp2d_dfact_panel(s+1)):
    the owners' sequence that no rank can overlap (broadcast latency excluded)."""
    L = E.N.lib()
    P, sh = E._ptr, E._stream_handle(dev)
    npad, n = GD.dfact_layout(spec, xt.shape[0])
    A = torch.empty((n, n), dtype=torch.float64, device=dev)
    desc = spec.desc()
    import ctypes
    E.N.check(L.gp2d_assemble(P(xt), xt.shape[0], npad, P(xt), xt.shape[0], npad, ctypes.byref(desc), 0.0025, 1,
                              P(A), n, sh), "assemble")
    pan = torch.empty(int(L.gp2d_dfact_panel_doubles(n)), dtype=torch.float64, device=dev)
    wb = int(L.gp2d_dfact_workspace(n))
    work = torch.empty(wb // 8 + 1, dtype=torch.float64, device=dev)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    nsb = n // GD.super_block()

    def run():
        E.N.check(L.gp2d_dfact_panel(P(A), n, n, 0, P(pan), P(info), P(work), wb, sh), "panel")
        for s in range(nsb - 1):
            E.N.check(L.gp2d_dfact_update(P(A), n, n, s, P(pan), 1, 0, s + 1, s + 2, sh), "update")
            E.N.check(L.gp2d_dfact_panel(P(A), n, n, s + 1, P(pan), P(info), P(work), wb, sh), "panel")
    t, _ = timed(run, 1)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,16384")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--emulate", default="2,8", help="P values whose per-rank share is timed")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for ntr in (int(s) for s in a.sizes.split(",")):
        x1, x2, u, v = D.synthetic_tracks(ntr, seed=2016)
        xt = torch.tensor(np.stack([x1, x2], 1), device=dev)
        yt = torch.tensor(np.concatenate([u, v]), device=dev)
        kind = "df" if ntr <= 4096 else "mixed"
        spec = E.KernelSpec(kind=kind, l_df=5.0, l_cf=5.0, ratio=1.0 if kind == "df" else 0.5)
        reps = a.reps if ntr <= 4096 else 1
        t_ref, gp = timed(lambda: E.fit(spec, xt, yt, 0.0025, device=dev, variance="ozaki"), reps)
        W0 = gp.W
        del gp
        t_d, gd = timed(lambda: GD.fit_distributed(spec, xt, yt, 0.0025, dev, variance="ozaki"), reps)
        rel = float(torch.linalg.norm(gd.W - W0) / torch.linalg.norm(W0))
        t_n, _ = timed(lambda: GD.fit_distributed(spec, xt, yt, 0.0025, dev, variance="ozaki", lookahead=False), 1)
        rec = {"n_train": ntr, "n": gd.n, "engine_fit_ms": t_ref, "fit_distributed_p1_ms": t_d,
               "fit_distributed_p1_no_lookahead_ms": t_n, "W_rel_diff": rel}
        del gd, W0
        torch.cuda.empty_cache()
        # one rank's share of a P-rank factorisation (no broadcast, no all-gather)
        for P in [int(p) for p in a.emulate.split(",") if p]:
            for r in sorted({0, P - 1}):
                t_e, g = timed(lambda: GD.fit_distributed(spec, xt, yt, 0.0025, dev, variance="ozaki",
                                                          emulate=(P, r)), 1)
                rec[f"rank_share_P{P}_r{r}_ms"] = t_e
                del g
        # the critical chain: per step, the next owner's column update + the panel factor
        rec["chain_ms"] = chain_ms(spec, xt, dev)
        print(json.dumps(rec), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
