"""BASELINE.json configs B, C, D on ONE MI355X (dev tool; output → profiles/r01_configs.log).

  H: div-free, N_train=4096, 256×256 grid (the bench.py headline workload)
  B: div-free, N_train=1024, 128×128 grid
  C: mixed (ratio 0.5), N_train=4096, 256×256 grid
  D: N_train=16384 (32768² K), 512×512 grid sharded over 8 GPUs — here ONE rank's shard
     (rank 0 of 8: 32768 points), the same code path every rank of the 8-GPU run executes

Per config: one warm fit+predict, then the median of three timed fit+predicts (Ozaki engine),
points/s, and accuracy: Ozaki vs the FP64-MFMA engine on the whole grid (normwise and
elementwise relative) and both vs the numpy oracle on a 256-point subset (B, C; D with
--oracle-d, a ~1-2 min CPU fit)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gp2d import data as D  # noqa: E402
from gp2d import engine as E  # noqa: E402
from oracle import gp2d_oracle as O  # noqa: E402

CONFIGS = {"H": ("df", 1.0, 4096, 256, 256, 1, 0),   # the bench.py headline workload
           "B": ("df", 1.0, 1024, 128, 128, 1, 0), "C": ("mixed", 0.5, 4096, 256, 256, 1, 0),
           "D": ("mixed", 0.5, 16384, 512, 512, 8, 0)}


def rel(a, b):
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


def run(name, oracle_d):
    kind, ratio, ntr, gx, gy, world, rank = CONFIGS[name]
    x1, x2, u, v = D.synthetic_tracks(ntr, seed=2016)
    x = torch.tensor(np.stack([x1, x2], 1), device="cuda")
    y = torch.tensor(np.concatenate([u, v]), device="cuda")
    _, _, xg_all = D.bbox_grid(x1, x2, gx, pad=5.0, Gy=gy)
    lo, hi = D.shard_range(xg_all.shape[0], world, rank)
    xg = torch.tensor(xg_all[lo:hi], device="cuda")
    ks = E.KernelSpec(kind=kind, l_df=5.0, l_cf=5.0, ratio=ratio)
    res = {}
    for eng in ("ozaki", "f64"):
        tfit, tpred = [], []
        for rep in range(4):               # one warm run, then the median of three
            if rep:
                del gp, mu, var
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gp = E.fit(ks, x, y, noise=0.0025, variance=eng)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            mu, var = E.Predictor(gp, 8192)(xg)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            if rep:
                tfit.append(t1 - t0)
                tpred.append(t2 - t1)
        res[eng] = (mu.cpu().numpy(), var.cpu().numpy(), float(np.median(tfit)), float(np.median(tpred)),
                    gp.extra["ozaki"][2] if "ozaki" in gp.extra else None)
        del gp, mu, var
        torch.cuda.empty_cache()
    mo, vo, tf, tp, nmod = res["ozaki"]
    mf, vf, tf64, tp64, _ = res["f64"]
    m = hi - lo
    line = (f"{name}: {kind} N={ntr} grid {gx}x{gy}" + (f" shard {rank}/{world} ({m} pts)" if world > 1 else f" ({m} pts)") +
            f" | ozaki: fit {1e3 * tf:.1f} ms predict {1e3 * tp:.1f} ms -> {m / (tf + tp):.3e} pts/s (nmod {nmod})"
            f" | f64 engine: {m / (tf64 + tp64):.3e} pts/s"
            f" | ozaki vs f64: var {rel(vo, vf):.1e} (elementwise {np.max(np.abs(vo - vf) / np.abs(vf)):.1e}),"
            f" mean {rel(mo, mf):.1e}; var>0 {bool(np.all(vo > 0))}")
    if name != "D" or oracle_d:
        sub = np.random.default_rng(0).choice(m, 256, replace=False)
        t0 = time.perf_counter()
        mr, vr = O.fit_predict(np.stack([x1, x2], 1), np.concatenate([u, v]), xg_all[lo:hi][sub], kind=kind,
                               l_df=5.0, l_cf=5.0, ratio=ratio, noise=0.0025)
        idx = np.concatenate([sub, m + sub])
        line += (f" | vs oracle (256 pts, {time.perf_counter() - t0:.0f} s CPU): ozaki var {rel(vo[idx], vr):.1e}"
                 f" mean {rel(mo[idx], mr):.1e}; f64 var {rel(vf[idx], vr):.1e} mean {rel(mf[idx], mr):.1e}")
    print(line, flush=True)


if __name__ == "__main__":
    names = [a for a in sys.argv[1:] if not a.startswith("-")] or ["B", "C", "D"]
    for nme in names:
        run(nme, "--oracle-d" in sys.argv)
