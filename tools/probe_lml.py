"""LML / gradient probe (dev tool): N=4096 div-free (config B size), per-stage wall times and
the config-E sweep rate (64 settings); run under rocprofv3 --kernel-trace --stats for the
per-kernel split."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np, torch
from gp2d import engine as E
from gp2d import hyper as H
from gp2d import data as D
ntr = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
nset = int(sys.argv[2]) if len(sys.argv) > 2 else 64
xx, yy, u, v = D.synthetic_tracks(ntr)
x = np.stack([xx, yy], 1)
y = np.concatenate([u, v])
ks = E.KernelSpec(kind="df", l_df=5.0)


def t(fn, reps=4):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        out.append(1e3 * (time.perf_counter() - t0))
    return min(out), r


tf, gp = t(lambda: E.fit(ks, x, y, 0.0025))
tl, _ = t(lambda: E.log_marginal_likelihood(gp))
tg, (v, g) = t(lambda: E.log_marginal_likelihood(gp, eval_gradient=True))
print(f"N={ntr}: fit {tf:.2f} ms, lml {tl:.3f} ms, lml+grad {tg:.2f} ms; lml={v:.6f} grad={g}", flush=True)
settings = [dict(l_df=float(l), noise=float(nz)) for l in np.linspace(2.0, 9.0, nset // 4)
            for nz in (0.001, 0.0025, 0.005, 0.01)]
for eg in (False, True):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    vals, _ = H.sweep(ks, x, y, settings, noise=0.0025, eval_gradient=eg)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"sweep {len(settings)} settings (grad={eg}): {dt:.3f} s, {len(settings) / dt:.2f} settings/s, "
          f"best l_df={settings[int(np.argmax(vals))]['l_df']:.3f}", flush=True)
torch.cuda.synchronize(); t0 = time.perf_counter()
res = H.optimize(E.KernelSpec(kind="df", l_df=3.0), x, y, 0.01)
torch.cuda.synchronize()
print(f"optimize: {time.perf_counter() - t0:.3f} s, nfev {res.nfev}, l_df {res.kernel.l_df:.4f} "
      f"noise {res.noise:.5f} lml {res.lml:.4f}", flush=True)
