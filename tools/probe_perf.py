"""Quick timing probe of the HIP path (dev tool, not the bench)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np, torch
from gp2d import engine as E

def run(ntr, G, kind="df", chunk=8192, reps=2, variance="f64"):
    rng = np.random.default_rng(2016)
    x = np.stack([rng.uniform(0, 60, ntr), rng.uniform(0, 45, ntr)], 1)
    y = rng.normal(0, 0.3, 2 * ntr)
    gx = np.linspace(-5, 65, G); gy = np.linspace(-5, 50, G)
    GX, GY = np.meshgrid(gx, gy)
    xg = np.stack([GX.ravel(), GY.ravel()], 1)
    ks = E.KernelSpec(kind=kind, l_df=5.0, l_cf=5.0, ratio=1.0 if kind == "df" else 0.5)
    xg_t = torch.tensor(xg, device="cuda")
    for r in range(reps):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        gp = E.fit(ks, x, y, noise=0.0025, variance=variance)
        torch.cuda.synchronize(); t1 = time.perf_counter()
        pr = E.Predictor(gp, chunk)
        E.timing_enable(True)
        torch.cuda.synchronize(); t2 = time.perf_counter()
        mu, var = pr(xg_t)
        torch.cuda.synchronize(); t3 = time.perf_counter()
        ms, cnt, fl = E.timing_read(); E.timing_enable(False)
        M = xg.shape[0]
        print(f"[{variance}] N={ntr} G={G} kind={kind}: fit {1e3*(t1-t0):.1f} ms, predict {1e3*(t3-t2):.1f} ms, "
              f"pts/s {M/(t3-t0):.3e}; colsq gemm {ms:.1f} ms in {cnt} launches = {fl/ms/1e9:.1f} TF/s", flush=True)

if __name__ == "__main__":
    v = sys.argv[1] if len(sys.argv) > 1 else "f64"
    run(1024, 128, variance=v)
    run(4096, 256, variance=v)
