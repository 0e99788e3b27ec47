"""Host-side (enqueue) cost of the per-job calls of distributed.krige_jobs_sharded at the
headline size: engine.fit(check=False), the Predictor call of an 8192-point shard, the
packing loop of broadcast_fit (root side) and ozaki_prepare — GPU work is not waited for."""
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

x1, x2, u, v = D.synthetic_tracks(4096, seed=2016)
xt = torch.tensor(np.stack([x1, x2], 1), device="cuda")
yt = torch.tensor(np.concatenate([u, v]), device="cuda")
_, _, xg = D.bbox_grid(x1, x2, 256, pad=5.0)
xg = torch.tensor(xg[:8192], device="cuda")
spec = E.KernelSpec(kind="df", l_df=5.0)
gp = E.fit(spec, xt, yt, 0.0025, variance="ozaki")
pred = E.Predictor(gp, 8192)
pred(xg)
torch.cuda.synchronize()


def host_ms(fn, reps=10):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        ts.append(1e3 * (time.perf_counter() - t))
    torch.cuda.synchronize()
    return float(np.median(ts))


blocks = GD.packed_blocks(gp.n)
packed = torch.empty(blocks[-1][2], dtype=torch.float64, device="cuda")


def pack():
    for r0, c1, off in blocks[:-1]:
        packed[off:off + GD.PACK_ROWS * c1].view(GD.PACK_ROWS, c1).copy_(gp.W[r0:r0 + GD.PACK_ROWS, :c1])


res = {"fit_enqueue_ms": host_ms(lambda: E.fit(spec, xt, yt, 0.0025, variance="ozaki", check=False)),
       "predict_8192_enqueue_ms": host_ms(lambda: pred(xg)),
       "pack_enqueue_ms": host_ms(pack),
       "ozaki_prepare_enqueue_ms": host_ms(lambda: E.ozaki_prepare(gp, diag_add=0.0025))}
print(res)
