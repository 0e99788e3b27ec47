"""Host-side (enqueue) cost of the per-job calls of distributed.krige_jobs_sharded at the
headline size: engine.fit(check=False), the Predictor call of an 8192-point shard, the
packing of broadcast_fit (root side; round 3: one gp2d_pack_lower launch, the round-2 per-block
copy loop beside it) and ozaki_prepare — GPU work is not waited for."""
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

NTR = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
G = int(sys.argv[2]) if len(sys.argv) > 2 else 256
x1, x2, u, v = D.synthetic_tracks(NTR, seed=2016)
xt = torch.tensor(np.stack([x1, x2], 1), device="cuda")
yt = torch.tensor(np.concatenate([u, v]), device="cuda")
_, _, xg = D.bbox_grid(x1, x2, G, pad=5.0)
xg = torch.tensor(xg[:8192], device="cuda")
xg_all = torch.tensor(D.bbox_grid(x1, x2, G, pad=5.0)[2], device="cuda")
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


def pack_loop():   # the round-2 per-block torch copies
    for r0, c1, off in blocks[:-1]:
        packed[off:off + GD.PACK_ROWS * c1].view(GD.PACK_ROWS, c1).copy_(gp.W[r0:r0 + GD.PACK_ROWS, :c1])


def pack():        # one gp2d_pack_lower launch (round 3)
    GD._pack_lower(gp.W, gp.n, packed, unpack=False)


res = {"fit_enqueue_ms": host_ms(lambda: E.fit(spec, xt, yt, 0.0025, variance="ozaki", check=False)),
       "predict_8192_enqueue_ms": host_ms(lambda: pred(xg)),
       "pack_enqueue_ms": host_ms(pack), "pack_loop_enqueue_ms": host_ms(pack_loop),
       "ozaki_prepare_enqueue_ms": host_ms(lambda: E.ozaki_prepare(gp, diag_add=0.0025))}
res["full_predict_enqueue_ms"] = host_ms(lambda: pred(xg_all))


def job_gpu():
    E.fit(spec, xt, yt, 0.0025, variance="ozaki", check=False)
    pred(xg_all)


ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
ev0.record()
for _ in range(10):
    job_gpu()
ev1.record()
torch.cuda.synchronize()
res["job_wall_ms"] = ev0.elapsed_time(ev1) / 10
res["job_enqueue_ms"] = host_ms(job_gpu)
print(NTR, G, res)
