"""World-size-2 gloo tests of the multi-GPU path (runs on CPU): factor broadcast,
tile-aligned grid sharding and rank-ordered reassembly.

The per-shard compute is injected (an elementwise stand-in), so the test checks
the sharding / communication logic bit-exactly; the HIP predict itself is
covered by tests/test_gpu_parity.py::test_sharded_predict_bit_identical.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_predict(xg, var_mode="latent", compute_var=True):
    x = torch.as_tensor(xg, dtype=torch.float64)
    mean = torch.cat([torch.sin(x[:, 0]) + x[:, 1], torch.cos(x[:, 1]) - x[:, 0]])
    var = torch.cat([x[:, 0] * x[:, 1], x[:, 0] - x[:, 1]])
    return mean, var


def _worker(rank, world, port, out_dir):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp2d import distributed as GD
    from gp2d import engine as E
    spec = E.KernelSpec(kind="df", l_df=5.0)
    n = 256
    if rank == 0:
        g = torch.Generator().manual_seed(7)
        W = torch.tril(torch.randn(n, n, generator=g, dtype=torch.float64))
        alpha = torch.randn(n, generator=g, dtype=torch.float64)
        X = torch.randn(100, 2, generator=g, dtype=torch.float64)
        gp = E.GPFit(kernel=spec, noise=0.01, x=X, n_train=100, n_pad=128, W=W, alpha=alpha,
                     device=torch.device("cpu"))
    else:
        gp = None
    comm = {}
    got = GD.broadcast_fit(gp, spec, 0.01, None, "cpu", comm=comm)
    cs = GD.comm_summary(comm)["bcast"]
    m = 1000
    xg = torch.stack([torch.linspace(0, 9, m, dtype=torch.float64), torch.linspace(3, -2, m, dtype=torch.float64)], 1)
    lo, hi, mean, var = GD.predict_shard(_fake_predict, xg)
    fm, fv = GD.gather_shards(m, 2, lo, hi, mean, var, "cpu")
    torch.save({"W": got.W, "alpha": got.alpha, "x": got.x, "n_pad": got.n_pad, "lo": lo, "hi": hi,
                "mean": fm, "var": fv, "comm": [cs["calls"], cs["bytes_sent"], cs["bytes_recv"], cs["ms"]]},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_broadcast_and_shards_world2(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [torch.load(os.path.join(tmp_path, f"rank{i}.pt"), weights_only=True) for i in range(world)]
    assert torch.equal(r[0]["W"], r[1]["W"]) and torch.equal(r[0]["alpha"], r[1]["alpha"])
    assert torch.equal(r[0]["x"], r[1]["x"]) and r[1]["n_pad"] == 128
    assert r[0]["lo"] == 0 and r[0]["hi"] == r[1]["lo"] and r[1]["hi"] == 1000 and r[0]["hi"] % 64 == 0
    m = 1000
    xg = torch.stack([torch.linspace(0, 9, m, dtype=torch.float64), torch.linspace(3, -2, m, dtype=torch.float64)], 1)
    em, ev = _fake_predict(xg)
    for i in range(world):
        assert torch.equal(r[i]["mean"], em) and torch.equal(r[i]["var"], ev)
    # the comm accounting (bench.py's N > 1 `comm` block): the root sends the payload once, the
    # other rank receives it — packed W (≈ n²/2 doubles), α and X_train
    from gp2d import distributed as GD
    payload = 8 * (GD._packed_len(256) + 256 + 100 * 2)
    assert r[0]["comm"][:3] == [1, payload, 0] and r[1]["comm"][:3] == [1, 0, payload]
    assert r[0]["comm"][3] >= 0 and r[1]["comm"][3] >= 0


def test_assemble_from_shards_numpy():
    from gp2d import distributed as GD
    m, bd = 777, 2
    full = np.arange(bd * m, dtype=np.float64)
    shards = []
    for lo, hi in GD.shard_layout(m, bd, 3):
        k = hi - lo
        vec = np.concatenate([full[c * m + lo:c * m + hi] for c in range(bd)])
        assert vec.size == bd * k
        shards.append((lo, hi, vec))
    assert np.array_equal(GD.assemble_from_shards(m, bd, shards), full)


def test_packed_blocks_cover_the_lower_triangle():
    from gp2d import distributed as GD
    for n in (128, 256, 1024):
        blocks = GD.packed_blocks(n)
        cover = np.zeros((n, n), int)
        for r0, c1, off in blocks[:-1]:
            cover[r0:r0 + GD.PACK_ROWS, :c1] += 1
        assert np.all(cover[np.tril_indices(n)] == 1)       # every lower entry once
        assert blocks[-1][2] == sum(GD.PACK_ROWS * c1 for _, c1, _ in blocks[:-1])
        assert blocks[-1][2] <= n * n // 2 + n * GD.PACK_ROWS


def _fail_worker(rank, world, port, out_dir):
    """Rank 0's fit fails (non-PD K_y): every rank must raise, none may hang in the broadcast."""
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp2d import distributed as GD
    from gp2d import engine as E
    spec = E.KernelSpec(kind="df", l_df=5.0)
    err = np.linalg.LinAlgError("K_y is not positive definite (leading minor of order 3)") if rank == 0 else None
    raised = "none"
    try:
        GD.broadcast_fit(None, spec, -1e-3, None, "cpu", error=err)
    except np.linalg.LinAlgError:
        raised = "LinAlgError"
    # gather_shards refuses a range that does not match its align
    bad = "none"
    try:
        lo, hi = GD.D.shard_range(1100, world, rank, 128)   # 640 | 576 with align 64
        GD.gather_shards(1100, 2, lo, hi, torch.zeros(2 * (hi - lo)), torch.zeros(2 * (hi - lo)), "cpu", align=64)
    except ValueError:
        bad = "ValueError"
    with open(os.path.join(out_dir, f"fail{rank}.txt"), "w") as f:
        f.write(f"{raised} {bad}")
    dist.barrier()
    dist.destroy_process_group()


def test_bcast_fit_failure_raises_on_every_rank(tmp_path):
    world = 2
    mp.spawn(_fail_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for i in range(world):
        raised, bad = open(os.path.join(tmp_path, f"fail{i}.txt")).read().split()
        assert raised == "LinAlgError", i
        assert bad == "ValueError", i


def _info_worker(rank, world, port, out_dir):
    """allreduce_first_failure: the first failing leading minor over the ranks (not the last)."""
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp2d import distributed as GD
    cases = [(0, 0, 0), (0, 513, 513), (700, 513, 513), (513, 0, 513), (300, 900, 300)]
    got = []
    for a, b, _ in cases:
        info = torch.tensor([a if rank == 0 else b], dtype=torch.int32)
        got.append(int(GD.allreduce_first_failure(info).item()))
    with open(os.path.join(out_dir, f"info{rank}.txt"), "w") as f:
        f.write(" ".join(map(str, got)))
    dist.barrier()
    dist.destroy_process_group()


def test_info_allreduce_reports_first_failure(tmp_path):
    world = 2
    mp.spawn(_info_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    want = "0 513 513 513 300"
    for i in range(world):
        assert open(os.path.join(tmp_path, f"info{i}.txt")).read() == want, i


def test_point_count_accepts_lists_arrays_tensors():
    """krige_jobs_sharded sizes a job's broadcast from x on every rank: x may be a nested list
    (engine.fit accepts them through _as_points), an array or a tensor."""
    from gp2d import engine as E
    pts = [[0.0, 1.0], [2.0, 3.0], [4.0, 5.0]]
    assert E._point_count(pts, 2) == 3
    assert E._point_count(np.asarray(pts), 2) == 3
    assert E._point_count(torch.tensor(pts), 2) == 3
    assert E._point_count([[0.0, 1.0, 2.0]] * 5, 3) == 5
