"""The multi-GPU path end to end on the GPU: two fresh rank processes (gloo process group,
both on the one card of the test box — the 8-GPU node is the driver's) run
fit_sharded(mode='bcast', variance='ozaki' / 'f64') → predict_shard → gather_shards, and the
gathered posterior must be bit-identical to the one-process fit + predict.

Rank 0 fits and broadcasts the packed W = L⁻¹, α and the (Morton-ordered) training points;
rank 1 derives its own INT8 residue planes from the received factor (a-priori moduli count,
as engine.fit does), so both ranks predict from identical operands.  The children are started
with the 'spawn' method (a new interpreter each), never by exec'ing this process.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

import torch.multiprocessing as mp  # noqa: E402

from conftest import PKG, ROOT  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem():
    rng = np.random.default_rng(1024)
    n, G = 1024, 96
    x = np.stack([rng.uniform(0, 60, n), rng.uniform(0, 45, n)], 1)
    y = np.concatenate([np.sin(x[:, 1] / 7), np.cos(x[:, 0] / 9)]) + rng.normal(0, 0.05, 2 * n)
    gx, gy = np.linspace(-5, 65, G), np.linspace(-5, 50, G + 7)
    GX, GY = np.meshgrid(gx, gy)
    return x, y, np.stack([GX.reshape(-1), GY.reshape(-1)], 1)


def _worker(rank, world, port, out_dir, variance, kind):
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp2d import distributed as GD
    from gp2d import engine as E
    x, y, xg = _problem()
    dev = torch.device("cuda", 0)
    spec = E.KernelSpec(kind=kind, l_df=5.0, l_cf=4.0, ratio=0.5 if kind == "mixed" else 1.0)
    gp = GD.fit_sharded(spec, torch.tensor(x, device=dev), torch.tensor(y, device=dev), 0.0025, dev,
                        mode="bcast", variance=variance)
    pred = E.Predictor(gp, 1024)
    lo, hi, mean, var = GD.predict_shard(pred, torch.tensor(xg, device=dev))
    fm, fv = GD.gather_shards(xg.shape[0], 2, lo, hi, mean, var, dev)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), mean=fm.cpu().numpy(), var=fv.cpu().numpy(), lo=lo, hi=hi,
             nmod=int(gp.extra["ozaki"][2]) if "ozaki" in gp.extra else 0)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("variance,kind", [("ozaki", "df"), ("ozaki", "mixed"), ("f64", "df")])
def test_bcast_fit_two_ranks_bit_identical(tmp_path, variance, kind):
    from gp2d import engine as E
    world = 2
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), variance, kind)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():  # pragma: no cover — a hung rank: end it, then fail
            p.kill()
    assert codes == [0, 0], codes
    x, y, xg = _problem()
    spec = E.KernelSpec(kind=kind, l_df=5.0, l_cf=4.0, ratio=0.5 if kind == "mixed" else 1.0)
    gp = E.fit(spec, x, y, 0.0025, variance=variance)
    mu, var = (t.cpu().numpy() for t in E.Predictor(gp, 1024)(xg))
    r = [np.load(os.path.join(tmp_path, f"rank{i}.npz")) for i in range(world)]
    assert int(r[0]["lo"]) == 0 and int(r[0]["hi"]) == int(r[1]["lo"]) and int(r[1]["hi"]) == xg.shape[0]
    assert int(r[0]["nmod"]) == int(r[1]["nmod"])
    for i in range(world):
        assert np.array_equal(r[i]["mean"], mu), i
        assert np.array_equal(r[i]["var"], var), i


def test_gp2d_bcast_native_rccl():
    """gp2d_bcast (the C ABI's factor broadcast for C/C++ hosts) on a one-rank RCCL
    communicator made with ncclCommInitAll: root 0 keeps its bytes, rc 0; a root outside the
    communicator comes back as −100 − ncclInvalidArgument with RCCL's message."""
    import ctypes
    from gp2d import _native as N
    L = N.lib()
    rccl = ctypes.CDLL("librccl.so.1")
    comm = ctypes.c_void_p()
    devs = (ctypes.c_int * 1)(torch.cuda.current_device())
    assert rccl.ncclCommInitAll(ctypes.byref(comm), 1, devs) == 0
    try:
        x = torch.arange(1 << 20, dtype=torch.float64, device="cuda")
        ref = x.clone()
        s = torch.cuda.current_stream()
        rc = L.gp2d_bcast(ctypes.c_void_p(x.data_ptr()), x.numel() * 8, 0, comm, ctypes.c_void_p(s.cuda_stream))
        assert rc == 0, L.gp2d_last_error()
        torch.cuda.synchronize()
        assert torch.equal(x, ref)
        rc = L.gp2d_bcast(ctypes.c_void_p(x.data_ptr()), 8, 1, comm, ctypes.c_void_p(s.cuda_stream))
        assert rc == -104 and b"ncclBroadcast" in L.gp2d_last_error(), (rc, L.gp2d_last_error())
    finally:
        rccl.ncclCommDestroy(comm)


def _lib_comm_worker(rank, world, port, out_dir):
    """One rank on RCCL (the 'nccl' backend) with GP2D_FORCE_COLLECTIVES=1: the library's own
    communicator (gp2d/comm.py, gp2d_comm_init from a unique id sent through torch's store)
    carries every collective of the job stream and of the distributed factor."""
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GP2D_FORCE_COLLECTIVES="1")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    from gp2d import comm as C
    from gp2d import distributed as GD
    c = C.get(dev)
    out = {}
    # the primitives on one rank: broadcast keeps the root's bytes, all-gather copies, the
    # reductions return the input, a send/receive to itself copies (RCCL's copy kernel)
    x = torch.arange(1 << 16, dtype=torch.float64, device=dev)
    y = x.clone()
    c.broadcast(y, 0)
    g = torch.empty_like(x)
    c.all_gather_into(g, x)
    i = torch.tensor([5, 0, 2147483647], dtype=torch.int32, device=dev)
    c.all_reduce(i, "min")
    f = torch.tensor([1.5, -2.0], dtype=torch.float64, device=dev)
    c.all_reduce(f, "sum")
    r = torch.empty_like(x)
    c.sendrecv(x, 0, r, 0)
    torch.cuda.synchronize()
    out.update(bcast_ok=torch.equal(y, x), gather_ok=torch.equal(g, x), sendrecv_ok=torch.equal(r, x),
               imin=i.cpu().numpy(), fsum=f.cpu().numpy())
    before = dict(c.calls)
    res = {}
    for j, (lo, hi, mean, var) in enumerate(GD.krige_jobs_sharded(_jobs(), variance="ozaki", chunk=1024)):
        res[f"mean{j}"], res[f"var{j}"] = mean.cpu().numpy(), var.cpu().numpy()
    stream_bcasts = c.calls.get("broadcast", 0) - before.get("broadcast", 0)
    xd, yd, _ = _dfit_problem(1024)
    spec = GD.E.KernelSpec(kind="df", l_df=5.0)
    before = dict(c.calls)
    gp = GD.fit_distributed(spec, torch.tensor(xd, device=dev), torch.tensor(yd, device=dev), 0.0025, dev)
    torch.cuda.synchronize()
    dfit_calls = {k: c.calls.get(k, 0) - before.get(k, 0) for k in c.calls}
    np.savez(os.path.join(out_dir, "libcomm.npz"), stream_bcasts=stream_bcasts, W_sha=_sha(gp.W),
             alpha=gp.alpha.cpu().numpy(), dfit_bcast=dfit_calls.get("broadcast", 0),
             dfit_gather=dfit_calls.get("all_gather", 0), dfit_reduce=dfit_calls.get("all_reduce", 0), **out, **res)
    torch.cuda.synchronize()
    dist.barrier()
    C.shutdown()
    dist.destroy_process_group()


def test_library_rccl_communicator_one_rank(tmp_path):
    """The multi-GPU data path on the library's own RCCL communicator: the
    primitives, the job stream's factor broadcasts (4 gp2d_bcast per job: status, packed W, α,
    X) and the distributed factor's panel broadcasts / all-gathers / status all-reduce, all
    through gp2d_comm_*; the results equal one process's without any collective, bit for bit."""
    from gp2d import distributed as GD
    from gp2d import engine as E
    _spawn(_lib_comm_worker, 1, str(tmp_path))
    r = np.load(os.path.join(tmp_path, "libcomm.npz"))
    assert bool(r["bcast_ok"]) and bool(r["gather_ok"]) and bool(r["sendrecv_ok"])
    assert r["imin"].tolist() == [5, 0, 2147483647] and r["fsum"].tolist() == [1.5, -2.0]
    jobs = _jobs()
    assert int(r["stream_bcasts"]) == 4 * len(jobs)
    for j, (spec, x, y, noise, xg) in enumerate(jobs):
        gp = E.fit(spec, x, y, noise, variance="ozaki")
        mu, var = (t.cpu().numpy() for t in E.Predictor(gp, 1024)(xg))
        assert np.array_equal(r[f"mean{j}"], mu) and np.array_equal(r[f"var{j}"], var), j
    xd, yd, _ = _dfit_problem(1024)
    gp1 = GD.fit_distributed(E.KernelSpec(kind="df", l_df=5.0), xd, yd, 0.0025)   # no process group
    assert np.array_equal(r["W_sha"], _sha(gp1.W)) and np.array_equal(r["alpha"], gp1.alpha.cpu().numpy())
    nsb = gp1.W.shape[0] // GD.super_block()
    assert int(r["dfit_bcast"]) == nsb and int(r["dfit_gather"]) == 3 and int(r["dfit_reduce"]) == 1


def _jobs(noises=None):
    """Five small jobs; noises (optional): per-job noise overrides (the accuracy guard's range)."""
    from gp2d import engine as E
    out = []
    for seed, n, G, kind in [(11, 700, 40, "df"), (12, 700, 44, "mixed"), (13, 900, 40, "df"), (14, 700, 36, "cf"),
                             (15, 900, 48, "mixed")]:
        rng = np.random.default_rng(seed)
        x = np.stack([rng.uniform(0, 60, n), rng.uniform(0, 45, n)], 1)
        y = np.concatenate([np.sin(x[:, 1] / 7), np.cos(x[:, 0] / 9)]) + rng.normal(0, 0.05, 2 * n)
        GX, GY = np.meshgrid(np.linspace(-5, 65, G), np.linspace(-5, 50, G + 5))
        xg = np.stack([GX.reshape(-1), GY.reshape(-1)], 1)
        spec = E.KernelSpec(kind=kind, l_df=4.0 + seed % 3, l_cf=3.0, ratio=0.5 if kind == "mixed" else 1.0)
        out.append((spec, x, y, 0.0025 if noises is None else noises[len(out)], xg))
    return out


# the guard's three outcomes across the job stream: default bits, more bits, the FP64 engine
GUARD_NOISES = (0.0025, 2e-5, 0.0025, 0.01, 1e-8)


def _rr_worker(rank, world, port, out_dir, variance, bad, noises=None):
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp2d import distributed as GD
    jobs = _jobs(noises)
    if bad is not None:   # a non-SPD job (negative noise) owned by rank bad % world
        s, x, y, _, xg = jobs[bad]
        jobs[bad] = (s, x, y, -100.0, xg)
    res, raised = {}, -1
    try:
        for j, (lo, hi, mean, var) in enumerate(GD.krige_jobs_sharded(jobs, variance=variance, chunk=1024)):
            res[f"lo{j}"], res[f"hi{j}"] = lo, hi
            res[f"mean{j}"], res[f"var{j}"] = mean.cpu().numpy(), var.cpu().numpy()
    except np.linalg.LinAlgError:
        raised = len([k for k in res if k.startswith("lo")])
    np.savez(os.path.join(out_dir, f"rr{rank}.npz"), raised=raised, **res)
    dist.barrier()
    dist.destroy_process_group()


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():  # pragma: no cover — a hung rank: end it, then fail
            p.kill()
    assert codes == [0] * world, codes


@pytest.mark.parametrize("variance", ["ozaki", "f64"])
def test_round_robin_jobs_two_ranks_bit_identical(tmp_path, variance):
    """krige_jobs_sharded: job j fitted on rank j mod 2 only, factor broadcast, every rank
    predicts its shard; the assembled shards equal one process's fit + predict, bit for bit."""
    from gp2d import distributed as GD
    from gp2d import engine as E
    world = 2
    _spawn(_rr_worker, world, str(tmp_path), variance, None)
    r = [np.load(os.path.join(tmp_path, f"rr{i}.npz")) for i in range(world)]
    for j, (spec, x, y, noise, xg) in enumerate(_jobs()):
        gp = E.fit(spec, x, y, noise, variance=variance)
        mu, var = (t.cpu().numpy() for t in E.Predictor(gp, 1024)(xg))
        m = xg.shape[0]
        shards_m = [(int(r[i][f"lo{j}"]), int(r[i][f"hi{j}"]), r[i][f"mean{j}"]) for i in range(world)]
        shards_v = [(int(r[i][f"lo{j}"]), int(r[i][f"hi{j}"]), r[i][f"var{j}"]) for i in range(world)]
        assert np.array_equal(GD.assemble_from_shards(m, 2, shards_m), mu), j
        assert np.array_equal(GD.assemble_from_shards(m, 2, shards_v), var), j


def test_round_robin_guard_decisions_two_ranks_bit_identical(tmp_path):
    """The accuracy guard across ranks: jobs whose statistics ask for more W / K* bits (noise
    2e-5) or for the FP64 engine (1e-8) — the receiving rank applies the owner's status block to
    the packed payload (re-prepared planes, or W unpacked) — still equal one process bit for bit."""
    from gp2d import distributed as GD
    from gp2d import engine as E
    world = 2
    _spawn(_rr_worker, world, str(tmp_path), "ozaki", None, GUARD_NOISES)
    r = [np.load(os.path.join(tmp_path, f"rr{i}.npz")) for i in range(world)]
    engines = []
    for j, (spec, x, y, noise, xg) in enumerate(_jobs(GUARD_NOISES)):
        gp = E.fit(spec, x, y, noise, variance="ozaki")
        g = gp.extra["guard"]
        engines.append((g["engine"], g["wbits"], g["kbits"]))
        mu, var = (t.cpu().numpy() for t in E.Predictor(gp, 1024)(xg))
        m = xg.shape[0]
        shards_m = [(int(r[i][f"lo{j}"]), int(r[i][f"hi{j}"]), r[i][f"mean{j}"]) for i in range(world)]
        shards_v = [(int(r[i][f"lo{j}"]), int(r[i][f"hi{j}"]), r[i][f"var{j}"]) for i in range(world)]
        assert np.array_equal(GD.assemble_from_shards(m, 2, shards_m), mu), j
        assert np.array_equal(GD.assemble_from_shards(m, 2, shards_v), var), j
    print("guard decisions:", engines)
    # all three outcomes: default bits, more bits, the FP64 engine
    assert engines[0] == ("ozaki", 49, 45) and engines[4][0] == "f64"
    assert engines[1][0] == "ozaki" and (engines[1][1], engines[1][2]) != (49, 45)


def _rr_noguard_worker(rank, world, port, out_dir):
    """The job stream with the accuracy guard off (GP2D_GUARD=0, read at import): the owner's
    status block carries the NaN "no guard ran" sentinel, so the receiving rank keeps the
    default precision instead of acting on the block's other bytes."""
    os.environ["GP2D_GUARD"] = "0"
    _rr_worker(rank, world, port, out_dir, "ozaki", None, GUARD_NOISES)


def test_round_robin_jobs_without_guard_bit_identical(tmp_path):
    from gp2d import distributed as GD
    from gp2d import engine as E
    world = 2
    _spawn(_rr_noguard_worker, world, str(tmp_path))
    r = [np.load(os.path.join(tmp_path, f"rr{i}.npz")) for i in range(world)]
    for j, (spec, x, y, noise, xg) in enumerate(_jobs(GUARD_NOISES)):
        if noise < 1e-6:
            continue   # noise 1e-8 without the guard: not a parity case (the guard routes it to FP64)
        gp = E.fit(spec, x, y, noise, variance="ozaki", guard=False)
        mu, var = (t.cpu().numpy() for t in E.Predictor(gp, 1024)(xg))
        m = xg.shape[0]
        shards_m = [(int(r[i][f"lo{j}"]), int(r[i][f"hi{j}"]), r[i][f"mean{j}"]) for i in range(world)]
        shards_v = [(int(r[i][f"lo{j}"]), int(r[i][f"hi{j}"]), r[i][f"var{j}"]) for i in range(world)]
        assert np.array_equal(GD.assemble_from_shards(m, 2, shards_m), mu), j
        assert np.array_equal(GD.assemble_from_shards(m, 2, shards_v), var), j


def test_round_robin_jobs_non_spd_raises_on_every_rank(tmp_path):
    """Job 3 (owned by rank 1) has a non-SPD K_y: both ranks raise LinAlgError after the
    three jobs before it, none hangs."""
    world = 2
    _spawn(_rr_worker, world, str(tmp_path), "ozaki", 3)
    for i in range(world):
        assert int(np.load(os.path.join(tmp_path, f"rr{i}.npz"))["raised"]) == 3, i


def _window_worker(rank, world, port, out_dir):
    """bench.py's timing pattern: a warmup generator drained, then t0, then a FRESH generator
    over the timed jobs; the fits this rank issues are stamped (stats)."""
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import time
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp2d import distributed as GD
    job = _jobs()[0]
    for _ in GD.krige_jobs_sharded([job] * 2, chunk=1024):
        pass
    torch.cuda.synchronize()
    dist.barrier()
    stats = {}
    t0 = time.perf_counter()
    n_out = sum(1 for _ in GD.krige_jobs_sharded([job] * 5, chunk=1024, stats=stats))
    torch.cuda.synchronize()
    dist.barrier()
    t1 = time.perf_counter()
    ts = np.asarray(stats.get("fit_issue_times", []))
    np.savez(os.path.join(out_dir, f"win{rank}.npz"), inside=int(((ts >= t0) & (ts <= t1)).sum()), total=len(ts),
             issued=int(stats.get("fits_issued", 0)), n_out=n_out)
    dist.barrier()
    dist.destroy_process_group()


def test_round_robin_timed_window_holds_every_fit(tmp_path):
    """With a fresh krige_jobs_sharded generator started after t0, the fits of all 5 timed jobs
    are issued inside [t0, t1] — 3 on rank 0 (jobs 0, 2, 4), 2 on rank 1 — and none before."""
    world = 2
    _spawn(_window_worker, world, str(tmp_path))
    r = [np.load(os.path.join(tmp_path, f"win{i}.npz")) for i in range(world)]
    assert [int(x["total"]) for x in r] == [3, 2]
    assert [int(x["inside"]) for x in r] == [3, 2]
    assert [int(x["issued"]) for x in r] == [3, 2]
    assert all(int(x["n_out"]) == 5 for x in r)


# ------------------------------------------------------------------ one job's factor over ranks
def _dfit_problem(n):
    rng = np.random.default_rng(4242 + n)
    x = np.stack([rng.uniform(0, 60, n), rng.uniform(0, 45, n)], 1)
    y = np.concatenate([np.sin(x[:, 1] / 7), np.cos(x[:, 0] / 9)]) + rng.normal(0, 0.05, 2 * n)
    GX, GY = np.meshgrid(np.linspace(-5, 65, 40), np.linspace(-5, 50, 43))
    return x, y, np.stack([GX.reshape(-1), GY.reshape(-1)], 1)


def _sha(t):
    import hashlib
    return np.frombuffer(hashlib.sha256(t.contiguous().cpu().numpy().tobytes()).digest(), np.uint8)


def _dfit_worker(rank, world, port, out_dir, n, kind, noise):
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp2d import distributed as GD
    from gp2d import engine as E
    x, y, xg = _dfit_problem(n)
    dev = torch.device("cuda", 0)
    spec = E.KernelSpec(kind=kind, l_df=5.0, l_cf=4.0, ratio=0.5 if kind == "mixed" else 1.0)
    out = {}
    try:
        gp = GD.fit_distributed(spec, torch.tensor(x, device=dev), torch.tensor(y, device=dev), noise, dev)
        lo, hi, mean, var = GD.predict_shard(E.Predictor(gp, 1024), torch.tensor(xg, device=dev))
        fm, fv = GD.gather_shards(xg.shape[0], 2, lo, hi, mean, var, dev)
        out = dict(W_sha=_sha(gp.W), alpha=gp.alpha.cpu().numpy(), mean=fm.cpu().numpy(),
                   var=fv.cpu().numpy(), nmod=int(gp.extra["ozaki"][2]), raised=0)
    except np.linalg.LinAlgError:
        out = dict(raised=1)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"dfit{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n,kind", [(1024, "df"), (700, "mixed"), (4096, "df")])
def test_distributed_fit_two_ranks_bit_identical(tmp_path, n, kind):
    """fit_distributed over two ranks (block-cyclic POTRF + TRTRI, a panel broadcast per
    512-column super-block, W columns all-gathered): both ranks hold the bits of the one-rank
    run of the same algorithm (W by SHA-256, α, and the sharded posterior), and agree with
    engine.fit's factor and posterior to 1e-12 / 1e-10 (relative, normwise).  N = 4096
    (n = 8192: 16 super-columns, 8 per rank) is the headline's size."""
    from gp2d import distributed as GD
    from gp2d import engine as E
    world = 2
    _spawn(_dfit_worker, world, str(tmp_path), n, kind, 0.0025)
    r = [np.load(os.path.join(tmp_path, f"dfit{i}.npz")) for i in range(world)]
    x, y, xg = _dfit_problem(n)
    spec = E.KernelSpec(kind=kind, l_df=5.0, l_cf=4.0, ratio=0.5 if kind == "mixed" else 1.0)
    gp1 = GD.fit_distributed(spec, x, y, 0.0025)                  # world 1: no process group here
    mu1, var1 = (t.cpu().numpy() for t in E.Predictor(gp1, 1024)(xg))
    W1 = gp1.W.cpu().numpy()
    assert W1.shape[0] // GD.super_block() >= 3                    # both ranks own super-columns
    for i in range(world):
        assert int(r[i]["raised"]) == 0
        assert np.array_equal(r[i]["W_sha"], _sha(gp1.W)), i
        assert np.array_equal(r[i]["alpha"], gp1.alpha.cpu().numpy()), i
        assert np.array_equal(r[i]["mean"], mu1) and np.array_equal(r[i]["var"], var1), i
    assert np.array_equal(np.triu(W1, 1), np.zeros_like(W1))       # W = L⁻¹ is lower-triangular
    gp = E.fit(spec, x, y, 0.0025, variance="ozaki")
    Wr = gp.W.cpu().numpy()
    k = Wr.shape[0]   # engine.fit pads to the same 256 multiple for the ozaki engine
    assert k == W1.shape[0]
    assert np.linalg.norm(W1 - Wr) / np.linalg.norm(Wr) < 1e-12
    mu, var = (t.cpu().numpy() for t in E.Predictor(gp, 1024)(xg))
    assert np.linalg.norm(mu1 - mu) / np.linalg.norm(mu) < 1e-10
    assert np.linalg.norm(var1 - var) / np.linalg.norm(var) < 1e-10


def test_distributed_fit_non_spd_raises_on_every_rank(tmp_path):
    world = 2
    _spawn(_dfit_worker, world, str(tmp_path), 700, "df", -100.0)
    for i in range(world):
        assert int(np.load(os.path.join(tmp_path, f"dfit{i}.npz"))["raised"]) == 1, i


def test_distributed_fit_one_rank_lookahead_and_f64():
    """One process: the look-ahead order changes no bits; the FP64 engine's posterior from the
    distributed factor matches engine.fit's (1e-10)."""
    from gp2d import distributed as GD
    from gp2d import engine as E
    x, y, xg = _dfit_problem(900)
    spec = E.KernelSpec(kind="df", l_df=5.0)
    a = GD.fit_distributed(spec, x, y, 0.0025, variance="f64")
    b = GD.fit_distributed(spec, x, y, 0.0025, variance="f64", lookahead=False)
    assert torch.equal(a.W, b.W) and torch.equal(a.alpha, b.alpha)
    mu1, var1 = (t.cpu().numpy() for t in E.Predictor(a, 1024)(xg))
    gp = E.fit(spec, x, y, 0.0025, variance="f64")
    mu, var = (t.cpu().numpy() for t in E.Predictor(gp, 1024)(xg))
    assert np.linalg.norm(mu1 - mu) / np.linalg.norm(mu) < 1e-10
    assert np.linalg.norm(var1 - var) / np.linalg.norm(var) < 1e-10


def _prep_fail_worker(rank, world, port, out_dir):
    """Job 1 (owned by rank 1): the owner's int8 preparation fails after a successful POTRF
    (fault injected into engine.ozaki_prepare inside that one fit).  The owner defers the error
    to check(); the status word it broadcasts must say "failed" (−1), so BOTH ranks raise at
    job 1 after yielding job 0 and neither waits in a later collective."""
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp2d import _native as N
    from gp2d import distributed as GD
    from gp2d import engine as E
    jobs = _jobs()[:3]
    real_fit, real_prep = E.fit, E.ozaki_prepare
    calls = [0]

    def fit(*a, **k):
        calls[0] += 1
        if rank == 1 and calls[0] == 1:   # rank 1's first fit is job 1

            def bad_prep(gp, diag_add=None):
                raise N.GP2DError("injected: gp2d_ozaki_prepare_async failed")
            E.ozaki_prepare = bad_prep
            try:
                return real_fit(*a, **k)
            finally:
                E.ozaki_prepare = real_prep
        return real_fit(*a, **k)

    E.fit = fit
    done, raised = 0, "none"
    try:
        for _ in GD.krige_jobs_sharded(jobs, chunk=1024):
            done += 1
    except Exception as e:   # noqa: BLE001 — the type is what the test checks
        raised = type(e).__name__
    torch.cuda.synchronize()
    with open(os.path.join(out_dir, f"prep{rank}.txt"), "w") as f:
        f.write(f"{done} {raised}")
    dist.barrier()
    dist.destroy_process_group()


def test_round_robin_owner_preparation_error_raises_on_every_rank(tmp_path):
    world = 2
    _spawn(_prep_fail_worker, world, str(tmp_path))
    got = [open(os.path.join(tmp_path, f"prep{i}.txt")).read().split() for i in range(world)]
    assert got[1] == ["1", "GP2DError"], got        # the owner: its own deferred error
    assert got[0] == ["1", "RuntimeError"], got     # the receiver: "failed on the rank that owned it"


def _list_worker(rank, world, port, out_dir):
    """krige_jobs_sharded with x, y, xg given as nested Python lists on every rank (engine.fit
    accepts lists): the receivers size the broadcast from the list."""
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp2d import distributed as GD
    jobs = [(s, x.tolist(), y.tolist(), nz, xg) for s, x, y, nz, xg in _jobs()[:2]]
    res = {}
    for j, (lo, hi, mean, var) in enumerate(GD.krige_jobs_sharded(jobs, chunk=1024)):
        res[f"lo{j}"], res[f"hi{j}"] = lo, hi
        res[f"mean{j}"], res[f"var{j}"] = mean.cpu().numpy(), var.cpu().numpy()
    np.savez(os.path.join(out_dir, f"list{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def test_round_robin_jobs_list_inputs(tmp_path):
    from gp2d import distributed as GD
    from gp2d import engine as E
    world = 2
    _spawn(_list_worker, world, str(tmp_path))
    r = [np.load(os.path.join(tmp_path, f"list{i}.npz")) for i in range(world)]
    for j, (spec, x, y, noise, xg) in enumerate(_jobs()[:2]):
        gp = E.fit(spec, x, y, noise, variance="ozaki")
        mu, var = (t.cpu().numpy() for t in E.Predictor(gp, 1024)(xg))
        m = xg.shape[0]
        assert np.array_equal(GD.assemble_from_shards(
            m, 2, [(int(r[i][f"lo{j}"]), int(r[i][f"hi{j}"]), r[i][f"mean{j}"]) for i in range(world)]), mu), j
        assert np.array_equal(GD.assemble_from_shards(
            m, 2, [(int(r[i][f"lo{j}"]), int(r[i][f"hi{j}"]), r[i][f"var{j}"]) for i in range(world)]), var), j


def _sweep_settings():
    return [dict(l_df=l, noise=nz) for l in (3.0, 5.0, 8.0) for nz in (0.0025, 0.01)] + [dict(noise=-50.0)]


def _sweep_tracks():
    rng = np.random.default_rng(31)
    x = np.stack([rng.uniform(0, 60, 400), rng.uniform(0, 45, 400)], 1)
    y = np.concatenate([np.sin(x[:, 1] / 7), np.cos(x[:, 0] / 9)]) + rng.normal(0, 0.05, 800)
    return x, y


def _sweep_worker(rank, world, port, out_dir):
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp2d import engine as E
    from gp2d import hyper as H
    x, y = _sweep_tracks()
    vals, grads = H.sweep(E.KernelSpec(kind="df", l_df=5.0), x, y, _sweep_settings(), noise=0.0025,
                          eval_gradient=True)   # the default: each rank's settings in one batched factorisation
    np.savez(os.path.join(out_dir, f"sweep{rank}.npz"), vals=vals, grads=grads)
    dist.barrier()
    dist.destroy_process_group()


def test_sweep_two_ranks_batched_bit_identical(tmp_path):
    """hyper.sweep over two ranks: each rank's settings (dealt round robin) fitted in one batched
    factorisation, the results all-reduced — every rank holds one process's sweep, bit for bit,
    the non-PD setting -inf."""
    from gp2d import engine as E
    from gp2d import hyper as H
    world = 2
    _spawn(_sweep_worker, world, str(tmp_path))
    x, y = _sweep_tracks()
    ref_v, ref_g = H.sweep(E.KernelSpec(kind="df", l_df=5.0), x, y, _sweep_settings(), noise=0.0025,
                           eval_gradient=True, batch=1)
    assert ref_v[-1] == -np.inf
    for r in range(world):
        got = np.load(os.path.join(tmp_path, f"sweep{r}.npz"))
        assert np.array_equal(got["vals"], ref_v) and np.array_equal(got["grads"], ref_g)
