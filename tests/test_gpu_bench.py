"""bench.py's one-line JSON contract (the driver parses it), on a tiny workload."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("variance", ["ozaki", "f64"])
def test_bench_json_contract(variance):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--ntrain", "256", "--grid", "32", "--steps", "2",
           "--warmup", "1", "--chunk", "1024", "--cpu-sample-points", "64", "--variance", variance]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=100, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["value"] > 0 and abs(d["value"] - 32 * 32 / (d["ms_per_step"] * 1e-3)) / d["value"] < 1e-6
    assert d["vs_baseline"] is None and d["scaling"] == "weak" and "workload" in d["config"]
    # every timed job's fit is issued inside the clock (a fresh job generator after t0)
    assert d["timed_fits"]["issued_in_window"] == d["timed_fits"]["issued_total"] == 2
    assert d["single_job"]["ms"] > 0
    r = d["roofline"]
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in r, key
    assert r["bound"] == "mfma" and 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
    c = d["cpu_baseline"]
    assert c["value"] > 0 and c["kind"] == "port" and c["cores"] >= 1 and c["sample"]
    # N = 1 readings beside the headline: the strict FP64 engine and the Krig drop-in surface
    assert d["f64_value"] > 0 and d["f64"]["steps"] == 5
    assert d["dropin"]["value"] > 0 and d["dropin"]["variance_engine"] in ("ozaki", "f64")
    assert d["dropin_f64"]["value"] > 0 and d["dropin_f64"]["variance_engine"] == "f64"   # Krig's default
    if variance == "ozaki":   # the accuracy guard's decision for the timed jobs
        assert d["guard"]["engine"] in ("ozaki", "f64") and d["guard"]["vmin_over_kss"] > 0
    # the job shape krige_jobs resolved: a batch only back to back, batch_ahead only for a batch
    assert d["batch_ahead"] is False or (d["fits_ahead"] == 0 and d["batch_fits"] > 1)


def test_bench_two_ranks_default_contract():
    """The N > 1 default (strong scaling, round-robin fits + factor broadcast) through
    torch.distributed.run with two ranks on the one card (gloo: RCCL refuses two ranks per
    device): one JSON line from rank 0, whole-job value over both ranks."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, GP2D_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--ntrain", "256", "--grid", "64", "--steps", "4", "--warmup", "1", "--chunk", "1024"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=200, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["api"] == "distributed.krige_jobs_sharded"
    assert abs(d["value"] - 64 * 64 / (d["ms_per_step"] * 1e-3)) / d["value"] < 1e-6
    assert "cpu_baseline" not in d and d["roofline"]["frac"] > 0
    # job j is fitted by rank j mod 2 only: the 4 timed jobs' 4 fits, all issued after t0
    assert d["timed_fits"]["issued_in_window"] == d["timed_fits"]["issued_total"] == 4
    assert d["timed_fits"]["warmup_jobs_run"] >= 2
    sj = d["single_job"]
    assert sj["ms"] > 0 and sj["distributed_fit"]["ms"] > 0 and sj["distributed_fit"]["fit_ms"] > 0
    # the N > 1 line's communication accounting: every job's factor reaches both ranks
    cb = d["comm"]["bcast"]
    assert cb["calls_per_job"] == 1 and cb["ms_per_job_max_over_ranks"] > 0
    n = 2 * 256   # padded matrix order at N_train = 256 (ozaki layout)
    # each rank fits (and sends) every other job's factor and receives the rest
    assert cb["bytes_recv_per_job_max"] + cb["bytes_sent_per_job_max"] >= 8 * n * n // 2
    # a rank prepares the int8 planes of the jobs it receives (every other one) from the payload
    rp = d["comm"]["recv_prepare"]
    assert rp["calls_per_job"] == 0.5 and rp["ms_per_job_max_over_ranks"] > 0 and rp["bytes_recv_per_job_max"] == 0
    dc = sj["distributed_fit"]["comm"]
    assert dc["panel_bcast"]["calls_per_job"] >= 1 and dc["w_allgather"]["calls_per_job"] == 1


def test_bench_multi_rank_paths_under_rccl():
    """The N > 1 code paths (round-robin fits with packed-W broadcasts, the distributed single
    job with its panel broadcasts, all_gather_into_tensor and all_reduce) under the REAL RCCL
    backend: one rank (GP2D_FORCE_COLLECTIVES=1 takes the multi-rank paths at world size 1;
    RCCL refuses two ranks on one device, so N = 2..8 are the driver's runs)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, GP2D_FORCE_COLLECTIVES="1")
    env.pop("GP2D_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "1",
           "--ntrain", "700", "--grid", "64", "--steps", "3", "--warmup", "1", "--chunk", "1024"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=200, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["api"] == "distributed.krige_jobs_sharded" and d["scaling"] == "strong"
    assert d["timed_fits"]["issued_in_window"] == d["timed_fits"]["issued_total"] == 3
    assert d["single_job"]["distributed_fit"]["ms"] > 0
    assert d["comm"]["bcast"]["calls_per_job"] == 1 and d["comm"]["bcast"]["ms_per_job_max_over_ranks"] > 0
    # the job stream's factor broadcasts went through the library's own RCCL communicator
    assert d["comm"]["transport"].startswith("the library's own RCCL communicator")
    assert d["comm"]["library_calls"]["broadcast"] >= 4 * (3 + 1)   # status + packed W + alpha + X per job


def test_bench_gpus2_self_launch():
    """`python bench.py --gpus 2` with NO launcher (the driver's command shape) starts the two
    rank processes itself (one child torch.distributed.run) and reports n_gpus = world_size = 2
    (gloo: RCCL refuses two ranks on the one card of this box)."""
    env = dict(os.environ, GP2D_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--ntrain", "256", "--grid", "64",
           "--steps", "4", "--warmup", "1", "--chunk", "1024"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=200, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and d["scaling"] == "strong"
    assert d["timed_fits"]["issued_in_window"] == d["timed_fits"]["issued_total"] == 4
    assert abs(d["value"] - 64 * 64 / (d["ms_per_step"] * 1e-3)) / d["value"] < 1e-6
