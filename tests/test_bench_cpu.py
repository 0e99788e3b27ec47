"""bench.py's --gpus / WORLD_SIZE contract, checked before any GPU call (runs on CPU).

`python bench.py --gpus N` (N > 1) without a launcher starts the N ranks itself
(tests/test_gpu_bench.py::test_bench_gpus2_self_launch runs that on the GPU box); under a
launcher --gpus must equal WORLD_SIZE, otherwise the bench refuses to run."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=120, cwd=ROOT, env=e)


def test_mismatched_gpus_exits_nonzero():
    out = _run(["--gpus", "2", "--steps", "1"], WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    assert out.returncode == 2, (out.returncode, out.stderr[-1000:])
    assert "WORLD_SIZE=3" in out.stderr and not out.stdout.strip()


def test_gpus_below_one_refused():
    out = _run(["--gpus", "0"])
    assert out.returncode != 0 and "--gpus must be >= 1" in out.stderr


def test_launcher_command_shape():
    """The self-launch is ONE child torch.distributed.run with the script's own arguments and a
    127.0.0.1 rendezvous (the parent never initialises HIP, never execs)."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert '"torch.distributed.run"' in src and '"--master-addr", "127.0.0.1"' in src
    assert "subprocess.Popen" in src and "os.exec" not in src
