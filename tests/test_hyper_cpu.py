"""Host logic of the hyperparameter fitting (gp2d.hyper) on CPU: parameter naming /
ordering, the unconstrained transforms and their derivatives, and the world-size-2
gloo path of the config-E sweep reduction (bit-exact, rank-independent)."""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT
from gp2d import engine as E
from gp2d import hyper as H


def test_param_names_and_roundtrip():
    ks = E.KernelSpec(kind="mixed", l_df=2.0, l_cf=3.0, ratio=0.25)
    assert E.param_names(ks) == ("l_df", "l_cf", "ratio", "noise")
    p = H.get_params(ks, 0.01)
    assert p == dict(l_df=2.0, l_cf=3.0, ratio=0.25, noise=0.01)
    k2, nz = H.set_params(ks, dict(p, l_cf=7.0))
    assert k2.l_cf == 7.0 and k2.kind == "mixed" and nz == 0.01
    ard = E.KernelSpec(family="ard", variances=(0.5, 0.2), lengthscales=((1.0, 2.0, 3.0), (4.0, 5.0, 6.0)))
    names = E.param_names(ard)
    assert names == ("variance_0", "lengthscale_0_0", "lengthscale_0_1", "lengthscale_0_2",
                     "variance_1", "lengthscale_1_0", "lengthscale_1_1", "lengthscale_1_2", "noise")
    pa = H.get_params(ard, 0.004)
    assert list(pa.values()) == [0.5, 1.0, 2.0, 3.0, 0.2, 4.0, 5.0, 6.0, 0.004]   # GPy param_array order
    a2, _ = H.set_params(ard, pa)
    assert a2 == ard


def test_free_names():
    assert H.free_names(E.KernelSpec(kind="df")) == ("l_df", "noise")
    assert H.free_names(E.KernelSpec(kind="cf")) == ("l_cf", "noise")
    assert H.free_names(E.KernelSpec(kind=0)) == ("l_df", "noise")
    assert H.free_names(E.KernelSpec(kind="mixed"), fix=("noise",)) == ("l_df", "l_cf", "ratio")


@pytest.mark.parametrize("name,v", [("l_df", 3.7), ("noise", 1e-4), ("ratio", 0.3), ("ratio", 0.999)])
def test_transforms(name, v):
    z = H._to_free(name, v)
    assert math.isclose(H._from_free(name, z), v, rel_tol=1e-12)
    h = 1e-6
    fd = (H._from_free(name, z + h) - H._from_free(name, z - h)) / (2 * h)
    assert math.isclose(H._dfree(name, v), fd, rel_tol=1e-6)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp2d import hyper as H
    S, P = 11, 4
    vals = np.zeros(S)
    grads = np.zeros((S, P))
    for i in range(rank, S, world):          # the round-robin deal of hyper.sweep
        vals[i] = -np.inf if i == 7 else math.sin(i + 0.1) * 1e3 + 1.0 / 3.0
        grads[i] = np.arange(P) * 0.1 + i / 7.0
    v, g = H.allreduce_disjoint(vals, grads)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), v=v, g=g)
    dist.barrier()
    dist.destroy_process_group()


def test_sweep_allreduce_world2(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    S, P = 11, 4
    ev = np.array([-np.inf if i == 7 else math.sin(i + 0.1) * 1e3 + 1.0 / 3.0 for i in range(S)])
    eg = np.array([np.arange(P) * 0.1 + i / 7.0 for i in range(S)])
    for r in range(world):
        z = np.load(os.path.join(tmp_path, f"r{r}.npz"))
        assert np.array_equal(z["v"], ev) and np.array_equal(z["g"], eg)
