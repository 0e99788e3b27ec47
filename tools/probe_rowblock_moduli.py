"""Probe for DESIGN.md §8 item 4: how many moduli each 256-row block of W = L⁻¹ needs.

The Ozaki-II variance GEMM uses one moduli count for the whole of W, set by the worst row
(gp2d.hip, gp2d_ozaki_prepare).  This probe restates that per-row bound (the smaller of
(a) l1_i·2^{pB−1} and (b) 2^{s_i+s_B}·2√kss + n·2^{pB−2} + l1_i + n) on the bench workload
and reports, per 256-row block, the count that block alone would need, plus the share of
the lower-triangular GEMM work (row block i reads 256(i+1) columns of K) that per-block
counts would skip against the data-driven and the a-priori uniform counts.

Run on the GPU box:  python tools/probe_rowblock_moduli.py
"""
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "2d-gp_amd"))
from gp2d import data as D  # noqa: E402
from gp2d import engine as E  # noqa: E402

MODULI = [256, 255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217, 211, 199, 197, 193]
PW, PB = 49, 45   # ozaki.hpp defaults


def nmod_bits(log2_pmax):
    need, bits = log2_pmax + 2.0, 0.0
    for l, m in enumerate(MODULI):
        bits += math.log2(m)
        if bits > need:
            return l + 1
    return -1


def main():
    dev = torch.device("cuda:0")
    ntrain = int(os.environ.get("NTRAIN", "4096"))
    x1, x2, u, v = D.synthetic_tracks(ntrain, seed=2016)
    x = torch.tensor(np.stack([x1, x2], 1), device=dev)
    y = torch.tensor(np.concatenate([u, v]), device=dev)
    spec = E.KernelSpec(kind="df", l_df=5.0, l_cf=5.0, ratio=1.0)
    noise = 0.0025
    gp = E.fit(spec, x, y, noise, device=dev, variance="f64")
    gp = E.ozaki_prepare(gp)                       # data-driven count
    _, rowscale, nmod_data = gp.extra["ozaki"]
    n = gp.n
    nmod_apriori = int(E.N.lib().gp2d_ozaki_nmod_apriori(n, __import__("ctypes").byref(spec.desc()),
                                                          float(noise)))
    M = float(np.prod([float(m) for m in MODULI[:nmod_data]]))
    W = torch.tril(gp.W).abs()
    mx = W.max(dim=1).values.cpu().numpy()
    e = np.array([math.frexp(v)[1] - 1 if v > 0 else 0 for v in mx])   # ilogb
    s = PW - 1 - e
    l1 = (torch.round(torch.tril(gp.W) * torch.tensor(np.ldexp(1.0, s), device=dev)[:, None]).abs()
          .sum(dim=1).cpu().numpy())
    ssb = np.log2(M / rowscale.cpu().numpy())      # s_i + s_B
    kd = spec.kdiag() if callable(spec.kdiag) else spec.kdiag
    sq = 2.0 * math.sqrt(kd)
    a = np.ldexp(l1 * 1.01, PB - 1)
    b = np.exp2(ssb) * sq + math.ldexp(n, PB - 2) + l1 + n
    bound = np.maximum(1.0, np.minimum(a, b))
    nb = (n + 255) // 256
    per_block = [nmod_bits(math.log2(bound[i * 256:(i + 1) * 256].max())) for i in range(nb)]
    work = np.arange(1, nb + 1, dtype=float)       # row block i: 256(i+1) columns of K
    used = float((np.array(per_block) * work).sum())
    print(f"n={n} row blocks={nb} nmod data-driven={nmod_data} a-priori={nmod_apriori}")
    print("per-block counts:", per_block)
    cap11 = sum(math.log2(m) for m in MODULI[:11]) - 2.0
    lb = [math.log2(bound[i * 256:(i + 1) * 256].max()) for i in range(nb)]
    print(f"log2 bound per block: min {min(lb):.2f} max {max(lb):.2f}; 11 moduli hold {cap11:.2f} bits")
    hist = {k: per_block.count(k) for k in sorted(set(per_block))}
    print("histogram:", hist)
    for name, u in (("data-driven", nmod_data), ("a-priori", nmod_apriori)):
        print(f"work saved vs uniform {name} ({u}): {1.0 - used / (u * work.sum()):.4f}")


if __name__ == "__main__":
    main()
