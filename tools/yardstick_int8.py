"""Vendor yardstick for the dominant kernel: what the ROCm library int8
GEMM (torch._int_mm → hipBLASLt) reaches on this chip at the variance product's shape,
M = 8192 (W rows, n at N_train = 4096), N = 16384 (one 8192-point chunk, u and v columns),
K = 8192, on random and on zero operands.  Dense count 2·M·N·K (the library does not know W is
triangular); our kernel's executed count is about half of it.

    python tools/yardstick_int8.py [--reps 20]
"""
import argparse
import json

import torch

PEAK = 5000.0   # dense int8 TOP/s (MI355X_MICROARCH.md: 2x the BF16 rate)


def bench(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--k", type=int, default=8192)
    a = ap.parse_args()
    M, N, K = a.m, a.n, a.k
    g = torch.Generator(device="cuda").manual_seed(0)
    res = {"shape": [M, N, K], "dense_ops": 2.0 * M * N * K, "peak_tops": PEAK}
    for data in ("random", "zeros"):
        if data == "random":
            A = torch.randint(-128, 128, (M, K), dtype=torch.int8, device="cuda", generator=g)
            Bt = torch.randint(-128, 128, (N, K), dtype=torch.int8, device="cuda", generator=g)
        else:
            A = torch.zeros((M, K), dtype=torch.int8, device="cuda")
            Bt = torch.zeros((N, K), dtype=torch.int8, device="cuda")
        for layout in ("NT", "NN"):
            B = Bt.t() if layout == "NT" else Bt.t().contiguous()
            try:
                ms = bench(lambda: torch._int_mm(A, B), a.reps)
                tops = 2.0 * M * N * K / (ms * 1e-3) / 1e12
                res[f"{data}_{layout}"] = {"ms": ms, "tops": tops, "frac": tops / PEAK}
            except Exception as e:  # noqa: BLE001
                res[f"{data}_{layout}"] = {"error": repr(e)[:300]}
            print(json.dumps({data + "_" + layout: res[f"{data}_{layout}"]}), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
