"""Which streams share a hardware queue (dev tool).  HIP maps streams onto at most
GPU_MAX_HW_QUEUES hardware queues per priority level; two streams on one queue run in order,
so a side stream that lands on the predict stream's queue cannot overlap it.  For each torch
pool stream handed out (normal and high priority): a ~20 ms spin kernel on the current
(null) stream, then an empty kernel on the candidate stream; if the candidate's kernel only
completes after the spin, the two share a queue.

    python tools/probe_queues.py [count]
"""
import json
import sys
import time

import torch


def shares_queue(a: torch.cuda.Stream, b: torch.cuda.Stream) -> bool:
    torch.cuda.synchronize()
    with torch.cuda.stream(a):
        torch.cuda._sleep(50_000_000)   # ≈ 20 ms of spinning
    ev = torch.cuda.Event()
    with torch.cuda.stream(b):
        x = torch.empty(1, device="cuda")
        x.zero_()
        ev.record(b)
    t0 = time.perf_counter()
    while not ev.query():
        if time.perf_counter() - t0 > 2.0:
            break
    dt = time.perf_counter() - t0
    torch.cuda.synchronize()
    return dt > 0.010


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    main_s = torch.cuda.current_stream()
    out = {"normal": [], "high": []}
    for i in range(n):
        s = torch.cuda.Stream()
        out["normal"].append(shares_queue(main_s, s))
    for i in range(n):
        s = torch.cuda.Stream(priority=-1)
        out["high"].append(shares_queue(main_s, s))
    print(json.dumps({"aliases_current_stream": out}))


if __name__ == "__main__":
    main()
