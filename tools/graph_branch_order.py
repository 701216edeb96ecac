"""HIP-graph replay of a main chain whose nodes each fork one node onto a side chain (the weight-gradient pattern
of backward): how much of the side chain overlaps the main chain? Prints the replay time against the serial and
the ideal (main chain + one side node) times, and the per-queue start order from HIP events."""
import os
import sys

import torch

torch.cuda.init()
cyc = int(os.environ.get("CYC", "100000"))
n = 20


def capture():
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        for i in range(n):
            torch.cuda._sleep(cyc)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                torch.cuda._sleep(cyc)
        cur.wait_stream(side)
    return g


def one():
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        torch.cuda._sleep(cyc)
    return g


def timed(g, reps=10):
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


t1 = timed(one())
tg = timed(capture())
print(f"{sys.argv[1:]} one sleep {t1:.3f} ms; graph {tg:.3f} ms; serial {2 * n * t1:.3f}; ideal {(n + 1) * t1:.3f}",
      flush=True)
