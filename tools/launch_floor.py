"""Per-launch floor of back-to-back kernels in one HIP graph replay: 100 tiny launches (a 1-element add), and 100
launches that each write 4 MB, timed with HIP events around the replay."""
import torch

torch.cuda.init()
x = torch.zeros(1, device="cuda")
big = torch.zeros(1 << 20, device="cuda")


def timed(fn, n=100, reps=20):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps / n * 1000


print(f"tiny add: {timed(lambda: x.add_(1)):.2f} us per launch", flush=True)
print(f"4 MB fill: {timed(lambda: big.fill_(1.0)):.2f} us per launch", flush=True)
print(f"4 MB add: {timed(lambda: big.add_(1.0)):.2f} us per launch", flush=True)
