"""Does a HIP graph replay run independent branches concurrently? Two spin kernels (torch.cuda._sleep), captured
once on one stream (serial) and once forked onto a side stream (parallel); prints both replay times."""
import torch

torch.cuda.init()
cyc = 2_000_000  # ~1 ms at the shader clock


def capture(parallel: bool):
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        if parallel:
            side.wait_stream(cur)
        torch.cuda._sleep(cyc)
        if parallel:
            with torch.cuda.stream(side):
                torch.cuda._sleep(cyc)
            cur.wait_stream(side)
        else:
            torch.cuda._sleep(cyc)
    return g


for parallel in (False, True, False, True):
    g = capture(parallel)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    print(f"parallel={parallel}: {s.elapsed_time(e) / 10:.3f} ms per replay", flush=True)

# eager reference: the same two sleeps on two streams
side = torch.cuda.Stream()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    cur = torch.cuda.current_stream()
    torch.cuda._sleep(cyc)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        torch.cuda._sleep(cyc)
    cur.wait_stream(side)
e.record()
torch.cuda.synchronize()
print(f"eager two streams (dependent fork): {s.elapsed_time(e) / 10:.3f} ms", flush=True)
s.record()
for _ in range(10):
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    torch.cuda._sleep(cyc)
    with torch.cuda.stream(side):
        torch.cuda._sleep(cyc)
    cur.wait_stream(side)
e.record()
torch.cuda.synchronize()
print(f"eager two streams (independent): {s.elapsed_time(e) / 10:.3f} ms", flush=True)
