"""Times the dependency-graph attention (small4 path) of C4 at its bench shape: qkv [B*L, G+1, 3D] bf16, H heads,
static_kv_first, dropout 0.1; forward and backward, median of graph-free repeats (HIP events)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from eventstreamgpt_amd import ops  # noqa: E402
from eventstreamgpt_amd.kernels import tickets  # noqa: E402

esgpt = ops.load()
BL, T, D, H = 32 * 256, 5, 256, 4
torch.manual_seed(0)
qkv = (torch.randn(BL, T, 3 * D, device="cuda") * 0.5).to(torch.bfloat16)
seed = torch.tensor([1234], dtype=torch.int64, device="cuda")
o, lse, keep = esgpt.attention(qkv, None, None, H, 0, True, 0.1, seed)
do = torch.randn_like(o)
tk = tickets(qkv.device)


def t(fn, n=20, reps=7):
    """Per-call device time: n calls captured in one HIP graph (no host launch gaps), median of reps replays."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / n)
    return sorted(ts)[reps // 2]


f = t(lambda: esgpt.attention(qkv, None, None, H, 0, True, 0.1, seed))
b = t(lambda: esgpt.attention_bwd(qkv, o, do, lse, None, None, H, 0, True, 0.1, seed, keep, tk))
ref = esgpt.attention_bwd(qkv, o, do, lse, None, None, H, 0, True, 0.1, seed, keep, tk)
o2, _, _ = esgpt.attention(qkv, None, None, H, 0, True, 0.1, seed)
print(f"ni={os.environ.get('ESGPT_SMALL4_NI', 'default')} fwd {f:.1f} us  bwd {b:.1f} us  "
      f"o_sum {o2.float().sum().item():.6f} dqkv_sum {ref.float().sum().item():.6f} "
      f"dq0_abs {ref[:, 0, :D].float().abs().max().item():.3g}", flush=True)
