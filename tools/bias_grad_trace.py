"""One eager Linear(256->1024) -> GELU -> Linear(1024->256) backward (f32, x without grad), the case whose first bias
gradient goes wrong under HIP-graph replay (tools/graph_blaslt_repro.py); run under
`rocprofv3 --hip-runtime-trace --kernel-trace` to see which kernels and runtime calls (memsets) it issues."""
import torch
import torch.nn as nn

torch.manual_seed(0)
m = nn.Sequential(nn.Linear(256, 1024), nn.GELU(), nn.Linear(1024, 256)).cuda()
x = torch.randn(8192, 256, device="cuda")
for _ in range(2):
    m.zero_grad(set_to_none=True)
    m(x).square().mean().backward()
torch.cuda.synchronize()
torch.cuda.nvtx.range_push("marker") if hasattr(torch.cuda, "nvtx") else None
m.zero_grad(set_to_none=True)
y = m(x).square().mean()
torch.cuda.synchronize()
y.backward()
torch.cuda.synchronize()
print("done")
