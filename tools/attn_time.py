"""Graph-timed attention forward and backward at the C2 / C3 / C5 / long layer shapes (tag = ESGPT_ATTN_ORDER)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from eventstreamgpt_amd import ops as O  # noqa: E402
from eventstreamgpt_amd.kernels import tickets  # noqa: E402
from tools.gemm_time import gtime  # noqa: E402

tag = os.environ.get("ESGPT_ATTN_ORDER", "-") + "/nw" + os.environ.get("ESGPT_ATTN_FWD_NW", "-")
esgpt = O.load()
for (B, L, H, hd, win, p) in [(32, 256, 4, 64, 0, 0.1), (32, 512, 8, 64, 0, 0.1), (32, 512, 8, 64, 32, 0.1),
                              (16, 1024, 4, 64, 0, 0.1), (4, 4096, 8, 64, 0, 0.0)]:
    D = H * hd
    em = torch.ones(B, L, dtype=torch.bool, device="cuda")
    if os.environ.get("PAD") == "1":  # right padding as in the bench batches: each subject keeps 50-100 % of L events
        lens = torch.randint(L // 2, L + 1, (B,), generator=torch.Generator().manual_seed(1)).cuda()
        em = torch.arange(L, device="cuda")[None] < lens[:, None]
    T = B * L * (L + 1) / 2 if not win else B * sum(min(i + 1, win) for i in range(L))
    qkv = (0.5 * torch.randn(B, L, 3 * D, device="cuda")).bfloat16()
    seed = torch.tensor([99], dtype=torch.int64, device="cuda") if p > 0 else None
    o, lse, keep = esgpt.attention(qkv, em, em, H, win, False, p, seed)
    do = torch.randn_like(o)
    tk = tickets(qkv.device)
    tf = gtime(lambda: esgpt.attention(qkv, em, em, H, win, False, p, seed))
    tb = gtime(lambda: esgpt.attention_bwd(qkv, o, do, lse, em, em, H, win, False, p, seed, keep, tk))
    print(f"order {tag} B={B} L={L} H={H} hd={hd} w={win} p={p}: fwd {tf:7.1f}us ({4 * H * hd * T / tf / 1e6:6.1f} "
          f"TF/s)  bwd {tb:7.1f}us ({8 * H * hd * T / tb / 1e6:6.1f} TF/s)", flush=True)
