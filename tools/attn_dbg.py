"""Debug: the attention forward at one shape under the current ESGPT_ATTN_FWD_NW, against a torch f32 restatement."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from eventstreamgpt_amd import ops as O  # noqa: E402

esgpt = O.load()
B, L, H, hd = [int(x) for x in os.environ.get("SHAPE", "2,260,4,16").split(",")]
p = float(os.environ.get("P", "0.0"))
D = H * hd
g = torch.Generator().manual_seed(5)
qkv = (torch.randn(B, L, 3 * D, generator=g) * 0.5).cuda().bfloat16()
lens = torch.randint(max(1, L // 2), L + 1, (B,), generator=torch.Generator().manual_seed(3))
km = (torch.arange(L)[None] < lens[:, None]).cuda()
seed = torch.tensor([7], dtype=torch.int64, device="cuda") if p > 0 else None
o, lse, keep = esgpt.attention(qkv, km, km, H, 0, False, p, seed)
q, k, v = qkv.float().split(D, -1)
q = q.view(B, L, H, hd).transpose(1, 2)
k = k.view(B, L, H, hd).transpose(1, 2)
v = v.view(B, L, H, hd).transpose(1, 2)
s = q @ k.transpose(-1, -2)
s = s.masked_fill(~torch.ones(L, L, dtype=torch.bool, device="cuda").tril(), -1e30)
s = s.masked_fill(~km[:, None, None, :], -1e30)
ref = (s.softmax(-1) @ v).transpose(1, 2).reshape(B, L, D)
ref = torch.where(km[..., None], ref, torch.zeros_like(ref))
err = torch.where(km[..., None], (o.float() - ref).abs(), torch.zeros_like(ref))
print(os.environ.get("ESGPT_ATTN_FWD_NW"), "shape", B, L, H, hd, "p", p, "max err", err.max().item(),
      "rows bad", int((err.amax(-1) > 0.05).sum()), "first bad", (err.amax(-1) > 0.05).nonzero()[:4].tolist())
