"""Attention backward: the fused kernel vs the split dK/dV + dQ kernels (tools build, ESGPT_ATTN_BWD_SPLIT2 read once
per process: 0 fused, 64 / 128 split with that many keys per dK/dV workgroup). Times graph-replayed launches at the
C2 / C3 / C5 / long layer shapes and saves dq|dk|dv for a cross-check between settings (tools/attn_split_cmp.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from eventstreamgpt_amd import ops as O  # noqa: E402
from eventstreamgpt_amd.kernels import tickets  # noqa: E402
from tools.gemm_time import gtime  # noqa: E402

SHAPES = [(32, 256, 4, 64, 0), (32, 512, 8, 64, 0), (32, 512, 8, 64, 32), (16, 1024, 4, 64, 0), (4, 4096, 8, 64, 0),
          (8, 300, 2, 32, 0), (4, 600, 4, 128, 0), (4, 520, 4, 16, 40)]


def main():
    tag = os.environ.get("ESGPT_ATTN_BWD_SPLIT2", "default")
    esgpt = O.load()
    out = {}
    for (B, L, H, hd, win) in SHAPES:
        D = H * hd
        g = torch.Generator(device="cuda").manual_seed(B * L + H + hd + win)
        em = torch.rand(B, L, device="cuda", generator=g) > 0.1
        em[:, 0] = True
        T = B * L * (L + 1) / 2 if not win else B * sum(min(i + 1, win) for i in range(L))
        for p in (0.0, 0.1):
            qkv = (0.5 * torch.randn(B, L, 3 * D, device="cuda", generator=g)).bfloat16()
            seed = torch.tensor([1234 + L], dtype=torch.int64, device="cuda") if p > 0 else None
            o, lse, keep = esgpt.attention(qkv, em, em, H, win, False, p, seed)
            do = torch.randn(o.shape, device="cuda", generator=g).bfloat16()
            tk = tickets(qkv.device)
            dqkv = esgpt.attention_bwd(qkv, o, do, lse, em, em, H, win, False, p, seed, keep, tk)
            out[f"{B}_{L}_{H}_{hd}_{win}_{p}"] = dqkv.float().cpu()
            tb = gtime(lambda: esgpt.attention_bwd(qkv, o, do, lse, em, em, H, win, False, p, seed, keep, tk))
            print(f"{tag:7s} B={B} L={L} H={H} hd={hd} w={win} p={p}: bwd {tb:8.1f}us "
                  f"({8 * H * hd * T / tb / 1e6:6.1f} TF/s)", flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    torch.save(out, f"gpurun_out/attn_split_{tag}.pt")


if __name__ == "__main__":
    main()
