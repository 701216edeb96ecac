"""Eager launches of the C2 attention forward / backward (B=32, L=256, H=4, hd=64; ATTN_SHAPE=long: B=4, L=4096,
H=8) for counter collection:
    rocprofv3 --pmc <counters> -- python tools/attn_pmc.py [p]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from eventstreamgpt_amd import ops as O  # noqa: E402
from eventstreamgpt_amd.kernels import next_dropout_seed, tickets  # noqa: E402


def main():
    p = float(sys.argv[1]) if len(sys.argv) > 1 else 0.0
    esgpt = O.load()
    B, L, H, hd = (4, 4096, 8, 64) if os.environ.get("ATTN_SHAPE") == "long" else (32, 256, 4, 64)
    D = H * hd
    em = torch.ones(B, L, dtype=torch.bool, device="cuda")
    qkv = (0.5 * torch.randn(B, L, 3 * D, device="cuda")).bfloat16()
    seed = next_dropout_seed(qkv.device) if p > 0 else None
    o, lse, keep = esgpt.attention(qkv, em, em, H, 0, False, p, seed)
    do = torch.randn_like(o)
    tk = tickets(qkv.device)
    for _ in range(5):
        esgpt.attention(qkv, em, em, H, 0, False, p, seed)
        esgpt.attention_bwd(qkv, o, do, lse, em, em, H, 0, False, p, seed, keep, tk)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
