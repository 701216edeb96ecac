"""Times the packed-QKV attention kernels (fwd, bwd) at the C2 / C5 layer shapes, with and without dropout, as
graph-replayed launches (tools/gemm_time.gtime), and prints achieved TFLOP/s against the algorithmic FLOPs (fwd
4*H*hd*T, bwd 8*H*hd*T over allowed (q, k) pairs)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from eventstreamgpt_amd import ops as O  # noqa: E402
from eventstreamgpt_amd.kernels import next_dropout_seed, tickets  # noqa: E402
from tools.gemm_time import gtime  # noqa: E402


def main():
    esgpt = O.load()
    for (B, L, H, hd, win) in [(32, 256, 4, 64, 0), (32, 512, 8, 64, 0), (32, 512, 8, 64, 32), (16, 1024, 4, 64, 0),
                              (4, 4096, 8, 64, 0)]:
        D = H * hd
        em = torch.ones(B, L, dtype=torch.bool, device="cuda")
        T = B * L * (L + 1) / 2 if not win else B * sum(min(i + 1, win) for i in range(L))
        for p in (0.0, 0.1):
            qkv = (0.5 * torch.randn(B, L, 3 * D, device="cuda")).bfloat16()
            seed = next_dropout_seed(qkv.device) if p > 0 else None
            o, lse, keep = esgpt.attention(qkv, em, em, H, win, False, p, seed)
            do = torch.randn_like(o)
            tk = tickets(qkv.device)
            tf = gtime(lambda: esgpt.attention(qkv, em, em, H, win, False, p, seed))
            tb = gtime(lambda: esgpt.attention_bwd(qkv, o, do, lse, em, em, H, win, False, p, seed, keep, tk))
            th = gtime(lambda: esgpt.attention_bwd(qkv, o, do, lse, em, em, H, win, False, p, seed, None, tk))
            print(f"B={B} L={L} H={H} hd={hd} w={win} p={p}: fwd {tf:7.1f}us ({4 * H * hd * T / tf / 1e6:6.1f} TF/s)  "
                  f"bwd {tb:7.1f}us ({8 * H * hd * T / tb / 1e6:6.1f} TF/s)  bwd re-hashing the mask {th:7.1f}us",
                  flush=True)


if __name__ == "__main__":
    main()
