"""Embedding-bag backward (esgpt_embed_bag_bwd, deterministic sorted-CSR form) at the C2 step's batch and the C5
step's batch: graph-replayed time per launch and the §8d per-occurrence bytes. Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import embed_bwd_bytes, graph_time_ms  # noqa: E402
from eventstreamgpt_amd import _lib as L  # noqa: E402
from eventstreamgpt_amd.kernels import bag_bwd  # noqa: E402
from eventstreamgpt_amd.synthetic import CONFIGS  # noqa: E402


def main():
    for name in ("C2", "C5"):
        bc = CONFIGS[name]
        cfg = bc.model_config()
        batch = bc.batch(0, device="cuda")
        B, Lq = batch.event_mask.shape
        D, V = cfg.hidden_size, cfg.vocab_size
        dsrc = torch.randn(B * Lq, D, device="cuda")
        fn = lambda: bag_bwd(batch, [], L.BAG_JOINT, L.EMB_STATIC, 0.5, 0.5, dsrc, D, D, V, 1)  # noqa: E731
        ms = graph_time_ms(fn)
        nb = embed_bwd_bytes(batch, cfg)
        print(json.dumps({"config": name, "B": B, "L": Lq, "us": round(ms * 1e3, 2), "bytes": nb,
                          "GBs": round(nb / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
