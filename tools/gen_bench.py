"""Generation throughput: ``CIPPTForGenerativeSequenceModeling.generate`` on the C2 model
(random init, f32, eval) from a left-padded synthetic prompt, with and without the KV cache.

    python tools/gen_bench.py [--batch 32] [--prompt 128] [--new 64]

Prints one JSON line: generated events/s (B·new ÷ wall time of the whole generate call) per mode, plus the decode
kernel's own time from the kernels' per-launch HIP-event timing.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from eventstreamgpt_amd import kernels as K  # noqa: E402
from eventstreamgpt_amd.synthetic import CONFIGS  # noqa: E402
from eventstreamgpt_amd.transformer.conditionally_independent_model import (  # noqa: E402
    CIPPTForGenerativeSequenceModeling,
)


def left_pad(batch):
    order = torch.argsort(batch.event_mask.to(torch.int8), dim=1, stable=True)
    for k in ("event_mask", "time_delta", "dynamic_indices", "dynamic_measurement_indices", "dynamic_values",
              "dynamic_values_mask"):
        t = getattr(batch, k)
        setattr(batch, k, t.gather(1, order.view(*order.shape, *([1] * (t.dim() - 2))).expand_as(t)))
    return batch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--new", type=int, default=64)
    args = ap.parse_args()
    bc = CONFIGS[args.config]
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    torch.manual_seed(0)
    model = CIPPTForGenerativeSequenceModeling(cfg).cuda().eval()
    batch = bc.batch(0, batch_size=args.batch)
    batch = left_pad(batch[:, : args.prompt]).to("cuda")
    out = {"config": args.config, "B": args.batch, "prompt_events": args.prompt, "new_events": args.new,
           "dtype": "f32", "data": "synthetic, random init"}
    for use_cache in (True, False):
        torch.manual_seed(1)
        model.generate(batch, max_new_events=2, use_cache=use_cache)  # warm-up
        torch.cuda.synchronize()
        torch.manual_seed(1)
        t0 = time.perf_counter()
        g = model.generate(batch, max_new_events=args.new, use_cache=use_cache)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        assert g.sequence_length == args.prompt + args.new
        key = "kv_cache" if use_cache else "no_cache"
        out[key] = {"generated_events_per_s": round(args.batch * args.new / dt, 1),
                    "ms_per_generated_event": round(1e3 * dt / args.new, 3)}
        if use_cache:  # per-launch kernel times from a second, instrumented run
            K.TIMING["events"].clear()
            K.TIMING["enabled"] = True
            torch.manual_seed(1)
            model.generate(batch, max_new_events=8, use_cache=True)
            K.TIMING["enabled"] = False
            out[key]["kernels"] = {k: {"launches": n, "mean_ms": round(ms, 5)} for k, (n, ms) in
                                   K.timing_summary().items() if k in ("attn_decode", "kv_append")}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
