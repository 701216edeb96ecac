"""Headline benchmark: CI-PPT training throughput (train events/sec) — BASELINE.json ``metric`` on ``configs[1]``
(C2: CI-PPT, 6 layers, d=256, L=256, global attention, synthetic EHR-shaped batches, one MI355X per rank).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2] [--no-graph] [--no-cpu-baseline]

A step = forward + backward + (RCCL gradient all-reduce) + AdamW + LR-schedule step on one batch of B=32
subjects per GPU (weak scaling). Inputs are resident in HBM before the timed region. Rank 0 prints ONE JSON line.
Also reported: the roofline of the dominant hot-path kernels (HIP events around each launch, averaged over an
instrumented pass of the same steps) and the CPU baseline (the f32 oracle port timed on this host's cores on a
bounded sample of the same workload).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from eventstreamgpt_amd import kernels as K  # noqa: E402
from eventstreamgpt_amd.synthetic import CONFIGS  # noqa: E402
from eventstreamgpt_amd.train import TrainStep, init_distributed  # noqa: E402
from eventstreamgpt_amd.transformer.config import OptimizationConfig  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def attention_flops_fwd(batch, cfg) -> float:
    """Algorithmic forward FLOPs per layer: 4 * H * hd * T, T = allowed (q, k) pairs over valid
    queries (causal: keys j <= i that are valid; local: also i - j < window)."""
    em = batch.event_mask.cpu()
    H, hd = cfg.num_attention_heads, cfg.head_dim
    cum = em.long().cumsum(1)
    T_glob = float((cum * em).sum())  # for each valid query: number of valid keys j <= i (global layers)
    return 4.0 * H * hd * T_glob


def embed_fwd_bytes(batch, cfg) -> float:
    """Algorithmic bytes of the JOINT input-layer kernel: gathered rows per occurrence + entries +
    output + static rows (gathered per event) + time/mask."""
    em = batch.event_mask.cpu()
    idx = batch.dynamic_indices.cpu()
    D = cfg.hidden_size
    valid = em.unsqueeze(-1) & (idx > 0)
    nnz = float(valid.sum())
    B, L, M = idx.shape
    S = batch.static_indices.shape[1]
    n_ev = float(em.sum())
    return nnz * D * 4 + B * L * M * 21 + B * L * D * 4 + n_ev * S * D * 4 + B * L * 5


def cpu_baseline(bc, seconds: float = 12.0) -> dict:
    """The f32 oracle (CPU port of the reference step: fwd + bwd + AdamW) on this host's cores, B=4 subjects."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import esgpt_oracle as O
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling

    threads = torch.get_num_threads()
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    torch.manual_seed(0)
    m = CIPPTForGenerativeSequenceModeling(cfg)
    trainable = {k for k, p in m.named_parameters() if p.requires_grad}
    params = {k: v.detach().clone().requires_grad_(k in trainable) for k, v in m.state_dict().items()}
    state = {}
    Bs = 4
    batch = bc.batch(0, batch_size=Bs)
    n_ev = float(batch.event_mask.sum())
    t0 = time.perf_counter()
    steps = 0
    while True:
        out = O.model_losses(params, cfg, batch)
        grads = torch.autograd.grad(out["loss"], [v for v in params.values() if v.requires_grad])
        named = dict(zip([k for k, v in params.items() if v.requires_grad], grads))
        with torch.no_grad():
            O.adamw_step({k: v for k, v in params.items() if v.requires_grad}, named, state, 1e-3, 0.01)
        steps += 1
        if time.perf_counter() - t0 > seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": steps * n_ev / dt, "unit": "train events/sec", "cores": threads, "kind": "port",
            "sample": f"{bc.name}: oracle f32 fwd+bwd+AdamW, B={Bs} subjects (L={bc.seq_len}), {steps} steps "
                      f"in {dt:.1f}s, torch.set_num_threads={threads}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    args = ap.parse_args()

    rank, world, local = init_distributed()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    bc = CONFIGS[args.config]
    # Reference defaults: dropout 0.1 on inputs, residuals and attention probabilities (config.py:517-519).
    cfg = bc.model_config(attention_dropout=0.1, input_dropout=0.1, resid_dropout=0.1)
    torch.manual_seed(0)
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    Model = (CIPPTForGenerativeSequenceModeling if cfg.structured_event_processing_mode == "conditionally_independent"
             else NAPPTForGenerativeSequenceModeling)
    model = Model(cfg).to(dev)
    model.train()
    opt_cfg = OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=10, max_training_steps=10_000)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    use_graph = not args.no_graph
    ts = TrainStep(model, opt_cfg, compute_dtype=dtype, use_graph=use_graph)

    n_batches = 4
    batches = [bc.batch(100 * rank + i, device=dev) for i in range(n_batches)]
    events = [float(b.event_mask.sum()) for b in batches]

    for i in range(args.warmup):
        ts.step(batches[i % n_batches])
    torch.cuda.synchronize()
    ts.check()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ts.step(batches[i % n_batches])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ts.check()
    local_events = sum(events[i % n_batches] for i in range(args.steps))
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        e = torch.tensor([local_events], device=dev, dtype=torch.float64)
        dist.all_reduce(e)
        local_events = float(e.item())
    value = local_events / elapsed

    # ---- instrumented pass: per-launch HIP events around the hot-path kernels (eager) ----
    K.TIMING["enabled"] = True
    K.TIMING["events"].clear()
    ts_eager_graph, ts.use_graph = ts.use_graph, False
    n_inst = min(args.steps, 5)
    for i in range(n_inst):
        ts.step(batches[i % n_batches])
    summ = K.timing_summary()
    K.TIMING["enabled"] = False
    ts.use_graph = ts_eager_graph

    b0 = batches[0]
    fl = attention_flops_fwd(b0, cfg)
    attn_ms = summ.get("attn_fwd", (0, float("nan")))[1]
    attn_tf = fl / (attn_ms * 1e-3) / 1e12
    peak_tf = PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_F32_TFLOPS
    eb = embed_fwd_bytes(b0, cfg)
    emb_ms = summ.get("embed_joint_fwd", (0, float("nan")))[1]
    emb_gbs = eb / (emb_ms * 1e-3) / 1e9
    roofline = {"kernel": "attn_fwd", "bound": "mfma", "achieved": round(attn_tf, 3), "peak": peak_tf,
                "unit": "TFLOP/s", "frac": round(attn_tf / peak_tf, 5), "traffic": None,
                "avg_ms": round(attn_ms, 5), "algorithmic_flops_per_launch": fl}
    aux = [{"kernel": "embed_joint_fwd", "bound": "hbm", "achieved": round(emb_gbs, 1), "peak": PEAK_HBM_GBS,
            "unit": "GB/s", "frac": round(emb_gbs / PEAK_HBM_GBS, 4), "avg_ms": round(emb_ms, 5),
            "algorithmic_bytes_per_launch": eb}]
    for k in ("attn_bwd", "embed_joint_bwd", "output_loss"):
        if k in summ:
            aux.append({"kernel": k, "avg_ms": round(summ[k][1], 5), "launches": summ[k][0]})

    result = {
        "metric": "train events/sec (node)",
        "value": round(value, 1),
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if dtype == torch.bfloat16 else "f32",
        "data": "synthetic (EHR-shaped batches, random-init weights)",
        "config": {"workload": f"{args.config}: {bc.name}", "model": "CIPPT" if "CI" in bc.name else "NAPPT",
                   "global_batch": bc.batch_size * world, "seq_len": bc.seq_len, "parallelism": f"dp{world}",
                   "events_per_step_per_gpu": round(sum(events) / n_batches, 1), "hip_graph": use_graph,
                   "dropout": {"input": 0.1, "resid": 0.1, "attention": 0.1}},
        "roofline": roofline,
        "roofline_aux": aux,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(bc)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
