"""Where the gradient exchange sits in a HIP-graph training step under DDP: two ranks on cuda:0
(gloo — RCCL refuses two ranks on one device), the C2 model through TrainStep with the graph cut into per-bucket
segments; rank 0 records its last step with torch.profiler (in-process tracer) and prints, for every device copy of
a bucket's exchange (gloo copies the bucket device -> host, reduces on the host and copies it back), how many of the
step's kernels ran on the device while that copy was in flight, and the step's kernel / copy timeline in order.

    python tools/ddp_overlap_trace.py [out.json]
"""
import json
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STEPS = 4


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import datetime

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    from eventstreamgpt_amd.synthetic import CONFIGS
    from eventstreamgpt_amd.train import TrainStep
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling
    from eventstreamgpt_amd.transformer.config import OptimizationConfig

    bc = CONFIGS["C2"]
    torch.manual_seed(0)
    m = CIPPTForGenerativeSequenceModeling(bc.model_config()).to("cuda:0").train()
    opt = OptimizationConfig(init_lr=1e-4, lr_num_warmup_steps=1, max_training_steps=100)
    ts = TrainStep(m, opt, torch.bfloat16, use_graph=True, bucket_mb=4.0)
    batches = [bc.batch(10 * rank + s, device="cuda:0").packed() for s in range(STEPS)]
    for b in batches[:-1]:
        ts.step(b)
    torch.cuda.synchronize()
    dist.barrier()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        ts.step(batches[-1])
        torch.cuda.synchronize()
    ts.check()
    if rank == 0:
        prof.export_chrome_trace(out)
        nseg = [len(e[0]) for e in ts.graphs.values() if e is not None]
        print(json.dumps({"buckets": len(ts.grad_buckets.buckets), "segments": nseg}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def analyse(path):
    ev = json.load(open(path))["traceEvents"]
    dev = [e for e in ev if e.get("ph") == "X" and e.get("cat") in ("kernel", "gpu_memcpy", "gpu_memset")]
    dev.sort(key=lambda e: e["ts"])
    kern = [e for e in dev if e["cat"] == "kernel"]
    copies = [e for e in dev if e["cat"] == "gpu_memcpy"]
    rows = []
    for c in copies:
        c0, c1 = c["ts"], c["ts"] + c["dur"]
        during = [k for k in kern if k["ts"] < c1 and k["ts"] + k["dur"] > c0]
        rows.append({"copy": c["name"][:40], "start_us": round(c0 - dev[0]["ts"], 1), "dur_us": round(c["dur"], 1),
                     "bytes": c.get("args", {}).get("bytes"), "kernels_in_flight": len(during),
                     "kernel_names": sorted({k["name"].split("(")[0][-40:] for k in during})[:4]})
    print(json.dumps({"kernels": len(kern), "copies": len(copies),
                      "span_us": round(dev[-1]["ts"] + dev[-1]["dur"] - dev[0]["ts"], 1)}))
    for r in rows:
        print(json.dumps(r))


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ddp_overlap_trace.json"
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    assert codes == [0, 0], codes
    analyse(out)


if __name__ == "__main__":
    main()
