"""Data-parallel semantics of eventstreamgpt_amd.train.TrainStep on a 2-rank gloo (CPU) process group.

Each rank computes its own per-rank loss (the reference's per-rank weighted_loss normalisation under DDP) on its
own subjects; TrainStep all-reduces the gradients in flat buckets and divides by the world size. The test
checks the updated parameters on both ranks against a single-process AdamW step on the mean of the per-rank
gradients.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Toy(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(6, 5)
        self.b = torch.nn.Linear(5, 3)

    def forward(self, x):
        class Out:
            pass

        o = Out()
        o.loss = self.b(torch.tanh(self.a(x))).pow(2).mean()
        return o


def _data(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(7, 6, generator=g)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eventstreamgpt_amd.train import TrainStep
    from eventstreamgpt_amd.transformer.config import OptimizationConfig

    torch.manual_seed(0)
    m = Toy()
    ts = TrainStep(m, OptimizationConfig(init_lr=0.1, lr_num_warmup_steps=0, max_training_steps=10),
                   compute_dtype=torch.float32, bucket_mb=2e-5)  # tiny buckets: exercise several all-reduces
    gb = ts.grad_buckets
    assert ts.distributed and len(gb.buckets) > 1
    launched_in_backward = []
    orig = gb._launch

    def spy(b):  # buckets launched by the post-accumulate-grad hooks, i.e. while backward is still running
        launched_in_backward.append((b, torch._C._current_graph_task_id() != -1))
        orig(b)

    gb._launch = spy
    loss = ts.step(_data(rank))
    # the logged loss (generative_modeling.py:317-318, sync_dist=True): the mean of the ranks' losses, carried in
    # the exchange's last bucket (no collective of its own)
    both = [torch.zeros(()) for _ in range(world)]
    dist.all_gather(both, loss.detach().reshape(()).clone())
    assert torch.allclose(ts.logged_loss, sum(both) / world, rtol=1e-6), (ts.logged_loss, both)
    assert not torch.equal(both[0], both[1])
    assert launched_in_backward and all(in_bwd for _, in_bwd in launched_in_backward)
    assert [b for b, _ in launched_in_backward] == list(range(len(gb.buckets)))  # index order, once each
    # every gradient is a view into the one flat exchange buffer
    base = gb.flat.data_ptr()
    for p in ts.params:
        assert base <= p.grad.data_ptr() < base + 4 * gb.flat.numel()
    q.put((rank, {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}))  # by value, not shm
    dist.destroy_process_group()


def test_two_rank_gradient_averaging():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    # single-process reference: mean of per-rank gradients, then one AdamW step at lr 0.1
    torch.manual_seed(0)
    ref = Toy()
    grads = None
    for r in range(world):
        ref.zero_grad()
        ref(_data(r)).loss.backward()
        g = [p.grad.clone() for p in ref.parameters()]
        grads = g if grads is None else [a + b for a, b in zip(grads, g)]
    for p, g in zip(ref.parameters(), grads):
        p.grad = g / world
    opt = torch.optim.AdamW(ref.parameters(), lr=0.1, weight_decay=0.01)
    opt.step()
    want = ref.state_dict()
    for r in range(world):
        for k, v in want.items():
            torch.testing.assert_close(torch.from_numpy(res[r][k]), v, rtol=1e-6, atol=1e-7)


# ---- gradient accumulation (generative_modeling.py:661-664: Lightning's accumulate_grad_batches) ----------------
ACCUM, WINDOWS = 2, 2


def _acc_data(rank, i):
    g = torch.Generator().manual_seed(1000 + 10 * rank + i)
    return torch.randn(5 + i, 6, generator=g)


def _acc_cfg():
    from eventstreamgpt_amd.transformer.config import OptimizationConfig

    return OptimizationConfig(init_lr=0.1, lr_num_warmup_steps=1, max_training_steps=10,
                              gradient_accumulation=ACCUM)


def _worker_accum(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eventstreamgpt_amd.train import TrainStep

    torch.manual_seed(0)
    m = Toy()
    ts = TrainStep(m, _acc_cfg(), compute_dtype=torch.float32, bucket_mb=2e-5)
    gb = ts.grad_buckets
    launched = []
    orig = gb._launch

    def spy(b):
        launched.append(b)
        orig(b)

    gb._launch = spy
    per_batch = []
    for i in range(ACCUM * WINDOWS):
        launched.clear()
        ts.step(_acc_data(rank, i))
        last = (i + 1) % ACCUM == 0
        # the exchange only on the window's last batch (no_sync before it), every bucket once, in index order
        per_batch.append(launched == (list(range(len(gb.buckets))) if last else []))
    q.put((rank, (per_batch, ts.sched_step, {k: v.detach().numpy().copy() for k, v in m.state_dict().items()})))
    dist.destroy_process_group()


def test_two_rank_gradient_accumulation():
    """accumulate_grad_batches = 2 under 2-rank DDP: each rank sums the gradients of its window's batches (each
    backward seeded with 1/2, as Lightning normalises the loss), the sums are averaged over the ranks once per window,
    and AdamW + the LR schedule step once per window — against a single process doing exactly that by hand."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker_accum, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    from eventstreamgpt_amd.train import poly_decay_lambda

    cfg = _acc_cfg()
    torch.manual_seed(0)
    ref = Toy()
    opt = torch.optim.AdamW(ref.parameters(), lr=cfg.init_lr, weight_decay=cfg.weight_decay)
    sched = torch.optim.lr_scheduler.LambdaLR(
        opt, poly_decay_lambda(cfg.lr_num_warmup_steps, cfg.max_training_steps, cfg.lr_decay_power, cfg.init_lr,
                               cfg.end_lr))
    for w in range(WINDOWS):
        tot = [torch.zeros_like(p) for p in ref.parameters()]
        for r in range(world):
            ref.zero_grad(set_to_none=True)
            for i in range(w * ACCUM, (w + 1) * ACCUM):
                (ref(_acc_data(r, i)).loss / ACCUM).backward()
            tot = [a + p.grad for a, p in zip(tot, ref.parameters())]
        for p, g in zip(ref.parameters(), tot):
            p.grad = g / world
        opt.step()
        sched.step()
    want = ref.state_dict()
    for r in range(world):
        per_batch, sched_step, sd = res[r]
        assert all(per_batch), per_batch
        assert sched_step == WINDOWS
        for k, v in want.items():
            torch.testing.assert_close(torch.from_numpy(sd[k]), v, rtol=1e-5, atol=1e-6)
