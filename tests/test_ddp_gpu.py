"""World-size-2 data parallelism of the real training step on the GPU: both ranks on cuda:0 with the
gloo backend (the box has one GPU; RCCL refuses two ranks on one device), the CI model through TrainStep with
FusedAdamW and the HIP graph cut into per-bucket segments, each rank on its own subjects. The ranks take different
paths in the same step — rank 1's batches change length (the collate pads each batch to its own longest subject,
pytorch_dataset.py:571), so it captures a new graph while rank 0 replays, and past max_graphs it runs eagerly — and
the exchange must still pair the same buckets. Compared with one process that computes each rank's gradients
(per-rank weighted_loss normalisation), averages them and takes the same optimizer steps
(generative_modeling.py:434-485 under Lightning DDP)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
STEPS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    from eventstreamgpt_amd.synthetic import CONFIGS
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling
    from eventstreamgpt_amd.transformer.config import OptimizationConfig

    bc = CONFIGS["C1"]
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    torch.manual_seed(0)
    m = CIPPTForGenerativeSequenceModeling(cfg).to("cuda:0").train()
    opt = OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=1, max_training_steps=100)
    return bc, m, opt


LENGTHS = {0: [256, 256, 256], 1: [256, 200, 184]}  # rank 1: capture, capture, eager (max_graphs = 2)


def _batches(bc, rank):
    return [bc.batch(10 * rank + s, batch_size=8, device="cuda:0")[:, :n].packed()
            for s, n in zip(range(STEPS), LENGTHS[rank])]


class _CopySpy(torch.utils._python_dispatch.TorchDispatchMode):
    """Records the gradient copies / adds of the exchange's release (GradBuckets._launch)."""

    def __init__(self):
        super().__init__()
        self.hits = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__.split(".")[0]
        if name in ("_foreach_copy_", "_foreach_add_"):
            self.hits.append(name)
        return func(*args, **(kwargs or {}))


def _worker(rank, world, port, q):
    import datetime
    import traceback

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
        from eventstreamgpt_amd.train import TrainStep

        bc, m, opt = _setup()
        ts = TrainStep(m, opt, torch.bfloat16, use_graph=True, bucket_mb=0.05, max_graphs=2)  # several buckets
        assert ts.use_graph and ts.distributed and len(ts.grad_buckets.buckets) > 1
        order = []
        orig = ts.grad_buckets._launch

        def spy(b):
            order.append(b)
            orig(b)

        ts.grad_buckets._launch = spy
        assert ts.grad_buckets.zero_copy
        copies = _CopySpy()
        losses = []
        for i, b in enumerate(_batches(bc, rank)):
            order.clear()
            with copies:  # capture (warm-up + segmented capture), replay and the eager step past max_graphs
                losses.append(float(ts.step(b)))
            nb = len(ts.grad_buckets.buckets)
            assert order == list(range(nb)), (i, order)  # one exchange per bucket, in index order, every step
            q.put(("progress", rank, f"step {i} loss {losses[-1]:.6f}"))
        ts.check()
        segs = [len(e[0]) for e in ts.graphs.values() if e is not None]
        assert len(ts.graphs) == (1 if rank == 0 else 2) and all(n > 1 for n in segs), segs
        gb = ts.grad_buckets
        # zero-copy exchange: every gradient was written by its backward kernel into its own view of the buffer
        # (the q|k|v, LayerNorm and head groups laid out adjacently by the warm-up's relayout); no copy kernel ran
        in_flat = all(p.grad.data_ptr() == gb.views[i].data_ptr() for i, p in enumerate(ts.params))
        assert copies.hits == [], copies.hits
        assert len(gb.laid_out) > 0, "no parameter groups recorded"
        q.put(("done", rank, (losses, in_flat, {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()})))
        dist.destroy_process_group()
    except BaseException:
        q.put(("error", rank, traceback.format_exc()))
        raise


def test_two_ranks_on_one_gpu_match_averaged_gradients():
    import queue
    import time

    from eventstreamgpt_amd.train import FusedAdamW, poly_decay_lambda

    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.time() + 150
    try:
        while len(res) < world:
            try:
                kind, r, payload = q.get(timeout=5)
            except queue.Empty:
                assert time.time() < deadline, "ranks did not finish in 150 s"
                assert all(p.is_alive() or p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
                continue
            if kind == "error":
                raise AssertionError(f"rank {r} failed:\n{payload}")
            if kind == "progress":
                print(f"rank {r}: {payload}", flush=True)
                continue
            res[r] = payload
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0

    # single process: per-rank losses / gradients on each rank's batch, averaged, then the same AdamW steps
    bc, m, opt_cfg = _setup()
    params = [p for p in m.parameters() if p.requires_grad]
    opt = FusedAdamW(params, lr=opt_cfg.init_lr, weight_decay=opt_cfg.weight_decay)
    lam = poly_decay_lambda(opt_cfg.lr_num_warmup_steps, opt_cfg.max_training_steps, opt_cfg.lr_decay_power,
                            opt_cfg.init_lr, opt_cfg.end_lr)
    batches = {r: _batches(bc, r) for r in range(world)}
    for s in range(STEPS):
        acc = [torch.zeros_like(p) for p in params]
        for r in range(world):
            for p in params:
                p.grad = None
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = m(batches[r][s]).loss
            loss.backward()
            assert abs(float(loss) - res[r][0][s]) <= 1e-3 * abs(float(loss)), (r, s)
            for a, p in zip(acc, params):
                a += p.grad
        for a, p in zip(acc, params):
            p.grad = a / world
        opt.step(opt_cfg.init_lr * lam(s))
    want = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    for r in range(world):
        assert res[r][1], "param.grad must be the exchange buffer's own views"
        for k, v in want.items():
            got = torch.from_numpy(res[r][2][k])
            assert (got.float() - v.float()).abs().max().item() < 1e-4, (r, k)


def _run_ranks(target, world=2, budget=150):
    """Spawns `world` ranks of `target(rank, world, port, q)`; returns {rank: payload} of their "done" messages."""
    import queue
    import time

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.time() + budget
    try:
        while len(res) < world:
            try:
                kind, r, payload = q.get(timeout=5)
            except queue.Empty:
                assert time.time() < deadline, f"ranks did not finish in {budget} s"
                assert all(p.is_alive() or p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
                continue
            if kind == "error":
                raise AssertionError(f"rank {r} failed:\n{payload}")
            if kind == "progress":
                print(f"rank {r}: {payload}", flush=True)
                continue
            res[r] = payload
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return res


def _worker_peer_error(rank, world, port, q):
    """Rank 1's second batch holds an out-of-range embedding index. Both ranks must skip that step's update and
    raise at the same step (rank 1 the reference's AssertionError, rank 0 the peer RuntimeError), then train on
    in lockstep."""
    import datetime
    import traceback

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
        from eventstreamgpt_amd.train import TrainStep

        bc, m, opt = _setup()
        ts = TrainStep(m, opt, torch.bfloat16, use_graph=True, bucket_mb=0.05)
        good = [bc.batch(10 * rank + s, batch_size=8, device="cuda:0").packed() for s in range(3)]
        bad = bc.batch(10 * rank + 1, batch_size=8)
        if rank == 1:
            bad.dynamic_indices[2, 3, 0] = m.config.vocab_size + 5
        bad = bad.to("cuda:0").packed()
        ts.step(good[0])
        ts.check()
        before = {k: v.detach().clone() for k, v in m.state_dict().items()}
        raised = None
        try:
            ts.step(bad)
            ts.check()
        except (AssertionError, RuntimeError) as e:
            raised = (type(e).__name__, str(e))
        untouched = all(torch.equal(v, before[k]) for k, v in m.state_dict().items())
        ts.step(good[2])
        ts.check()
        q.put(("done", rank, (raised, untouched, ts.opt.steps[:3],
                              {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()})))
        dist.destroy_process_group()
    except BaseException:
        q.put(("error", rank, traceback.format_exc()))
        raise


def test_device_error_on_one_rank_is_a_collective_decision():
    res = _run_ranks(_worker_peer_error)
    assert res[1][0] is not None and res[1][0][0] == "AssertionError" and "Invalid embedding!" in res[1][0][1], res[1][0]
    assert res[0][0] is not None and res[0][0][0] == "RuntimeError" and "another data-parallel rank" in res[0][0][1]
    for r in (0, 1):
        assert res[r][1], f"rank {r} updated its parameters on the failed step"
        assert res[r][2] == [2, 2, 2], res[r][2]  # AdamW counts: the failed step rolled back on both ranks
    for k in res[0][3]:  # still in lockstep after the failed step
        assert (torch.from_numpy(res[0][3][k]).float() - torch.from_numpy(res[1][3][k]).float()).abs().max() == 0, k


def _worker_rccl_single(rank, world, port, q):
    """One rank over RCCL ("nccl"): the bucketed exchange with ReduceOp.AVG, issued between HIP-graph segment
    replays, on the real collective library (a one-GPU box cannot host two RCCL ranks; the AVG of one rank is the
    identity, so the run must equal the same steps without DDP)."""
    import datetime
    import traceback

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        torch.cuda.set_device(0)
        from eventstreamgpt_amd.train import GradBuckets, TrainStep

        def run(ddp):
            bc, m, opt = _setup()
            ts = TrainStep(m, opt, torch.bfloat16, use_graph=True, bucket_mb=0.05)
            if ddp:
                ts.grad_buckets = GradBuckets(ts.params, 1, 0.05, err_check=True)
                ts.grad_buckets.zero_copy = True  # the backward kernels write into the RCCL exchange buffer
                assert ts.grad_buckets.avg and len(ts.grad_buckets.buckets) > 1
            for s in range(STEPS):
                ts.step(bc.batch(s, batch_size=8, device="cuda:0").packed())
            ts.check()
            segs = [len(e[0]) for e in ts.graphs.values() if e is not None]
            return {k: v.detach().clone() for k, v in m.state_dict().items()}, segs

        dist.init_process_group("nccl", rank=0, world_size=1, timeout=datetime.timedelta(seconds=60))
        assert dist.get_backend() == "nccl"
        got, segs = run(True)
        want, _ = run(False)
        diff = max((got[k].float() - want[k].float()).abs().max().item() for k in want)
        q.put(("done", rank, (diff, segs)))
        dist.destroy_process_group()
    except BaseException:
        q.put(("error", rank, traceback.format_exc()))
        raise


def test_rccl_exchange_single_rank_matches_no_ddp():
    res = _run_ranks(_worker_rccl_single, world=1)
    diff, segs = res[0]
    assert segs and all(n > 1 for n in segs), segs  # the captured step was cut into per-bucket segments
    # equal to f32 rounding: the segmented capture flushes the deferred LayerNorm column sums at each segment
    # boundary, a different launch grouping of the same sums (measured: 7.5e-9 after three steps)
    assert diff < 1e-6, diff


def _worker_peer_error_no_check(rank, world, port, q):
    """As _worker_peer_error, but without check() between steps: the error of step k must be raised on BOTH ranks at
    the submission of step k + 2, never earlier on one rank because its event happened to be complete (then the
    other rank would run step k + 1's collectives alone)."""
    import datetime
    import traceback

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
        from eventstreamgpt_amd.train import TrainStep

        bc, m, opt = _setup()
        ts = TrainStep(m, opt, torch.bfloat16, use_graph=True, bucket_mb=0.05)
        batches = [bc.batch(10 * rank + s, batch_size=8) for s in range(6)]
        if rank == 1:
            batches[1].dynamic_indices[2, 3, 0] = m.config.vocab_size + 5
        batches = [b.to("cuda:0").packed() for b in batches]
        raised_at = []
        for i, b in enumerate(batches):
            torch.cuda.synchronize()  # every earlier step's event is complete when step i is submitted
            try:
                ts.step(b)
            except (AssertionError, RuntimeError) as e:
                raised_at.append((i, type(e).__name__))
        ts.check()
        q.put(("done", rank, (raised_at, {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()})))
        dist.destroy_process_group()
    except BaseException:
        q.put(("error", rank, traceback.format_exc()))
        raise


def test_device_error_raised_at_the_same_step_on_every_rank_without_check():
    res = _run_ranks(_worker_peer_error_no_check)
    assert res[1][0] == [(3, "AssertionError")], res[1][0]
    assert res[0][0] == [(3, "RuntimeError")], res[0][0]
    for k in res[0][1]:  # in lockstep afterwards
        assert (torch.from_numpy(res[0][1][k]).float() - torch.from_numpy(res[1][1][k]).float()).abs().max() == 0, k


def test_bench_two_ranks_end_to_end():
    """bench.py --gpus 2 as the driver's scaling run launches it (its own torch.distributed.run child, the ranks'
    barriers, the MAX / SUM reductions of the timed region, rank 0's one JSON line), rehearsed on the one-GPU box:
    both ranks on device 0 over gloo (init_distributed's ESGPT_DIST_BACKEND / ESGPT_DIST_ONE_DEVICE test override)."""
    import json
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ESGPT_DIST_BACKEND="gloo", ESGPT_DIST_ONE_DEVICE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--no-roofline", "--no-cpu-baseline", "--no-hbm-line"], cwd=repo, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 2 * 32 and d["scaling"] == "weak"
    # value = the events of BOTH ranks over the max-over-ranks wall time of the 3 timed steps
    per_rank_events = d["config"]["events_per_step_per_gpu"]
    assert d["value"] > 0 and abs(d["value"] * d["ms_per_step"] * 1e-3 - 2 * per_rank_events) < 0.25 * 2 * per_rank_events
