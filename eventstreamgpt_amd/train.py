"""Minimal Lightning-free training step (``generative_modeling.py:434-485``) for one GPU or DDP over RCCL.

* loss = model(batch).loss (per-rank weighted_loss normalisation, exactly like the reference under DDP);
* AdamW(lr=init_lr, weight_decay) + transformers' polynomial-decay-with-warmup schedule, stepped every step;
* gradients are reset to ``None`` before each backward (Lightning's ``zero_grad(set_to_none=True)``), so autograd
  hands each parameter its gradient without an accumulate-add; parameters without a gradient are skipped by
  AdamW exactly as in the reference;
* data parallelism: one process per GPU (``torch.distributed`` "nccl" = RCCL over xGMI). Gradients are packed
  into size-capped flat buckets, all-reduced and divided by world size (the DDP gradient-averaging semantics of
  the reference's Lightning trainer); a parameter without a gradient contributes zeros.
* optional HIP-graph capture of forward+backward (static shapes; batches are copied into static buffers).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .data.types import PytorchBatch
from .kernels import begin_dropout_step, check_errors, end_dropout_step
from .transformer.config import OptimizationConfig


def poly_decay_lambda(warmup: int, total: int, power: float, init_lr: float, end_lr: float):
    """``transformers.get_polynomial_decay_schedule_with_warmup`` as a multiplier of ``init_lr``."""

    def f(step: int) -> float:
        if step < warmup:
            return float(step) / float(max(1, warmup))
        if step > total:
            return end_lr / init_lr
        rem = 1 - (step - warmup) / (total - warmup)
        return ((init_lr - end_lr) * rem**power + end_lr) / init_lr

    return f


class FusedAdamW:
    """``torch.optim.AdamW`` (default betas / eps, decoupled weight decay; ``generative_modeling.py:460-466``) as ONE
    gfx950 kernel launch per step over every parameter (csrc/misc.hip ``esgpt_adamw``), instead of torch's
    multi-tensor launches. Parameters whose ``.grad`` is None are skipped, like torch. The tensor table (device
    pointers of p / grad / exp_avg / exp_avg_sq) is rebuilt only when a gradient's storage changes (never under
    HIP-graph replay, where gradients live in the graph's pool)."""

    def __init__(self, params, lr: float, weight_decay: float = 0.01, betas=(0.9, 0.999), eps: float = 1e-8):
        from . import _lib as L

        self.L = L
        self.lib = L.load()
        self.params = list(params)
        self.lr, self.weight_decay, self.betas, self.eps = lr, weight_decay, betas, eps
        self.exp_avg = [torch.zeros_like(p, memory_format=torch.contiguous_format) for p in self.params]
        self.exp_avg_sq = [torch.zeros_like(p, memory_format=torch.contiguous_format) for p in self.params]
        self.steps = [0] * len(self.params)
        self._key = None
        self._table = self._blocks = None
        self._active = []

    def zero_grad(self, set_to_none: bool = True):
        for p in self.params:
            p.grad = None

    def _plan(self):
        items = [i for i, p in enumerate(self.params) if p.grad is not None]
        for i in items:
            g = self.params[i].grad
            if not (g.is_contiguous() and g.dtype == torch.float32 and self.params[i].is_contiguous()):
                raise RuntimeError("FusedAdamW needs contiguous f32 parameters and gradients")
        key = tuple((i, self.params[i].grad.data_ptr()) for i in items)
        if key == self._key:
            return
        chunk = int(self.lib.esgpt_adamw_chunk())
        rows, blocks = [], []
        for t, i in enumerate(items):
            p = self.params[i]
            rows.append([p.data_ptr(), p.grad.data_ptr(), self.exp_avg[i].data_ptr(), self.exp_avg_sq[i].data_ptr(),
                         p.numel()])
            blocks += [(t << 40) | s for s in range(0, p.numel(), chunk)]
        dev = self.params[0].device
        self._table = torch.tensor(rows, dtype=torch.int64).to(dev)
        self._blocks = torch.tensor(blocks, dtype=torch.int64).to(dev)
        self._key = key
        self._active = items

    @torch.no_grad()
    def step(self, lr: float | None = None):
        self._plan()
        if not self._active:
            return
        # torch keeps one step counter per parameter; they advance together for parameters updated every step
        step = self.steps[self._active[0]] + 1
        for i in self._active:
            self.steps[i] += 1
        b1, b2 = self.betas
        self.L.check(self.lib.esgpt_adamw(self._table.data_ptr(), self._blocks.data_ptr(), self._blocks.numel(),
                                          float(self.lr if lr is None else lr), b1, b2, self.eps,
                                          self.weight_decay, step, self.L.stream()), "adamw")

    def state_dict(self):
        return {"state": {i: {"step": self.steps[i], "exp_avg": self.exp_avg[i], "exp_avg_sq": self.exp_avg_sq[i]}
                          for i in range(len(self.params))},
                "param_groups": [{"lr": self.lr, "betas": self.betas, "eps": self.eps,
                                  "weight_decay": self.weight_decay}]}


def graph_safe(model) -> bool:
    """True when the model's training step runs entirely through the fused CI path (capturable)."""
    from .fused import fused_supported
    from .transformer.config import StructuredEventProcessingMode

    import os

    if os.environ.get("ESGPT_FORCE_GRAPH") == "1":  # diagnostics (tools/na_graph_check.py)
        return True
    enc = getattr(model, "encoder", None)
    cfg = getattr(model, "config", None)
    if enc is None or cfg is None:
        return False
    if cfg.structured_event_processing_mode != StructuredEventProcessingMode.CONDITIONALLY_INDEPENDENT:
        return False
    return fused_supported(enc)


class TrainStep:
    def __init__(self, model: torch.nn.Module, opt_cfg: OptimizationConfig, compute_dtype=torch.bfloat16,
                 bucket_mb: float = 25.0, use_graph: bool = False):
        self.model = model
        self.cfg = opt_cfg
        self.dtype = compute_dtype
        self.distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.world = dist.get_world_size() if self.distributed else 1
        params = [p for p in model.parameters() if p.requires_grad]
        self.params = params
        dev = params[0].device
        # buckets of parameter indices in reverse order (the last layers' gradients are final first)
        self.buckets, cur, size = [], [], 0
        lim = int(bucket_mb * 2**20 / 4)
        for i in reversed(range(len(params))):
            cur.append(i)
            size += params[i].numel()
            if size >= lim:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        total = opt_cfg.max_training_steps or 1_000_000
        warm = opt_cfg.lr_num_warmup_steps or 0
        self.lr_lambda = poly_decay_lambda(warm, total, opt_cfg.lr_decay_power, opt_cfg.init_lr, opt_cfg.end_lr)
        self.sched_step = 0  # LambdaLR semantics: the first optimizer step uses lambda(0)
        if dev.type == "cuda":
            self.opt = FusedAdamW(params, lr=opt_cfg.init_lr, weight_decay=opt_cfg.weight_decay)
            self.sched = None
        else:
            self.opt = torch.optim.AdamW(params, lr=opt_cfg.init_lr, weight_decay=opt_cfg.weight_decay)
            self.sched = torch.optim.lr_scheduler.LambdaLR(self.opt, self.lr_lambda)
        # HIP-graph capture only for the fully fused CI step (every kernel ours). The module-by-module paths (NA
        # blocks, unsupported CI shapes) run PyTorch-ROCm GEMMs whose bias-gradient results were garbage on graph
        # replay (tools/na_graph_check.py: c_fc.bias gradients ~1e38 from the second replay on); they run eagerly.
        self.use_graph = use_graph and graph_safe(model)
        self.graph = None
        self.static_batch = None
        self.static_loss = None

    # --------------------------------------------------------------------------------------------------------
    def _fwd_bwd(self, batch: PytorchBatch):
        # The autocast weight-cast cache must be off under HIP-graph capture (cached casts would outlive capture).
        dev = self.params[0].device
        if dev.type == "cuda":
            begin_dropout_step(dev)
        with torch.autocast("cuda", dtype=self.dtype, enabled=self.dtype != torch.float32,
                            cache_enabled=not self.use_graph):
            out = self.model(batch)
        out.loss.backward()
        if dev.type == "cuda":
            end_dropout_step(dev)
        return out.loss.detach()

    def _allreduce(self):
        if not self.distributed:
            return
        for idx in self.buckets:
            ps = [self.params[i] for i in idx]
            for p in ps:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
            grads = [p.grad for p in ps]
            flat = torch._utils._flatten_dense_tensors(grads)
            dist.all_reduce(flat)
            flat.div_(self.world)
            torch._foreach_copy_(grads, torch._utils._unflatten_dense_tensors(flat, grads))

    def _copy_into_static(self, batch: PytorchBatch):
        # one D2D copy when the batch is packed (native collate / .packed()), else one per field
        self.static_batch.copy_(batch, non_blocking=True)

    def step(self, batch: PytorchBatch) -> torch.Tensor:
        if not self.use_graph:
            self.opt.zero_grad(set_to_none=True)
            loss = self._fwd_bwd(batch)
        else:
            if self.graph is None:
                self._capture(batch)
            self._copy_into_static(batch)
            self.graph.replay()
            loss = self.static_loss
        self._allreduce()
        if self.sched is None:
            self.opt.step(self.cfg.init_lr * self.lr_lambda(self.sched_step))
        else:
            self.opt.step()
            self.sched.step()
        self.sched_step += 1
        return loss

    def _capture(self, batch: PytorchBatch):
        self.static_batch = batch.packed()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):  # warm up allocator / lazy init outside the graph
                self.opt.zero_grad(set_to_none=True)
                self._fwd_bwd(self.static_batch)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        # gradients are (re)allocated inside the capture from the graph's pool and stay static across replays
        self.opt.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_loss = self._fwd_bwd(self.static_batch)
        torch.cuda.synchronize()

    def check(self):
        check_errors()


def init_distributed():
    """Initialises the process group from torchrun's env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*)."""
    import os

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1, 0
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        backend = "nccl"
    else:
        backend = "gloo"
    dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def n_params(model) -> int:
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def grad_bytes(model) -> int:
    return 4 * n_params(model)

