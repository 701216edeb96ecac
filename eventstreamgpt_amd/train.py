"""Minimal Lightning-free training step (``generative_modeling.py:434-485``) for one GPU or DDP over RCCL.

* loss = model(batch).loss (per-rank weighted_loss normalisation, exactly like the reference under DDP);
* AdamW(lr=init_lr, weight_decay) + transformers' polynomial-decay-with-warmup schedule, stepped every step
  (``configure_optimizers``, ``generative_modeling.py:460-485``); one step count per parameter, as torch keeps;
* gradients are reset to ``None`` before each backward (Lightning's ``zero_grad(set_to_none=True)``), so autograd
  hands each parameter its gradient without an accumulate-add; parameters without a gradient are skipped by
  AdamW exactly as in the reference;
* data-dependent errors (bad embedding index, NaN TTE log-likelihood, subject without an observed TTE) are raised
  with the reference's exception type and message. The kernels flag them in a device error block whose flag word
  each step's first launch starts afresh (each step's flags are its own), moving the previous step's flags into a
  sticky word; the AdamW kernel skips its update while either is set. So the failing step k AND every step
  already queued behind it leave the parameters untouched (the reference raises before its optimizer step and
  never runs k + 1: the parameters stay at their pre-error values). ``step`` raises the error of step k at the
  latest when step k + 2 is submitted (the host never waits for the step it just queued), ``check()`` at once; the
  AdamW and LR-schedule counters of step k and of the discarded later steps are rolled back, and the block
  (sticky word included) is cleared, before the raise;
* data parallelism: one process per GPU (``torch.distributed`` "nccl" = RCCL over xGMI); a device error on any rank
  is a collective decision carried by the gradient exchange (GradBuckets): every rank skips the step and raises.
  Every ``param.grad`` ends
  the step as a view into one flat f32 buffer laid out last-layer-first and cut into buckets; every step issues
  exactly one all-reduce (average) per bucket, in bucket-index order on every rank, whichever path (eager, graph
  capture, graph replay) the rank takes. A bucket is launched as soon as backward has produced its gradients and
  those of every lower-index bucket, so the exchange overlaps the rest of backward. Under HIP
  graphs the captured step is split at those points into segment graphs; each segment's buckets are exchanged
  while the next segment replays;
* the LayerNorm backwards' column sums (d ln_w, d ln_b) of a whole backward pass in one launch (``defer_colsums``);
* optionally (``overlap_weight_grads``) the projections' weight / bias gradients run on a second stream (joined
  before the exchange and AdamW), off backward's critical path;
* optional HIP-graph capture of forward+backward, one graph per batch shape signature (static shapes; batches are
  copied into the graph's static buffers). A batch whose signature matches no captured graph is captured (up to
  ``max_graphs``) or run eagerly — never broadcast into the wrong buffers. A signature whose warm-up pass runs any
  ATen GEMM (a module-by-module fallback through PyTorch-ROCm BLAS, e.g. a token count the fused blocks do not
  take) or any ATen reduction (whose semaphore memset does not replay correctly) is never captured: it runs
  eagerly.
"""
from __future__ import annotations

import weakref
from collections import deque

import torch
import torch.distributed as dist

from .data.types import PytorchBatch
from .kernels import (begin_dropout_step, check_errors, colsum_deferral_active, deferred_colsums,
                      end_dropout_step, err_word, flush_colsums, grad_destinations, join_weight_grads,
                      raise_for_error, weight_grad_overlap, weight_grad_overlap_active)
from ._lib import FLAG_PEER_RANK
from .transformer.config import OptimizationConfig


def poly_decay_lambda(warmup: int, total: int, power: float, init_lr: float, end_lr: float):
    """``transformers.get_polynomial_decay_schedule_with_warmup`` (its ``lr_lambda``) as a multiplier of
    ``init_lr``; raises the same ValueError when ``end_lr`` is not below ``init_lr``."""
    if not (init_lr > end_lr):
        raise ValueError(f"lr_end ({end_lr}) must be smaller than initial lr ({init_lr})")

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
    gfx950 kernel launch per step over every parameter (``torch.ops.esgpt.adamw`` → csrc/misc.hip ``esgpt_adamw``),
    instead of torch's multi-tensor launches. Parameters whose ``.grad`` is None are skipped and keep their step count, like torch;
    when the active parameters' step counts differ, their bias corrections go to the kernel as a per-tensor table.
    The tensor table (device pointers of p / grad / exp_avg / exp_avg_sq) is rebuilt only when a gradient's storage
    changes (never under HIP-graph replay, where gradients live in the graph's pool). The launch is a no-op while
    the device error block holds a flag (``err``)."""

    def __init__(self, params, lr: float, weight_decay: float = 0.01, betas=(0.9, 0.999), eps: float = 1e-8):
        from . import _lib as L
        from . import ops

        self.L = L
        self.lib = L.load()
        self.ops = ops.load()
        self.params = list(params)
        self.lr, self.weight_decay, self.betas, self.eps = lr, weight_decay, betas, eps
        self.exp_avg = [torch.zeros_like(p, memory_format=torch.contiguous_format) for p in self.params]
        self.exp_avg_sq = [torch.zeros_like(p, memory_format=torch.contiguous_format) for p in self.params]
        self.steps = [0] * len(self.params)  # host mirror of the device counters (state_dict, error rollback)
        self._key = None
        self._plan_cur = None
        self._active = []
        dev = self.params[0].device
        # device state of the step: per-parameter step counts + the schedule's step (esgpt_adamw_prepare), the step's lr
        self._counters = torch.zeros(len(self.params) + 1, dtype=torch.int64, device=dev)
        self._lr_dev = torch.empty(1, dtype=torch.float32, device=dev)
        # (kind, warmup, total, power, init_lr, end_lr): kind 0 = constant lr; TrainStep installs its polynomial decay
        self.schedule = (0, 0, 1, 1.0, float(lr), 0.0)

    def zero_grad(self, set_to_none: bool = True):
        for p in self.params:
            p.grad = None

    def make_plan(self, items: list | None = None, fill: bool = True) -> dict:
        """The launch tables of the parameters that hold a gradient now (or of ``items``): tensor table (p / grad /
        exp_avg / exp_avg_sq pointers), chunk list, active indices (host and device) and the per-tensor
        bias-correction buffer. A captured optimizer step keeps its own plan alive (its graph reads these buffers).
        ``fill=False``: the table's pointers are written later (``fill_table``) — a plan made before a HIP-graph
        capture whose gradients the capture itself allocates (the kernel reads the table when it runs)."""
        if items is None:
            items = [i for i, p in enumerate(self.params) if p.grad is not None]
        chunk = int(self.lib.esgpt_adamw_chunk())
        blocks = []
        for t, i in enumerate(items):
            blocks += [(t << 40) | s for s in range(0, self.params[i].numel(), chunk)]
        dev = self.params[0].device
        plan = {"active": list(items), "table": torch.zeros(len(items), 5, dtype=torch.int64, device=dev),
                "blocks": torch.tensor(blocks, dtype=torch.int64).to(dev),
                "active_dev": torch.tensor(items, dtype=torch.int32).to(dev),
                "per": torch.empty(2 * max(1, len(items)), dtype=torch.float32, device=dev)}
        if fill:
            self.fill_table(plan)
        return plan

    def fill_table(self, plan: dict) -> None:
        """Writes the plan's tensor table from the parameters' current gradients."""
        rows = []
        for i in plan["active"]:
            p, g = self.params[i], self.params[i].grad
            if g is None or not (g.is_contiguous() and g.dtype == torch.float32 and p.is_contiguous()):
                raise RuntimeError("FusedAdamW needs contiguous f32 parameters and gradients")
            rows.append([p.data_ptr(), g.data_ptr(), self.exp_avg[i].data_ptr(), self.exp_avg_sq[i].data_ptr(),
                         p.numel()])
        if rows:
            plan["table"].copy_(torch.tensor(rows, dtype=torch.int64))
        plan["key"] = tuple((i, self.params[i].grad.data_ptr()) for i in plan["active"])

    def _plan(self):
        key = tuple((i, p.grad.data_ptr()) for i, p in enumerate(self.params) if p.grad is not None)
        if self._plan_cur is None or key != self._key:
            self._plan_cur = self.make_plan()
            self._key = key
            self._active = self._plan_cur["active"]
        return self._plan_cur

    def launch(self, plan: dict, lr: float | None = None, hand=None) -> bool:
        """The device step over ``plan``: esgpt_adamw_prepare (counters, lr, per-tensor bias corrections — torch's
        one ``step`` per parameter) + the update, both no-ops while the device error block holds a flag. No host
        arguments change between steps (``lr=None``: the installed schedule), so the launch replays in a graph.
        ``hand`` = (src, ring, ring_ctr, ring_tab, host_words): the step's hand-off entry written by the prepare launch
        (src — the step's loss — and the error block into ring entry ring_ctr % len(ring_tab), the error words also into
        the mapped host words when host_words != 0; TrainStep._claim). Returns whether the launch (and so the hand-off)
        happened."""
        if not plan["active"]:
            return False
        kind, warm, total, power, init_lr, end_lr = self.schedule
        if lr is not None:
            kind, init_lr = 0, float(lr)
        b1, b2 = self.betas
        self.ops.adamw_dev(plan["table"], plan["blocks"], self._counters, plan["active_dev"], len(self.params),
                           int(kind), int(warm), int(total), float(power), float(init_lr), float(end_lr), float(b1),
                           float(b2), float(self.eps), float(self.weight_decay), plan["per"], self._lr_dev,
                           err_word(self.params[0].device), *(hand if hand is not None else (None, None, None, None, 0)))
        return True

    def note_step(self, active):
        """Host mirror of the device counters: one step for each active parameter."""
        for i in active:
            self.steps[i] += 1

    @torch.no_grad()
    def step(self, lr: float | None = None, hand=None) -> bool:
        """One optimizer step; returns whether ``hand`` (see ``launch``) was written by it."""
        plan = self._plan()
        done = False
        if self.host_args:
            self._step_host_args(plan, lr)
        else:
            done = self.launch(plan, lr, hand)
        self.note_step(plan["active"])
        return done

    host_args = False  # measurement hook (bench.py --opt-host-args): round 3's launch with host lr / bias corrections

    def _step_host_args(self, plan, lr):
        if not plan["active"]:
            return
        lr = float(self.lr if lr is None else lr)
        b1, b2 = self.betas
        steps = [self.steps[i] + 1 for i in plan["active"]]
        per = None
        if any(s != steps[0] for s in steps):
            vals = []
            for s in steps:
                vals += [lr / (1.0 - b1**s), (1.0 - b2**s) ** 0.5]
            self._per_host = torch.tensor(vals, dtype=torch.float32).pin_memory()
            plan["per"][: len(vals)].copy_(self._per_host, non_blocking=True)
            per = plan["per"]
        self.ops.adamw(plan["table"], plan["blocks"], lr, b1, b2, self.eps, self.weight_decay, steps[0], per,
                       err_word(self.params[0].device))

    def state_dict(self):
        # the step counts AdamW actually used: the device counters (a step discarded on the device — an error flag
        # up with TrainStep(check_errors=False) — advanced the host mirror but not them); the host-argument
        # measurement path keeps no device counters
        steps = self.steps if self.host_args else [int(c) for c in self._counters[:-1].tolist()]
        return {"state": {i: {"step": steps[i], "exp_avg": self.exp_avg[i], "exp_avg_sq": self.exp_avg_sq[i]}
                          for i in range(len(self.params))},
                "param_groups": [{"lr": self.lr, "betas": self.betas, "eps": self.eps,
                                  "weight_decay": self.weight_decay}]}


def graph_safe(model, compute_dtype=torch.bfloat16) -> bool:
    """True when the model's training step is capturable as one HIP graph: the CI model through the fused encoder,
    or the NA model in bf16 (its blocks through fused.inner_block_fused; the structured-attention glue — where, pad,
    cat — is stream-ordered ATen work with static shapes). Pinned by tests/test_train_paths.py's graph-vs-eager NA
    test with host allocations between replays."""
    from .fused import fused_supported
    from .transformer.config import StructuredEventProcessingMode

    enc = getattr(model, "encoder", None)
    cfg = getattr(model, "config", None)
    if enc is None or cfg is None or not fused_supported(enc):
        return False
    mode = cfg.structured_event_processing_mode
    if mode == StructuredEventProcessingMode.CONDITIONALLY_INDEPENDENT:
        return True
    return mode == StructuredEventProcessingMode.NESTED_ATTENTION and compute_dtype == torch.bfloat16


class GradBuckets:
    """DDP gradient exchange: one flat f32 buffer holding every trainable parameter's gradient, laid out in reverse
    registration order (the last layers' gradients are produced first in backward) and cut into buckets of
    ~``bucket_mb``. A post-accumulate-grad hook counts each bucket's gradients; buckets are released strictly in
    index order — bucket b once it and every bucket below it are complete — so every rank issues the same collective
    sequence. What a release does depends on ``mode``:
      "launch"  the bucket's gradients that are not already views of the buffer are copied in (one multi-tensor
                copy), ``p.grad`` is re-pointed at its view, and the bucket is all-reduced in place (average)
                asynchronously, overlapping the rest of backward;
      "mark"    (HIP-graph capture) ``on_boundary(buckets)`` is called instead: the capture is cut there;
      "off"     nothing (graph warm-up passes: no collectives).
    ``finish()`` launches the buckets not yet launched (zero-filling gradients that were never produced), in index
    order, waits for every exchange on the current stream, and leaves every ``param.grad`` a view of the buffer
    (what FusedAdamW reads).

    Device errors are a collective decision (``err_check``): one f32 slot past the last gradient rides in the last
    bucket, set by each rank to 1 when its step raised a device error flag; after the exchange it is non-zero on
    every rank iff some rank failed, and each rank ORs ESGPT_FLAG_PEER_RANK into its error block — so every rank's
    AdamW skips the step and every rank raises at the same step (the failing rank its own exception, the others
    RuntimeError), instead of the healthy ranks running on into a collective the failing rank never joins. No
    extra collective: the flag travels with the gradients.

    Zero-copy exchange (``zero_copy``; TrainStep turns it on without gradient accumulation): the backward formulas
    write their dW / db / table / column-sum outputs straight into the buffer (kernels.grad_destinations), so a
    release only re-points ``p.grad`` and launches the all-reduce — no copy kernel, eager or under HIP-graph
    capture. One kernel output may cover several parameters (q|k|v, a LayerNorm's (w, b) sums + the unused bias
    row, the padded head): the forward records those groups (``note_group``) and ``relayout()`` — run by TrainStep
    before anything has been captured, at the same point on every rank — keeps each group adjacent, in its kernel's
    row order and followed by its scratch pad, at the position of its first member in the reversed order. Any
    gradient the kernels did not write into the buffer is still copied in at release."""

    def __init__(self, params: list, world: int, bucket_mb: float = 25.0, err_check: bool = False):
        self.params = params
        self.world = world
        dev = params[0].device
        self.avg = dist.get_backend() == "nccl"  # RCCL has ncclAvg; gloo sums (divided afterwards)
        self.err_check = err_check and dev.type == "cuda"
        self.lim = int(bucket_mb * 2**20 / 4)
        self.index = {id(p): i for i, p in enumerate(params)}
        self.groups: dict = {}  # tuple of parameter indices -> pad elements (recorded by the forward)
        self.laid_out: dict = {}  # the groups the current layout honours
        self.zero_copy = False
        self._claimed: set = set()
        self._layout()
        self.mode = "launch"
        self.on_boundary = None
        # gradient accumulation (TrainStep, OptimizationConfig.gradient_accumulation): the buffer already holds the
        # window's earlier batches — a release ADDS the batch's gradients instead of copying them
        self.add = False
        self.loss_src = None  # the current step's loss (TrainStep sets it before backward / the replay)
        self.reset()
        self._hooks = [params[i].register_post_accumulate_grad_hook(self._make_hook(i)) for i in range(len(params))]

    def _layout(self):
        """Flat buffer, per-parameter views and buckets for the groups in ``self.laid_out``."""
        params = self.params
        member = {}
        for g, pad in self.laid_out.items():
            for i in g:
                member[i] = (g, pad)
        seq, placed = [], set()
        for i in reversed(range(len(params))):
            if i in placed:
                continue
            g, pad = member.get(i, ((i,), 0))
            seq.append((g, pad))
            placed.update(g)
        total = sum(sum(params[i].numel() for i in g) + pad for g, pad in seq)
        self.flat = torch.zeros(total + 2, dtype=torch.float32, device=params[0].device)
        self.slot = self.flat[total:total + 1]  # the any-rank-failed flag (last bucket)
        # the step's loss (last bucket): after the exchange, the mean of the ranks' losses — the reference's
        # self.log("train_loss", ..., sync_dist=True) (generative_modeling.py:317-318) at no extra collective
        self.loss_slot = self.flat[total + 1:total + 2]
        self.views, self.offset, self.pad_after, self.bucket_of, self.buckets = {}, {}, {}, {}, []
        off, start, cur = 0, 0, []
        for g, pad in seq:
            for i in g:
                n = params[i].numel()
                self.views[i] = self.flat[off: off + n].view_as(params[i])
                self.offset[i] = off
                cur.append(i)
                off += n
            self.pad_after[g[-1]] = pad
            off += pad
            if off - start >= self.lim:
                self.buckets.append((cur, start, off))
                cur, start = [], off
        if cur:
            self.buckets.append((cur, start, off))
        idx, s0, e0 = self.buckets[-1]
        self.buckets[-1] = (idx, s0, e0 + 2)  # + the error and loss slots
        for b, (idx, _, _) in enumerate(self.buckets):
            for i in idx:
                self.bucket_of[i] = b

    # ---- zero-copy destinations (kernels.grad_destinations) ----------------------------------------------------
    def note_group(self, tensors, pad: int):
        idx = tuple(self.index.get(id(t), -1) for t in tensors)
        if -1 in idx or (len(idx) == 1 and pad == 0) or idx in self.groups:
            return
        if any(i in g for g in self.groups for i in idx):  # overlapping groups: the first one recorded wins
            return
        self.groups[idx] = int(pad)

    def layout_stale(self) -> bool:
        return self.zero_copy and self.groups != self.laid_out

    def relayout(self):
        """Re-cuts the buffer for the recorded groups. Only while no captured graph writes into the buffer and no
        exchange is in flight; ``param.grad`` views of the old buffer stay valid until replaced."""
        self.laid_out = dict(self.groups)
        self._layout()
        self.reset()

    def begin_pass(self):
        self._claimed.clear()

    def region(self, tensors, pad: int):
        idx = [self.index.get(id(t), -1) for t in tensors]
        if -1 in idx or any(i in self._claimed for i in idx):
            return None
        if self.pad_after.get(idx[-1], 0) != pad and not (pad == 0 and len(idx) == 1):
            return None
        off = self.offset[idx[0]]
        for a, b in zip(idx, idx[1:]):  # adjacent in the kernel's row order
            if self.offset[b] != self.offset[a] + self.params[a].numel():
                return None
        self._claimed.update(idx)
        n = sum(self.params[i].numel() for i in idx) + pad
        return self.flat[off: off + n]

    def _make_hook(self, i: int):
        def hook(p):
            b = self.bucket_of[i]
            self._ready[b] += 1
            if self._ready[b] == len(self.buckets[b][0]):
                self._complete[b] = True
                self._release()

        return hook

    def _release(self):
        newly = []
        while self._next < len(self.buckets) and self._complete[self._next]:
            newly.append(self._next)
            self._next += 1
        if not newly:
            return
        if self.mode == "launch":
            for b in newly:
                self._launch(b)
        elif self.mode == "mark":
            self.on_boundary(newly)

    def reset(self):
        self._ready = [0] * len(self.buckets)
        self._complete = [False] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._next = 0
        self._works = []

    def _launch(self, b: int):
        idx, s, e = self.buckets[b]
        src, dst = [], []
        dev = self.flat.device
        if weight_grad_overlap_active(dev):  # the bucket's weight gradients may still be in flight on their stream
            join_weight_grads(dev)
        if colsum_deferral_active(dev):  # LayerNorm gradients whose column sums are still pending
            flush_colsums(dev)
        with torch.no_grad():
            for i in idx:
                p, v = self.params[i], self.views[i]
                if p.grad is None:
                    if not self.add:
                        v.zero_()
                elif p.grad.data_ptr() != v.data_ptr():
                    src.append(p.grad)
                    dst.append(v)
            if src:
                if self.add:
                    torch._foreach_add_(dst, src)
                else:
                    torch._foreach_copy_(dst, src)
            for i in idx:
                self.params[i].grad = self.views[i]
            if b == len(self.buckets) - 1:  # this rank's verdict on its step: 1 = a device error flag is up
                if self.err_check:
                    # the flag word or the sticky word: an earlier batch of an accumulation window that failed
                    # holds only the sticky word by now (symmetric across ranks otherwise: a failed exchange
                    # raised the peer flag on every rank)
                    ew = err_word(dev)[0:1]
                    self.slot.copy_(ew.ne(0))
                else:
                    self.slot.zero_()
                if self.loss_src is not None:
                    self.loss_slot.copy_(self.loss_src.detach().reshape(1))
                else:
                    self.loss_slot.zero_()
            seg = self.flat[s:e]
            op = dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM
            self._works.append((dist.all_reduce(seg, op=op, async_op=True), seg))
        self._launched[b] = True

    def finish(self):
        for b in range(len(self.buckets)):
            if not self._launched[b]:
                self._launch(b)
        for w, seg in self._works:
            w.wait()
            if not self.avg:
                seg.div_(self.world)
        if self.err_check:  # some rank failed this step: every rank's AdamW skips it and every rank raises
            ew = err_word(self.flat.device)[0:1]
            ew.bitwise_or_(self.slot.gt(0).to(torch.int64) * FLAG_PEER_RANK)
        self.reset()


# the replayed step's loss copy rides in the optimizer's prepare launch (False, measurement hook: the pack kernel)
LOSS_IN_OPT = True


def _storage_users(t: torch.Tensor) -> int:
    """Use count of t's storage (every tensor viewing it holds one reference)."""
    return torch._C._storage_Use_Count(t.untyped_storage()._cdata)


def _copy_scalar(t: torch.Tensor) -> torch.Tensor:
    """A device copy of a small f32 tensor (one esgpt::pack launch)."""
    from . import _lib as L
    from .kernels import _ops

    return _ops().pack([t.reshape(-1)], [1], [0], [L.F32])[0].view(t.shape)


class _GemmSpy(torch.utils._python_dispatch.TorchDispatchMode):
    """Records the ATen ops of a step that must not be captured into a HIP graph (forward or backward: the mode
    follows autograd into its worker threads):
      * GEMMs — a step that left the HIP kernels for a PyTorch-ROCm BLAS fallback (the module-by-module path);
      * reductions — ATen's cross-block reduce kernel zeroes its semaphores with hipMemsetAsync, and a captured
        memset node does not re-run correctly on replay on this ROCm stack (tools/graph_blaslt_repro.py: the buffer
        holds garbage from the second replay on; fill kernels replay correctly). That is the cause of round 1's NA
        graph divergence: the module path's bias gradients are such column sums.
    The library's own kernels zero-fill with kernels, never hipMemsetAsync."""
    GEMMS = ("mm", "addmm", "bmm", "baddbmm", "matmul", "linear", "_addmm_activation", "addbmm", "_scaled_mm")
    REDUCTIONS = ("sum", "mean", "amax", "amin", "max", "min", "norm", "linalg_vector_norm", "var", "std", "prod",
                  "any", "all", "argmax", "argmin", "logsumexp", "var_mean", "std_mean", "nansum", "aminmax")

    def __init__(self):
        super().__init__()
        self.hits = set()

    BINARY = ("other", "out")  # aten.max.other / min.other (and their out= forms) are elementwise, not reductions

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__.split(".")[0]
        if func.namespace == "aten" and (name in self.GEMMS or name in self.REDUCTIONS):  # torch.ops.esgpt.* are ours
            if not (name in ("max", "min") and func._overloadname in self.BINARY):
                self.hits.add(name)
        return func(*args, **(kwargs or {}))


class TrainStep:
    def __init__(self, model: torch.nn.Module, opt_cfg: OptimizationConfig, compute_dtype=torch.bfloat16,
                 bucket_mb: float = 25.0, use_graph: bool = False, check_errors: bool = True,
                 max_graphs: int = 4, overlap_weight_grads: bool = False, defer_colsums: bool = True,
                 capture_optimizer: bool = False, zero_copy_grads: bool = True, fuse_optimizer: bool = False,
                 _force_graph: bool = False):
        self.model = model
        self.cfg = opt_cfg
        self.dtype = compute_dtype
        self.distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.world = dist.get_world_size() if self.distributed else 1
        params = [p for p in model.parameters() if p.requires_grad]
        self.params = params
        dev = params[0].device
        self.device = dev
        total = opt_cfg.max_training_steps or 1_000_000
        warm = opt_cfg.lr_num_warmup_steps or 0
        self.lr_lambda = poly_decay_lambda(warm, total, opt_cfg.lr_decay_power, opt_cfg.init_lr, opt_cfg.end_lr)
        self.sched_step = 0  # LambdaLR semantics: the first optimizer step uses lambda(0)
        if dev.type == "cuda":
            self.opt = FusedAdamW(params, lr=opt_cfg.init_lr, weight_decay=opt_cfg.weight_decay)
            # the schedule runs on the device (esgpt_adamw_prepare), so the optimizer step replays inside the graph
            self.opt.schedule = (1, warm, total, float(opt_cfg.lr_decay_power), float(opt_cfg.init_lr),
                                 float(opt_cfg.end_lr))
            self.sched = None
        else:
            self.opt = torch.optim.AdamW(params, lr=opt_cfg.init_lr, weight_decay=opt_cfg.weight_decay)
            self.sched = torch.optim.lr_scheduler.LambdaLR(self.opt, self.lr_lambda)
        self.grad_buckets = (GradBuckets(params, self.world, bucket_mb, err_check=check_errors and dev.type == "cuda")
                             if self.distributed else None)
        # HIP-graph capture for the capturable steps (graph_safe). `_force_graph` is for diagnostics of the other
        # paths (tools/na_graph_*.py).
        self.use_graph = use_graph and (_force_graph or graph_safe(model, compute_dtype))
        self.max_graphs = max_graphs
        # the optimizer step as its own graph replayed after the step's segments (no host launch per step). Off by
        # default: measured on the C2 step, same box, alternating runs, it costs ~10 us (1.7118 / 1.7115 vs 1.6981 /
        # 1.7045 ms) — the extra graph launch costs more than the two kernel launches it replaces.
        # gradient accumulation (generative_modeling.py:661-664: Lightning's accumulate_grad_batches): each batch's
        # backward is seeded with 1 / k (Lightning normalises the closure loss), the gradients of k batches are
        # summed, and the optimizer / LR schedule step (and, under DDP, the exchange) happen on every k-th batch
        self.accum = max(1, int(opt_cfg.gradient_accumulation or 1))
        if self.grad_buckets is not None:  # gradients written into the exchange buffer by the backward kernels
            self.grad_buckets.zero_copy = zero_copy_grads and self.accum == 1 and dev.type == "cuda"
        self._micro = 0  # batches already accumulated in the current window
        self._acc = None  # (flat f32 buffer, per-parameter views) without DDP; GradBuckets' buffer under DDP
        self._touched: set = set()  # parameters that received a gradient in the current window
        self.capture_optimizer = capture_optimizer and self.accum == 1
        # single process, no accumulation: the optimizer step (esgpt_adamw_prepare + esgpt_adamw_dev, with the step's
        # loss / error-block hand-off) captured at the end of the step's own graph — no host launch after the replay.
        # Off by default: the ~9 us gap a replay's completion costs the next launch moves to the next step's first
        # launch instead (C2, same box, tools/host_bound.py: 1.657 vs 1.650 ms with error checks, 1.636 vs 1.642
        # without)
        self.fuse_optimizer = fuse_optimizer and self.accum == 1 and self.grad_buckets is None
        self.graphs: dict = {}  # shape signature -> (segments, static batch, static loss, grads) | None (eager)
        self.capture_report: dict = {}  # shape signature -> ATen GEMMs / reductions seen in its warm-up pass
        self.check_errors = check_errors and dev.type == "cuda"
        # projection weight gradients on a second stream beside the rest of backward (kernels.weight_grad_overlap).
        # Off by default: measured on the C2 step (HIP graph) it gains nothing — the graph executor starts the side
        # chain late and every fork costs the main stream a ~4.5 us barrier gap.
        self.overlap_weight_grads = overlap_weight_grads and dev.type == "cuda"
        # the LayerNorm backwards' column sums in one launch per backward pass (kernels.deferred_colsums)
        self.defer_colsums = defer_colsums and dev.type == "cuda"
        if dev.type == "cuda":
            # a second gradient contribution to a parameter is added on the current stream: the first one may still
            # be pending (a deferred LayerNorm column sum, or a weight gradient in flight on its stream) — settle it
            for p in params:
                p.register_hook(self._make_accumulate_guard(p))
        self._pending: deque = deque()  # (event, pinned error block copy, batch) of submitted steps
        # the optimizer launch's hand-off ring (esgpt_adamw_prepare_tab): entry k = [loss, pad x3, error block x4
        # words] of the k-th launch; the returned loss of a replayed step is a view of its entry (the entry is given a
        # fresh allocation before reuse while anything still shares it), the error words go to the host for check()
        self.ring_len = 64
        self._ring_tab = None
        self._host_words = None
        self._slots: list = []
        self._ring_n = 0  # host mirror of the device ring counter
        self._vocab = getattr(getattr(model, "config", None), "vocab_size", None)
        self._copy_stream = None
        self._staging: dict = {}
        self._prefetched = None
        self._release = None
        # the step's loss as the reference logs it (train_loss, sync_dist=True): under DDP the mean over ranks,
        # carried in the exchange's last bucket (a view of the exchange buffer, valid until the next step);
        # otherwise the step's own loss
        self.logged_loss = None

    def _ones(self, loss: torch.Tensor) -> torch.Tensor:
        """d(loss)/d(loss) = 1 as a persistent tensor (no fill launch in the step; under HIP-graph capture the graph
        reads it in place)."""
        one = getattr(self, "_one", None)
        if one is None or one.shape != loss.shape or one.dtype != loss.dtype or one.device != loss.device:
            one = self._one = torch.full_like(loss, 1.0 / self.accum)
        return one

    # ---- optimizer hand-off ring -------------------------------------------------------------------------------
    # Entry k is its own 8-float allocation ([loss, pad x3, error block x4 words]) reached through a device table of
    # entry addresses (esgpt_adamw_prepare_tab). A returned loss is a view of its entry; when the entry comes round
    # again while ANY tensor still shares its storage (the returned object, a detach(), a view, an index — counted by
    # the storage's use count, not by object identity), the entry gets a fresh allocation and its table slot is
    # re-pointed (one stream-ordered fill) — the caller's tensors keep their value and nothing is copied.
    # The error words of entry k also land in coherent mapped host memory (esgpt_host_words_alloc), which check()
    # reads once the step's event has completed: no D2H copy launch per step (a 16-byte copy to pinned memory costs
    # its launch plus a ~15 us idle gap on the compute stream).
    def _ring_state(self):
        if self._ring_tab is None:
            self._slots = [torch.zeros(8, dtype=torch.float32, device=self.device) for _ in range(self.ring_len)]
            self._ring_tab = torch.tensor([t.data_ptr() for t in self._slots], dtype=torch.int64, device=self.device)
            self._ring_ctr = torch.zeros(1, dtype=torch.int64, device=self.device)
            self._slot_users = _storage_users(self._slots[0])  # the ring's own reference alone
            if HOST_ERROR_WORDS and self.device.type == "cuda":
                self._host_words = _HostWords(self.ring_len)
        hw = self._host_words
        return None, self._ring_ctr, self._ring_tab, (hw.dev if hw is not None else 0)

    def _claim(self) -> int:
        """The ring entry the next optimizer launch writes (its device counter advances with every launch); an entry
        whose storage is still shared by a tensor the caller holds is given a fresh allocation first."""
        self._ring_state()
        slot = self._ring_n % self.ring_len
        if _storage_users(self._slots[slot]) > self._slot_users:
            new = torch.zeros_like(self._slots[slot])
            self._slots[slot] = new
            self._ring_tab[slot].fill_(new.data_ptr())  # stream-ordered before the launch that writes the entry
        self._ring_n += 1
        return slot

    def _unclaim(self):
        self._ring_n -= 1  # no launch happened: the device counter did not advance

    def _ring_loss(self, slot: int, like: torch.Tensor) -> torch.Tensor:
        loss = self._slots[slot][: like.numel()].view(like.shape)
        return loss if like.dtype == torch.float32 else loss.to(like.dtype)

    def _hand(self, src: torch.Tensor):
        return (src.detach().reshape(-1).float(),) + self._ring_state()

    # ---- gradient accumulation -------------------------------------------------------------------------------
    def _acc_views(self):
        if self.grad_buckets is not None:
            return self.grad_buckets.views
        if self._acc is None:
            flat = torch.zeros(sum(p.numel() for p in self.params), dtype=torch.float32, device=self.device)
            views, off = {}, 0
            for i, p in enumerate(self.params):
                views[i] = flat[off: off + p.numel()].view_as(p)
                off += p.numel()
            self._acc = (flat, views)
        return self._acc[1]

    @torch.no_grad()
    def _accumulate(self):
        """Adds this batch's gradients into the window's buffer (one multi-tensor add; torch's accumulate order)."""
        views = self._acc_views()
        src, dst = [], []
        for i, p in enumerate(self.params):
            if p.grad is not None:
                src.append(p.grad)
                dst.append(views[i])
                self._touched.add(i)
        if src:
            torch._foreach_add_(dst, src)

    @torch.no_grad()
    def _reset_accumulation(self):
        """Ends the window. The buffer is zeroed lazily, at the start of the next window (_zero_window), so the
        gradients the optimizer just read (``param.grad`` views of it) stay readable until the next ``step``."""
        self._micro = 0
        self._touched.clear()
        self._acc_dirty = self.accum > 1

    @torch.no_grad()
    def _zero_window(self):
        if getattr(self, "_acc_dirty", False):
            if self.grad_buckets is not None:
                self.grad_buckets.flat.zero_()
            elif self._acc is not None:
                self._acc[0].zero_()
            self._acc_dirty = False

    @torch.no_grad()
    def flush(self):
        """Applies a partial accumulation window (Lightning steps the optimizer on an epoch's last, incomplete
        window of ``accumulate_grad_batches``): the exchange (under DDP every rank must call it at the same point), the
        optimizer and the LR schedule step on the window's sums. As in Lightning, each batch's loss was scaled by
        1 / gradient_accumulation whatever the window's length. Returns whether a step was taken."""
        if self.accum == 1 or self._micro == 0:
            return False
        gb = self.grad_buckets
        views = self._acc_views()
        for i, p in enumerate(self.params):  # the sums are already in the buffer: a release must not add them again
            p.grad = views[i] if i in self._touched else None
        if gb is not None:
            gb.add, gb.loss_src = True, None
            gb.finish()
        if self.sched is None:
            if self.sched_step == self.lr_lambda_warm_total():
                self.lr_lambda(self.sched_step)
            self.opt.step(self.cfg.init_lr * self.lr_lambda(self.sched_step) if self.opt.host_args else None)
            active = list(self.opt._active)
        else:
            self.opt.step()
            self.sched.step()
            active = []
        self.sched_step += 1
        self._reset_accumulation()
        if self.check_errors:
            self._record_pending(None, active, True)
        return True

    def _maybe_relayout(self):
        """Zero-copy exchange: adopt the parameter groups the last forward recorded — only before any graph has been
        captured (a captured backward writes into the buffer it was captured with) and between windows. Every rank
        reaches this at the same step with the same groups (same model, same code path)."""
        gb = self.grad_buckets
        if (gb is not None and gb.layout_stale() and self._micro == 0
                and not any(e is not None for e in self.graphs.values())):
            torch.cuda.synchronize(self.device)  # the old buffer's last readers (AdamW, all-reduce) are done
            gb.relayout()

    @staticmethod
    def _make_accumulate_guard(p):
        def hook(grad):
            if p.grad is not None:
                if colsum_deferral_active(grad.device):
                    flush_colsums(grad.device)
                if weight_grad_overlap_active(grad.device):
                    join_weight_grads(grad.device)
            return None

        return hook

    # --------------------------------------------------------------------------------------------------------
    def _fwd_bwd(self, batch: PytorchBatch, autocast_cache: bool = True):
        dev = self.device
        if dev.type == "cuda":
            begin_dropout_step(dev, reset_errors=True)  # this step's error flags start clear
        gb = self.grad_buckets
        rec = gb if (gb is not None and gb.zero_copy) else None
        # the backward writes gradients into the exchange buffer only on a pass whose release copies (not adds) them
        dest = rec if (rec is not None and rec.mode != "off" and not rec.add) else None
        with grad_destinations(dev, rec, dest):
            # The autocast weight-cast cache must be off under HIP-graph capture (cached casts would outlive it).
            with torch.autocast("cuda", dtype=self.dtype, enabled=self.dtype != torch.float32,
                                cache_enabled=autocast_cache):
                out = self.model(batch)
            if gb is not None:
                gb.loss_src = out.loss
            with deferred_colsums(dev, enabled=self.defer_colsums), \
                    weight_grad_overlap(dev, enabled=self.overlap_weight_grads):
                out.loss.backward(self._ones(out.loss))
        if dev.type == "cuda":
            end_dropout_step(dev)
        return out.loss.detach()

    def _capture(self, batch: PytorchBatch):
        """Captures this batch signature's step (forward + backward) as HIP graph segments, or records that it
        runs eagerly (None). Two warm-up passes on a side stream first (allocator / lazy init; no collectives); the
        first runs under _GemmSpy: a signature whose step reaches an ATen GEMM or reduction is not captured. Under DDP the
        capture is cut wherever GradBuckets releases buckets, so each segment's buckets can be exchanged while the
        next segment replays."""
        if self.check_errors:
            self._raise_pending(keep=0)  # earlier steps' errors are theirs, not this batch's
        sig = batch.shape_signature()
        static = batch.packed()
        gb = self.grad_buckets
        if gb is not None:
            gb.mode = "off"
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        spy = _GemmSpy()
        try:
            fuse = (self.fuse_optimizer and isinstance(self.opt, FusedAdamW) and self.sched is None
                    and not self.opt.host_args and not self.capture_optimizer)
            items = None
            with torch.cuda.stream(s):
                for k in range(2):  # warm up allocator / lazy init outside the graph
                    self.opt.zero_grad(set_to_none=True)
                    if k == 0:
                        with spy:
                            self._fwd_bwd(static, autocast_cache=False)
                    else:
                        self._fwd_bwd(static, autocast_cache=False)
                        items = [i for i, p in enumerate(self.params) if p.grad is not None]
                    if gb is not None:
                        gb.reset()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            check_errors(self.device, self._vocab)  # a warm-up error is this batch's error: raise it now
            self._maybe_relayout()  # the warm-up recorded the gradient kernels' parameter groups
            self.opt.zero_grad(set_to_none=True)
            self.capture_report[sig] = sorted(spy.hits)
            if spy.hits:  # a PyTorch-ROCm BLAS fallback or ATen reduction in the step: not captured
                self.graphs[sig] = None
                return
            pool = torch.cuda.graph_pool_handle()
            # the fused optimizer's plan, made before the capture; its table is written once the capture has
            # allocated the gradients
            fplan = self.opt.make_plan(items, fill=False) if fuse and items else None
            ring_ctr = self._ring_state() if fplan is not None else None
            segs = []
            cur = {"g": torch.cuda.CUDAGraph()}
            # a segment ends on the autograd worker thread that runs the bucket hook, and the next begins there:
            # capture sequences that cross threads must be "relaxed" (HIP refuses to end a global-mode capture
            # from another thread)
            mode = "relaxed" if gb is not None else "global"
            if gb is not None:
                def boundary(buckets):  # runs on the autograd worker thread, on the capturing stream
                    dev = self.device
                    if weight_grad_overlap_active(dev):
                        join_weight_grads(dev)
                    if colsum_deferral_active(dev):  # the released buckets' LayerNorm sums belong to this segment
                        flush_colsums(dev)
                    cur["g"].capture_end()
                    segs.append((cur["g"], list(buckets)))
                    cur["g"] = torch.cuda.CUDAGraph()
                    cur["g"].capture_begin(pool=pool, capture_error_mode=mode)

                gb.mode, gb.on_boundary = "mark", boundary
                gb.reset()
            with torch.cuda.stream(s):
                cur["g"].capture_begin(pool=pool, capture_error_mode=mode)
                loss = self._fwd_bwd(static, autocast_cache=False)
                if fplan is not None:
                    self.opt.launch(fplan, hand=(loss.reshape(-1).float(),) + ring_ctr)
                cur["g"].capture_end()
                segs.append((cur["g"], []))
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            if fplan is not None:
                if [i for i, p in enumerate(self.params) if p.grad is not None] != fplan["active"]:
                    raise RuntimeError("TrainStep: the captured step's gradients differ from its warm-up's")
                self.opt.fill_table(fplan)
            # the optimizer step as its own small graph over the captured gradients (its plan's tables are built
            # here, outside any capture, and kept alive with the entry): no host launch per replayed step
            opt_graph = plan = None
            if isinstance(self.opt, FusedAdamW) and self.capture_optimizer:
                if gb is not None:  # under DDP the step reads the exchanged gradients: the flat buffer's views
                    saved = [p.grad for p in self.params]
                    for i, p in enumerate(self.params):
                        p.grad = gb.views[i]
                    plan = self.opt.make_plan()
                    for p, g in zip(self.params, saved):
                        p.grad = g
                else:
                    plan = self.opt.make_plan()
                opt_graph = torch.cuda.CUDAGraph()
                with torch.cuda.stream(s):
                    opt_graph.capture_begin(pool=pool)
                    self.opt.launch(plan)
                    opt_graph.capture_end()
                torch.cuda.current_stream().wait_stream(s)
                torch.cuda.synchronize()
        finally:
            if gb is not None:
                gb.mode, gb.on_boundary = "launch", None
                gb.reset()
        grads = [p.grad for p in self.params]
        if fplan is not None:
            opt_graph, plan = "fused", fplan
        self.graphs[sig] = (segs, static, loss, grads, opt_graph, plan)

    def _raise_pending(self, keep: int):
        """Raises the first device error among submitted steps, waiting only for steps older than the newest
        ``keep`` (``keep = 0``: all of them)."""
        # Under DDP a step's error is raised exactly at the submission of step k + 2 (or at check()), never earlier
        # because its event happens to have completed: every rank then raises at the same step, whatever its
        # timing, and no rank runs step k + 1's collectives alone.
        while len(self._pending) > keep or (not self.distributed and self._pending and self._pending[0][0].query()):
            ev, host, batch, active, stepped = self._pending.popleft()
            ev.synchronize()
            code, mx = host[0].read(host[1]) if isinstance(host, tuple) else (int(host[0]), int(host[1]))
            if code & 0xFFFFFFFF:
                # the failing step's AdamW was a no-op on the device, and so is every step queued behind it (the
                # sticky word): take back their step counts and LR steps. The block is cleared after them in
                # stream order.
                discarded = [(active, stepped)] + [(e[3], e[4]) for e in self._pending]
                self._pending.clear()
                err_word(self.device).zero_()
                for act, st in discarded:
                    if isinstance(self.opt, FusedAdamW):
                        for i in act:
                            self.opt.steps[i] -= 1
                    if st:
                        self.sched_step -= 1
                self._reset_accumulation()  # the window's partial sums belong to the discarded batches
                raise_for_error(code, mx, self._vocab, batch)

    def prefetch(self, batch: PytorchBatch) -> None:
        """Starts the host -> device copy of a (pinned, packed) host batch on a side stream, so it overlaps the step
        in flight; the next ``step(batch)`` with the same object waits for that copy instead of issuing its own.
        Two staging buffers per shape signature alternate, so a copy never overwrites a batch still being read."""
        if batch.device.type != "cpu" or self.device.type != "cuda":
            return
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(self.device)
        sig = batch.shape_signature()
        ring = self._staging.setdefault(sig, [None, None, 0])
        k = ring[2]
        ring[2] ^= 1
        slot = ring[k]
        if slot is None:
            dst = batch.packed().to(self.device)
            slot = ring[k] = [dst, torch.cuda.Event()]
            slot[1].record()  # no reader yet
        dst, free_ev = slot
        cs = self._copy_stream
        cs.wait_event(free_ev)  # the previous reader of this buffer is done
        with torch.cuda.stream(cs):
            dst.copy_(batch, non_blocking=True)
            ready = torch.cuda.Event()
            ready.record(cs)
        self._prefetched = (batch, dst, ready, free_ev)

    def _to_device(self, batch: PytorchBatch) -> PytorchBatch:
        if batch.device.type == self.device.type or self.device.type != "cuda":
            return batch
        pf = self._prefetched
        if pf is not None and pf[0] is batch:
            self._prefetched = None
            _, dst, ready, free_ev = pf
            torch.cuda.current_stream().wait_event(ready)
            self._release = free_ev
            return dst
        return batch.to(self.device, non_blocking=True)

    def step(self, batch: PytorchBatch) -> torch.Tensor:
        """One optimizer step on ``batch`` (device-resident, or a pinned host batch: the H2D copy is part of the
        step, overlapped when ``prefetch(batch)`` was called during the previous step)."""
        if self.check_errors:
            self._raise_pending(keep=1)
        host_batch = batch  # the caller's object (named in an error message; device staging buffers get reused)
        batch = self._to_device(batch)
        entry = None
        if self.use_graph:
            sig = batch.shape_signature()
            # only real graphs count against max_graphs (a signature recorded as eager holds no graph memory)
            if sig not in self.graphs and sum(g is not None for g in self.graphs.values()) < self.max_graphs:
                self._capture(batch)
            entry = self.graphs.get(sig)
        gb = self.grad_buckets
        accumulating = self.accum > 1
        last = self._micro + 1 >= self.accum  # this batch closes the accumulation window: exchange + step
        if accumulating and self._micro == 0:
            self._zero_window()  # the previous window's sums, left readable until now
        exchange = gb is not None and last
        if gb is not None:
            gb.add = accumulating
        opt_graph = plan = None
        if entry is None:
            self.opt.zero_grad(set_to_none=True)
            self._maybe_relayout()
            if gb is not None and not exchange:
                gb.mode = "off"  # Lightning's no_sync on the window's earlier batches
            try:
                loss = self._fwd_bwd(batch)
            finally:
                if gb is not None:
                    gb.mode = "launch"
        else:
            segs, static, sloss, grads, opt_graph, plan = entry
            fused_slot = None
            if opt_graph == "fused" and self.sched_step == self.lr_lambda_warm_total():
                self.lr_lambda(self.sched_step)  # warmup == total: the reference's lambda raises here
            static.copy_(batch, non_blocking=True)
            if self._release is not None:  # the staging buffer is consumed: the next prefetch may refill it
                self._release.record()
                self._release = None
            for p, gr in zip(self.params, grads):  # the graph writes its gradients into its own pool
                p.grad = gr
            if gb is not None:
                gb.loss_src = sloss
            if opt_graph == "fused":  # the optimizer step (and its ring entry) ends the step's graph
                fused_slot = self._claim()
            try:
                for g, released in segs:
                    g.replay()
                    if exchange:  # exchanged while the next segment replays
                        for b in released:
                            gb._launch(b)
            except BaseException:
                if fused_slot is not None:
                    self._unclaim()
                raise
            # the next replay overwrites the static loss: hand back a copy — written by the optimizer's prepare launch
            # into the hand-off ring when this step runs one (no launch of its own, no host-launch gap), else by the
            # library's pack kernel (not clone()'s D2D blit: ~5 us of device time for 4 bytes)
            loss = self._ring_loss(fused_slot, sloss) if fused_slot is not None else None
        if loss is None and not (LOSS_IN_OPT and last and opt_graph is None and self.sched is None
                                 and not self.opt.host_args):
            loss = _copy_scalar(sloss)  # no device optimizer launch to carry the copy
        if accumulating and not exchange:
            self._accumulate()  # into the window's buffer (GradBuckets' under DDP)
        self.logged_loss = loss if gb is None else None
        if not last:
            self._micro += 1
            if self._release is not None:
                self._release.record()
                self._release = None
            if self.check_errors:
                self._record_pending(host_batch, [], False)
            return loss
        self._micro = 0
        if gb is not None:
            gb.finish()
            self.logged_loss = gb.loss_slot.view(())
        elif accumulating:  # the window's sums are the gradients AdamW reads
            views = self._acc_views()
            for i, p in enumerate(self.params):
                p.grad = views[i] if i in self._touched else None
        if self.sched is None and self.sched_step == self.lr_lambda_warm_total():
            self.lr_lambda(self.sched_step)  # warmup == total: the reference's lambda raises ZeroDivisionError here
        slot = None
        if opt_graph == "fused":  # replayed with the step
            self.opt.note_step(plan["active"])
            active = list(plan["active"])
            slot = fused_slot
        elif opt_graph is not None:
            opt_graph.replay()
            self.opt.note_step(plan["active"])
            active = list(plan["active"])
        elif self.sched is None:
            # the installed schedule, on the device (or, measurement hook, round 3's host-computed lr); the prepare
            # launch writes the step's hand-off entry (the replayed step's loss, the error block)
            pending = loss is None
            slot = None if self.opt.host_args else self._claim()
            try:
                done = self.opt.step(self.cfg.init_lr * self.lr_lambda(self.sched_step) if self.opt.host_args else None,
                                     hand=self._hand(sloss if pending else loss) if slot is not None else None)
            except BaseException:  # no launch: the device ring counter did not advance
                if slot is not None:
                    self._unclaim()
                raise
            if slot is not None and not done:  # no active parameter: no launch wrote the entry
                self._unclaim()
                slot = None
            if pending:
                loss = self._ring_loss(slot, sloss) if slot is not None else sloss.clone()
            active = list(self.opt._active)
        else:
            self.opt.step()
            self.sched.step()
            active = []
        self.sched_step += 1
        if accumulating:
            self._reset_accumulation()  # stream-ordered after the optimizer's reads
        if self._release is not None:  # the staging buffer may be refilled once this step has consumed it
            self._release.record()
            self._release = None
        if self.check_errors:
            self._record_pending(host_batch, active, True, slot)
        return loss

    def _record_pending(self, host_batch, active, stepped: bool, slot: int | None = None):
        # the step's error block: the words its optimizer launch wrote into ring entry `slot`, else the live block.
        # (Copied on the compute stream: on a side stream — waiting on an event recorded after the step — the C2
        # step measured ~50 us slower, tools/host_bound.py.)
        if slot is not None and self._host_words is not None:
            host = (self._host_words, slot)  # written by the optimizer launch straight into mapped host memory
        else:
            host = torch.empty(2, dtype=torch.int64, pin_memory=True)
            host.copy_(err_word(self.device) if slot is None else self._slots[slot][4:8].view(torch.int64),
                       non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._pending.append((ev, host, host_batch, active, stepped))

    def lr_lambda_warm_total(self) -> int:
        """The schedule step at which warmup == max_training_steps makes the reference's lambda divide 0 / 0
        (-1: never)."""
        total = self.cfg.max_training_steps or 1_000_000
        warm = self.cfg.lr_num_warmup_steps or 0
        return total if total == warm else -1

    def check(self):
        """Waits for every submitted step and raises the first device error (the reference's exception)."""
        if self.check_errors:
            self._raise_pending(keep=0)
        check_errors(self.device if self.device.type == "cuda" else None, self._vocab)


HOST_ERROR_WORDS = True  # measurement hook (bench.py --err-copy): False = round 5's per-step D2H copy


class _HostWords:
    """ring_len x 4 int32 words of coherent, device-mapped host memory (esgpt_host_words_alloc); freed with the
    owner. ``read(k)`` = entry k's (flags | sticky << 32, max bad index), as the D2H copy of the error block gave."""

    def __init__(self, n: int):
        import ctypes

        from . import _lib as L

        lib = L.load()
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        L.check(lib.esgpt_host_words_alloc(16 * n, ctypes.byref(h), ctypes.byref(d)), "host_words_alloc")
        self.dev = int(d.value)
        self._words = (ctypes.c_int64 * (2 * n)).from_address(h.value)
        self._fin = weakref.finalize(self, lib.esgpt_host_words_free, ctypes.c_void_p(h.value))

    def read(self, k: int):
        return int(self._words[2 * k]), int(self._words[2 * k + 1])


def init_distributed():
    """Initialises the process group from torchrun's env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*): RCCL ("nccl")
    with one GPU per rank, gloo without a GPU. Test override (the multi-rank bench rehearsed on a one-GPU box):
    ESGPT_DIST_BACKEND=gloo with ESGPT_DIST_ONE_DEVICE=1 puts every rank on device 0 (RCCL refuses two ranks on one
    device)."""
    import os

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1, 0
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if os.environ.get("ESGPT_DIST_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("ESGPT_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def n_params(model) -> int:
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def grad_bytes(model) -> int:
    return 4 * n_params(model)
