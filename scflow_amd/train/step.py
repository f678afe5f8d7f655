"""One training iteration of the refinement model (the reference runs it
through mmengine's OptimWrapper: configs/refine_models/scflow_ycbv_real.py:285-305 — AdamW
lr 4e-4, betas (0.9, 0.999), eps 1e-8, weight decay 1e-4, clip_grad max_norm 10, and the
OneCycleLR schedule of :299-306 — schedule.py — stepped once per iteration).

Data parallel = one process per GPU (torch.distributed over RCCL).  Gradients live in a few
flat fp32 buckets (every ``param.grad`` is a view into one), so the exchange is one all-reduce
per bucket, sized for xGMI (default 8 MB, 4 buckets for the 32.7 MB model: large enough that
the ring is link-bound).  By default the buckets are reduced right after the backward pass,
all issued before the first wait (the 32.7 MB exchange is ≈0.3 ms against a ≈40 ms step at
B = 16 per GPU, so overlapping it buys < 1 %); ``overlap=True`` instead issues each bucket's all-reduce from a
post-accumulate-grad hook as soon as its last gradient is written (buckets filled in reverse
registration order ≈ the order backward produces gradients).  No per-parameter collectives,
no DDP wrapper.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from .._lib import bump_weights_generation
from .functions import capture_cache, direct_weight_grads
from .model import refiner_train_forward
from .schedule import OneCycleLR, reference_schedule

Tensor = torch.Tensor
_MT_BACKWARD = os.environ.get("SCFLOW_TRAIN_MT_BACKWARD", "1") == "1"  # A/B switch (tuning)


def trainable_parameters(refiner) -> List[torch.nn.Parameter]:
    """The refiner's parameters, each once (the shared render / real feature encoder appears
    under both names) and only those that require grad (``freeze_encoder`` clears it on the
    feature encoder) — what the gradient buckets and the optimizer hold."""
    return [p for p in dict.fromkeys(refiner.parameters()) if p.requires_grad]


class GradBuckets:
    """Flat gradient buckets all-reduced (averaged) over the process group, after the backward
    pass or (``overlap``) from post-accumulate-grad hooks during it."""

    def __init__(self, params: Sequence[torch.nn.Parameter], bucket_bytes: int = 8 << 20,
                 group=None, overlap: bool = False) -> None:
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.buckets: List[Tensor] = []
        self.members: List[List[torch.nn.Parameter]] = []
        cur: List[torch.nn.Parameter] = []
        size = 0
        for p in reversed(self.params):
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= bucket_bytes:
                self.members.append(cur)
                cur, size = [], 0
        if cur:
            self.members.append(cur)
        self._bucket_of = {}
        for bi, mem in enumerate(self.members):
            dev = mem[0].device
            flat = torch.zeros(sum(p.numel() for p in mem), device=dev, dtype=mem[0].dtype)
            off = 0
            for p in mem:
                p.grad = flat[off:off + p.numel()].view_as(p)
                off += p.numel()
                self._bucket_of[p] = bi
            self.buckets.append(flat)
        self._pending = [0] * len(self.members)
        self._work: List[Optional[object]] = [None] * len(self.members)
        self._hooks = []
        if self.world > 1 and overlap:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def _on_grad(self, p) -> None:
        bi = self._bucket_of[p]
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._work[bi] = dist.all_reduce(self.buckets[bi], op=dist.ReduceOp.SUM, group=self.group,
                                             async_op=True)

    def zero(self) -> None:
        for b in self.buckets:
            b.zero_()
        for bi, mem in enumerate(self.members):
            self._pending[bi] = len(mem)
            self._work[bi] = None

    def finish(self) -> None:
        """Wait for every bucket's all-reduce (issuing any whose hooks did not all fire — a
        parameter without a gradient this step) and average."""
        if self.world == 1:
            return
        for bi, flat in enumerate(self.buckets):
            if self._work[bi] is None:
                self._work[bi] = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group,
                                                 async_op=True)
        for bi, flat in enumerate(self.buckets):
            self._work[bi].wait()
            flat.mul_(1.0 / self.world)
            self._work[bi] = None

    def clip_(self, max_norm: float) -> Tensor:
        """clip_grad_norm_ (L2 over all parameters) on the flat buckets."""
        norms = torch.stack([b.norm() for b in self.buckets])
        total = norms.norm()
        coef = (max_norm / (total + 1e-6)).clamp(max=1.0)
        for b in self.buckets:
            b.mul_(coef)
        return total


class TrainStep:
    """forward (HIP) → losses → backward (HIP) → bucketed all-reduce → clip → AdamW.

    ``graph=True`` (off by default): the forward + backward (≈3000 kernel
    launches) are captured once into a hipGraph on the third call and replayed on every later
    call with the batch copied into the captured input buffers; the gradient all-reduce stays
    eager between two replays, and clipping + AdamW (``capturable``: step counts on the device)
    are a second captured graph.  The weights are re-packed inside the graph, so optimizer
    updates are seen by every replay.  The learning rate is a device tensor in graph mode (the
    schedule's value is written into it before every step, so the captured AdamW reads it), a
    float in eager mode.  ``lr_schedule``: "onecycle" (default: the configured OneCycleLR with
    ``eta_max = lr``, ``total_steps``, ``pct_start`` and linear annealing), a ``OneCycleLR``-like
    object with ``lr_at(step)``, or None for a constant ``lr``.  Every kernel of the forward + backward is one of ours (no vendor
    GEMM: see functions.py), and eager steps and the capture run on the step's own stream."""

    def __init__(self, refiner, model_points: Sequence[Tensor], diameters: Sequence[float],
                 lr: float = 4e-4, weight_decay: float = 1e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 max_norm: float = 10.0, bucket_bytes: int = 8 << 20, iters: Optional[int] = None,
                 group=None, overlap: bool = False, graph: bool = False,
                 lr_schedule="onecycle", total_steps: int = 100100, pct_start: float = 0.05) -> None:
        self.refiner = refiner
        self.graph = graph
        self._g = None
        self._g_opt = None
        self._gn = None
        self._static = None
        self._out = None
        self._calls = 0
        self.model_points = list(model_points)
        self.diameters = list(diameters)
        self.max_norm = max_norm
        self.iters = iters
        if lr_schedule == "onecycle":
            lr_schedule = (reference_schedule(lr) if (total_steps, pct_start) == (100100, 0.05) else
                           OneCycleLR(lr, total_steps, pct_start, anneal_strategy="linear"))
        self.lr_schedule = lr_schedule
        self.iteration = 0  # training iterations taken (the schedule's step)
        params = trainable_parameters(refiner)
        self.grads = GradBuckets(params, bucket_bytes, group, overlap)
        dev = self.grads.params[0].device
        lr0 = lr if lr_schedule is None else lr_schedule.lr_at(0)
        self._lr_const = float(lr)
        # graph mode: the captured AdamW must read the lr from memory
        self._lr_t = torch.tensor(lr0, dtype=torch.float32, device=dev) if graph else None
        self.opt = torch.optim.AdamW(self.grads.params, lr=lr0 if self._lr_t is None else self._lr_t,
                                     betas=betas, eps=eps, weight_decay=weight_decay, foreach=True,
                                     capturable=graph)
        self.stream = torch.cuda.Stream(device=dev)
        self.diam_t = torch.as_tensor(self.diameters, dtype=torch.float32, device=dev)
        if dist.is_initialized() and dist.get_world_size(group) > 1:
            self.broadcast_parameters()

    def state_dict(self) -> Dict:
        """The step's resumable state: the schedule position and the optimizer state (the model's
        own state_dict holds the weights and BN statistics)."""
        return dict(iteration=self.iteration, optimizer=self.opt.state_dict())

    def load_state_dict(self, state: Dict) -> None:
        """Resume: the schedule continues at ``state['iteration']`` (warm-up is not repeated)."""
        self.iteration = int(state["iteration"])
        self.opt.load_state_dict(state["optimizer"])
        self._set_lr()

    def broadcast_parameters(self, src: int = 0) -> None:
        """Start every rank from rank 0's weights and BN statistics."""
        for t in list(self.refiner.parameters()) + list(self.refiner.buffers()):
            dist.broadcast(t.data, src, group=self.grads.group)

    @property
    def lr(self) -> float:
        """The learning rate of the next step."""
        if self.lr_schedule is None:
            return self._lr_const
        return self.lr_schedule.lr_at(self.iteration)

    def _set_lr(self) -> None:
        if self.lr_schedule is None:
            return
        v = self.lr_schedule.lr_at(self.iteration)
        if self._lr_t is not None:
            self._lr_t.fill_(v)  # stream-ordered write (no host sync), read by the captured AdamW
        else:
            for g in self.opt.param_groups:
                g["lr"] = v

    def _fwd_bwd(self, batch: Dict[str, Tensor]) -> Dict[str, Tensor]:
        self.grads.zero()
        out = refiner_train_forward(self.refiner, batch, self.model_points, self.diam_t, self.iters)
        # SCFLOW_TRAIN_MT_BACKWARD=0 runs backward on the calling thread (measured equal)
        with torch.autograd.set_multithreading_enabled(_MT_BACKWARD):
            if self.grads._hooks:  # per-parameter hooks must see every accumulation
                out["loss"].backward()
            else:
                with direct_weight_grads():  # its exit sums uses the pass did not reach
                    out["loss"].backward()
        # detached: a returned tensor must not keep this step's autograd graph (and its
        # AccumulateGrad nodes) alive into the next step or a capture
        return {k: _detach(v) for k, v in out.items()}

    def _capture(self, batch: Dict[str, Tensor]) -> None:
        self._static = {k: v.clone() for k, v in batch.items()}
        bufs = [b.clone() for b in self.refiner.buffers()]  # the warm-up must not move BN stats
        self._fwd_bwd(self._static)  # allocator warm-up on the step's stream (capture recipe)
        for b, c in zip(self.refiner.buffers(), bufs):
            b.copy_(c)
        self._g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g, stream=self.stream), capture_cache():
            self._out = self._fwd_bwd(self._static)

    def _step(self, batch: Dict[str, Tensor]) -> Dict[str, Tensor]:
        if self.graph and self._calls > 2:
            if self._g is None:
                self._capture(batch)
            else:
                if set(batch) != set(self._static):  # a replay reads exactly the captured inputs
                    raise ValueError(f"TrainStep(graph=True): batch keys {sorted(batch)} differ from "
                                     f"the captured ones {sorted(self._static)}")
                for k, v in batch.items():
                    self._static[k].copy_(v)
            self._g.replay()
            # scalars are copied out (the graph overwrites its outputs on the next replay);
            # the per-iteration lists stay views of the graph's buffers
            out = {k: (v.clone() if isinstance(v, Tensor) and v.dim() == 0 else v)
                   for k, v in self._out.items()}
            self.grads.finish()
            if self._g_opt is None:  # optimizer state exists (eager calls 1-2): capture clip + AdamW
                self._g_opt = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self._g_opt, stream=self.stream):
                    self._gn = self.grads.clip_(self.max_norm)
                    self.opt.step()
            self._g_opt.replay()
            # the replay wrote the parameters without moving their version counters: make every
            # weight-derived cache (packed / flipped forms) re-derive before its next eager use
            bump_weights_generation()
            out["grad_norm"] = self._gn.clone()
            return out
        out = self._fwd_bwd(batch)
        self.grads.finish()
        out["grad_norm"] = self.grads.clip_(self.max_norm)
        self.opt.step()
        return out

    def __call__(self, batch: Dict[str, Tensor]) -> Dict[str, Tensor]:
        """One step, enqueued on the step's own stream (eager steps and the captured graph see
        the same stream, so autograd's gradient accumulation never crosses streams), ordered
        after and before the caller's current stream."""
        self.refiner.train()
        self._calls += 1
        lr = self.lr
        self._set_lr()
        cur = torch.cuda.current_stream(self.stream.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            out = self._step(batch)
        cur.wait_stream(self.stream)
        out["lr"] = lr
        self.iteration += 1
        return out


def _detach(v):
    if isinstance(v, Tensor):
        return v.detach()
    if isinstance(v, tuple) and hasattr(v, "_fields"):  # named tuple (losses.LowRes)
        return type(v)(*(_detach(x) for x in v))
    if isinstance(v, (list, tuple)):
        return type(v)(_detach(x) for x in v)
    return v
