"""Data-parallel sharding of refinement batches over GPUs (one process per GPU).

Every tensor on the hot path is per image pair: the correlation volume, the
GRU state, the pose and the 2D-3D points are all indexed by the pair, so a batch splits
contiguously across ranks and each rank runs the whole decoder on its shard with NO
collective inside the refinement loop.  Results are gathered once at the end — the
reference's eval pattern (``tools/eval.py:186-216``: pad to the largest shard, all_gather,
trim), here for the refined poses and flows.  With the NCCL backend (= RCCL on ROCm) the
gather runs over xGMI; the CPU tests use gloo.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

Tensor = torch.Tensor


def shard_range(batch: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, end) of ``batch`` items owned by ``rank`` (sizes differ by ≤ 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_batch(batch: Dict[str, Tensor], rank: int, world: int, batch_dim: int = 0,
                head_label_key: Optional[str] = "label") -> Dict[str, Tensor]:
    """Slice every per-pair tensor of a decoder input dict to this rank's shard.

    The reference's pose head picks the class head of ``label[0]`` for the WHOLE batch
    (``pose_head.py:208-209``), so a shard whose first label differs from the global batch's
    would pick a different head than the unsharded forward.  With ``head_label_key`` set (the
    default, ``"label"``) the shard also carries ``head_label`` = the global ``label[:1]``,
    which ``SCFlowDecoder.forward`` / ``SCFlowRefiner.get_pose`` / the training step take as
    the pose head's label: sharded output then equals unsharded output for multi-class
    batches.  (The reference's own DDP runs — ``train.py:42-45``, ``tools/eval.py`` — shard
    through the data loader, so there every rank uses its local ``label[0]``; pass
    ``head_label_key=None`` for that behaviour.  Training shards should: the reference's DDP
    gradient is the mean of per-replica gradients, each with its local ``label[0]`` and its
    own BatchNorm statistics — ``shard_train_batch``.)"""
    sizes = {v.shape[batch_dim] for v in batch.values() if isinstance(v, Tensor) and v.dim() > 0}
    if len(sizes) != 1:
        raise ValueError(f"inconsistent batch sizes {sizes}")
    b = sizes.pop()
    s, e = shard_range(b, rank, world)
    out = {k: (v.narrow(batch_dim, s, e - s) if isinstance(v, Tensor) and v.dim() > 0 else v)
           for k, v in batch.items()}
    if head_label_key is not None and head_label_key in batch and "head_label" not in batch:
        out["head_label"] = batch[head_label_key].narrow(batch_dim, 0, 1)
    return out


def shard_train_batch(batch: Dict[str, Tensor], rank: int, world: int) -> Dict[str, Tensor]:
    """``shard_batch`` for the training step, with the reference's DDP semantics: no global
    ``head_label`` — each replica's pose head takes its local ``label[0]`` (pose_head.py:208-209
    under the DataLoader's per-rank sampling, train.py:42-45), and its context-encoder BatchNorm
    normalises with its own shard's statistics (plain BN, scflow_ycbv_real.py:198), so the
    all-reduced gradient is the mean of the per-shard single-process gradients
    (tests/test_train_dist_cpu.py)."""
    return shard_batch(batch, rank, world, head_label_key=None)


def gather_shards(x: Tensor, group=None) -> Tensor:
    """all_gather of per-rank shards of possibly different lengths along dim 0, in rank order."""
    world = dist.get_world_size(group)
    n = torch.tensor([x.shape[0]], device=x.device, dtype=torch.long)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(v.item()) for v in ns]
    m = max(ns)
    pad = x.new_zeros((m,) + tuple(x.shape[1:]))
    pad[: x.shape[0]] = x
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad.contiguous(), group=group)
    return torch.cat([b[:k] for b, k in zip(bufs, ns)], 0)


def gather_results(results: Sequence[Sequence[Tensor]], which: Sequence[int] = (0, 1, 2, 3),
                   last_only: bool = True, group=None) -> List[Tensor]:
    """Gather the decoder's output lists (7-tuple of per-iteration lists) across ranks.

    Returns, for each requested output index, the full-batch tensor of the last iteration
    (``last_only``) — e.g. the refined rotations/translations the refiner keeps
    (``scflow_refiner.py:160-176``)."""
    out = []
    for i in which:
        lst = results[i]
        t = lst[-1] if last_only else torch.stack(list(lst), 1)
        out.append(gather_shards(t.contiguous(), group))
    return out
