"""Training losses of SCFlowRefiner (models/loss/sequence_loss.py:7-80,
point_matching_loss.py:106-218; composition scflow_refiner.py:182-256; weights from
configs/refine_models/scflow_ycbv_real.py:231-262), batched over the samples.

The point-matching loss runs all B samples at once when every class's model-point set has the
same size (one [B, P, 3] gather + batched matmuls); ragged point sets fall back to a per-sample
loop.  Symmetric classes (SYMMETRIC_CLASSES) replace pytorch3d ``knn_points(K=1)`` by a
brute-force nearest neighbour (squared distances + argmin; indices carry no gradient, as with
knn_points).
"""
from __future__ import annotations

import os
from typing import NamedTuple, Sequence, Tuple

import torch
import torch.nn.functional as F

from .. import ops

Tensor = torch.Tensor

SYMMETRIC_CLASSES = (12, 15, 18, 19, 20)  # 0-based labels of cls_13, cls_16, cls_19, cls_20, cls_21 (config :34-40)
POSE_WEIGHT, FLOW_WEIGHT, MASK_WEIGHT, GAMMA = 10.0, 0.1, 10.0, 0.8
_KNN_TORCH = os.environ.get("SCFLOW_TRAIN_KNN_TORCH", "0") == "1"  # A/B switch (tuning)
_PM_TORCH = os.environ.get("SCFLOW_TRAIN_PM_TORCH", "0") == "1"    # A/B switch (tuning)


class LowRes(NamedTuple):
    """A prediction kept at the decoder's resolution (channels-last [N, h, w, C]) whose loss
    upsamples it inside the fused kernel (functions.up_l1_loss); value_scale multiplies the
    upsampled values (the flow's ×8)."""
    lr: Tensor
    value_scale: float


def flow_valid(gt: Tensor, valid: Tensor, max_flow: float = 400.) -> Tensor:
    """RAFTLoss's pixel mask (sequence_loss.py:15-23): valid ≥ 0.5 and |gt| < max_flow."""
    return ((valid >= 0.5) & (gt.pow(2).sum(1).sqrt() < max_flow)).to(gt)


def flow_l1_loss(pred: Tensor, gt: Tensor, valid: Tensor, max_flow: float = 400.,
                 weight: float = FLOW_WEIGHT, eps: float = 1e-10, v: Tensor = None) -> Tensor:
    """RAFTLoss (sequence_loss.py:15-23): valid-masked L1 of the flow (``v``: the mask from
    flow_valid, when the caller computes it once for all iterations)."""
    if v is None:
        v = flow_valid(gt, valid, max_flow)
    return weight * (v[:, None] * (pred - gt).abs()).sum() / (v.sum() + eps)


def mask_l1_loss(pred: Tensor, gt: Tensor, weight: float = MASK_WEIGHT) -> Tensor:
    """L1Loss (sequence_loss.py:34-36)."""
    return weight * (pred - gt).abs().mean()


def matmul3(a: Tensor, b: Tensor) -> Tensor:
    """Batched a @ b for a tiny inner dimension (3×3 rotations, [B, P, 3] point sets) as
    broadcast multiply-adds: no vendor GEMM kernel in the training step (it must stay
    capturable into one hipGraph)."""
    return (a[..., :, :, None] * b[..., None, :, :]).sum(-2)


def _pm_terms(pts: Tensor, pred_r: Tensor, pred_t: Tensor, gt_r: Tensor, gt_t: Tensor,
              sym: Tensor) -> Tensor:
    """[B] per-sample (l_rot + l_z + l_xy), l1 norms, disentangle_z."""
    gt_rot = matmul3(pts, gt_r.transpose(1, 2))
    gt_rt = gt_rot + gt_t[:, None]
    pred_rot = matmul3(pts, pred_r.transpose(1, 2)) + gt_t[:, None]
    if sym is not None:  # symmetric samples: nearest predicted point per GT point (no host sync)
        with torch.no_grad():  # knn_points' squared distance; HIP kernel on the device
            if gt_rt.is_cuda and not _KNN_TORCH:
                idx = ops.knn1(gt_rt.float().contiguous(), pred_rot.float().contiguous())
            else:
                idx = ((gt_rt[:, :, None] - pred_rot[:, None]) ** 2).sum(-1).argmin(-1)  # [B, P]
        matched = torch.gather(pred_rot, 1, idx[..., None].expand(-1, -1, 3))
        pred_rot = torch.where(sym[:, None, None], matched, pred_rot)
    l_rot = (pred_rot - gt_rt).abs().sum(-1).mean(-1)
    tz = torch.cat([gt_t[:, :2], pred_t[:, 2:]], 1)
    txy = torch.cat([pred_t[:, :2], gt_t[:, 2:]], 1)
    l_z = (gt_rot + tz[:, None] - gt_rt).abs().sum(-1).mean(-1)
    l_xy = (gt_rot + txy[:, None] - gt_rt).abs().sum(-1).mean(-1)
    return l_rot + l_z + l_xy


class _PointMatchingLoss(torch.autograd.Function):
    """The disentangled L1 point-matching loss of one iteration as three HIP launches forward
    (points, nearest-point matching, loss) and one backward (scflow_pm_loss), instead of ~25
    torch kernels forward and ~40 backward; gradients w.r.t. the predicted rotation and
    translation (the GT pose and the model points carry none)."""

    @staticmethod
    def forward(ctx, pred_r, pred_t, gt_r, gt_t, pts, sym, diam, weight):
        pred_r, pred_t = pred_r.contiguous().float(), pred_t.contiguous().float()
        loss, ws = ops.pm_loss(pts, gt_r, gt_t, pred_r, pred_t, sym, diam, weight)
        ctx.save_for_backward(pts, pred_t, gt_t, diam, *[w for w in ws if w is not None])
        ctx.has_sym = sym is not None
        ctx.sym = sym
        ctx.weight = weight
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        pts, pred_t, gt_t, diam, gt_rt, pred_rot, *rest = ctx.saved_tensors
        idx = rest[0] if ctx.has_sym else None
        g_r, g_t = ops.pm_loss_backward(g.reshape(1).contiguous().float(), pts, (gt_rt, pred_rot, idx),
                                        ctx.sym, pred_t, gt_t, diam, ctx.weight)
        return g_r, g_t, None, None, None, None, None, None


def point_matching_loss(pred_r: Tensor, pred_t: Tensor, gt_r: Tensor, gt_t: Tensor, labels: Tensor,
                        points: Sequence[Tensor], diameters: Tensor,
                        weight: float = POSE_WEIGHT, any_symmetric: bool = True,
                        pts: Tensor = None, hoisted: Tuple[Tensor, Tensor] = None) -> Tensor:
    """DisentanglePointMatchingLoss (point_matching_loss.py:159-218) with loss_type l1,
    disentangle_z, no xy/depth scaling, reduction mean.  ``any_symmetric=False`` (the caller
    knows no label is a symmetric class) skips the nearest-neighbour matching.  ``hoisted``:
    (symmetric mask, per-sample diameter) from ``label_terms``, computed once per step."""
    B = pred_r.shape[0]
    labels = labels.long()
    sym, diam = hoisted if hoisted is not None else label_terms(labels, diameters, any_symmetric)
    if len({int(p.shape[0]) for p in points}) == 1:
        if pts is None:
            pts = torch.stack(list(points))[labels]
        if pred_r.is_cuda and not _PM_TORCH:
            return _PointMatchingLoss.apply(
                pred_r, pred_t, gt_r.contiguous().float(), gt_t.contiguous().float(),
                pts.contiguous().float(), None if sym is None else sym.float().contiguous(),
                diam.contiguous().float(), float(weight))
        per = _pm_terms(pts, pred_r, pred_t, gt_r, gt_t, sym)
    else:
        per = torch.cat([_pm_terms(points[int(labels[i])][None], pred_r[i:i + 1], pred_t[i:i + 1],
                                   gt_r[i:i + 1], gt_t[i:i + 1], None if sym is None else sym[i:i + 1])
                         for i in range(B)])
    return weight * (per / diam).sum() / B


def label_terms(labels: Tensor, diameters: Tensor, any_symmetric: bool = True):
    """(symmetric-class mask or None, diameter per sample) of a batch's labels."""
    labels = labels.long()
    sym = None
    if any_symmetric:
        for c in SYMMETRIC_CLASSES:
            sym = (labels == c) if sym is None else (sym | (labels == c))
    return sym, diameters[labels]


def sequence_loss(values: Sequence[Tensor], gamma: float = GAMMA) -> Tensor:
    """SequenceLoss (sequence_loss.py:59-80): Σ γ^(n−i−1)·loss_i."""
    n = len(values)
    return sum(gamma ** (n - i - 1) * v for i, v in enumerate(values))


def filter_flow_by_mask(flow: Tensor, gt_mask: Tensor, invalid_num: float = 400.) -> Tensor:
    """filter_flow_by_mask (models/utils/flow.py:6-26)."""
    N, _, H, W = flow.shape
    bad = (flow[:, 0] >= invalid_num) & (flow[:, 1] >= invalid_num)
    yy = torch.arange(H, device=flow.device, dtype=flow.dtype)[:, None]
    xx = torch.arange(W, device=flow.device, dtype=flow.dtype)[None]
    gx = (xx + flow[:, 0]) * 2. / max(W - 1, 1) - 1.
    gy = (yy + flow[:, 1]) * 2. / max(H - 1, 1) - 1.
    m = F.grid_sample(gt_mask[:, None].to(flow.dtype), torch.stack([gx, gy], -1), mode="bilinear",
                      padding_mode="zeros", align_corners=False)
    bad = (m[:, 0] < 0.9) | bad
    return torch.where(bad[:, None].expand_as(flow), torch.full_like(flow, invalid_num), flow)


def refine_losses(outs, gt_r: Tensor, gt_t: Tensor, gt_flow: Tensor, render_mask: Tensor,
                  labels: Tensor, points: Sequence[Tensor], diameters, max_flow: float = 400.
                  ) -> Tuple[Tensor, Tensor, Tensor]:
    """(loss_pose, loss_flow, loss_mask) from the decoder's 7 lists (scflow_refiner.py:200-242)."""
    _, flow_pred, Rs, ts, masks, _, _ = outs
    diam = diameters if isinstance(diameters, Tensor) else torch.as_tensor(
        diameters, dtype=gt_r.dtype, device=gt_r.device)
    pts = torch.stack(list(points))[labels.long()] if len({int(p.shape[0]) for p in points}) == 1 else None
    hoisted = label_terms(labels, diam)  # iteration-invariant label work, once per step
    n = len(Rs)
    fused = gt_r.is_cuda and pts is not None and flow_pred and isinstance(flow_pred[0], LowRes)
    if fused:
        if not _PM_TORCH:  # the kernel's operand types, converted once
            hoisted = (None if hoisted[0] is None else hoisted[0].float(), hoisted[1].float().contiguous())
        # the fused HIP losses scale by their weight argument: fold SequenceLoss's γ^(n−i−1)
        # into it and sum the 8 terms with one stack + sum instead of 2·8 scalar ops
        gam = [GAMMA ** (n - i - 1) for i in range(n)]
        lp = torch.stack([point_matching_loss(R, t, gt_r, gt_t, labels, points, diam, pts=pts,
                                              hoisted=hoisted, weight=POSE_WEIGHT * gam[i]).reshape(())
                          for i, (R, t) in enumerate(zip(Rs, ts))]).sum()
    else:
        lp = sequence_loss([point_matching_loss(R, t, gt_r, gt_t, labels, points, diam, pts=pts,
                                                hoisted=hoisted)
                            for R, t in zip(Rs, ts)])  # (symmetric matching always evaluated: no sync)
    v = flow_valid(gt_flow, render_mask, max_flow)  # iteration-invariant
    occ = (gt_flow.sum(1) < max_flow).to(gt_flow)
    if flow_pred and isinstance(flow_pred[0], LowRes):  # fused upsample + L1 (HIP)
        from .functions import up_l1_loss
        denom = (v.sum() + 1e-10).reshape(1)
        gt = gt_flow.contiguous()
        gam = [GAMMA ** (len(flow_pred) - i - 1) for i in range(len(flow_pred))]
        lf = torch.stack([up_l1_loss(f.lr, gt, v, f.value_scale, denom, 0.0, FLOW_WEIGHT * gam[i]).reshape(())
                          for i, f in enumerate(flow_pred)]).sum()
        occ4 = occ[:, None].contiguous()
        gam = [GAMMA ** (len(masks) - i - 1) for i in range(len(masks))]
        lm = torch.stack([up_l1_loss(m.lr, occ4, None, m.value_scale, None, float(occ.numel()),
                                     MASK_WEIGHT * gam[i]).reshape(()) for i, m in enumerate(masks)]).sum()
        return lp, lf, lm
    lf = sequence_loss([flow_l1_loss(f, gt_flow, render_mask, max_flow, v=v) for f in flow_pred])
    lm = sequence_loss([mask_l1_loss(m[:, 0], occ) for m in masks])
    return lp, lf, lm
