"""Pose-accuracy metrics: the numeric core of the reference's ``ADD``
metric (metrics/add.py) — ``eval_pose_error`` :354-400 (ADD / ADD-S normalised by the object
diameter, mean 2D reprojection error) and the class-wise precision of ``parse_error_to_metric``
:261-330 — on device tensors, batched per class.

What stays the reference's: BOP annotation loading, prediction↔GT matching
(``match_results``), result dumping — data-set I/O (no YCB-V data exists here).  ADD-S (the
symmetric classes of ``mesh_symmetry``) matches each GT point to the nearest predicted point
(brute force, chunked) exactly like the reference's numpy argmin; the reference also
sub-samples 1000 vertices per mesh at random (:157) — pass the points to use.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import torch

Tensor = torch.Tensor


def project(points: Tensor, K: Tensor, R: Tensor, t: Tensor) -> Tuple[Tensor, Tensor]:
    """datasets/pose.py:18-75 project_3d_point (multi-image): [P,3] points, [N,3,3] K and R,
    [N,3] t → (2D [N,P,2] with the 1e-8 guard, camera-frame 3D [N,P,3])."""
    cam = torch.einsum("nij,pj->npi", R, points) + t[:, None, :]
    uvw = torch.einsum("nij,npj->npi", K, cam)
    uv = uvw[..., :2] / (uvw[..., 2:] + 1e-8)
    return uv, cam


def _nearest(gt: Tensor, pred: Tensor, chunk: int = 2048) -> Tensor:
    """For each GT point the nearest predicted point (ADD-S), per image, chunked over GT."""
    out = torch.empty_like(gt)
    for s in range(0, gt.shape[1], chunk):
        d = torch.cdist(gt[:, s:s + chunk], pred)  # [N, c, P]
        idx = d.argmin(-1)
        out[:, s:s + chunk] = torch.gather(pred, 1, idx[..., None].expand(-1, -1, 3))
    return out


def pose_errors(points: Sequence[Tensor], gt_R: Tensor, gt_t: Tensor, pred_R: Tensor, pred_t: Tensor,
                labels: Tensor, K: Tensor, symmetric: Sequence[int], diameters: Sequence[float]
                ) -> Dict[str, Tensor]:
    """ADD(-S)/diameter ('add'), mean reprojection error in px ('rep') and ADD(-S) in model units
    ('add_mm') per prediction (metrics/add.py:354-400).  points[label]: [P,3] model points;
    ``symmetric``: labels evaluated with ADD-S."""
    n = labels.shape[0]
    dev = gt_R.device
    add = torch.empty(n, device=dev, dtype=gt_R.dtype)
    rep = torch.empty_like(add)
    add_mm = torch.empty_like(add)
    sym = set(int(s) for s in symmetric)
    for lab in torch.unique(labels).tolist():
        m = labels == lab
        pts = points[lab].to(dev, gt_R.dtype)
        g2, g3 = project(pts, K[m], gt_R[m], gt_t[m])
        p2, p3 = project(pts, K[m], pred_R[m], pred_t[m])
        if lab in sym:
            p3 = _nearest(g3, p3)
        e3 = (g3 - p3).norm(dim=-1).mean(-1)
        add_mm[m] = e3
        add[m] = e3 / float(diameters[lab])
        rep[m] = (g2 - p2).norm(dim=-1).mean(-1)
    return {"add": add, "rep": rep, "add_mm": add_mm}


def classwise_precision(errors: Tensor, labels: Tensor, thresholds: Sequence[float],
                        class_names: Sequence[str]) -> Tuple[Dict[str, List[float]], List[float]]:
    """parse_error_to_metric (:309-330): per class the fraction of predictions with
    error < thr for each threshold (−1 for a class with no prediction), and the average over
    the classes that have predictions."""
    per_class: Dict[str, List[float]] = {}
    sums = [0.0] * len(thresholds)
    count = 0
    for c, name in enumerate(class_names):
        e = errors[labels == c]
        if e.numel() == 0:
            per_class[name] = [-1.0] * len(thresholds)
            continue
        vals = [float((e < thr).float().mean()) for thr in thresholds]
        per_class[name] = vals
        sums = [a + b for a, b in zip(sums, vals)]
        count += 1
    avg = [s / count if count else -1.0 for s in sums]
    return per_class, avg
