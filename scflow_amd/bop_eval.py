"""BOP-format pose evaluation: the host side of the reference's ``ADD``
metric (metrics/add.py) around the numeric core in ``metrics.py``.

* ``load_bop_annotations`` — per sequence ``scene_gt.json`` / ``scene_camera.json`` /
  ``scene_gt_info.json`` (add.py:71-89 ``_load_pose_annots``; the BOP layout ``{seq:06d}/…``).
* ``match_results`` — prediction ↔ GT matching (add.py:184-255): for every GT object of an
  image, the one prediction of its class, or — several predictions of that class — the one with
  the smallest normalised ADD(-S), or none (invalid; errors filled with the reference's 1 / 50 px
  / 110 values, add.py:158-160).
* ``parse_error_to_metric`` — class-wise precision at the thresholds (add.py:261-330: per class
  the fraction with error < thr, −1 for an absent class, the average over present classes per
  threshold) and the ``{class}/{metric}`` dictionary of ``parse_metric_to_tensorboard``.
* ``evaluate`` — compute_metrics (add.py:134-180): match, ADD(-S)/diameter + reprojection error
  (``metrics.pose_errors``), the table.
* ``format_results`` — predictions dumped as BOP ``scene_gt.json`` per sequence (add.py:402-446).

Inputs are plain dicts / arrays (the reference's ``results`` entries: ``img_metas.img_path``,
``pred.labels / rotations / translations``); model points are passed in (the reference samples
1000 mesh vertices at random per class with trimesh — once in match_results, add.py:190, and
again in compute_metrics, add.py:157 — trimesh and the meshes are absent here, so the caller
supplies both point sets).  Parity: pinned by ``tests/golden/golden_metric_add.npz``, generated
from the reference's own ``ADD`` class (constructed with its real ``__init__`` on a synthetic BOP
tree, ``make_golden.py metric``) — compute_metrics end to end, match_results, eval_pose_error,
parse_error_to_metric and the scene_gt.json text (tests/test_metric_golden.py).
"""
from __future__ import annotations

import json
import os
import os.path as osp
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .metrics import pose_errors

POSE_JSON = "{:06d}/scene_gt.json"
INFO_JSON = "{:06d}/scene_gt_info.json"
CAMERA_JSON = "{:06d}/scene_camera.json"


def load_bop_annotations(annots_root: str, sequences: Sequence[str]) -> Dict[str, dict]:
    """{sequence: {'pose': scene_gt, 'camera': scene_camera, 'gt_info': scene_gt_info (if any)}}."""
    out = {}
    for seq in sequences:
        sid = int(seq)
        d = {}
        for key, tmpl in (("pose", POSE_JSON), ("camera", CAMERA_JSON), ("gt_info", INFO_JSON)):
            path = osp.join(annots_root, tmpl.format(sid))
            if osp.exists(path):
                with open(path) as f:
                    d[key] = json.load(f)
        out[seq] = d
    return out


def _seq_and_image(img_path: str) -> Tuple[str, int]:
    """add.py:193-198: '…/{seq}/rgb/{img}.png' → (seq, image id)."""
    parts = img_path.rsplit("/", 3)
    seq, img_name = (parts[0], parts[2]) if len(parts) == 3 else (parts[1], parts[3])
    return seq, int(osp.splitext(img_name)[0])


def _errors(points, gt_r, gt_t, pred_r, pred_t, labels0, k, symmetric, diameters):
    """metrics.pose_errors on float64 CPU tensors → numpy (add, rep, add_mm)."""
    t = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float64)  # noqa: E731
    e = pose_errors([t(p) for p in points], t(gt_r), t(gt_t), t(pred_r), t(pred_t),
                    torch.as_tensor(np.asarray(labels0), dtype=torch.int64), t(k), symmetric, diameters)
    return e["add"].numpy(), e["rep"].numpy(), e["add_mm"].numpy()


def match_results(results: Sequence[dict], gt_annots: Dict[str, dict], points: Sequence[np.ndarray],
                  symmetric: Sequence[int], diameters: Sequence[float],
                  inverse_label_mapping: Optional[Dict[int, int]] = None):
    """(gt_R [M,3,3], gt_t [M,3], pred_R, pred_t, labels0 [M] (0-based), valid [M] bool, K [M,3,3])
    over every GT object of every result's image (add.py:184-255)."""
    inv = inverse_label_mapping or {}
    gR, gT, pR, pT, K, valid, labels = [], [], [], [], [], [], []
    for res in results:
        seq, img_id = _seq_and_image(res["img_metas"]["img_path"])
        ann = gt_annots[seq]
        gt_objs = ann["pose"][str(img_id)]
        k = np.asarray(ann["camera"][str(img_id)]["cam_K"], dtype=np.float32).reshape(3, 3)
        pred = res["pred"]
        pl = np.array([inv.get(int(l) + 1, int(l) + 1) for l in np.asarray(pred["labels"])], dtype=np.int64)
        prs = np.asarray(pred["rotations"], dtype=np.float32).reshape(-1, 3, 3)
        pts = np.asarray(pred["translations"], dtype=np.float32).reshape(-1, 3)
        for obj in gt_objs:
            oid = int(obj["obj_id"])
            R = np.asarray(obj["cam_R_m2c"], dtype=np.float32).reshape(3, 3)
            tt = np.asarray(obj["cam_t_m2c"], dtype=np.float32).reshape(-1)
            gR.append(R)
            gT.append(tt)
            K.append(k)
            labels.append(oid)
            m = pl == oid
            nm = int(m.sum())
            if nm == 1:
                j = int(np.nonzero(m)[0][0])
                pR.append(prs[j])
                pT.append(pts[j])
                valid.append(True)
            elif nm > 1:  # the candidate with the smallest normalised ADD(-S)
                add, _, _ = _errors(points, np.repeat(R[None], nm, 0), np.repeat(tt[None], nm, 0),
                                    prs[m], pts[m], np.full(nm, oid - 1), np.repeat(k[None], nm, 0),
                                    symmetric, diameters)
                full = np.full(m.shape[0], 100.0, dtype=np.float32)
                full[m] = add
                j = int(np.argmin(full))
                pR.append(prs[j])
                pT.append(pts[j])
                valid.append(True)
            else:
                pR.append(np.zeros((3, 3), np.float32))
                pT.append(np.zeros(3, np.float32))
                valid.append(False)
    return (np.stack(gR), np.stack(gT), np.stack(pR), np.stack(pT),
            np.asarray(labels, np.int64) - 1, np.asarray(valid, bool), np.stack(K))


def parse_error_to_metric(error_dict: Dict[str, np.ndarray], labels: np.ndarray,
                          metrics: Dict[str, Sequence[float]], class_names: Sequence[str]):
    """(metric_dict {'average': [...], class: [...]}, headers) as add.py:261-330 for the
    thresholded metrics ('add', 'rep'); metrics outside those two are skipped, as there."""
    metric_dict: Dict[str, List[float]] = {"average": []}
    headers = ["class"]
    per_class = {c: [] for c in class_names}
    avg_total: List[List[float]] = []
    for metric, thresholds in metrics.items():
        if metric not in ("add", "rep"):
            continue
        err = error_dict[metric]
        thresholds = list(thresholds)
        if not thresholds:  # already a per-sample quantity: class means
            headers.append(metric)
            for l, name in enumerate(class_names):
                sel = err[labels == l]
                per_class[name].append(-1 if sel.size == 0 else float(sel.mean()))
            avg_total.append(err.tolist())
            continue
        for thr in thresholds:
            headers.append("{}_{:0>2d}".format(metric, int(thr * 100)) if thr < 1
                           else "{}_{:0>2d}".format(metric, thr))
        avg = [[] for _ in thresholds]
        for l, name in enumerate(class_names):
            sel = err[labels == l]
            if sel.shape[0] == 0:
                per_class[name].extend([-1.0] * len(thresholds))
                continue
            for i, thr in enumerate(thresholds):
                v = float((sel < thr).sum() / sel.shape[0])
                per_class[name].append(v)
                avg[i].append(v)
        avg_total.extend(avg)
    metric_dict.update(per_class)
    metric_dict["average"] = [sum(p) / len(p) for p in avg_total]
    return metric_dict, headers


def to_flat_dict(metric_dict: Dict[str, List[float]], headers: Sequence[str]) -> Dict[str, float]:
    """parse_metric_to_tensorboard (add.py:344-351): {'{class}/{metric}': value}."""
    out = {}
    for name, vals in metric_dict.items():
        for i, h in enumerate(headers):
            if h != "class":
                out[f"{name}/{h}"] = vals[i - 1]
    return out


def evaluate(results: Sequence[dict], gt_annots: Dict[str, dict], points: Sequence[np.ndarray],
             class_names: Sequence[str], symmetric: Sequence[int], diameters: Sequence[float],
             metrics: Optional[Dict[str, Sequence[float]]] = None,
             inverse_label_mapping: Optional[Dict[int, int]] = None,
             match_points: Optional[Sequence[np.ndarray]] = None,
             round_digits: Optional[int] = 4) -> Dict[str, float]:
    """compute_metrics (add.py:134-180) → the flat '{class}/{metric}' dictionary.

    ``points``: the model points the errors are measured on (add.py:157); ``match_points``: those
    the duplicate-prediction matching uses (add.py:190; default ``points`` — the reference draws
    the two sets separately).  ``round_digits``: the reference's print_metric rounds every value
    to 4 decimals in place before parse_metric_to_tensorboard (add.py:334-339), so its returned
    dictionary holds rounded values; None keeps full precision."""
    metrics = metrics if metrics is not None else {"auc": [], "add": [0.05, 0.10, 0.20, 0.50]}
    gR, gT, pR, pT, labels, valid, K = match_results(
        results, gt_annots, points if match_points is None else match_points, symmetric, diameters,
        inverse_label_mapping)
    add = np.ones(labels.shape, np.float32)
    rep = np.full(labels.shape, 50.0, np.float32)
    if valid.any():
        a, r, _ = _errors(points, gR[valid], gT[valid], pR[valid], pT[valid], labels[valid], K[valid],
                          symmetric, diameters)
        add[valid] = a
        rep[valid] = r
    md, headers = parse_error_to_metric({"add": add, "rep": rep}, labels, metrics, class_names)
    if round_digits is not None:
        md = {k: [round(x, round_digits) for x in v] for k, v in md.items()}
    return to_flat_dict(md, headers)


def dumps_json(data, indent: int = 2, depth: int = 2) -> str:
    """JSON text as the reference's BOP dumps write it (datasets/utils.py:39-67): indented
    ``indent`` spaces per level, except that every container whose children would sit deeper
    than ``depth`` levels is written compactly on its opening line — for scene_gt.json, one line
    per predicted object."""
    def enc(v, level):
        if isinstance(v, (dict, list)) and v:
            if level >= depth:
                return json.dumps(v)
            pad = " " * (indent * (level + 1))
            end = "\n" + " " * (indent * level)
            if isinstance(v, dict):
                body = ",\n".join(f"{pad}{json.dumps(k)}: {enc(x, level + 1)}" for k, x in v.items())
                return "{\n" + body + end + "}"
            body = ",\n".join(pad + enc(x, level + 1) for x in v)
            return "[\n" + body + end + "]"
        return json.dumps(v)
    return enc(data, 0)


def format_results(results: Sequence[dict], data_root: str, save_dir: str,
                   inverse_label_mapping: Optional[Dict[int, int]] = None,
                   time: Optional[float] = None) -> List[str]:
    """Predictions written as BOP ``scene_gt.json`` per sequence under save_dir (add.py:402-446,
    the reference's dumps_json layout); returns the written paths."""
    inv = inverse_label_mapping or {}
    per_seq: Dict[str, Dict[str, list]] = {}
    for res in results:
        dst = res["img_metas"]["img_path"].replace(data_root, save_dir)
        seq_dir = os.path.dirname(os.path.dirname(dst))
        img_id = str(int(os.path.splitext(os.path.basename(dst))[0]))
        pred = res["pred"]
        rs = np.asarray(pred["rotations"], dtype=np.float64).reshape(-1, 3, 3)
        ts = np.asarray(pred["translations"], dtype=np.float64).reshape(-1, 3)
        objs = []
        for i, l in enumerate(np.asarray(pred["labels"])):
            d = dict(cam_R_m2c=rs[i].reshape(-1).tolist(), cam_t_m2c=ts[i].tolist(),
                     obj_id=inv.get(int(l) + 1, int(l) + 1))
            if time is not None:
                d["time"] = time
            objs.append(d)
        entries = per_seq.setdefault(seq_dir, {})
        if img_id in entries:
            raise ValueError(f"duplicate image {img_id} in {seq_dir}")
        entries[img_id] = objs
    paths = []
    for seq_dir, content in per_seq.items():
        os.makedirs(seq_dir, exist_ok=True)
        path = os.path.join(seq_dir, "scene_gt.json")
        with open(path, "w") as f:
            f.write(dumps_json(content))
        paths.append(path)
    return paths
