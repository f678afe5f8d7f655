"""Deterministic synthetic inputs and weights for the SCFlow refinement hot path.

There is no dataset, renderer or checkpoint in this environment,
so every test, golden fixture and benchmark draws its inputs from here:

* decoder inputs shaped like ``SCFlowRefiner.get_pose`` hands them to the decoder
  (``/root/reference/models/refiner/scflow_refiner.py:108-138``): render/real features
  ``[B,256,S/8,S/8]``, ``h=tanh(.)``, ``cxt=relu(.)`` (``scflow_refiner.py:101-104``),
  reference pose, rendered depth ``[B,S,S]``, intrinsics ``[B,3,3]``, labels, zero init flow;
* a YCB-V-like scene: object diameters from ``configs/refine_models/scflow_ycbv_real.py:19-21``,
  t_z ~ U(600, 1200) mm, K with f = S·t_z/(1.1·d_obj) (crop/resize maths of
  ``datasets/pipelines/geometry_transform.py`` ``Crop``/``RemapPose``), depth of an analytic
  ellipsoid standing in for the pytorch3d zbuf (``models/utils/rendering.py:185-248``);
* deterministic per-parameter weights (PCG64 seeded by the crc32 of the state-dict key),
  with the pose head's zero-initialised output layers (``models/head/pose_head.py:187-198``)
  perturbed so the pose actually moves (SURVEY.md §7 "Hard parts" 5).

Everything is generated in float64 with numpy's PCG64 and cast to float32, so the same
arrays come out on every machine (here, and on the GPU box).
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, Iterable, Tuple

import numpy as np

# YCB-V object diameters (mm), configs/refine_models/scflow_ycbv_real.py:19-21
YCBV_DIAMETERS = (172.16, 269.58, 198.38, 120.66, 199.79, 90.17, 142.58, 114.39, 129.73,
                  198.40, 263.60, 260.76, 162.27, 126.86, 230.44, 237.30, 204.11, 121.46,
                  183.08, 231.39, 102.92)


def _rot_zyx(az: float, ay: float, ax: float) -> np.ndarray:
    cz, sz = math.cos(az), math.sin(az)
    cy, sy = math.cos(ay), math.sin(ay)
    cx, sx = math.cos(ax), math.sin(ax)
    rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    return rz @ ry @ rx


def _random_rotation(rng: np.random.Generator) -> np.ndarray:
    q = rng.standard_normal(4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def ellipsoid_depth(R: np.ndarray, t: np.ndarray, K: np.ndarray, size: int,
                    semi_axes: np.ndarray) -> np.ndarray:
    """z-buffer depth of an ellipsoid (object frame semi-axes ``semi_axes``) posed at (R, t).

    Pixel (u, v) casts the ray X = s·K⁻¹[u, v, 1]ᵀ (z-component 1, so s is the depth);
    the nearest intersection with (Rᵀ(X−t))ᵀ D (Rᵀ(X−t)) = 1 is the depth; 0 = background,
    matching the renderer's zbuf convention (models/utils/rendering.py, decoder uses depth>0).
    """
    v, u = np.meshgrid(np.arange(size, dtype=np.float64), np.arange(size, dtype=np.float64),
                       indexing="ij")
    rays = np.stack([u, v, np.ones_like(u)], -1) @ np.linalg.inv(K).T  # [S,S,3], z = 1
    D = np.diag(1.0 / semi_axes ** 2)
    dr = rays @ R  # Rᵀ d for every ray (row vectors)
    tr = R.T @ t
    a = np.einsum("hwi,ij,hwj->hw", dr, D, dr)
    b = -2.0 * np.einsum("hwi,ij,j->hw", dr, D, tr)
    c = float(tr @ D @ tr - 1.0)
    disc = b * b - 4 * a * c
    hit = disc > 0
    s = np.where(hit, (-b - np.sqrt(np.where(hit, disc, 0.0))) / (2 * a), 0.0)
    return np.where(hit & (s > 0), s, 0.0)


def make_scene(batch: int, size: int, seed: int = 0, num_class: int = 21) -> Dict[str, np.ndarray]:
    """Labels, reference poses, intrinsics and rendered depth for ``batch`` image pairs."""
    rng = np.random.default_rng(seed + 7919)
    labels = rng.integers(0, num_class, batch)
    Rs, ts, Ks, depths = [], [], [], []
    for b in range(batch):
        d_obj = YCBV_DIAMETERS[int(labels[b]) % len(YCBV_DIAMETERS)]
        tz = rng.uniform(600.0, 1200.0)
        txy = rng.normal(0.0, 15.0, 2)
        t = np.array([txy[0], txy[1], tz])
        # reference pose = a random orientation jittered like PoseJitter (datasets/pipelines/jitter.py:51-79)
        ang = np.clip(rng.normal(0.0, math.radians(15.0), 3), -math.radians(45), math.radians(45))
        R = _rot_zyx(*ang) @ _random_rotation(rng)
        f = size * tz / (1.1 * d_obj)
        # principal point at the patch centre, shifted so the object centre projects near it
        K = np.array([[f, 0.0, size / 2.0 - f * t[0] / t[2]],
                      [0.0, f, size / 2.0 - f * t[1] / t[2]],
                      [0.0, 0.0, 1.0]])
        semi = np.array([0.5, 0.38, 0.3]) * d_obj
        depths.append(ellipsoid_depth(R, t, K, size, semi))
        Rs.append(R)
        ts.append(t)
        Ks.append(K)
    return dict(labels=labels.astype(np.int64), ref_rotation=np.stack(Rs).astype(np.float32),
                ref_translation=np.stack(ts).astype(np.float32),
                internel_k=np.stack(Ks).astype(np.float32),
                depth=np.stack(depths).astype(np.float32))


def make_decoder_inputs(batch: int, size: int, seed: int = 0, feat_channels: int = 256,
                        h_channels: int = 128, cxt_channels: int = 128,
                        num_class: int = 21) -> Dict[str, np.ndarray]:
    """All inputs of ``SCFlowDecoder.forward`` (scflow_decoder.py:151-156) as float32 numpy."""
    rng = np.random.default_rng(seed)
    h = w = size // 8
    feat_render = rng.standard_normal((batch, feat_channels, h, w))
    # the real image is the rendered one moved by a couple of feature cells plus noise, so the
    # correlation volume has a real peak away from the identity
    feat_real = np.roll(feat_render, shift=(1, -2), axis=(2, 3)) + 0.3 * rng.standard_normal(
        feat_render.shape)
    h_feat = np.tanh(rng.standard_normal((batch, h_channels, h, w)))
    cxt_feat = np.maximum(rng.standard_normal((batch, cxt_channels, h, w)), 0.0)
    out = dict(feat_render=feat_render.astype(np.float32), feat_real=feat_real.astype(np.float32),
               h_feat=h_feat.astype(np.float32), cxt_feat=cxt_feat.astype(np.float32))
    out.update(make_scene(batch, size, seed, num_class))
    out["init_flow"] = np.zeros((batch, 2, size, size), np.float32)
    return out


def make_images(batch: int, size: int, seed: int = 0) -> Dict[str, np.ndarray]:
    """Rendered / real image pair batch: rendered ~ U[0,1) (the config's
    Normalize is mean 0 / std 255, scflow_ycbv_real.py:42-43, so images enter in [0, 1]),
    real = rendered rolled by (3, −2) px plus N(0, 0.02) noise."""
    rng = np.random.default_rng(seed + 7919)
    render = rng.uniform(0.0, 1.0, (batch, 3, size, size))
    real = np.roll(render, shift=(3, -2), axis=(2, 3)) + 0.02 * rng.standard_normal(render.shape)
    return dict(render_images=render.astype(np.float32), real_images=real.astype(np.float32))


def _param_rng(key: str, seed: int) -> np.random.Generator:
    return np.random.default_rng(zlib.crc32(key.encode()) ^ (seed * 0x9E3779B1 & 0xFFFFFFFF))


def param_value(key: str, shape: Tuple[int, ...], seed: int = 0) -> np.ndarray:
    """Deterministic value for one decoder parameter, by its reference state-dict key.

    conv/linear weights: U(-1,1)·√(3/fan_in) (unit-variance pre-activations);
    biases: U(-0.1, 0.1); GroupNorm affine: 1+U(-.1,.1) / U(-.1,.1).
    The pose head's output layers (zero-initialised in the reference, pose_head.py:187-198)
    get small weights and the identity ortho6d bias plus a perturbation, so Δpose ≠ identity.
    """
    rng = _param_rng(key, seed)
    u = rng.uniform(-1.0, 1.0, size=shape)
    if "rotation_pred" in key or "translation_pred" in key:
        if key.endswith("weight"):
            return (u * 2e-3).astype(np.float32)
        if "rotation_pred" in key:  # ortho6d identity [1,0,0,0,1,0] per class + noise
            base = np.tile(np.array([1.0, 0, 0, 0, 1.0, 0]), shape[0] // 6)
            return (base + 2e-2 * u).astype(np.float32)
        return (2e-2 * u).astype(np.float32)
    if key.endswith("running_var"):  # encoder BatchNorm statistics (context encoder)
        return (1.0 + 0.25 * u).astype(np.float32)
    if key.endswith("running_mean"):
        return (0.1 * u).astype(np.float32)
    if key.endswith(".gn.weight") or (key.endswith("weight") and len(shape) == 1):
        return (1.0 + 0.1 * u).astype(np.float32)
    if key.endswith(".gn.bias") or key.endswith("bias"):
        return (0.1 * u).astype(np.float32)
    fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else int(shape[0])
    return (u * math.sqrt(3.0 / max(fan_in, 1))).astype(np.float32)


def make_state_dict(shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int = 0) -> Dict[str, np.ndarray]:
    """Values for every (key, shape) pair; keys are the reference decoder's state-dict keys."""
    return {k: param_value(k, tuple(s), seed) for k, s in shapes}


def fill_module_(module, seed: int = 0) -> None:
    """Overwrite every parameter of a torch module with ``param_value`` (in place)."""
    import torch
    with torch.no_grad():
        for k, p in module.state_dict().items():
            if not p.is_floating_point():
                continue
            v = torch.from_numpy(param_value(k, tuple(p.shape), seed))
            p.copy_(v.to(p.dtype))


ELLIPSOID_AXES = (0.5, 0.38, 0.3)  # semi-axes / diameter of the stand-in object (make_scene)


def make_model_points(num_points: int = 512, num_class: int = 21, seed: int = 0) -> np.ndarray:
    """[num_class, P, 3] model points on each class's stand-in ellipsoid surface (mm) — the
    meshes the point-matching loss reads (point_matching_loss.py:148-155) are absent here."""
    rng = np.random.default_rng(seed + 104729)
    out = np.empty((num_class, num_points, 3))
    for c in range(num_class):
        d = rng.standard_normal((num_points, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        out[c] = d * np.array(ELLIPSOID_AXES) * YCBV_DIAMETERS[c % len(YCBV_DIAMETERS)]
    return out.astype(np.float32)


def make_train_targets(scene: Dict[str, np.ndarray], size: int, seed: int = 0,
                       rot_deg: float = 5.0, trans_xy: float = 8.0, trans_z: float = 0.03
                       ) -> Dict[str, np.ndarray]:
    """Ground-truth pose (the reference pose perturbed like PoseJitter,
    datasets/pipelines/jitter.py:51-79, here small so the GT flow stays in range) and the GT
    mask (the stand-in ellipsoid rendered at the GT pose) for a ``make_scene`` batch."""
    rng = np.random.default_rng(seed + 15485863)
    Rs, ts, masks = [], [], []
    for b in range(len(scene["labels"])):
        ang = rng.normal(0.0, math.radians(rot_deg), 3)
        R = _rot_zyx(*ang) @ scene["ref_rotation"][b].astype(np.float64)
        t = scene["ref_translation"][b].astype(np.float64).copy()
        t[:2] += rng.normal(0.0, trans_xy, 2)
        t[2] *= 1.0 + rng.normal(0.0, trans_z)
        d_obj = YCBV_DIAMETERS[int(scene["labels"][b]) % len(YCBV_DIAMETERS)]
        masks.append(ellipsoid_depth(R, t, scene["internel_k"][b].astype(np.float64), size,
                                     np.array(ELLIPSOID_AXES) * d_obj) > 0)
        Rs.append(R)
        ts.append(t)
    return dict(gt_rotation=np.stack(Rs).astype(np.float32),
                gt_translation=np.stack(ts).astype(np.float32), gt_masks=np.stack(masks))


def make_train_batch(batch: int, size: int, seed: int = 0, labels=None) -> Dict[str, np.ndarray]:
    """One supervised training batch (the fields SCFlowRefiner.loss reads after
    format_data_train_sup, base_refiner.py:154-225): image pair, reference + GT pose, rendered
    depth, intrinsics, labels, GT mask."""
    scene = make_scene(batch, size, seed=seed)
    if labels is not None:
        scene["labels"] = np.asarray(labels, np.int64)
    out = {**make_images(batch, size, seed=seed), **scene, **make_train_targets(scene, size, seed=seed)}
    out["label"] = out.pop("labels")
    return out


def ellipsoid_mesh(semi_axes, n_lat: int = 24, n_lon: int = 48) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """UV-sphere triangle mesh of the stand-in object (the models_1024 meshes the renderer reads,
    scflow_ycbv_real.py:262, are absent): verts [V,3] float32 (mm), faces [F,3] int64
    (outward-consistent winding), vertex colours [V,3] in [0, 1] (a smooth pattern)."""
    a = np.asarray(semi_axes, np.float64)
    verts = [[0.0, 0.0, a[2]]]
    for i in range(1, n_lat):
        th = math.pi * i / n_lat
        for j in range(n_lon):
            ph = 2 * math.pi * j / n_lon
            verts.append([a[0] * math.sin(th) * math.cos(ph), a[1] * math.sin(th) * math.sin(ph),
                          a[2] * math.cos(th)])
    verts.append([0.0, 0.0, -a[2]])
    verts = np.asarray(verts)
    faces = []
    ring = lambda i, j: 1 + (i - 1) * n_lon + (j % n_lon)  # noqa: E731
    for j in range(n_lon):
        faces.append([0, ring(1, j), ring(1, j + 1)])
    for i in range(1, n_lat - 1):
        for j in range(n_lon):
            faces.append([ring(i, j), ring(i + 1, j), ring(i + 1, j + 1)])
            faces.append([ring(i, j), ring(i + 1, j + 1), ring(i, j + 1)])
    last = len(verts) - 1
    for j in range(n_lon):
        faces.append([last, ring(n_lat - 1, j + 1), ring(n_lat - 1, j)])
    u = verts / a
    colors = 0.5 + 0.4 * np.stack([u[:, 0], u[:, 1] * u[:, 2], np.cos(3 * u[:, 0])], 1)
    return verts.astype(np.float32), np.asarray(faces, np.int64), colors.astype(np.float32)
