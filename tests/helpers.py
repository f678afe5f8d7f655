"""Shared test helpers: golden fixtures, synthetic inputs, the oracle's state dict."""
import os
from functools import lru_cache

import numpy as np
import torch

from scflow_amd import synthetic

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_FILES = {"ops": "golden_ops.npz", "e2e": "golden_e2e_b2_s256_it4.npz",
          "enc": "golden_enc_b1_s128.npz", "refine": "golden_refine_b2_s256_it4.npz",
          "render_wiring": "golden_render_wiring.npz"}


@lru_cache(maxsize=None)
def golden(name):
    with np.load(os.path.join(GOLDEN, _FILES[name]), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def t(a, dtype=None):
    x = torch.from_numpy(np.ascontiguousarray(a))
    return x if dtype is None else x.to(dtype)


def reference_state_shapes():
    g = golden("e2e")
    return [(str(k), tuple(int(s) for s in str(v).split(",") if s))
            for k, v in zip(g["state_keys"], g["state_shapes"])]


def oracle_state_dict(seed=0, dtype=torch.float32):
    vals = synthetic.make_state_dict(reference_state_shapes(), seed=seed)
    return {k: torch.from_numpy(v).to(dtype) for k, v in vals.items()}


def decoder_inputs(B, S, seed, g=None, dtype=torch.float32, device="cpu"):
    """Regenerate the decoder inputs; when a golden dict is given, check they are the same."""
    raw = synthetic.make_decoder_inputs(B, S, seed=seed)
    if g is not None:
        for k in ("feat_render", "feat_real", "h_feat", "cxt_feat"):
            ref = g[f"sum_{k}"]
            got = np.array([raw[k].astype(np.float64).sum(), np.abs(raw[k]).astype(np.float64).sum()])
            np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-6)
        for k in ("labels", "ref_rotation", "ref_translation", "internel_k", "depth"):
            np.testing.assert_array_equal(raw[k], g[f"in_{k}"])
    out = {}
    for k, v in raw.items():
        x = torch.from_numpy(v)
        if x.is_floating_point():
            x = x.to(dtype)
        out[k] = x.to(device)
    out["label"] = out.pop("labels")
    return out


def encoder_state_shapes(norm):
    """(key, shape) of the reference RAFTEncoder with norm 'IN' / 'BN' (from the fixture)."""
    g = golden("enc")
    return [(str(k), tuple(int(x) for x in str(v).split(",") if x))
            for k, v in zip(g[f"keys_{norm}"], g[f"shapes_{norm}"])
            if not str(k).endswith("num_batches_tracked")]


def encoder_state_dict(norm, seed, prefix="", dtype=torch.float32):
    vals = synthetic.make_state_dict(encoder_state_shapes(norm), seed=seed)
    return {prefix + k: torch.from_numpy(v).to(dtype) for k, v in vals.items()}


def refiner_state_dict(dtype=torch.float32):
    """Flat oracle state dict of the refinement model: the shared feature encoder (seed 1) under
    both attribute names, the context encoder (seed 2), the decoder (seed 0)."""
    sd = oracle_state_dict(seed=0, dtype=dtype)
    sd.update(encoder_state_dict("IN", 1, "real_encoder.", dtype))
    sd.update(encoder_state_dict("IN", 1, "render_encoder.", dtype))
    sd.update(encoder_state_dict("BN", 2, "context.", dtype))
    return sd


def refine_inputs(B, S, seed, g=None, dtype=torch.float32, device="cpu"):
    """Images + scene of the refinement fixture; checked against the fixture's checksums."""
    imgs = synthetic.make_images(B, S, seed=seed)
    scene = synthetic.make_scene(B, S, seed=seed)
    if g is not None:
        got = np.array([imgs["render_images"].astype(np.float64).sum(),
                        imgs["real_images"].astype(np.float64).sum()])
        np.testing.assert_allclose(got, g["sum_images"], rtol=1e-12)
    out = {k: torch.from_numpy(v) for k, v in {**imgs, **scene}.items()}
    for k, v in out.items():
        if v.is_floating_point():
            out[k] = v.to(dtype)
        out[k] = out[k].to(device)
    out["label"] = out.pop("labels")
    return out


# ------------------------------------------------------------------ §8(f)-4 BOP tree
def _rot_np(rng):
    q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
    return (q * np.sign(np.linalg.det(q))).astype(np.float32)


def make_bop_case(root, seed=11, n_class=21, n_verts=1500):
    """A synthetic BOP tree under ``root`` (data/{seq}/scene_gt|scene_camera|scene_gt_info.json,
    an image list, keypoints, empty obj_XXXXXX.ply mesh files) and the reference-format results:
    per image single, duplicate (2–3 candidates), missing and spurious predictions, symmetric
    classes included.  Returns (results, mesh vertices [n_class, n_verts, 3], image list lines)."""
    import json as _json
    rng = np.random.default_rng(seed)
    verts = synthetic.make_model_points(n_verts, n_class, seed=seed)
    data = os.path.join(root, "data")
    os.makedirs(os.path.join(root, "models_eval"), exist_ok=True)
    for c in range(n_class):
        open(os.path.join(root, "models_eval", f"obj_{c + 1:06d}.ply"), "w").close()
    with open(os.path.join(root, "bbox.json"), "w") as f:
        _json.dump(rng.standard_normal((n_class, 8, 3)).round(3).tolist(), f)
    results, lines = [], []
    for seq in (48, 55):
        scene_gt, scene_cam, scene_info = {}, {}, {}
        for img in range(1, 7):
            f = 500.0 + 100 * rng.random()
            K = [[f, 0, 320.0], [0, f, 240.0], [0, 0, 1]]
            objs, pl, pr, pt = [], [], [], []
            for oid in rng.choice(np.arange(1, n_class + 1), size=4, replace=False):
                oid = int(oid)
                R = _rot_np(rng)
                t = np.array([rng.normal() * 60, rng.normal() * 60, 600 + 500 * rng.random()], np.float32)
                objs.append(dict(cam_R_m2c=R.reshape(-1).tolist(), cam_t_m2c=t.tolist(), obj_id=oid))
                mode = int(rng.integers(0, 5))
                if mode == 4:  # missed object
                    continue
                ncand = 1 if mode < 2 else int(rng.integers(2, 4))
                for k in range(ncand):
                    noise = float(rng.choice([0.5, 5.0, 30.0, 120.0]))
                    Rn = R if rng.random() < 0.6 else _rot_np(rng)
                    pl.append(oid - 1)
                    pr.append(Rn)
                    pt.append(t + rng.normal(size=3).astype(np.float32) * noise)
            if rng.random() < 0.5:  # a spurious prediction of a class not in the image
                extra = int(rng.integers(1, n_class + 1))
                if all(o["obj_id"] != extra for o in objs):
                    pl.append(extra - 1)
                    pr.append(_rot_np(rng))
                    pt.append(np.array([0, 0, 800], np.float32))
            scene_gt[str(img)] = objs
            scene_cam[str(img)] = dict(cam_K=np.asarray(K).reshape(-1).tolist(), depth_scale=0.1)
            scene_info[str(img)] = [dict(bbox_obj=[0, 0, 10, 10], visib_fract=1.0) for _ in objs]
            rel = f"{seq:06d}/rgb/{img:06d}.png"
            lines.append(rel)
            results.append(dict(img_metas=dict(img_path=os.path.join(data, rel)),
                                pred=dict(labels=np.asarray(pl, np.int64),
                                          rotations=np.asarray(pr, np.float32).reshape(-1, 3, 3),
                                          translations=np.asarray(pt, np.float32).reshape(-1, 3))))
        d = os.path.join(data, f"{seq:06d}")
        os.makedirs(d, exist_ok=True)
        for name, content in (("scene_gt", scene_gt), ("scene_camera", scene_cam),
                              ("scene_gt_info", scene_info)):
            with open(os.path.join(d, f"{name}.json"), "w") as f:
                _json.dump(content, f)
    with open(os.path.join(root, "test.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    return results, verts, lines
