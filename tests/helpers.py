"""Shared test helpers: golden fixtures, synthetic inputs, the oracle's state dict."""
import os
from functools import lru_cache

import numpy as np
import torch

from scflow_amd import synthetic

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_FILES = {"ops": "golden_ops.npz", "e2e": "golden_e2e_b2_s256_it4.npz",
          "enc": "golden_enc_b1_s128.npz", "refine": "golden_refine_b2_s256_it4.npz"}


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
