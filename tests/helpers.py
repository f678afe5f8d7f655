"""Shared test helpers: golden fixtures, synthetic inputs, the oracle's state dict."""
import os
from functools import lru_cache

import numpy as np
import torch

from scflow_amd import synthetic

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_FILES = {"ops": "golden_ops.npz", "e2e": "golden_e2e_b2_s256_it4.npz"}


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
