"""SCFlowRefiner — the inference data flow around the decoder, on the HIP encoders + decoder.

Reference: ``models/refiner/scflow_refiner.py`` — ``__init__`` :17-63 (the feature encoder is
shared by the real and rendered images unless ``seperate_encoder``, base_refiner.py:33-40;
the context encoder is separate), ``extract_feat`` :84-106, ``get_pose`` :108-138.

Only the refinement path is here (SURVEY.md §8 scope): the renderer, data pre-processing,
losses and the training loop of the reference refiner are out of scope, so the loss / renderer
configuration arguments are accepted and ignored.

``get_pose`` runs the work MI355X-first rather than call by call:

* the shared feature encoder runs ONCE on cat[real, rendered] (2B images; InstanceNorm is per
  image, so batching is exact) and writes channels-last features;
* the context encoder writes tanh(h) | relu(cxt) — the split activation fused into its last
  conv — straight into the decoder's channels-last GRU working buffer;
* the decoder then runs with that buffer (no NCHW round trip for h / cxt).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple, Union

import torch
import torch.nn as nn

from . import ops
from ._lib import ScflowError
from .encoder import RAFTEncoder
from .registry import MODELS

Tensor = torch.Tensor


def _build(cfg):
    if isinstance(cfg, nn.Module):
        return cfg
    return MODELS.build(cfg)


@MODELS.register_module()
class SCFlowRefiner(nn.Module):
    def __init__(self, cxt_channels: int, h_channels: int, seperate_encoder: bool, cxt_encoder: dict,
                 encoder: dict, decoder: dict, renderer=None, render_augmentations=None,
                 pose_loss_cfg=None, flow_loss_cfg=None, mask_loss_cfg=None, max_flow: float = 400.,
                 filter_invalid_flow: bool = True, freeze_encoder: bool = False,
                 freeze_bn: bool = False, train_cfg: Optional[dict] = None,
                 test_cfg: Optional[dict] = None, init_cfg=None) -> None:
        super().__init__()
        self.seperate_encoder = seperate_encoder
        if seperate_encoder:
            self.render_encoder = _build(encoder)
            self.real_encoder = _build(encoder)
        else:
            enc = _build(encoder)
            self.render_encoder = enc
            self.real_encoder = enc
        self.decoder = _build(decoder)
        self.context = _build(cxt_encoder)
        self.h_channels, self.cxt_channels = h_channels, cxt_channels
        assert self.h_channels == self.decoder.h_channels
        assert self.cxt_channels == self.decoder.cxt_channels
        assert self.h_channels + self.cxt_channels == self.context.out_channels
        self.max_flow = max_flow
        self.filter_invalid_flow = filter_invalid_flow
        self.train_cfg = train_cfg or {}
        self.test_cfg = test_cfg or {}
        self.test_iter_num = self.test_cfg.get("iters", self.decoder.iters)

    # ------------------------------------------------------------------ reference API
    def extract_feat(self, render_images: Tensor, real_images: Tensor
                     ) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
        """scflow_refiner.py:84-106 — NCHW (render_feat, real_feat, tanh(h), relu(cxt))."""
        real_feat = self.real_encoder(real_images)
        render_feat = self.render_encoder(render_images)
        n = render_images.shape[0]
        c = self.context.forward_cl(render_images.contiguous().float(), act="Tanh", act2="ReLU",
                                    act_split=self.h_channels)
        _, h, w, _ = c.shape
        h_feat = ops.chan_to_nchw(ops.Chan(c, 0, self.h_channels), n, h, w)
        cxt_feat = ops.chan_to_nchw(ops.Chan(c, self.h_channels, self.cxt_channels), n, h, w)
        return render_feat, real_feat, h_feat, cxt_feat

    def get_pose(self, render_images: Tensor, real_images: Tensor, ref_rotation: Tensor,
                 ref_translation: Tensor, depth: Tensor, internel_k: Tensor, label: Tensor,
                 init_flow: Optional[Tensor] = None):
        """scflow_refiner.py:108-138 — images → encoders → SCFlowDecoder outputs (7 lists)."""
        if render_images.device.type != "cuda":
            raise ScflowError("SCFlowRefiner runs on the gfx950 HIP kernels only (no CPU fallback)")
        with torch.no_grad():
            return self._get_pose(render_images.contiguous().float(), real_images.contiguous().float(),
                                  ref_rotation, ref_translation, depth, internel_k, label, init_flow)

    def forward(self, *args, **kwargs):
        return self.get_pose(*args, **kwargs)

    # ------------------------------------------------------------------ fused path
    def _get_pose(self, render, real, R, t, depth, K, label, init_flow):
        N, _, H, W = real.shape
        dev = real.device
        dec = self.decoder
        # feature encoder(s): one launch sequence over cat[real, render] when shared
        if self.real_encoder is self.render_encoder:
            both = torch.cat([real, render], 0)
            fcl = self.real_encoder.forward_cl(both)
            n2, h, w, C = fcl.shape
            feats = ops.chan_to_nchw(ops.Chan.whole(fcl), n2, h, w)
            real_feat, render_feat = feats[:N], feats[N:]
        else:
            real_feat = self.real_encoder(real)
            render_feat = self.render_encoder(render)
            h, w = real_feat.shape[-2:]
        # context encoder → tanh(h) | relu(cxt) straight into the decoder's GRU buffer
        hx = torch.empty(N * h * w, dec.hx_channels, device=dev)
        self.context.forward_cl(render, out=hx.view(N, h, w, dec.hx_channels), act="Tanh",
                                act2="ReLU", act_split=self.h_channels)
        if init_flow is None:
            init_flow = torch.zeros(N, 2, H, W, device=dev)
        return dec._forward(render_feat.contiguous(), real_feat.contiguous(), None, None, R, t, depth,
                            K, label, init_flow, 0.0, hx=hx)
