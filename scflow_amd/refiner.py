"""SCFlowRefiner — the inference data flow around the decoder, on the HIP encoders + decoder.

Reference: ``models/refiner/scflow_refiner.py`` — ``__init__`` :17-63 (the feature encoder is
shared by the real and rendered images unless ``seperate_encoder``, base_refiner.py:33-40;
the context encoder is separate), ``extract_feat`` :84-106, ``get_pose`` :108-138.

Also here: the renderer-driven inference loop of ``BaseRefiner`` (base_refiner.py: the render
step of ``format_data_test`` :106-117, ``update_data`` :239-252, ``forward_multiple_pass``
:301-312, test cycles from ``test_cfg['cycles']``) as ``render`` / ``refine`` when a
``renderer`` config is given (the HIP renderer, scflow_amd/renderer.py).  Data loading /
pre-processing stay the reference's; the loss configuration arguments are accepted and the
losses live in ``scflow_amd.train``.

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
        self.test_cycle_num = self.test_cfg.get("cycles", 1)
        self.renderer = None
        if renderer is not None:
            from .renderer import Renderer
            self.renderer = renderer if isinstance(renderer, Renderer) else Renderer(**renderer)
        # scflow_refiner.py:58-61.  The flags are kept and re-applied by train(): the reference
        # applies them once in __init__, so mmengine's later model.train() puts its BatchNorms
        # back in train mode; here a frozen module stays frozen (requires_grad=False persists
        # in both).
        self.freeze_bn_flag, self.freeze_encoder_flag = bool(freeze_bn), bool(freeze_encoder)
        if freeze_bn:
            self.freeze_bn()
        if freeze_encoder:
            self.freeze_encoder()

    def freeze_encoder(self) -> None:
        """scflow_refiner.py:65-73: the feature encoders (real and rendered; one module when
        shared) in eval mode with requires_grad=False.  The context encoder stays trainable."""
        self.freeze_encoder_flag = True
        for enc in (self.real_encoder, self.render_encoder):
            for m in enc.modules():
                m.eval()
                for p in m.parameters():
                    p.requires_grad = False

    def freeze_bn(self) -> None:
        """scflow_refiner.py:75-78: every BatchNorm2d in eval mode (running statistics, no
        update); its affine parameters stay trainable."""
        self.freeze_bn_flag = True
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eval()

    def train(self, mode: bool = True):
        super().train(mode)
        if mode and self.freeze_bn_flag:
            self.freeze_bn()
        if mode and self.freeze_encoder_flag:
            for enc in (self.real_encoder, self.render_encoder):
                enc.eval()
        return self

    def to(self, *args, **kwargs):  # base_refiner.py:69-72: the renderer's meshes move too
        if self.renderer is not None:
            dev = args[0] if args else kwargs.get("device")
            if dev is not None and not isinstance(dev, torch.dtype):
                self.renderer.to(dev)
        return super().to(*args, **kwargs)

    def cuda(self, device=None):
        if self.renderer is not None:
            self.renderer.to("cuda" if device is None else torch.device("cuda", device))
        return super().cuda(device)

    # ------------------------------------------------------------------ renderer-driven loop
    def render(self, rotations: Tensor, translations: Tensor, internel_k: Tensor, labels: Tensor,
               norm_mean=(0.0, 0.0, 0.0), norm_std=(255.0, 255.0, 255.0)):
        """format_data_test's render step (base_refiner.py:106-117): rendered images (RGB,
        normalised with img_norm_cfg /255 — mean 0 / std 255 in the config, i.e. identity),
        rendered depth (zbuf), rendered masks (depth > 0)."""
        if self.renderer is None:
            raise RuntimeError("SCFlowRefiner was built without a renderer config")
        out = self.renderer(rotations, translations, internel_k, labels)
        img = out["images"][..., :3].permute(0, 3, 1, 2).contiguous()
        mean = torch.tensor(norm_mean, device=img.device).view(1, 3, 1, 1) / 255.0
        std = torch.tensor(norm_std, device=img.device).view(1, 3, 1, 1) / 255.0
        img = (img - mean) / std
        depth = out["fragments"].zbuf[..., 0]
        return img, depth, (depth > 0).float()

    def refine(self, real_images: Tensor, ref_rotations: Tensor, ref_translations: Tensor,
               internel_k: Tensor, labels: Tensor, cycles: Optional[int] = None):
        """Test-time refinement (base_refiner.py:301-312 + scflow_refiner.py:142-177): for each
        cycle render the current pose, run ``get_pose`` with ``test_cfg['iters']`` iterations and
        take the last pose; returns (rotations, translations, last get_pose outputs)."""
        cycles = self.test_cycle_num if cycles is None else cycles
        R, t = ref_rotations, ref_translations
        iters = self.decoder.iters
        self.decoder.iters = self.test_iter_num
        try:
            for _ in range(cycles):
                img, depth, _ = self.render(R, t, internel_k, labels)
                out = self.get_pose(img, real_images, R, t, depth, internel_k, labels)
                R, t = out[2][-1], out[3][-1]
        finally:
            self.decoder.iters = iters
        return R, t, out

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
                 init_flow: Optional[Tensor] = None, head_label: Optional[Tensor] = None):
        """scflow_refiner.py:108-138 — images → encoders → SCFlowDecoder outputs (7 lists)."""
        if render_images.device.type != "cuda":
            raise ScflowError("SCFlowRefiner runs on the gfx950 HIP kernels only (no CPU fallback)")
        with torch.no_grad():
            return self._get_pose(render_images.contiguous().float(), real_images.contiguous().float(),
                                  ref_rotation, ref_translation, depth, internel_k, label, init_flow,
                                  head_label)

    def forward(self, *args, **kwargs):
        return self.get_pose(*args, **kwargs)

    # ------------------------------------------------------------------ fused path
    def _get_pose(self, render, real, R, t, depth, K, label, init_flow, head_label=None):
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
                            K, label, init_flow, 0.0, hx=hx, head_label=head_label)
