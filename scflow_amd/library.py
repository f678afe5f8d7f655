"""The hot-path HIP ops as ``torch.library`` custom ops ("called from the build's
SCFlowDecoder through torch.library.custom_op wrappers").

Registered under the ``scflow`` namespace, each with a fake (meta) implementation so FX tracing,
``torch.compile`` and ``torch.library.opcheck`` see through them, and the two differentiable
ones with their HIP adjoints (``register_autograd``):

=============================  =====================================================  =========
op                             reference                                              backward
=============================  =====================================================  =========
``scflow::corr_pyramid``       CorrelationPyramid.forward, raft_decoder.py:35-58      yes
``scflow::corr_lookup``        CorrLookup.forward, corr_lookup.py:102-136             pyramid
``scflow::pose_update_flow``   get_pose_from_delta_pose + get_flow_from_delta_pose_   no (the
                               and_points, pose.py:66-88,124-169                      decoder
                                                                                      detaches)
=============================  =====================================================  =========

The two backward formulas are ops of their own (``scflow::corr_pyramid_backward``,
``scflow::corr_lookup_backward``), so AOT autograd traces the backward graph as well.

The pyramid travels as ONE flat fp32 buffer (levels back to back, each ``[N·H·W, 1, H_l, W_l]``
row-major — ``ops.pyramid_views`` turns it into the reference's list); the modules
``CorrelationPyramid`` / ``CorrLookup`` (modules.py) call these ops.  Every op runs the HIP
kernel on the inputs' current stream; there is no CPU implementation (the product path fails
loudly off-GPU, ``ScflowError``).
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import ops

Tensor = torch.Tensor


def pyramid_numel(n: int, h: int, w: int, num_levels: int) -> int:
    """Elements of the flat pyramid buffer: N·H·W maps per level of (H>>l)·(W>>l)."""
    return n * h * w * sum((h >> l) * (w >> l) for l in range(num_levels))


# ------------------------------------------------------------------------------------ a1
@torch.library.custom_op("scflow::corr_pyramid", mutates_args=(), device_types="cuda")
def corr_pyramid(feat1: Tensor, feat2: Tensor, num_levels: int) -> Tensor:
    """feat1, feat2 [N, C, H, W] fp32 → flat pyramid buffer (level 0 = f1ᵀf2/√C, levels 1.. =
    AvgPool2d(2, 2) over the target dims)."""
    buf, _ = ops.corr_pyramid(feat1.contiguous(), feat2.contiguous(), num_levels)
    return buf


@corr_pyramid.register_fake
def _(feat1, feat2, num_levels):
    n, _, h, w = feat1.shape
    return feat1.new_empty(pyramid_numel(n, h, w, num_levels))


def _corr_pyramid_setup(ctx, inputs, output):
    feat1, feat2, num_levels = inputs
    ctx.save_for_backward(feat1, feat2)
    ctx.num_levels = num_levels


@torch.library.custom_op("scflow::corr_pyramid_backward", mutates_args=(), device_types="cuda")
def corr_pyramid_backward(dbuf: Tensor, feat1: Tensor, feat2: Tensor, num_levels: int
                          ) -> Tuple[Tensor, Tensor]:
    """AvgPool adjoint down the levels, then dF1 = F2·dCᵀ, dF2 = F1·dC on the HIP GEMM (the
    training step's adjoint, train/functions.py _CorrPyramid)."""
    n, c, h, w = feat1.shape
    P = h * w
    levels = ops.pyramid_views(dbuf.contiguous(), n, h, w, num_levels)
    g = levels[-1]
    for lv in reversed(levels[:-1]):
        hl, wl = lv.shape[-2:]
        up = torch.zeros_like(lv)
        up[..., : (hl // 2) * 2, : (wl // 2) * 2] = \
            g.repeat_interleave(2, -2).repeat_interleave(2, -1) * 0.25
        g = lv + up
    dC = g.reshape(n, P, P) / (c ** 0.5)
    f1 = feat1.contiguous().view(n, c, P)
    f2 = feat2.contiguous().view(n, c, P)
    df1 = ops.gemm(f2, dC.transpose(1, 2)).view_as(feat1)
    df2 = ops.gemm(f1, dC).view_as(feat2)
    return df1, df2


@corr_pyramid_backward.register_fake
def _(dbuf, feat1, feat2, num_levels):
    return torch.empty_like(feat1, memory_format=torch.contiguous_format), \
        torch.empty_like(feat2, memory_format=torch.contiguous_format)


def _corr_pyramid_backward(ctx, dbuf):
    feat1, feat2 = ctx.saved_tensors
    df1, df2 = corr_pyramid_backward(dbuf, feat1, feat2, ctx.num_levels)
    return df1, df2, None


corr_pyramid.register_autograd(_corr_pyramid_backward, setup_context=_corr_pyramid_setup)


# ------------------------------------------------------------------------------------ a2
@torch.library.custom_op("scflow::corr_lookup", mutates_args=(), device_types="cuda")
def corr_lookup(pyramid: Tensor, flow: Tensor, num_levels: int, radius: int,
                align_corners: bool) -> Tensor:
    """pyramid (flat buffer of ``corr_pyramid``), flow [B, 2, H, W] → [B, L·(2r+1)², H, W]."""
    B, _, H, W = flow.shape
    return ops.corr_lookup(pyramid.contiguous(), flow.contiguous(), B, H, W, num_levels, radius,
                           align_corners=align_corners)


@corr_lookup.register_fake
def _(pyramid, flow, num_levels, radius, align_corners):
    B, _, H, W = flow.shape
    return flow.new_empty(B, num_levels * (2 * radius + 1) ** 2, H, W)


def _corr_lookup_setup(ctx, inputs, output):
    pyramid, flow, num_levels, radius, align_corners = inputs
    ctx.save_for_backward(flow)
    ctx.cfg = (pyramid.numel(), num_levels, radius, align_corners)


@torch.library.custom_op("scflow::corr_lookup_backward", mutates_args=(), device_types="cuda")
def corr_lookup_backward(dout: Tensor, flow: Tensor, numel: int, num_levels: int, radius: int
                         ) -> Tensor:
    """Gradient w.r.t. the pyramid only (the decoder detaches the flow, scflow_decoder.py:193-194):
    the adjoint scatter with grid_sample's tap weights (scflow_corr_lookup_backward,
    align_corners=True)."""
    B, _, H, W = flow.shape
    dpyr = torch.zeros(numel, device=dout.device, dtype=torch.float32)
    # channels-last gradient and flow: the layouts of the training step's lookup backward
    ops.corr_lookup_backward(dout.permute(0, 2, 3, 1).contiguous().view(B * H * W, -1),
                             flow.permute(0, 2, 3, 1).contiguous(), dpyr, B, H, W, num_levels,
                             radius)
    return dpyr


@corr_lookup_backward.register_fake
def _(dout, flow, numel, num_levels, radius):
    return dout.new_empty(numel)


def _corr_lookup_backward(ctx, dout):
    (flow,) = ctx.saved_tensors
    numel, L, r, ac = ctx.cfg
    if not ac:
        raise NotImplementedError("scflow::corr_lookup backward: align_corners=True only "
                                  "(SCFlow's configuration)")
    if ctx.needs_input_grad[1]:
        # grid_sample would also give the sampling coordinates a gradient (corr_lookup.py:
        # 102-136); every SCFlow caller detaches the flow first (scflow_decoder.py:193-194), and a
        # silent zero gradient would be wrong, so an attached flow is an error
        raise NotImplementedError("scflow::corr_lookup backward: no gradient w.r.t. flow — "
                                  "detach the flow (as SCFlowDecoder does)")
    return corr_lookup_backward(dout, flow, numel, L, r), None, None, None, None


corr_lookup.register_autograd(_corr_lookup_backward, setup_context=_corr_lookup_setup)


# ------------------------------------------------------------------------------------ a8 + a10
@torch.library.custom_op("scflow::pose_update_flow", mutates_args=(), device_types="cuda")
def pose_update_flow(drot: Tensor, dt: Tensor, R: Tensor, t: Tensor, K: Tensor, points: Tensor,
                     invalid_num: float, weight: float, depth_transform: str
                     ) -> Tuple[Tensor, Tensor, Tensor]:
    """Δpose (ortho6d [n, 6] or quaternion [n, 4], Δt [n, 3]) applied to (R, t) → (R', t') and
    the pose-induced flow [n, 2, H, W] of the lifted object points [n, H, W, 4] under K."""
    n, H, W, _ = points.shape
    R_out, t_out = torch.empty_like(R), torch.empty_like(t)
    flow = torch.empty(n, 2, H, W, device=R.device, dtype=torch.float32)
    ops.pose_update_flow(drot.contiguous(), dt.contiguous(), R.contiguous(), t.contiguous(),
                         K.contiguous(), points.contiguous(), R_out, t_out, flow, invalid_num,
                         weight, depth_transform)
    return R_out, t_out, flow


@pose_update_flow.register_fake
def _(drot, dt, R, t, K, points, invalid_num, weight, depth_transform):
    n, H, W, _ = points.shape
    return torch.empty_like(R), torch.empty_like(t), R.new_empty(n, 2, H, W)
