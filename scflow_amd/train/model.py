"""Training forward of SCFlowRefiner on the HIP autograd Functions.

``refiner_train_forward`` reproduces ``SCFlowRefiner.loss`` (models/refiner/scflow_refiner.py:
182-256) for synthetic batches: shared feature encoder on real + rendered images, context
encoder (BatchNorm in train mode), the decoder loop with the configured detaches
(detach_flow / detach_pose / detach_depth_for_xy, scflow_decoder.py:193-236) and back-prop
through the 8 GRU steps, then the three sequence losses.  Activations are channels-last; every
convolution is ``conv2d_nhwc`` (HIP forward + backward); the correlation pyramid and lookup are
HIP Functions; the detached per-iteration geometry (2D-3D lift, pose-induced flow, flow
downsampling, GT flow) runs on the inference kernels without autograd.  Normalisations,
activations, the GRU gate algebra, the pose update and the losses are torch ops (pointwise /
per-sample); FCs are plain library GEMMs.
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import Chan
from .functions import (ResidualGrad, batch_norm_nhwc, begin_forward, bn_fusable, conv2d_nhwc,
                        conv2d_nhwc_split, corr_lookup, corr_pyramid, dual_conv2d_nhwc,
                        group_norm_nhwc, gru_step, instance_norm_nhwc,
                        instance_norm_residual_relu_nhwc, linear, pose_update6, share_weight,
                        upsample_bilinear_ac)
from .losses import LowRes, filter_flow_by_mask, matmul3, refine_losses

Tensor = torch.Tensor
_GRU_FUSED = os.environ.get("SCFLOW_TRAIN_GRU_FUSED", "1") != "0"  # A/B switch (tuning)
_FUSED_LOSS = os.environ.get("SCFLOW_TRAIN_FUSED_LOSS", "1") != "0"  # A/B switch (tuning)
_GN_FUSED = os.environ.get("SCFLOW_TRAIN_GN_FUSED", "1") != "0"  # A/B switch (tuning)
_RES_GRAD = os.environ.get("SCFLOW_TRAIN_RES_GRAD", "1") != "0"  # A/B switch (tuning)
_BN_FUSED = os.environ.get("SCFLOW_TRAIN_BN_FUSED", "1") != "0"  # A/B switch (tuning)
_HEADS_FUSED = os.environ.get("SCFLOW_TRAIN_HEADS_FUSED", "1") != "0"  # A/B switch (tuning)


def _act(x: Tensor, act) -> Tensor:
    if act == "ReLU":
        return torch.relu(x)
    if act == "Sigmoid":
        return torch.sigmoid(x)
    if act == "Tanh":
        return torch.tanh(x)
    return x


def _cm(x: Tensor, m, x1: Tensor = None) -> Tensor:
    """mmcv ConvModule (conv → act, fused; the decoder's ConvModules have no norm); ``x1``: a
    second input concatenated along channels (read in place)."""
    c = m.conv
    return conv2d_nhwc(x, c.weight, c.bias, c.stride[0], c.padding, act=m.act_type, x1=x1)


def _conv(x: Tensor, c, res_grad=None) -> Tensor:
    if res_grad is None:
        return conv2d_nhwc(x, c.weight, c.bias, c.stride[0], c.padding)
    return conv2d_nhwc(x, c.weight, c.bias, c.stride[0], c.padding, res_grad=res_grad)


# ------------------------------------------------------------------------------- encoders
def _norm(x: Tensor, mod, relu: bool = False) -> Tensor:
    """InstanceNorm2d (affine=False; HIP statistics / apply / backward, the ReLU fused) or
    BatchNorm2d (train mode: batch statistics, running-stat update) on a channels-last tensor."""
    if isinstance(mod, torch.nn.InstanceNorm2d):
        c = x.shape[-1]
        if x.is_cuda and c % 4 == 0 and c <= 256 and not mod.affine:
            return instance_norm_nhwc(x, mod.eps, relu)
        m = x.mean(dim=(1, 2), keepdim=True)
        v = x.var(dim=(1, 2), unbiased=False, keepdim=True)
        y = (x - m) / torch.sqrt(v + mod.eps)
        return torch.relu(y) if relu else y
    if _BN_FUSED and bn_fusable(mod, x):
        return batch_norm_nhwc(x, mod, relu)
    y = F.batch_norm(x.permute(0, 3, 1, 2), mod.running_mean, mod.running_var, mod.weight, mod.bias,
                     training=mod.training, momentum=mod.momentum, eps=mod.eps)
    if mod.training and mod.num_batches_tracked is not None:
        mod.num_batches_tracked.add_(1)
    y = y.permute(0, 2, 3, 1)
    return torch.relu(y) if relu else y


def encoder_train(enc, x_nhwc: Tensor) -> Tensor:
    """RAFTEncoder.forward (raft_encoder.py:286-314) with autograd; channels-last in and out."""
    x = _norm(_conv(x_nhwc, enc.conv1), enc.norm1, relu=True)
    for name in enc.res_layers:
        for blk in getattr(enc, name):
            n2 = blk.norm2
            in_tail = (isinstance(n2, torch.nn.InstanceNorm2d) and not n2.affine and x.is_cuda
                       and x.shape[-1] % 4 == 0 and x.shape[-1] <= 256)
            bn_tail = _BN_FUSED and bn_fusable(n2, x)
            fused_tail = in_tail or bn_tail
            # identity block: its input's two gradients (conv1's dX, the identity) summed in
            # conv1's dX epilogue (ResidualGrad)
            rg = ResidualGrad() if (fused_tail and blk.downsample is None and _RES_GRAD and
                                    blk.conv1.stride[0] == 1) else None
            out = _norm(_conv(x, blk.conv1, rg), blk.norm1, relu=True)
            ident = x if blk.downsample is None else _norm(_conv(x, blk.downsample[0]), blk.downsample[1])
            y2 = _conv(out, blk.conv2)
            if fused_tail and y2.shape[-1] % 4 == 0 and y2.shape[-1] <= 256 and ident.shape == y2.shape:
                if in_tail:
                    x = instance_norm_residual_relu_nhwc(y2, ident, n2.eps, rg)  # norm + sum + ReLU
                else:
                    x = batch_norm_nhwc(y2, n2, res=ident, res_grad=rg)
            else:
                x = torch.relu(_norm(y2, n2) + ident)
    return _conv(x, enc.conv2)


# ------------------------------------------------------------------------------- pose head
def pose_head_train(head, x: Tensor, label: Tensor) -> Tuple[Tensor, Tensor]:
    """MultiClassPoseHead.forward (pose_head.py:201-211), label[0] quirk kept."""
    for m in head.conv_layers:
        c = m.conv
        y = conv2d_nhwc(x, c.weight, c.bias, c.stride[0], c.padding)
        gn = m.gn
        if y.is_cuda and _GN_FUSED and gn.affine and y.shape[-1] == 4 * gn.num_groups:
            x = group_norm_nhwc(y, gn.weight, gn.bias, gn.num_groups, gn.eps, relu=True)
            continue
        y = F.group_norm(y.permute(0, 3, 1, 2), gn.num_groups, gn.weight, gn.bias, gn.eps)
        x = torch.relu(y).permute(0, 2, 3, 1)
    v = x.permute(0, 3, 1, 2).reshape(x.shape[0], -1)  # nn.Flatten of NCHW
    for fc in head.fc_layers:
        v = torch.relu(linear(v, fc[0].weight, fc[0].bias))
    n = v.shape[0]
    t = linear(v, head.translation_pred.weight, head.translation_pred.bias).view(n, head.num_class, 3)
    r = linear(v, head.rotation_pred.weight, head.rotation_pred.bias).view(
        n, head.num_class, head.rotation_out_channels)
    # index_select(dim=1, index=label)[:, 0]: every sample takes class label[0] (the quirk), as a
    # gather whose backward is a plain scatter-add (index_select's index_add backward: ~48 µs)
    lab = label[:1].view(1, 1, 1)
    t = t.gather(1, lab.expand(n, 1, 3))[:, 0]
    r = r.gather(1, lab.expand(n, 1, r.shape[-1]))[:, 0]
    return r, t


# ------------------------------------------------------------------------------- pose maths
def _normalize(v: Tensor) -> Tensor:
    return v / v.norm(dim=1, keepdim=True).clamp_min(1e-12)


def pose_update(drot: Tensor, dt: Tensor, R: Tensor, t: Tensor, weight: float = 10.0,
                depth_transform: str = "exp", detach_depth_for_xy: bool = True) -> Tuple[Tensor, Tensor]:
    """get_pose_from_delta_pose + get_rotation_matrix_from_ortho6d (pose.py:124-169); a [n, 4]
    drot is a quaternion (x, y, z, w; pose.py:132-133, see oracle.rotation_from_quaternion_xyzw)."""
    if drot.shape[1] == 6 and drot.is_cuda and depth_transform in ("exp", "linear"):
        return pose_update6(drot, dt, R, t, weight, depth_transform == "exp", detach_depth_for_xy)
    if drot.shape[1] == 4:
        q = drot / drot.norm(dim=1, keepdim=True).clamp_min(1e-12)
        qx, qy, qz, qw = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
        tx, ty, tz = 2.0 * qx, 2.0 * qy, 2.0 * qz
        one = torch.ones_like(qx)
        D = torch.stack([one - (ty * qy + tz * qz), ty * qx - tz * qw, tz * qx + ty * qw,
                         ty * qx + tz * qw, one - (tx * qx + tz * qz), tz * qy - tx * qw,
                         tz * qx - ty * qw, tz * qy + tx * qw, one - (tx * qx + ty * qy)],
                        dim=-1).view(-1, 3, 3)
        Rd = matmul3(D, R)
    else:
        x = _normalize(drot[:, 0:3])
        z = _normalize(torch.cross(x, drot[:, 3:6], dim=1))
        y = torch.cross(z, x, dim=1)
        Rd = matmul3(torch.stack([x, y, z], dim=2), R)
    vz = t[:, 2] / torch.exp(dt[:, 2]) if depth_transform == "exp" else t[:, 2] * (dt[:, 2] + 1)
    vzxy = vz.detach() if detach_depth_for_xy else vz
    vx = vzxy * (dt[:, 0] / weight + t[:, 0] / t[:, 2])
    vy = vzxy * (dt[:, 1] / weight + t[:, 1] / t[:, 2])
    return Rd, torch.stack([vx, vy, vz], dim=-1)


# ------------------------------------------------------------------------------- decoder
def decoder_train(dec, feat_render: Tensor, feat_real: Tensor, h: Tensor, cxt: Tensor, R0: Tensor,
                  t0: Tensor, depth: Tensor, K: Tensor, label: Tensor, iters: int,
                  invalid_flow_num: float = 0.0) -> Tuple[List[Tensor], ...]:
    """SCFlowDecoder.forward with autograd (scflow_decoder.py:151-252); features channels-last
    [N, h, w, C].  Returns (flow_from_pose, flow_from_pred, R, t, mask, Δrot, Δt) lists."""
    if not dec.detach_flow or dec.mask_flow or dec.mask_corr:
        raise NotImplementedError("training path follows the configured decoder: detach_flow=True, "
                                  "mask_flow=mask_corr=False (scflow_ycbv_real.py:213-218)")
    N, hh, ww, _ = feat_render.shape
    _, H, W = depth.shape
    dt = feat_render.dtype
    L, r = dec.num_levels, dec.radius
    scale = 2 ** (L - 1)
    pyr = corr_pyramid(feat_render.permute(0, 3, 1, 2), feat_real.permute(0, 3, 1, 2), L)
    depth = depth.contiguous().to(dt)
    K = K.contiguous().to(dt)
    with torch.no_grad():
        points = ops.lift_points(depth, K, R0.contiguous().to(dt), t0.contiguous().to(dt))
    flow_full = torch.zeros(N, 2, H, W, device=depth.device, dtype=dt)
    R, t = R0.to(dt), t0.to(dt)
    label = label.long()
    outs = ([], [], [], [], [], [], [])
    enc = dec.encoder
    gru = dec.gru
    hc, cc = dec.h_channels, dec.cxt_channels
    # loop-invariant context contribution of every GRU conv, once per forward (its gradient is
    # the sum over the iterations, so dgrad/wgrad of the context part also run once)
    it_w, ctx_pre = [], []
    for zc, rc, qc in zip(gru.conv_z, gru.conv_r, gru.conv_q):
        z, rr, q = zc.conv, rc.conv, qc.conv
        wzr = torch.cat([z.weight, rr.weight], 0)
        bzr = torch.cat([z.bias, rr.bias], 0)
        ctx_pre.append((conv2d_nhwc(cxt, wzr[:, hc:hc + cc], bzr, 1, q.padding),
                        conv2d_nhwc(cxt, q.weight[:, hc:hc + cc], q.bias, 1, q.padding)))
        w_zr = torch.cat([wzr[:, :hc], wzr[:, hc + cc:]], 1)
        w_q = torch.cat([q.weight[:, :hc], q.weight[:, hc + cc:]], 1)
        if _GRU_FUSED:  # one batched weight gradient over the 8 iterations' uses
            w_zr, w_q = share_weight(w_zr), share_weight(w_q)
        it_w.append((w_zr, w_q, q.padding))
    fl, ml = dec.flow_pred.layers, dec.mask_pred.layers
    heads_fused = (_HEADS_FUSED and len(fl) == 1 and len(ml) == 1 and h.is_cuda
                   and fl[0].conv.kernel_size == ml[0].conv.kernel_size
                   and fl[0].conv.padding == ml[0].conv.padding and fl[0].conv.stride == (1, 1)
                   and ml[0].conv.stride == (1, 1) and fl[0].act_type == ml[0].act_type
                   and (fl[0].conv.bias is None) == (ml[0].conv.bias is None))
    for _ in range(iters):
        with torch.no_grad():  # flow is detached every iteration (detach_flow=True)
            f2 = torch.empty(N * hh * ww, 2, device=depth.device, dtype=dt)
            ops.flow_downsample(flow_full.contiguous(), Chan.whole(f2), hh, ww, 1.0 / scale)
        f2 = f2.view(N, hh, ww, 2)
        corr = corr_lookup(pyr, f2, N, hh, ww, L, r)
        c = corr
        for m in enc.corr_net:
            c = _cm(c, m)
        f = f2
        for m in enc.flow_net:
            f = _cm(f, m)
        out = _cm(c, enc.out_net[0], x1=f)
        for m in enc.out_net[1:]:
            out = _cm(out, m)
        motion = torch.cat([out, f2], -1)
        for (w_zr, w_q, pad), (pre_zr, pre_q) in zip(it_w, ctx_pre):  # SeqConv: 1×5 then 5×1
            if _GRU_FUSED:
                h = gru_step(h, motion, w_zr, w_q, pre_zr, pre_q, pad)  # (1 − z)·h + z·q
            else:  # the same step as separate autograd ops (A/B reference)
                z, rg = conv2d_nhwc_split(h, w_zr, hc, None, 1, pad, act="Sigmoid", x1=motion,
                                          bias_map=pre_zr)
                qq = conv2d_nhwc(rg * h, w_q, None, 1, pad, act="Tanh", x1=motion, bias_map=pre_q)
                h = torch.lerp(h, qq, z)
        fl, ml = dec.flow_pred.layers, dec.mask_pred.layers
        if heads_fused:  # both XHeads' hidden convs as one launch each way
            fh, mh = dual_conv2d_nhwc(h, fl[0].conv.weight, fl[0].conv.bias, ml[0].conv.weight,
                                      ml[0].conv.bias, fl[0].conv.padding, fl[0].act_type)
        else:
            fh = h
            for m in fl:
                fh = _cm(fh, m)
            mh = h
            for m in ml:
                mh = _cm(mh, m)
        dflow = _conv(fh, dec.flow_pred.predict_layer)
        pl = dec.mask_pred.predict_layer
        mask = conv2d_nhwc(mh, pl.weight, pl.bias, 1, pl.padding, act="Sigmoid")
        dff = dflow
        for m in dec.delta_flow_encoder:
            dff = _cm(dff, m)
        mf = mask
        for m in dec.mask_encoder:
            mf = _cm(mf, m)
        drot, dtr = pose_head_train(dec.pose_pred, torch.cat([h, dff, mf], -1), label)
        if depth.is_cuda and _FUSED_LOSS:  # the losses upsample inside their fused kernel
            flow_pred = LowRes(f2 + dflow, float(scale))
            up_mask = LowRes(mask, 1.0)
        else:
            flow_pred = scale * upsample_bilinear_ac((f2 + dflow).permute(0, 3, 1, 2), scale)
            up_mask = upsample_bilinear_ac(mask.permute(0, 3, 1, 2), scale)
        if dec.detach_pose:
            R, t = R.detach(), t.detach()
        R, t = pose_update(drot, dtr, R, t, depth_transform=dec.depth_transform,
                           detach_depth_for_xy=dec.detach_depth_for_xy)
        with torch.no_grad():
            flow_full = torch.empty(N, 2, H, W, device=depth.device, dtype=dt)
            ops.pose_flow(R.detach().contiguous(), t.detach().contiguous(), K, points,
                          float(invalid_flow_num), out=flow_full)
        for lst, v in zip(outs, (flow_full, flow_pred, R, t, up_mask, drot, dtr)):
            lst.append(v)
    return outs


def refiner_train_forward(refiner, batch: Dict[str, Tensor], model_points: Sequence[Tensor],
                          diameters: Sequence[float], iters: int = None) -> Dict[str, Tensor]:
    """Images → losses (SCFlowRefiner.loss), autograd graph attached.  ``batch`` keys:
    render_images, real_images [N,3,S,S]; ref_rotation, ref_translation, gt_rotation,
    gt_translation, internel_k, depth, label; optional head_label (the pose head's class label,
    default label — a data-parallel shard passes the global batch's label[:1], dist.shard_batch)."""
    begin_forward()  # per-weight use counts of this pass (batched weight gradients)
    dec = refiner.decoder
    iters = int(dec.iters if iters is None else iters)
    real = batch["real_images"].permute(0, 2, 3, 1).contiguous()
    render = batch["render_images"].permute(0, 2, 3, 1).contiguous()
    N = real.shape[0]
    dt = real.dtype
    if refiner.real_encoder is refiner.render_encoder:  # shared: one batch of 2N images
        feats = encoder_train(refiner.real_encoder, torch.cat([real, render], 0))
        feat_real, feat_render = feats[:N], feats[N:]
    else:
        feat_real = encoder_train(refiner.real_encoder, real)
        feat_render = encoder_train(refiner.render_encoder, render)
    cx = encoder_train(refiner.context, render)
    hc = refiner.h_channels
    h, cxt = torch.tanh(cx[..., :hc]), torch.relu(cx[..., hc:])
    outs = decoder_train(dec, feat_render, feat_real, h, cxt, batch["ref_rotation"],
                         batch["ref_translation"], batch["depth"], batch["internel_k"],
                         batch.get("head_label", batch["label"]), iters)
    with torch.no_grad():  # GT flow: lift with the reference pose, project with the GT pose
        depth = batch["depth"].contiguous().to(dt)
        K = batch["internel_k"].contiguous().to(dt)
        pts = ops.lift_points(depth, K, batch["ref_rotation"].contiguous().to(dt),
                              batch["ref_translation"].contiguous().to(dt))
        gt_flow = torch.empty(N, 2, *depth.shape[1:], device=depth.device, dtype=dt)
        ops.pose_flow(batch["gt_rotation"].contiguous().to(dt), batch["gt_translation"].contiguous().to(dt),
                      K, pts, refiner.max_flow, out=gt_flow)
        if refiner.filter_invalid_flow and "gt_masks" in batch:
            gt_flow = filter_flow_by_mask(gt_flow, batch["gt_masks"], refiner.max_flow)
        render_mask = (depth > 0).to(dt)
    lp, lf, lm = refine_losses(outs, batch["gt_rotation"].to(dt), batch["gt_translation"].to(dt),
                               gt_flow, render_mask, batch["label"], model_points, diameters,
                               refiner.max_flow)
    return dict(loss=lp + lf + lm, loss_pose=lp, loss_flow=lf, loss_mask=lm, outs=outs, gt_flow=gt_flow)
