"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

CPU restatement (PyTorch on CPU, float32 or float64) of SCFlow's recurrent correlation-flow
hot path, written from the reference's behaviour, function by function, each citing the
reference ``/root/reference/<file>:<line>`` it follows.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module,
and only as the checker / CPU baseline.

Parity pinning: the restatement is checked against golden vectors produced by running the
reference's own modules (``tests/golden/make_golden.py``, fixtures in ``tests/golden/*.npz``;
see ``tests/test_oracle_golden.py``).  The reference ships no tests of its own
(SURVEY.md §4), so those generated fixtures are the pin.

Parameters are passed as a flat state dict whose keys are exactly the reference
``SCFlowDecoder`` state-dict keys (SURVEY.md §8(b) "Weights / state dict").

Where the reference calls a torch primitive that *is* the definition of the operation
(``F.conv2d``, ``torch.matmul``, ``nn.AvgPool2d``, ``F.interpolate``, ``F.group_norm``,
``F.linear``), the oracle calls it too.  The index-heavy parts — the pyramid lookup
(grid_sample with the normalise/unnormalise round trip), the 2D-3D lift and the
reprojection scatter — are restated explicitly and densely (no ``nonzero``/Python loop over
samples) so they check the HIP kernels' index maths independently.
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
StateDict = Dict[str, Tensor]


# ---------------------------------------------------------------------------------------------
# a1 — correlation pyramid (models/decoder/raft_decoder.py:35-58)
# ---------------------------------------------------------------------------------------------
def corr_pyramid(feat1: Tensor, feat2: Tensor, num_levels: int = 4) -> List[Tensor]:
    """``corr = (f1ᵀ f2)/√C`` as ``[N·H·W,1,H,W]`` then AvgPool2d(2,2) per level.

    raft_decoder.py:47-52 (matmul + /sqrt(tensor(C).float())), :53-57 (pooling of the previous
    level, kernel 2 stride 2, floor for odd sizes).
    """
    N, C, H, W = feat1.shape
    corr = torch.matmul(feat1.reshape(N, C, H * W).permute(0, 2, 1), feat2.reshape(N, C, H * W))
    corr = corr.reshape(N * H * W, 1, H, W) / torch.sqrt(torch.tensor(C, dtype=feat1.dtype))
    pyr = [corr]
    for _ in range(num_levels - 1):
        pyr.append(F.avg_pool2d(pyr[-1], kernel_size=2, stride=2))
    return pyr


# ---------------------------------------------------------------------------------------------
# a2 — pyramid lookup (models/utils/corr_lookup.py:102-136, bilinear_sample :31-67)
# ---------------------------------------------------------------------------------------------
def _sample_zero_pad(img: Tensor, ix: Tensor, iy: Tensor) -> Tensor:
    """Bilinear sample of img[M,Hl,Wl] at pixel coords ix/iy [M,K]; taps outside → 0.

    The tap weights follow grid_sample's bilinear kernel (nw, ne, sw, se) with zero padding
    (``padding_mode='zeros'``, corr_lookup.py:67 → F.grid_sample).
    """
    M, Hl, Wl = img.shape
    x0 = torch.floor(ix)
    y0 = torch.floor(iy)
    wx1 = ix - x0
    wy1 = iy - y0
    wx0 = 1 - wx1
    wy0 = 1 - wy1
    x0i = x0.long()
    y0i = y0.long()
    flat = img.reshape(M, Hl * Wl)
    out = torch.zeros_like(ix)
    for dy, dx, wgt in ((0, 0, wx0 * wy0), (0, 1, wx1 * wy0), (1, 0, wx0 * wy1), (1, 1, wx1 * wy1)):
        xx = x0i + dx
        yy = y0i + dy
        ok = (xx >= 0) & (xx < Wl) & (yy >= 0) & (yy < Hl)
        idx = (yy.clamp(0, Hl - 1) * Wl + xx.clamp(0, Wl - 1))
        v = torch.gather(flat, 1, idx)
        out = out + torch.where(ok, v * wgt, torch.zeros_like(v))
    return out


def corr_lookup(pyramid: Sequence[Tensor], flow: Tensor, radius: int = 4,
                align_corners: bool = True) -> Tensor:
    """``CorrLookup.forward`` (corr_lookup.py:102-136), zeros padding; ``align_corners`` True
    (SCFlow's config) or False (bilinear_sample's default, corr_lookup.py:35: grid_sample maps back with
    ``((g+1)·W − 1)/2``).

    * grid = pixel coords (x, y) + flow (coords_grid, :11-28; :114-115);
    * level i: centroid = grid / 2**i, window point = centroid + (dy[i'], dx[j']) where
      ``delta = stack(meshgrid(dy, dx), -1)`` (:117-121) — the FIRST grid component (x)
      receives the window's ROW offset.  So output channel ``k = lvl·(2r+1)² + a·(2r+1) + b``
      samples x = cx + (a−r), y = cy + (b−r);
    * bilinear_sample normalises ``g·2/max(W−1,1) − 1`` (:63-64) and grid_sample with
      align_corners=True maps back with ``((g+1)/2)·(W−1)``; that round trip is kept;
    * output ``[B, L·(2r+1)², H, W]`` cast to float (:135-136).
    """
    B, _, H, W = flow.shape
    dt = flow.dtype
    xs = torch.arange(W, dtype=dt).view(1, 1, W)
    ys = torch.arange(H, dtype=dt).view(1, H, 1)
    gx = (xs + flow[:, 0]).reshape(B * H * W, 1)
    gy = (ys + flow[:, 1]).reshape(B * H * W, 1)
    d = torch.arange(-radius, radius + 1, dtype=dt)
    n = 2 * radius + 1
    off_x = d.view(n, 1).expand(n, n).reshape(1, n * n)  # row offset a-r  → x
    off_y = d.view(1, n).expand(n, n).reshape(1, n * n)  # col offset b-r  → y
    outs = []
    for lvl, corr in enumerate(pyramid):
        Hl, Wl = corr.shape[-2:]
        sx = gx / 2 ** lvl + off_x
        sy = gy / 2 ** lvl + off_y
        nx = sx * 2.0 / max(Wl - 1, 1) - 1.0
        ny = sy * 2.0 / max(Hl - 1, 1) - 1.0
        if align_corners:
            ix = (nx + 1) / 2 * (Wl - 1)
            iy = (ny + 1) / 2 * (Hl - 1)
        else:
            ix = ((nx + 1) * Wl - 1) / 2
            iy = ((ny + 1) * Hl - 1) / 2
        outs.append(_sample_zero_pad(corr.reshape(-1, Hl, Wl), ix, iy).reshape(B, H, W, n * n))
    out = torch.cat(outs, dim=-1)
    return out.permute(0, 3, 1, 2).contiguous()


# ---------------------------------------------------------------------------------------------
# mmcv ConvModule semantics used by every conv in the path: conv → (GroupNorm) → activation,
# conv bias present iff there is no norm (mmcv ``bias='auto'``).
# ---------------------------------------------------------------------------------------------
_ACTS = {
    None: lambda x: x,
    "ReLU": torch.relu,
    "Sigmoid": torch.sigmoid,
    "Tanh": torch.tanh,
}


def conv_module(x: Tensor, sd: StateDict, prefix: str, act: str | None = "ReLU",
                stride=1, padding=0, gn_groups: int | None = None) -> Tensor:
    w = sd[prefix + ".conv.weight"]
    b = sd.get(prefix + ".conv.bias")
    y = F.conv2d(x, w.to(x.dtype), None if b is None else b.to(x.dtype), stride=stride,
                 padding=padding)
    if gn_groups is not None:
        y = F.group_norm(y, gn_groups, sd[prefix + ".gn.weight"].to(x.dtype),
                         sd[prefix + ".gn.bias"].to(x.dtype), eps=1e-5)
    return _ACTS[act](y)


# ---------------------------------------------------------------------------------------------
# a3 — MotionEncoder 'Basic' (raft_decoder.py:75-85 tables, :152-166 forward)
# ---------------------------------------------------------------------------------------------
def motion_encoder(sd: StateDict, corr: Tensor, flow: Tensor, act: str | None = "ReLU",
                   prefix: str = "encoder") -> Tensor:
    c = conv_module(corr, sd, f"{prefix}.corr_net.0", act, padding=0)      # 1×1 324→256
    c = conv_module(c, sd, f"{prefix}.corr_net.1", act, padding=1)         # 3×3 256→192
    f = conv_module(flow, sd, f"{prefix}.flow_net.0", act, padding=3)      # 7×7 2→128
    f = conv_module(f, sd, f"{prefix}.flow_net.1", act, padding=1)         # 3×3 128→64
    o = conv_module(torch.cat([c, f], 1), sd, f"{prefix}.out_net.0", act, padding=1)  # 256→126
    return torch.cat([o, flow], 1)


# ---------------------------------------------------------------------------------------------
# a4 — ConvGRU 'SeqConv' (raft_decoder.py:180-181 kernels, :200-221 act, :235-253 forward)
# ---------------------------------------------------------------------------------------------
GRU_KERNELS = {"SeqConv": (((1, 5), (0, 2)), ((5, 1), (2, 0))), "Conv": (((3, 3), (1, 1)),)}


def conv_gru(sd: StateDict, h: Tensor, x: Tensor, net_type: str = "SeqConv",
             prefix: str = "gru") -> Tensor:
    prefix = prefix + "." if prefix else ""
    for i, (_, pad) in enumerate(GRU_KERNELS[net_type]):
        hx = torch.cat([h, x], 1)
        z = conv_module(hx, sd, f"{prefix}conv_z.{i}", "Sigmoid", padding=pad)
        r = conv_module(hx, sd, f"{prefix}conv_r.{i}", "Sigmoid", padding=pad)
        q = conv_module(torch.cat([r * h, x], 1), sd, f"{prefix}conv_q.{i}", "Tanh", padding=pad)
        h = (1 - z) * h + z * q
    return h


# ---------------------------------------------------------------------------------------------
# a5 — XHead (raft_decoder.py:256-294); ConvModule defaults → ReLU after the hidden conv
# ---------------------------------------------------------------------------------------------
def xhead(sd: StateDict, h: Tensor, prefix: str, kind: str) -> Tensor:
    y = conv_module(h, sd, f"{prefix}.layers.0", "ReLU", padding=1)
    pad = 1 if kind == "flow" else 0
    return F.conv2d(y, sd[f"{prefix}.predict_layer.weight"].to(h.dtype),
                    sd[f"{prefix}.predict_layer.bias"].to(h.dtype), padding=pad)


# ---------------------------------------------------------------------------------------------
# a7 — MultiClassPoseHead (models/head/pose_head.py:110-211)
# ---------------------------------------------------------------------------------------------
def pose_head(sd: StateDict, x: Tensor, label: Tensor, num_class: int = 21,
              rot_ch: int = 6, gn_groups: int = 32, prefix: str = "pose_pred") -> Tuple[Tensor, Tensor]:
    for i in range(3):  # 3× [3×3 s2 conv (no bias) + GN(32) + ReLU], pose_head.py:148-160
        x = conv_module(x, sd, f"{prefix}.conv_layers.{i}", "ReLU", stride=2, padding=1,
                        gn_groups=gn_groups)
    x = x.flatten(1)
    for i in range(2):  # FC 2048→1024→256 + ReLU, pose_head.py:163-170
        x = torch.relu(F.linear(x, sd[f"{prefix}.fc_layers.{i}.0.weight"].to(x.dtype),
                                sd[f"{prefix}.fc_layers.{i}.0.bias"].to(x.dtype)))
    t = F.linear(x, sd[f"{prefix}.translation_pred.weight"].to(x.dtype),
                 sd[f"{prefix}.translation_pred.bias"].to(x.dtype))
    r = F.linear(x, sd[f"{prefix}.rotation_pred.weight"].to(x.dtype),
                 sd[f"{prefix}.rotation_pred.bias"].to(x.dtype))
    t = t.view(-1, num_class, 3)
    rot_ch = sd[f"{prefix}.rotation_pred.bias"].numel() // num_class  # 6 ortho6d / 4 quaternion
    r = r.view(-1, num_class, rot_ch)
    idx = label.long()
    ar = torch.arange(x.shape[0])
    # index_select(dim=1, index=label)[:, 0, :] (pose_head.py:208-209): with B>1 labels the
    # reference selects ALL labels for every sample, then keeps entry 0 → label[0] for everyone.
    return r[ar, idx[0].expand_as(ar)], t[ar, idx[0].expand_as(ar)]


# ---------------------------------------------------------------------------------------------
# a8 — pose update (models/utils/pose.py:124-149, ortho6d :153-169)
# ---------------------------------------------------------------------------------------------
def _normalize(v: Tensor, eps: float = 1e-12) -> Tensor:  # F.normalize(p=2, dim=1)
    return v / v.norm(dim=1, keepdim=True).clamp_min(eps)


def rotation_from_ortho6d(o6: Tensor) -> Tensor:
    x = _normalize(o6[:, 0:3])
    z = _normalize(torch.cross(x, o6[:, 3:6], dim=1))
    y = torch.cross(z, x, dim=1)
    return torch.stack([x, y, z], dim=2)  # columns x, y, z (pose.py:163-169)


def rotation_from_quaternion_xyzw(q: Tensor) -> Tensor:
    """kornia.geometry.conversions.quaternion_to_rotation_matrix (pose.py:132-133; kornia is
    unpinned in requirements.txt and absent here — PARITY UNPINNED: restated from kornia's
    published implementation): q normalised (F.normalize, eps 1e-12), then the unit-quaternion
    matrix.  Coefficient order x, y, z, w: kornia ≤ 0.6's default, and the order the pose
    head's identity bias [0, 0, 0, 1] assumes (pose_head.py:192-194)."""
    q = _normalize(q)
    x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    tx, ty, tz = 2.0 * x, 2.0 * y, 2.0 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    one = torch.ones_like(x)
    return torch.stack([one - (tyy + tzz), txy - twz, txz + twy,
                        txy + twz, one - (txx + tzz), tyz - twx,
                        txz - twy, tyz + twx, one - (txx + tyy)], dim=-1).view(-1, 3, 3)


def pose_update(drot: Tensor, dt: Tensor, R: Tensor, t: Tensor, weight: float = 10.0,
                depth_transform: str = "exp", detach_depth_for_xy: bool = False) -> Tuple[Tensor, Tensor]:
    """get_pose_from_delta_pose (pose.py:124-149); detach_depth_for_xy only changes gradients.
    ``drot`` [n, 6] ortho6d or [n, 4] quaternion (x, y, z, w)."""
    dR = rotation_from_quaternion_xyzw(drot) if drot.shape[1] == 4 else rotation_from_ortho6d(drot)
    Rd = torch.bmm(dR, R)
    if depth_transform == "exp":
        vz = t[:, 2] / torch.exp(dt[:, 2])
    else:
        vz = t[:, 2] * (dt[:, 2] + 1)
    vzxy = vz.detach() if detach_depth_for_xy else vz
    vx = vzxy * (dt[:, 0] / weight + t[:, 0] / t[:, 2])
    vy = vzxy * (dt[:, 1] / weight + t[:, 1] / t[:, 2])
    return Rd, torch.stack([vx, vy, vz], dim=-1)


# ---------------------------------------------------------------------------------------------
# a9 — 2D-3D correspondences, dense form (pose.py:26-64)
# ---------------------------------------------------------------------------------------------
def lift_points(depth: Tensor, K: Tensor, R: Tensor, t: Tensor) -> Tuple[Tensor, Tensor]:
    """Object-frame 3D point for every pixel + validity (depth>0), ``[B,H,W,3]``, ``[B,H,W]``.

    ``P_cam = K⁻¹ [x·d, y·d, d]`` (lift_2d_to_3d :35-37), ``P_obj = R⁻¹ (P_cam − t)`` (:39),
    pixels enumerated by ``nonzero(depth>0)`` (:60) — here all pixels, masked.
    """
    B, H, W = depth.shape
    dt = depth.dtype
    ys, xs = torch.meshgrid(torch.arange(H, dtype=dt), torch.arange(W, dtype=dt), indexing="ij")
    homo = torch.stack([xs.expand(B, H, W), ys.expand(B, H, W), torch.ones(B, H, W, dtype=dt)], -1)
    pc = homo * depth[..., None]
    pc = torch.einsum("bij,bhwj->bhwi", torch.inverse(K.to(dt)), pc)
    po = torch.einsum("bij,bhwj->bhwi", torch.inverse(R.to(dt)), pc - t.to(dt)[:, None, None, :])
    return po, depth > 0


# ---------------------------------------------------------------------------------------------
# a10 — pose-induced flow (pose.py:66-88), dense
# ---------------------------------------------------------------------------------------------
def pose_flow(R: Tensor, t: Tensor, K: Tensor, points: Tensor, valid: Tensor,
              invalid_num: float = 400.0) -> Tensor:
    B, H, W, _ = points.shape
    dt = points.dtype
    cam = torch.einsum("bij,bhwj->bhwi", R.to(dt), points) + t.to(dt)[:, None, None, :]
    uv = torch.einsum("bij,bhwj->bhwi", K.to(dt), cam)
    ys, xs = torch.meshgrid(torch.arange(H, dtype=dt), torch.arange(W, dtype=dt), indexing="ij")
    fx = uv[..., 0] / uv[..., 2] - xs
    fy = uv[..., 1] / uv[..., 2] - ys
    flow = torch.stack([fx, fy], 1)
    return torch.where(valid[:, None], flow, torch.full_like(flow, invalid_num))


def flow_from_delta_pose_and_depth(R_src: Tensor, t_src: Tensor, R_dst: Tensor, t_dst: Tensor,
                                   depth: Tensor, K: Tensor, invalid_num: float = 400.0) -> Tensor:
    """GT flow for training (pose.py:92-121): lift with the source pose, project with dst."""
    pts, valid = lift_points(depth, K, R_src, t_src)
    return pose_flow(R_dst, t_dst, K, pts, valid, invalid_num)


# ---------------------------------------------------------------------------------------------
# a11 — flow resampling (scflow_decoder.py:197-198, :223-228)
# ---------------------------------------------------------------------------------------------
def downsample_flow(flow: Tensor, scale: int) -> Tensor:
    return 1.0 / scale * F.interpolate(flow, scale_factor=(1 / scale, 1 / scale), mode="bilinear",
                                       align_corners=True)


def upsample(x: Tensor, scale: int) -> Tensor:
    return F.interpolate(x, scale_factor=(scale, scale), mode="bilinear", align_corners=True)


# ---------------------------------------------------------------------------------------------
# a12 — SCFlowDecoder.forward (models/decoder/scflow_decoder.py:151-252)
# ---------------------------------------------------------------------------------------------
def decoder_forward(sd: StateDict, feat_render: Tensor, feat_real: Tensor, h_feat: Tensor,
                    cxt_feat: Tensor, ref_rotation: Tensor, ref_translation: Tensor,
                    depth: Tensor, internel_k: Tensor, label: Tensor, init_flow: Tensor,
                    invalid_flow_num: float = 0.0, iters: int = 8, num_levels: int = 4,
                    radius: int = 4, act: str | None = "ReLU", gru_type: str = "SeqConv",
                    num_class: int = 21, depth_transform: str = "exp", mask_flow: bool = False,
                    mask_corr: bool = False, hooks: dict | None = None, train: bool = False,
                    head_label: Tensor | None = None):
    """Returns the reference's 7 lists (scflow_decoder.py:252).  ``head_label``: the labels
    whose first entry picks the pose head's class (default ``label``; the reference's label[0]
    quirk, pose_head.py:208-209) — a data-parallel shard passes the global batch's label[:1].  ``train``: apply the configured
    detaches for autograd (detach_flow / detach_pose / detach_depth_for_xy = True,
    scflow_decoder.py:193-196,231-236; config scflow_ycbv_real.py:211-214) — values unchanged."""
    dt = feat_render.dtype
    sd = {k: v.to(dt) if v.is_floating_point() else v for k, v in sd.items()}
    pyr = corr_pyramid(feat_render, feat_real, num_levels)
    scale = 2 ** (num_levels - 1)
    N, H, W = depth.shape
    points, valid = lift_points(depth.to(dt), internel_k.to(dt), ref_rotation.to(dt),
                                ref_translation.to(dt))
    R, t = ref_rotation.to(dt), ref_translation.to(dt)
    K = internel_k.to(dt)
    mask = F.interpolate(torch.ones(N, 1, H, W, dtype=dt), scale_factor=(1 / scale, 1 / scale),
                         mode="bilinear", align_corners=True)
    flow = init_flow.to(dt)
    h = h_feat
    outs = ([], [], [], [], [], [], [])
    for it in range(iters):
        if train:
            flow = flow.detach()
        flow = downsample_flow(flow, scale)
        corr = corr_lookup(pyr, flow, radius)
        if mask_corr:
            corr = corr * mask
        motion = motion_encoder(sd, corr, flow * mask if mask_flow else flow, act)
        x = torch.cat([cxt_feat, motion], 1)
        h = conv_gru(sd, h, x, gru_type)
        dflow = xhead(sd, h, "flow_pred", "flow")
        mask = torch.sigmoid(xhead(sd, h, "mask_pred", "mask"))
        dff = conv_module(conv_module(dflow, sd, "delta_flow_encoder.0", act, padding=3), sd,
                          "delta_flow_encoder.1", act, padding=1)
        mf = conv_module(conv_module(mask, sd, "mask_encoder.0", act, padding=1), sd,
                         "mask_encoder.1", act, padding=1)
        drot, dtr = pose_head(sd, torch.cat([h, dff, mf], 1),
                              label if head_label is None else head_label, num_class)
        flow_pred = scale * upsample(flow + dflow, scale)
        up_mask = upsample(mask, scale)
        if train:
            R, t = R.detach(), t.detach()
        R, t = pose_update(drot, dtr, R, t, depth_transform=depth_transform,
                           detach_depth_for_xy=train)
        flow = pose_flow(R, t, K, points, valid, invalid_flow_num)
        if hooks is not None:
            hooks.setdefault("h", []).append(h)
            hooks.setdefault("corr", []).append(corr)
        for lst, v in zip(outs, (flow, flow_pred, R, t, up_mask, drot, dtr)):
            lst.append(v)
    return outs


def cal_epe_mean(flow_tgt: Tensor, flow_pred: Tensor, mask: Tensor | None = None,
                 max_flow: float = 400.0) -> Tensor:
    """Per-sample mean EPE, ``cal_epe(..., reduction='mean')['mean']`` (models/utils/flow.py:64-78)."""
    mag = torch.sum(flow_tgt ** 2, dim=1).sqrt()
    valid = (mag < max_flow) if mask is None else ((mag < max_flow) & (mask >= 0.5))
    err = torch.sum((flow_tgt - flow_pred) ** 2, dim=1).sqrt()
    return (err * valid.to(err)).sum(dim=(-1, -2)) / (valid.sum(dim=(-1, -2)) + 1e-10)


# ---------------------------------------------------------------------------------------------
# §8(f)-1 — RAFTEncoder 'Basic' (models/encoder/raft_encoder.py:286-314) and the refiner's
# feature extraction (models/refiner/scflow_refiner.py:84-106, 108-138)
# ---------------------------------------------------------------------------------------------
def _enc_norm(x: Tensor, sd: StateDict, key: str, norm: str, eps: float = 1e-5,
              train: bool = False) -> Tensor:
    """mmcv build_norm_layer: IN → InstanceNorm2d(affine=False), BN → BatchNorm2d (eval: running
    stats; ``train``: batch statistics, running stats left untouched here)."""
    if norm == "IN":
        return F.instance_norm(x, eps=eps)
    if train:
        return F.batch_norm(x, None, None, sd[key + ".weight"], sd[key + ".bias"], training=True, eps=eps)
    return F.batch_norm(x, sd[key + ".running_mean"], sd[key + ".running_var"], sd[key + ".weight"],
                        sd[key + ".bias"], training=False, eps=eps)


def _basic_block(sd: StateDict, p: str, x: Tensor, stride: int, norm: str,
                 train: bool = False) -> Tensor:
    """BasicBlock.forward (models/backbone/resnet.py:65-92); downsample = ResLayer's
    1×1/stride conv + norm (resnet.py:707-729)."""
    ab = "in" if norm == "IN" else "bn"
    out = F.conv2d(x, sd[p + "conv1.weight"], sd[p + "conv1.bias"], stride=stride, padding=1)
    out = F.relu(_enc_norm(out, sd, p + ab + "1", norm, train=train))
    out = F.conv2d(out, sd[p + "conv2.weight"], sd[p + "conv2.bias"], padding=1)
    out = _enc_norm(out, sd, p + ab + "2", norm, train=train)
    if p + "downsample.0.weight" in sd:
        identity = F.conv2d(x, sd[p + "downsample.0.weight"], sd[p + "downsample.0.bias"], stride=stride)
        identity = _enc_norm(identity, sd, p + "downsample.1", norm, train=train)
    else:
        identity = x
    return F.relu(out + identity)


def raft_encoder(sd: StateDict, x: Tensor, norm: str, prefix: str = "",
                 strides: Sequence[int] = (1, 2, 2), blocks: Sequence[int] = (2, 2, 2),
                 train: bool = False) -> Tensor:
    """RAFTEncoder.forward, net_type='Basic', scale 1/8 (stem stride 2)."""
    ab = "in" if norm == "IN" else "bn"
    x = F.conv2d(x, sd[prefix + "conv1.weight"], sd[prefix + "conv1.bias"], stride=2, padding=3)
    x = F.relu(_enc_norm(x, sd, prefix + ab + "1", norm, train=train))
    for i, (s, nb) in enumerate(zip(strides, blocks)):
        for b in range(nb):
            x = _basic_block(sd, f"{prefix}res_layer{i + 1}.{b}.", x, s if b == 0 else 1, norm, train)
    return F.conv2d(x, sd[prefix + "conv2.weight"], sd[prefix + "conv2.bias"])


def extract_feat(sd: StateDict, render_images: Tensor, real_images: Tensor,
                 h_channels: int = 128, cxt_channels: int = 128, train: bool = False):
    """SCFlowRefiner.extract_feat (scflow_refiner.py:84-106): one shared feature encoder
    (``real_encoder`` is ``render_encoder`` when ``seperate_encoder=False``,
    base_refiner.py:33-40), context encoder on the rendered image, split + tanh / relu."""
    real = raft_encoder(sd, real_images, "IN", "real_encoder.")
    render = raft_encoder(sd, render_images, "IN", "render_encoder.")
    cxt = raft_encoder(sd, render_images, "BN", "context.", train=train)
    h, c = torch.split(cxt, [h_channels, cxt_channels], dim=1)
    return render, real, torch.tanh(h), torch.relu(c)


# ---------------------------------------------------------------------------------------------
# §8(f)-2 — training losses (models/loss/sequence_loss.py:7-80, point_matching_loss.py:106-218,
# the SCFlowRefiner.loss composition scflow_refiner.py:182-256; weights from
# configs/refine_models/scflow_ycbv_real.py:231-262)
# ---------------------------------------------------------------------------------------------
SYMMETRIC_CLASSES = (12, 15, 18, 19, 20)  # 0-based labels of cls_13, cls_16, cls_19, cls_20, cls_21 (config :34-40)


def raft_loss(pred: Tensor, gt: Tensor, valid: Tensor, weight: float = 0.1, max_flow: float = 400.,
              eps: float = 1e-10) -> Tensor:
    """RAFTLoss.forward (sequence_loss.py:15-23)."""
    mag = torch.sum(gt ** 2, dim=1).sqrt()
    v = ((valid >= 0.5) & (mag < max_flow)).to(gt)
    loss = (v[:, None] * (pred - gt).abs()).sum() / (v.sum() + eps)
    return weight * loss


def l1_loss(pred: Tensor, gt: Tensor, weight: float = 10.0) -> Tensor:
    """L1Loss.forward (sequence_loss.py:34-36)."""
    return weight * torch.mean(torch.abs(pred - gt))


def point_matching_loss(pred_r: Tensor, pred_t: Tensor, gt_r: Tensor, gt_t: Tensor, labels: Tensor,
                        points: Sequence[Tensor], diameters: Sequence[float],
                        weight: float = 10.0) -> Tensor:
    """DisentanglePointMatchingLoss.forward, l1, disentangle_z, no xy/depth scaling
    (point_matching_loss.py:159-218); symmetric classes match each GT point to its nearest
    predicted point (brute force in place of pytorch3d knn_points, :183-186)."""
    loss = 0.
    B = len(pred_r)
    for i in range(B):
        P = points[int(labels[i])]
        gt_rot = P @ gt_r[i].T
        gt_rt = gt_rot + gt_t[i][None]
        pred_rot = P @ pred_r[i].T + gt_t[i][None]
        if int(labels[i]) in SYMMETRIC_CLASSES:
            idx = torch.cdist(gt_rt, pred_rot).argmin(dim=1)
            pred_rot = pred_rot[idx]
        l_rot = torch.mean(torch.linalg.norm(pred_rot - gt_rt, dim=-1, ord=1))
        tz = torch.cat([gt_t[i][:2], pred_t[i][2:]])
        l_z = torch.mean(torch.linalg.norm(gt_rot + tz[None] - gt_rt, dim=-1, ord=1))
        txy = torch.cat([pred_t[i][:2], gt_t[i][2:]])
        l_xy = torch.mean(torch.linalg.norm(gt_rot + txy[None] - gt_rt, dim=-1, ord=1))
        loss = loss + (l_z + l_xy + l_rot) / diameters[int(labels[i])]
    return weight * loss / B


def filter_flow_by_mask(flow: Tensor, gt_mask: Tensor, invalid_num: float = 400.) -> Tensor:
    """filter_flow_by_mask (models/utils/flow.py:6-26): a flow whose target falls outside the
    target mask (bilinear sample < 0.9, align_corners=False, zero padding) becomes invalid."""
    N, _, H, W = flow.shape
    bad = (flow[:, 0] >= invalid_num) & (flow[:, 1] >= invalid_num)
    yy, xx = torch.meshgrid(torch.arange(H, dtype=flow.dtype), torch.arange(W, dtype=flow.dtype),
                            indexing="ij")
    gx = (xx[None] + flow[:, 0]) * 2. / max(W - 1, 1) - 1.
    gy = (yy[None] + flow[:, 1]) * 2. / max(H - 1, 1) - 1.
    m = F.grid_sample(gt_mask[:, None].to(flow.dtype), torch.stack([gx, gy], -1), mode="bilinear",
                      padding_mode="zeros", align_corners=False)
    bad = (m[:, 0] < 0.9) | bad
    return torch.where(bad[:, None].expand_as(flow), torch.full_like(flow, invalid_num), flow)


def sequence_loss(values: Sequence[Tensor], gamma: float = 0.8) -> Tensor:
    """SequenceLoss.forward (sequence_loss.py:59-80): Σ γ^(n−i−1)·loss_i."""
    n = len(values)
    return sum(gamma ** (n - i - 1) * v for i, v in enumerate(values))


def refine_train_loss(outs, gt_R: Tensor, gt_t: Tensor, gt_flow: Tensor, render_mask: Tensor,
                      labels: Tensor, points: Sequence[Tensor], diameters: Sequence[float],
                      max_flow: float = 400.) -> Tuple[Tensor, Tensor, Tensor]:
    """(loss_pose, loss_flow, loss_mask) of SCFlowRefiner.loss (scflow_refiner.py:200-242)
    from the decoder's 7 lists; gt_flow already filtered (filter_flow_by_mask)."""
    fp, fpred, Rs, ts, masks, _, _ = outs
    loss_pose = sequence_loss([point_matching_loss(R, t, gt_R, gt_t, labels, points, diameters)
                               for R, t in zip(Rs, ts)])
    loss_flow = sequence_loss([raft_loss(f, gt_flow, render_mask) for f in fpred])
    occ = (torch.sum(gt_flow, dim=1) < max_flow).to(gt_flow)
    loss_mask = sequence_loss([l1_loss(m[:, 0], occ) for m in masks])
    return loss_pose, loss_flow, loss_mask


def refine_train_forward(sd: StateDict, render_images: Tensor, real_images: Tensor,
                         ref_rotation: Tensor, ref_translation: Tensor, gt_rotation: Tensor,
                         gt_translation: Tensor, depth: Tensor, internel_k: Tensor, label: Tensor,
                         points: Sequence[Tensor], diameters: Sequence[float],
                         gt_masks: Tensor | None = None, iters: int = 8, max_flow: float = 400.):
    """SCFlowRefiner.loss (scflow_refiner.py:182-256) for the configured model: features (BN in
    train mode), decoder with the training detaches, GT flow (lift with the reference pose,
    project with the GT pose, invalid = max_flow; filter by the GT mask), the three losses.
    Returns (loss, loss_pose, loss_flow, loss_mask, outs, gt_flow)."""
    dt = render_images.dtype
    render, real, h, c = extract_feat(sd, render_images, real_images, train=True)
    N, H, W = depth.shape
    outs = decoder_forward(sd, render, real, h, c, ref_rotation, ref_translation, depth, internel_k,
                           label, torch.zeros(N, 2, H, W, dtype=dt), iters=iters, train=True)
    with torch.no_grad():
        pts, valid = lift_points(depth.to(dt), internel_k.to(dt), ref_rotation.to(dt),
                                 ref_translation.to(dt))
        gt_flow = pose_flow(gt_rotation.to(dt), gt_translation.to(dt), internel_k.to(dt), pts, valid,
                            max_flow)
        if gt_masks is not None:
            gt_flow = filter_flow_by_mask(gt_flow, gt_masks, max_flow)
    lp, lf, lm = refine_train_loss(outs, gt_rotation.to(dt), gt_translation.to(dt), gt_flow,
                                   (depth > 0).to(dt), label, [p.to(dt) for p in points], diameters,
                                   max_flow)
    return lp + lf + lm, lp, lf, lm, outs, gt_flow
