"""CPU: the training forward's host composition (scflow_amd/train/model.py + losses.py) against
the oracle's SCFlowRefiner.loss restatement (oracle.refine_train_forward), fp64.

The HIP pieces the model calls (conv Function, correlation pyramid / lookup Functions, the 2D-3D
lift, pose-induced flow and flow downsampling kernels) are swapped for plain torch equivalents
here — this test checks the wiring (detaches, BN train mode, the GRU split, pose-head quirk, GT
flow + mask filtering, the loss weights and the sequence weighting) and the gradients that flow
through it; the HIP Functions themselves are covered by tests/test_gpu_train_ops.py and the whole
HIP training step by tests/test_gpu_train.py."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tests.helpers import refiner_state_dict

orc = pytest.importorskip("oracle.scflow_oracle")


def _patch_torch_ops(monkeypatch):
    from scflow_amd import ops
    from scflow_amd.train import model

    def conv(x, w, b=None, stride=1, padding=0, act=None, x1=None, bias_map=None):
        if x1 is not None:
            x = torch.cat([x, x1], -1)
        y = F.conv2d(x.permute(0, 3, 1, 2), w, b, stride, padding).permute(0, 2, 3, 1)
        if bias_map is not None:
            y = y + bias_map
        return {None: y, "ReLU": torch.relu(y), "Sigmoid": torch.sigmoid(y), "Tanh": torch.tanh(y)}[act]

    def conv_split(x, w, split, b=None, stride=1, padding=0, act=None, x1=None, bias_map=None):
        y = conv(x, w, b, stride, padding, act, x1, bias_map)
        return y[..., :split], y[..., split:]

    def pyramid(f1, f2, L=4):
        return orc.corr_pyramid(f1, f2, L)

    def lookup(levels, flow_nhwc, n, h, w, L=4, r=4):
        return orc.corr_lookup(levels, flow_nhwc.detach().permute(0, 3, 1, 2), r).permute(0, 2, 3, 1)

    def lift(depth, K, R, t):
        p, v = orc.lift_points(depth, K, R, t)
        return torch.cat([p, v[..., None].to(p)], -1)

    def pose_flow(R, t, K, pts, inv, out=None):
        f = orc.pose_flow(R, t, K, pts[..., :3], pts[..., 3] > 0, inv)
        if out is None:
            return f
        out.copy_(f)
        return out

    def downsample(flow, out0, h, w, value_scale, out1=None):
        f = orc.downsample_flow(flow, int(round(1 / value_scale)))
        out0.buf.view(-1, out0.buf.shape[-1])[:, out0.off:out0.off + 2] = f.permute(0, 2, 3, 1).reshape(-1, 2)

    monkeypatch.setattr(model, "conv2d_nhwc", conv)
    def gru(h, x, w_zr, w_q, pre_zr, pre_q, pad):
        c = h.shape[-1]
        zr = conv(h, w_zr, None, 1, pad, "Sigmoid", x, pre_zr)
        z, r = zr[..., :c], zr[..., c:]
        q = conv(r * h, w_q, None, 1, pad, "Tanh", x, pre_q)
        return torch.lerp(h, q, z)

    monkeypatch.setattr(model, "gru_step", gru)
    monkeypatch.setattr(model, "linear", F.linear)
    monkeypatch.setattr(model, "upsample_bilinear_ac", lambda x, s: F.interpolate(
        x, scale_factor=(s, s), mode="bilinear", align_corners=True))
    monkeypatch.setattr(model, "corr_pyramid", pyramid)
    monkeypatch.setattr(model, "corr_lookup", lookup)
    monkeypatch.setattr(ops, "lift_points", lift)
    monkeypatch.setattr(ops, "pose_flow", pose_flow)
    monkeypatch.setattr(ops, "flow_downsample", downsample)


def build_train_refiner(iters, dtype=torch.float32, **kw):
    from scflow_amd import MODELS
    from tests.test_gpu_decoder import decoder_cfg
    enc = dict(type="RAFTEncoder", in_channels=3, out_channels=256, net_type="Basic",
               norm_cfg=dict(type="IN"))
    ctx = dict(type="RAFTEncoder", in_channels=3, out_channels=256, net_type="Basic",
               norm_cfg=dict(type="BN"))
    r = MODELS.build(dict(type="SCFlowRefiner", cxt_channels=128, h_channels=128,
                          seperate_encoder=False, encoder=enc, cxt_encoder=ctx,
                          decoder=dict(type="SCFlowDecoder", **decoder_cfg(iters)), **kw))
    missing, unexpected = r.load_state_dict(
        {("decoder." + k if not k.startswith(("real_encoder.", "render_encoder.", "context.")) else k): v
         for k, v in refiner_state_dict().items()}, strict=False)
    assert not unexpected and all(k.endswith("num_batches_tracked") for k in missing), missing
    return r.to(dtype).train()


def train_batch(B, S, seed, labels=None, dtype=torch.float32, device="cpu"):
    """Synthetic training batch (images, reference + GT pose, depth, K, GT mask) + model points."""
    from scflow_amd import synthetic
    out = {}
    for k, v in synthetic.make_train_batch(B, S, seed=seed, labels=labels).items():
        x = torch.from_numpy(np.ascontiguousarray(v))
        out[k] = (x.to(dtype) if x.is_floating_point() else x).to(device)
    pts = torch.from_numpy(synthetic.make_model_points(256)).to(dtype).to(device)
    return out, list(pts), list(synthetic.YCBV_DIAMETERS)


def oracle_loss_and_grads(batch, points, diameters, iters, names, dtype=torch.float64):
    """CPU autograd (fp64 by default) of the oracle's SCFlowRefiner.loss restatement; grads keyed
    by the product module's parameter names."""
    sd = {k: v.to(dtype).requires_grad_(v.is_floating_point()) for k, v in refiner_state_dict().items()}
    b = {k: (v.to(dtype) if v.is_floating_point() else v).cpu() for k, v in batch.items()}
    loss, lp, lf, lm, outs, gt_flow = orc.refine_train_forward(
        sd, b["render_images"], b["real_images"], b["ref_rotation"], b["ref_translation"],
        b["gt_rotation"], b["gt_translation"], b["depth"], b["internel_k"], b["label"],
        [p.to(dtype).cpu() for p in points], diameters, gt_masks=b["gt_masks"], iters=iters)
    loss.backward()
    grads = {}
    for n in names:
        k = n if n.startswith(("real_encoder.", "render_encoder.", "context.")) else n[len("decoder."):]
        if k.startswith(("real_encoder.", "render_encoder.")):  # shared: both oracle copies
            tail = k.split(".", 1)[1]
            g = sd["real_encoder." + tail].grad
            gr = sd["render_encoder." + tail].grad
            grads[n] = None if g is None and gr is None else (
                (g if g is not None else 0) + (gr if gr is not None else 0))
        else:
            grads[n] = sd[k].grad
    return (loss, lp, lf, lm), outs, gt_flow, grads


def test_train_forward_host_matches_oracle(monkeypatch):
    from scflow_amd.train.model import refiner_train_forward
    _patch_torch_ops(monkeypatch)
    iters = 2
    r = build_train_refiner(iters, torch.float64)
    batch, points, diam = train_batch(2, 256, seed=5, labels=[12, 4], dtype=torch.float64)
    res = refiner_train_forward(r, batch, points, diam)
    res["loss"].backward()
    names = [n for n, _ in r.named_parameters()]
    (loss, lp, lf, lm), outs, gt_flow, grads = oracle_loss_and_grads(batch, points, diam, iters, names)
    np.testing.assert_allclose(res["gt_flow"].numpy(), gt_flow.numpy(), rtol=1e-9, atol=1e-6)
    for a, b in ((res["loss_pose"], lp), (res["loss_flow"], lf), (res["loss_mask"], lm)):
        np.testing.assert_allclose(a.item(), b.item(), rtol=1e-9)
    checked = 0
    for n, p in r.named_parameters():
        g = grads[n]
        if g is None:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, n
            continue
        np.testing.assert_allclose(p.grad.numpy(), g.numpy(), rtol=1e-7, atol=1e-9 * (1 + float(g.abs().max())),
                                   err_msg=n)
        checked += 1
    assert checked > 100
    # BN running stats were updated in train mode (SCFlowRefiner.train())
    assert int(r.context.norm1.num_batches_tracked) == 1


def test_freeze_bn_and_encoder(monkeypatch):
    """freeze_bn / freeze_encoder (scflow_refiner.py:58-79): BatchNorms in eval mode (no running
    statistics update, batch statistics not used), the feature encoder in eval mode with
    requires_grad=False — and both survive train(), which the training loop calls."""
    from scflow_amd.train.model import refiner_train_forward
    _patch_torch_ops(monkeypatch)
    r = build_train_refiner(1, torch.float64, freeze_bn=True, freeze_encoder=True)
    bns = [m for m in r.modules() if isinstance(m, torch.nn.BatchNorm2d)]
    assert bns and not any(m.training for m in bns)
    assert not any(m.training for m in r.real_encoder.modules())
    assert not any(p.requires_grad for p in r.real_encoder.parameters())
    assert all(p.requires_grad for p in r.context.parameters())
    assert r.decoder.training and r.context.training
    rm0 = r.context.norm1.running_mean.clone()
    batch, points, diam = train_batch(1, 256, seed=3, labels=[4], dtype=torch.float64)
    res = refiner_train_forward(r, batch, points, diam)
    res["loss"].backward()
    assert all(p.grad is None for p in r.real_encoder.parameters())
    assert r.context.norm1.weight.grad is not None  # BN affine stays trainable
    assert int(r.context.norm1.num_batches_tracked) == 0
    assert torch.equal(r.context.norm1.running_mean, rm0)
    # frozen BN = eval-mode batch_norm (running statistics) in the training forward
    from scflow_amd.train.model import _norm
    x = torch.randn(1, 8, 8, r.context.norm1.num_features, dtype=torch.float64)
    ref = F.batch_norm(x.permute(0, 3, 1, 2), r.context.norm1.running_mean, r.context.norm1.running_var,
                       r.context.norm1.weight, r.context.norm1.bias, training=False,
                       eps=r.context.norm1.eps).permute(0, 2, 3, 1)
    torch.testing.assert_close(_norm(x, r.context.norm1), ref)
    # TrainStep only optimises what requires grad
    from scflow_amd.train.step import trainable_parameters
    names = {id(p) for p in trainable_parameters(r)}
    assert not any(id(p) in names for p in r.real_encoder.parameters())
    # without the flags: train mode everywhere
    r2 = build_train_refiner(1, torch.float64)
    assert all(m.training for m in r2.modules() if isinstance(m, torch.nn.BatchNorm2d))
    assert all(p.requires_grad for p in r2.real_encoder.parameters())


def test_upsample_adjoint_matches_autograd(monkeypatch):
    """The training step's ×8 upsampling backward (two GEMMs on the interpolation matrices, here
    on torch.matmul in place of the HIP GEMM) equals autograd of F.interpolate(align_corners)."""
    from scflow_amd.train import functions as fn
    monkeypatch.setattr(fn.ops, "gemm", lambda a, b: torch.matmul(a, b))
    g = torch.Generator().manual_seed(5)
    for (h, w, s) in ((32, 32, 8), (7, 5, 4)):
        x = torch.randn(2, 3, h, w, generator=g, dtype=torch.float64)
        xr = x.clone().requires_grad_()
        yr = F.interpolate(xr, scale_factor=(s, s), mode="bilinear", align_corners=True)
        gy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
        (yr * gy).sum().backward()
        xg = x.float().requires_grad_()
        y = fn.upsample_bilinear_ac(xg, s)
        (y * gy.float()).sum().backward()
        assert torch.allclose(y.double(), yr.detach(), atol=1e-5)
        assert torch.allclose(xg.grad.double(), xr.grad, rtol=1e-5, atol=1e-4)


def test_channel_slice_views_are_read_in_place():
    """The training convs read a channel slice of a wider channels-last buffer in place
    (functions._chan_view: the XHeads' dual conv output feeding the predictors): slices map to
    (buffer, channel offset, channels); anything that is not a packed channel slice — a pixel
    sub-range, a transposed view, a slice of a non-contiguous tensor — is refused (copied)."""
    import torch
    from scflow_amd.train.functions import _chan, _chan_or_contiguous, _chan_view
    buf = torch.arange(2 * 4 * 4 * 12, dtype=torch.float32).view(2, 4, 4, 12)
    a, b = buf[..., :5], buf[..., 5:]
    ca, cb = _chan_view(a), _chan_view(b)
    assert (ca.off, ca.c, ca.stride) == (0, 5, 12) and (cb.off, cb.c, cb.stride) == (5, 7, 12)
    assert ca.buf.data_ptr() == buf.data_ptr() and ca.buf.shape == (32, 12)
    # the kernel's view of the slice: rows of `stride` floats from ptr, `c` of them used
    flat = ca.buf.view(-1)
    rows = torch.stack([flat[r * 12 + cb.off: r * 12 + cb.off + cb.c] for r in range(32)])
    assert torch.equal(rows.view(2, 4, 4, 7), b)
    assert _chan_or_contiguous(b) is b
    assert _chan(buf).c == 12 and _chan(buf).off == 0
    for bad in (buf[:, 1:3, :, :5], buf.transpose(1, 2)[..., :5], buf[..., ::2]):
        assert _chan_view(bad) is None
        assert _chan_or_contiguous(bad).is_contiguous()
