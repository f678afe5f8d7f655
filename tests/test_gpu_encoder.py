"""GPU parity of the RAFT encoders (§8(f) rank 1) and of the whole refinement forward
(images → encoders → decoder, SCFlowRefiner.get_pose) vs the reference and the oracle.

* encoder kernels one by one against plain PyTorch fp32 convs (CPU) — stride 1/2, 1×1/3×3,
  normalisation on load, BN affine + residual epilogue, split activation, column tiles;
* RAFTEncoder (IN and BN) against the reference's own output (golden, 128²) and the oracle at
  256² and 512²;
* SCFlowRefiner.get_pose against the reference fixture (B=2, 256², 4 iterations): mean flow EPE
  ≤ 1e-3 px, translations within 1e-3 mm.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tests.helpers import encoder_state_dict, golden, refine_inputs, refiner_state_dict, t

orc = pytest.importorskip("oracle.scflow_oracle")
pytestmark = pytest.mark.gpu


def build_encoder(norm, seed):
    from scflow_amd import MODELS
    enc = MODELS.build(dict(type="RAFTEncoder", in_channels=3, out_channels=256, net_type="Basic",
                            norm_cfg=dict(type=norm)))
    missing, unexpected = enc.load_state_dict(encoder_state_dict(norm, seed), strict=False)
    assert not unexpected and all(k.endswith("num_batches_tracked") for k in missing)
    return enc.eval().cuda()


def _cl(x):  # NCHW → channels-last contiguous
    return x.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("cin,cout,k,stride,h,w", [
    (64, 64, 3, 1, 128, 128),   # layer1 (whole-row tiles of 128)
    (64, 96, 3, 2, 128, 128),   # layer2 first conv (stride 2 → 64²)
    (96, 128, 3, 2, 64, 64),    # layer3 first conv (→ 32²)
    (64, 96, 1, 2, 128, 128),   # downsample 1×1/2
    (96, 128, 1, 2, 32, 32),    # downsample to 16² (4-row tiles)
    (128, 256, 1, 1, 32, 32),   # conv2
    (64, 64, 3, 1, 64, 512),    # column tiles (width 512 = 4 tiles of 128)
    (128, 128, 3, 1, 16, 16),   # 16-wide rows (128² images)
])
def test_enc_conv_matches_torch(cin, cout, k, stride, h, w):
    from scflow_amd import ops
    g = torch.Generator().manual_seed(cin * 7 + cout + k + stride)
    n = 2
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    pad = k // 2
    ref = F.conv2d(x, wt, b, stride=stride, padding=pad)
    oh, ow = ref.shape[-2:]
    out = torch.empty(n, oh, ow, cout, device="cuda")
    ops.enc_conv(_cl(x).cuda(), ops.enc_conv_pack(wt.cuda()), b.cuda(), n, h, w, cin, cout, k, stride,
                 pad, out)
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().permute(0, 3, 1, 2).numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


def test_enc_conv_fused_transforms_match_torch():
    """Input IN+ReLU on load, BN affine, residual and split tanh|relu epilogue."""
    from scflow_amd import ops
    g = torch.Generator().manual_seed(5)
    n, cin, cout, h, w = 2, 64, 128, 32, 32
    x = torch.randn(n, cin, h, w, generator=g) * 2 + 0.5
    wt = torch.randn(cout, cin, 3, 3, generator=g) / 24
    b = torch.randn(cout, generator=g) * 0.1
    isc = torch.rand(n, cin, generator=g) + 0.5
    ish = torch.randn(n, cin, generator=g) * 0.2
    osc = torch.rand(cout, generator=g) + 0.5
    osh = torch.randn(cout, generator=g) * 0.2
    res = torch.randn(n, cout, h, w, generator=g)
    xin = torch.relu(x * isc[:, :, None, None] + ish[:, :, None, None])
    v = F.conv2d(xin, wt, b, padding=1) * osc[None, :, None, None] + osh[None, :, None, None] + res
    ref = torch.cat([torch.tanh(v[:, :40]), torch.relu(v[:, 40:])], 1)
    out = torch.empty(n, h, w, cout + 8, device="cuda")  # pixel stride > cout
    ops.enc_conv(_cl(x).cuda(), ops.enc_conv_pack(wt.cuda()), b.cuda(), n, h, w, cin, cout, 3, 1, 1, out,
                 in_scale=isc.cuda(), in_shift=ish.cuda(), out_scale=osc.cuda(), out_shift=osh.cuda(),
                 res=_cl(res).cuda(), act="Tanh", act2="ReLU", act_split=40)
    torch.cuda.synchronize()
    got = out[..., :cout].cpu().permute(0, 3, 1, 2)
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


def test_enc_stem_stats_apply_match_torch():
    from scflow_amd import ops
    g = torch.Generator().manual_seed(9)
    n = 3
    x = torch.rand(n, 3, 256, 256, generator=g)
    wt = torch.randn(64, 3, 7, 7, generator=g) / 12
    b = torch.randn(64, generator=g) * 0.1
    ref = F.conv2d(x, wt, b, stride=2, padding=3)
    out = torch.empty(n, 128, 128, 64, device="cuda")
    ops.enc_stem(x.cuda(), ops.enc_stem_pack(wt.cuda()), b.cuda(), 64, 7, 2, 3, out)
    sc = torch.empty(n, 64, device="cuda")
    sh = torch.empty(n, 64, device="cuda")
    ops.enc_instance_norm_stats(out, n, 128 * 128, 64, sc, sh)
    idt = torch.randn(n, 128, 128, 64, generator=g)
    y = torch.empty_like(out)
    ops.enc_apply(out, sc, sh, y, n, 128 * 128, 64, id=idt.cuda())
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().permute(0, 3, 1, 2).numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
    ref_y = torch.relu(F.instance_norm(ref, eps=1e-5) + idt.permute(0, 3, 1, 2))
    np.testing.assert_allclose(y.cpu().permute(0, 3, 1, 2).numpy(), ref_y.numpy(), rtol=1e-4, atol=2e-4)


@pytest.mark.parametrize("norm,seed", [("IN", 1), ("BN", 2)])
def test_encoder_matches_reference_golden(norm, seed):
    from scflow_amd import synthetic
    g = golden("enc")
    B, S, iseed = (int(v) for v in g["meta"])
    x = t(synthetic.make_images(B, S, seed=iseed)["render_images"]).cuda()
    out = build_encoder(norm, seed)(x)
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().numpy(), g[f"enc_{norm}"], rtol=1e-4, atol=2e-4)


@pytest.mark.parametrize("norm,seed,B,S", [("IN", 1, 4, 256), ("BN", 2, 4, 256), ("IN", 1, 1, 512)])
def test_encoder_matches_oracle(norm, seed, B, S):
    from scflow_amd import synthetic
    x = t(synthetic.make_images(B, S, seed=21)["real_images"])
    ref = orc.raft_encoder(encoder_state_dict(norm, seed), x, norm)
    out = build_encoder(norm, seed)(x.cuda())
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=3e-4)


def build_refiner():
    from scflow_amd import MODELS
    from tests.test_gpu_decoder import decoder_cfg
    enc = dict(type="RAFTEncoder", in_channels=3, out_channels=256, net_type="Basic",
               norm_cfg=dict(type="IN"))
    ctx = dict(type="RAFTEncoder", in_channels=3, out_channels=256, net_type="Basic",
               norm_cfg=dict(type="BN"))
    r = MODELS.build(dict(type="SCFlowRefiner", cxt_channels=128, h_channels=128,
                          seperate_encoder=False, encoder=enc, cxt_encoder=ctx,
                          decoder=dict(type="SCFlowDecoder", **decoder_cfg(4))))
    missing, unexpected = r.load_state_dict(
        {("decoder." + k if not k.startswith(("real_encoder.", "render_encoder.", "context.")) else k): v
         for k, v in refiner_state_dict().items()}, strict=False)
    assert not unexpected and all(k.endswith("num_batches_tracked") for k in missing), missing
    return r.eval().cuda()


def test_refiner_get_pose_matches_reference_golden():
    g = golden("refine")
    B, S, iters, seed = (int(v) for v in g["meta"])
    inp = {k: v.cuda() for k, v in refine_inputs(B, S, seed, g).items()}
    r = build_refiner()
    r.decoder.iters = iters
    out = r.get_pose(inp["render_images"], inp["real_images"], inp["ref_rotation"],
                     inp["ref_translation"], inp["depth"], inp["internel_k"], inp["label"])
    torch.cuda.synchronize()
    fp, fpred, Rs, ts = (x[-1].cpu() for x in out[:4])
    assert float(orc.cal_epe_mean(t(g["flow_pose_last"]), fp).max()) <= 1e-3
    assert float(orc.cal_epe_mean(t(g["flow_pred_last"]), fpred).max()) <= 1e-3
    np.testing.assert_allclose(torch.stack([x.cpu() for x in out[3]]).numpy(), g["t"], rtol=1e-6, atol=1e-3)
    np.testing.assert_allclose(torch.stack([x.cpu() for x in out[2]]).numpy(), g["R"], atol=1e-5)


def test_refiner_extract_feat_matches_oracle():
    g = golden("refine")
    B, S, _, seed = (int(v) for v in g["meta"])
    inp = refine_inputs(B, S, seed, g)
    ref = orc.extract_feat(refiner_state_dict(), inp["render_images"], inp["real_images"])
    r = build_refiner()
    got = r.extract_feat(inp["render_images"].cuda(), inp["real_images"].cuda())
    torch.cuda.synchronize()
    for a, b in zip(got, ref):
        np.testing.assert_allclose(a.cpu().numpy(), b.numpy(), rtol=1e-4, atol=3e-4)


def test_refiner_rejects_cpu_tensors():
    from scflow_amd._lib import ScflowError
    r = build_refiner()
    x = torch.zeros(1, 3, 256, 256)
    with pytest.raises(ScflowError):
        r.get_pose(x, x, torch.eye(3)[None], torch.zeros(1, 3), torch.zeros(1, 256, 256),
                   torch.eye(3)[None], torch.zeros(1, dtype=torch.long))
