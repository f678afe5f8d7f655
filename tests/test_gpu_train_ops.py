"""GPU: training-step autograd Functions (HIP forward + backward) against CPU autograd of the
plain torch ops (fp64) — convolution (every variant the path uses, strides 1 and 2), the
correlation pyramid, the pyramid lookup (adjoint of CorrLookup, corr_lookup.py:102-136), the
feature encoder's InstanceNorm (+ ReLU) and the GRU's split-output z | r conv."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
orc = pytest.importorskip("oracle.scflow_oracle")


def _close(a, b, rtol, atol, what):
    a = a.detach().double().cpu().numpy()
    b = b.detach().double().cpu().numpy()
    err = np.abs(a - b).max()
    scale = np.abs(b).max() + 1e-12
    assert err <= atol + rtol * scale, f"{what}: max err {err:.3e} (scale {scale:.3e})"


@pytest.mark.parametrize("case", [
    # (n, h, w, cin, cout, k, stride, pad)      path exercised
    (2, 32, 32, 128, 64, 3, 1, 1),              # decoder MFMA 3×3
    (2, 32, 32, 256, 128, (1, 5), 1, (0, 2)),   # GRU 1×5
    (2, 32, 32, 324, 256, 1, 1, 0),             # corr_net.0 1×1 (cin not a multiple of 16)
    (2, 32, 32, 2, 128, 7, 1, 3),               # small-cin 7×7 (flow encoders)
    (2, 32, 32, 256, 2, 3, 1, 1),               # thin 3×3 → 2 (flow head)
    (2, 32, 32, 224, 128, 3, 2, 1),             # pose head conv1 (stride 2)
    (2, 64, 64, 64, 96, 3, 2, 1),               # encoder layer2 first conv
    (2, 64, 64, 64, 96, 1, 2, 0),               # encoder downsample 1×1/2
    (2, 64, 64, 3, 64, 7, 2, 3),                # encoder stem 7×7/2
    (2, 16, 16, 128, 128, 3, 1, 1),             # 16-wide (pose head / 128² encoder)
    (2, 32, 32, 1, 64, 3, 1, 1),                # mask encoder (cin 1: scalar wgrad staging)
    (2, 32, 32, 256, 128, (5, 1), 1, (2, 0)),   # GRU 5×1
    (2, 8, 8, 128, 128, 3, 2, 1),               # pose head conv3 (4×4 output)
    (3, 128, 128, 64, 64, 3, 1, 1),             # encoder layer1 (wide rows)
    (2, 32, 32, 256, 126, 3, 1, 1),             # out_net (cout not a multiple of 4)
    (2, 33, 31, 16, 40, 3, 2, 1),               # stride 2 on odd sizes (col2im dX)
    (2, 17, 15, 6, 8, 5, 2, 2),                 # stride 2, 5×5, channels not a multiple of 4
])
def test_conv2d_nhwc_forward_backward(case):
    from scflow_amd.train.functions import conv2d_nhwc
    n, h, w, cin, cout, k, stride, pad = case
    g = torch.Generator().manual_seed(hash(case) % 2 ** 31)
    kk = (k, k) if isinstance(k, int) else k
    x = torch.randn(n, h, w, cin, generator=g)
    wt = torch.randn(cout, cin, *kk, generator=g) / np.sqrt(cin * kk[0] * kk[1])
    b = torch.randn(cout, generator=g) * 0.1
    # reference: fp64 CPU autograd
    xr = x.double().permute(0, 3, 1, 2).requires_grad_()
    wr = wt.double().requires_grad_()
    br = b.double().requires_grad_()
    yr = F.conv2d(xr, wr, br, stride=stride, padding=pad)
    gy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    (yr * gy).sum().backward()
    # HIP
    xg = x.cuda().requires_grad_()
    wg = wt.cuda().requires_grad_()
    bg = b.cuda().requires_grad_()
    y = conv2d_nhwc(xg, wg, bg, stride, pad)
    (y * gy.float().permute(0, 2, 3, 1).cuda()).sum().backward()
    torch.cuda.synchronize()
    K = cin * kk[0] * kk[1]
    _close(y.permute(0, 3, 1, 2), yr, 1e-5, 1e-5 * np.sqrt(K), f"{case} y")
    _close(xg.grad.permute(0, 3, 1, 2), xr.grad, 1e-5, 1e-5 * np.sqrt(cout * kk[0] * kk[1]), f"{case} dx")
    _close(wg.grad, wr.grad, 1e-5, 1e-4 * np.sqrt(n * h * w), f"{case} dw")
    _close(bg.grad, br.grad, 1e-5, 1e-4 * np.sqrt(n * h * w), f"{case} db")


@pytest.mark.parametrize("act,two,bmap", [("Sigmoid", True, True), ("Tanh", True, True),
                                          ("ReLU", True, False), ("ReLU", False, False)])
def test_conv2d_nhwc_fused_act_two_sources_bias_map(act, two, bmap):
    """act(conv(cat[x0, x1]) + bias_map): the GRU's fused form (1×5, h ⊕ motion, hoisted context
    map) and the motion encoder's cat[c, f] — values and all five gradients vs fp64 autograd."""
    from scflow_amd.train.functions import conv2d_nhwc
    g = torch.Generator().manual_seed(11)
    n, h, w, c0, c1, cout = 2, 32, 32, 128, 128 if two else 0, 256
    x0 = torch.randn(n, h, w, c0, generator=g)
    x1 = torch.randn(n, h, w, c1, generator=g) if two else None
    wt = torch.randn(cout, c0 + c1, 1, 5, generator=g) / np.sqrt((c0 + c1) * 5)
    b = torch.randn(cout, generator=g) * 0.1 if not bmap else None
    bm = torch.randn(n, h, w, cout, generator=g) * 0.5 if bmap else None
    fn = {"Sigmoid": torch.sigmoid, "Tanh": torch.tanh, "ReLU": torch.relu}[act]
    leaves = [t.double().requires_grad_() if t is not None else None for t in (x0, x1, wt, b, bm)]
    xr = leaves[0] if not two else torch.cat([leaves[0], leaves[1]], -1)
    yr = F.conv2d(xr.permute(0, 3, 1, 2), leaves[2], leaves[3], padding=(0, 2)).permute(0, 2, 3, 1)
    if bmap:
        yr = yr + leaves[4]
    dev = [t.cuda().requires_grad_() if t is not None else None for t in (x0, x1, wt, b, bm)]
    y = conv2d_nhwc(dev[0], dev[2], dev[3], 1, (0, 2), act=act, x1=dev[1], bias_map=dev[4])
    _close(y, fn(yr.detach()), 1e-5, 1e-5 * np.sqrt(5 * (c0 + c1)), "y")
    # ReLU's derivative jumps at 0: the reference backward takes the device forward's active set,
    # so a pre-activation within fp32 rounding of 0 cannot flip a whole gradient element
    yr = yr * (y.detach().cpu().double() > 0) if act == "ReLU" else fn(yr)
    gy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    (yr * gy).sum().backward()
    (y * gy.float().cuda()).sum().backward()
    torch.cuda.synchronize()
    for name, a, r in zip(("x0", "x1", "w", "b", "bias_map"), dev, leaves):
        if a is not None:
            _close(a.grad, r.grad, 1e-5, 1e-4 * np.sqrt(n * h * w), name)


def test_dual_conv_heads_and_channel_slice_consumers():
    """dual_conv2d_nhwc (the XHeads' hidden convs as one launch each way) and convs reading its
    channel-view outputs in place (the predictors): values and every gradient — x, both weight /
    bias pairs, the predictors' weights — against fp64 autograd of the separate convs, over
    three uses of the same weights (the batched weight gradient across uses)."""
    from scflow_amd.train.functions import conv2d_nhwc, direct_weight_grads, dual_conv2d_nhwc
    g = torch.Generator().manual_seed(17)
    n, h, w, cin, ch = 2, 32, 32, 128, 256
    mk = lambda *s_, sc=1.0: (torch.randn(*s_, generator=g) * sc)
    wa, ba = mk(ch, cin, 3, 3, sc=cin ** -0.5 / 3), mk(ch, sc=0.1)
    wb, bb = mk(ch, cin, 3, 3, sc=cin ** -0.5 / 3), mk(ch, sc=0.1)
    wf, bf = mk(2, ch, 3, 3, sc=ch ** -0.5 / 3), mk(2, sc=0.1)
    wm, bm = mk(1, ch, 1, 1, sc=ch ** -0.5), mk(1, sc=0.1)
    xs = [mk(n, h, w, cin) for _ in range(3)]
    gys = [(mk(n, h, w, 2), mk(n, h, w, 1)) for _ in range(3)]
    leaves = [t.double().requires_grad_() for t in (wa, ba, wb, bb, wf, bf, wm, bm)]
    xr = [x.double().requires_grad_() for x in xs]
    tot = 0
    for x, (gf, gm) in zip(xr, gys):
        xc = x.permute(0, 3, 1, 2)
        fa = torch.relu(F.conv2d(xc, leaves[0], leaves[1], padding=1))
        fb = torch.relu(F.conv2d(xc, leaves[2], leaves[3], padding=1))
        of = F.conv2d(fa, leaves[4], leaves[5], padding=1).permute(0, 2, 3, 1)
        om = torch.sigmoid(F.conv2d(fb, leaves[6], leaves[7])).permute(0, 2, 3, 1)
        tot = tot + (of * gf.double()).sum() + (om * gm.double()).sum()
    tot.backward()
    dev = [t.cuda().requires_grad_() for t in (wa, ba, wb, bb, wf, bf, wm, bm)]
    for t in dev:
        t.grad = torch.zeros_like(t)
    xg = [x.cuda().requires_grad_() for x in xs]
    outs = []
    with direct_weight_grads():
        from scflow_amd.train.functions import begin_forward
        begin_forward()
        tot = 0
        for x, (gf, gm) in zip(xg, gys):
            fa, fb = dual_conv2d_nhwc(x, dev[0], dev[1], dev[2], dev[3], 1, "ReLU")
            of = conv2d_nhwc(fa, dev[4], dev[5], 1, 1)
            om = conv2d_nhwc(fb, dev[6], dev[7], 1, 0, act="Sigmoid")
            outs.append(of)
            tot = tot + (of * gf.cuda()).sum() + (om * gm.cuda()).sum()
        tot.backward()
    torch.cuda.synchronize()
    K = cin * 9
    for i in range(3):
        assert xg[i].grad is not None
        _close(xg[i].grad, xr[i].grad, 1e-5, 1e-4 * np.sqrt(K), f"dx[{i}]")
    for name, a, r in zip(("wa", "ba", "wb", "bb", "wf", "bf", "wm", "bm"), dev, leaves):
        _close(a.grad, r.grad, 1e-5, 1e-4 * np.sqrt(3 * n * h * w), name)


def test_conv_wgrad_accumulate_and_split():
    """scflow_conv_wgrad directly: a Chan slice as the second source, accumulate = 1 adds onto
    dw / db, and a batch large enough to split the pixel reduction over many workgroups."""
    from scflow_amd import ops
    from scflow_amd.ops import Chan
    g = torch.Generator().manual_seed(12)
    n, h, w, c0, c1, cout = 8, 64, 64, 64, 32, 96
    x0 = torch.randn(n, h, w, c0, generator=g)
    buf = torch.randn(n, h, w, 48, generator=g)  # second source = channels 8..40 of a wider buffer
    x1 = buf[..., 8:8 + c1]
    dy = torch.randn(n, h, w, cout, generator=g)
    ref = torch.nn.grad.conv2d_weight(torch.cat([x0, x1], -1).permute(0, 3, 1, 2).double(),
                                      (cout, c0 + c1, 3, 3), dy.permute(0, 3, 1, 2).double(), padding=1)
    dw = torch.ones(cout, c0 + c1, 3, 3).cuda()
    db = torch.ones(cout).cuda()
    bufc = buf.cuda()
    ops.conv_wgrad(dy.cuda().view(-1, cout), x0.cuda(), Chan(bufc.view(-1, 48), 8, c1), dw, db, n, h, w,
                   3, 3, 1, 1, 1, accumulate=True)
    torch.cuda.synchronize()
    _close(dw - 1, ref, 1e-5, 1e-4 * np.sqrt(n * h * w), "dw")
    _close(db - 1, dy.double().sum((0, 1, 2)), 1e-5, 1e-4 * np.sqrt(n * h * w), "db")


@pytest.mark.parametrize("case", [
    # (n, h, w, c0, c1, cout, kh, kw, stride)   thin side
    (16, 32, 32, 128, 128, 2, 3, 3, 1),       # cout 2, two sources (Chan slice), 256 workgroups
    (16, 32, 32, 256, 0, 1, 1, 1, 1),         # cout 1, 1×1 (mask predictor)
    (4, 32, 32, 1, 0, 64, 3, 3, 1),           # cin 1 (mask encoder)
    (2, 33, 31, 3, 0, 64, 3, 3, 2),           # cin 3, 3×3 / 2, odd sizes
    (2, 32, 32, 2, 0, 128, 5, 1, 1),          # cin 2, 5×1 (rows over grid.y, one tap per row)
    (2, 16, 16, 64, 0, 4, 1, 5, 2),           # cout 4, 1×5 / 2
])
def test_conv_wgrad_thin(case):
    """The thin-channel weight gradient (one side ≤ 4 channels): fp64 reference, accumulate = 1
    onto dw / db, a Chan slice as the second source."""
    from scflow_amd import ops
    from scflow_amd.ops import Chan
    n, h, w, c0, c1, cout, kh, kw, s = case
    g = torch.Generator().manual_seed(sum(case))
    ph, pw = kh // 2, kw // 2
    x0 = torch.randn(n, h, w, c0, generator=g)
    buf = torch.randn(n, h, w, c1 + 8, generator=g)
    x1 = buf[..., 4:4 + c1]
    oh, ow = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    dy = torch.randn(n, oh, ow, cout, generator=g)
    xc = torch.cat([x0, x1], -1) if c1 else x0
    ref = torch.nn.grad.conv2d_weight(xc.permute(0, 3, 1, 2).double(), (cout, c0 + c1, kh, kw),
                                      dy.permute(0, 3, 1, 2).double(), stride=s, padding=(ph, pw))
    dw = torch.ones(cout, c0 + c1, kh, kw).cuda()
    db = torch.ones(cout).cuda()
    src1 = Chan(buf.cuda().view(-1, c1 + 8), 4, c1) if c1 else None
    ops.conv_wgrad(dy.cuda().view(-1, cout), x0.cuda(), src1, dw, db, n, h, w, kh, kw, s, ph, pw,
                   accumulate=True)
    torch.cuda.synchronize()
    _close(dw - 1, ref, 1e-5, 1e-4 * np.sqrt(n * oh * ow), "dw")
    _close(db - 1, dy.double().sum((0, 1, 2)), 1e-5, 1e-4 * np.sqrt(n * oh * ow), "db")


@pytest.mark.parametrize("case", [
    # (n, h, w, c0, c1, cout, kh, kw, bias)
    (4, 32, 32, 128, 128, 256, 1, 5, False),   # GRU z | r 1×5 (h ⊕ motion), configs' width
    (4, 32, 32, 128, 128, 128, 5, 1, False),   # GRU q 5×1
    (3, 32, 32, 128, 0, 256, 1, 5, True),      # the hoisted context part (bias)
    (2, 64, 36, 64, 32, 96, 5, 1, True),       # ragged cout / cin blocks, two column chunks
    (2, 8, 64, 64, 32, 96, 1, 5, False),
])
def test_conv_wgrad_wino5(case):
    """The Winograd F(4, 5) weight gradient of the GRU's 1×5 / 5×1 convs (wgrad_wino5.h) vs an
    fp64 reference, accumulate = 1 onto dw / db, a Chan slice as the second source.  Tolerance:
    the transform-domain sums carry Winograd's larger fp32 rounding (points up to ±8 / ±5.25 in
    A / Bᵀ), bounded here at 2e-5 of the gradient's magnitude."""
    from scflow_amd import ops
    from scflow_amd.ops import Chan
    n, h, w, c0, c1, cout, kh, kw, bias = case
    g = torch.Generator().manual_seed(sum(case))
    ph, pw = kh // 2, kw // 2
    x0 = torch.randn(n, h, w, c0, generator=g)
    buf = torch.randn(n, h, w, c1 + 8, generator=g)
    x1 = buf[..., 4:4 + c1]
    dy = torch.randn(n, h, w, cout, generator=g)
    xc = torch.cat([x0, x1], -1) if c1 else x0
    ref = torch.nn.grad.conv2d_weight(xc.permute(0, 3, 1, 2).double(), (cout, c0 + c1, kh, kw),
                                      dy.permute(0, 3, 1, 2).double(), padding=(ph, pw))
    dw = torch.ones(cout, c0 + c1, kh, kw).cuda()
    db = torch.ones(cout).cuda() if bias else None
    src1 = Chan(buf.cuda().view(-1, c1 + 8), 4, c1) if c1 else None
    ops.conv_wgrad(dy.cuda().view(-1, cout), x0.cuda(), src1, dw, db, n, h, w, kh, kw, 1, ph, pw,
                   accumulate=True)
    torch.cuda.synchronize()
    err = float(((dw - 1).cpu().double() - ref).abs().max() / ref.abs().max())
    print(f"wino5 wgrad {case}: max error / max |dW| = {err:.2e}")
    _close(dw - 1, ref, 2e-5, 0.0, "dw")
    if bias:
        _close(db - 1, dy.double().sum((0, 1, 2)), 1e-5, 1e-4 * np.sqrt(n * h * w), "db")


@pytest.mark.parametrize("case", [
    # (segs, n, h, w, c0, c1, cout, kh, kw, bias)
    (8, 2, 32, 32, 128, 128, 256, 1, 5, False),   # the GRU's 8 iterations, z | r 1×5
    (8, 2, 32, 32, 128, 128, 128, 5, 1, False),   # q 5×1
    (8, 2, 32, 32, 256, 0, 192, 3, 3, True),      # corr_net.1 over 8 iterations (bias)
    (3, 2, 32, 64, 64, 32, 96, 3, 3, True),       # 3 segments, ragged channel blocks
])
def test_conv_wgrad_batched(case):
    """scflow_conv_wgrad_batched (one launch over equally shaped segments) = the sum of the
    segments' fp64 weight gradients, accumulate = 1 onto dw / db, Chan slices as second sources."""
    from scflow_amd import ops
    from scflow_amd.ops import Chan
    segs, n, h, w, c0, c1, cout, kh, kw, bias = case
    g = torch.Generator().manual_seed(sum(case))
    ph, pw = kh // 2, kw // 2
    ref = torch.zeros(cout, c0 + c1, kh, kw, dtype=torch.float64)
    dys, s0, s1, dbr = [], [], [], torch.zeros(cout, dtype=torch.float64)
    for _ in range(segs):
        x0 = torch.randn(n, h, w, c0, generator=g)
        buf = torch.randn(n, h, w, c1 + 8, generator=g)
        dy = torch.randn(n, h, w, cout, generator=g)
        xc = torch.cat([x0, buf[..., 4:4 + c1]], -1) if c1 else x0
        ref += torch.nn.grad.conv2d_weight(xc.permute(0, 3, 1, 2).double(), (cout, c0 + c1, kh, kw),
                                           dy.permute(0, 3, 1, 2).double(), padding=(ph, pw))
        dbr += dy.double().sum((0, 1, 2))
        dys.append(dy.cuda().view(-1, cout))
        s0.append(x0.cuda())
        s1.append(Chan(buf.cuda().view(-1, c1 + 8), 4, c1))
    dw = torch.ones(cout, c0 + c1, kh, kw).cuda()
    db = torch.ones(cout).cuda() if bias else None
    ops.conv_wgrad_batched(dys, s0, s1 if c1 else None, dw, db, n, h, w, kh, kw, 1, ph, pw,
                           accumulate=True)
    torch.cuda.synchronize()
    _close(dw - 1, ref, 2e-5, 0.0, "dw")
    if bias:
        _close(db - 1, dbr, 1e-5, 1e-4 * np.sqrt(segs * n * h * w), "db")


@pytest.mark.parametrize("case", [
    # (segs, n, h, w, c0, c1, cout, k, stride, bias)
    (8, 2, 32, 32, 324, 0, 256, 1, 1, True),    # corr_net.0 1×1 over 8 iterations (wgrad_1x1.h)
    (3, 2, 32, 32, 128, 64, 96, 1, 1, False),   # 1×1, two sources, ragged 128-blocks
    (2, 2, 33, 31, 64, 0, 96, 1, 2, True),      # 1×1 / 2 on odd sizes (encoder downsample)
    (8, 2, 32, 32, 128, 128, 2, 3, 1, True),    # thin: flow head 3×3 256 → 2, Chan second source
    (8, 2, 32, 32, 256, 0, 1, 1, 1, True),      # thin: mask head 1×1 256 → 1
    (8, 2, 32, 32, 1, 0, 64, 3, 1, True),       # thin: mask encoder 3×3 1 → 64
    (5, 1, 20, 24, 2, 0, 64, 5, 2, False),      # thin 5×5 / 2, ragged pixel runs
])
def test_conv_wgrad_batched_1x1_thin(case):
    """scflow_conv_wgrad_batched on the 1×1 kernel and the thin kernel (segments over grid.z):
    the sum of the segments' fp64 weight gradients, accumulate = 1."""
    from scflow_amd import ops
    from scflow_amd.ops import Chan
    segs, n, h, w, c0, c1, cout, k, s, bias = case
    g = torch.Generator().manual_seed(sum(case))
    p = k // 2
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    ref = torch.zeros(cout, c0 + c1, k, k, dtype=torch.float64)
    dys, s0, s1, dbr = [], [], [], torch.zeros(cout, dtype=torch.float64)
    for _ in range(segs):
        x0 = torch.randn(n, h, w, c0, generator=g)
        buf = torch.randn(n, h, w, c1 + 8, generator=g)
        dy = torch.randn(n, oh, ow, cout, generator=g)
        xc = torch.cat([x0, buf[..., 4:4 + c1]], -1) if c1 else x0
        ref += torch.nn.grad.conv2d_weight(xc.permute(0, 3, 1, 2).double(), (cout, c0 + c1, k, k),
                                           dy.permute(0, 3, 1, 2).double(), stride=s, padding=p)
        dbr += dy.double().sum((0, 1, 2))
        dys.append(dy.cuda().view(-1, cout))
        s0.append(x0.cuda())
        s1.append(Chan(buf.cuda().view(-1, c1 + 8), 4, c1))
    dw = torch.ones(cout, c0 + c1, k, k).cuda()
    db = torch.ones(cout).cuda() if bias else None
    ops.conv_wgrad_batched(dys, s0, s1 if c1 else None, dw, db, n, h, w, k, k, s, p, p,
                           accumulate=True)
    torch.cuda.synchronize()
    _close(dw - 1, ref, 1e-5, 1e-4 * np.sqrt(segs * n * oh * ow), "dw")
    if bias:
        _close(db - 1, dbr, 1e-5, 1e-4 * np.sqrt(segs * n * oh * ow), "db")


@pytest.mark.parametrize("acc", [False, True])
def test_concat_gemm_wgrad_7x7(acc):
    """The flow encoders' 7×7 2 → 128 weight gradient summed over 8 uses as one GEMM
    (functions._concat_gemm_wgrad) vs the fp64 sum, with the bias, accumulate on / off."""
    from scflow_amd.train import functions as fn
    g = torch.Generator().manual_seed(77)
    segs, n, h, w, cin, cout = 8, 2, 32, 32, 2, 128
    ref = torch.zeros(cout, cin, 7, 7, dtype=torch.float64)
    dbr = torch.zeros(cout, dtype=torch.float64)
    items = []
    for _ in range(segs):
        x = torch.randn(n, h, w, cin, generator=g)
        dy = torch.randn(n, h, w, cout, generator=g)
        ref += torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).double(), (cout, cin, 7, 7),
                                           dy.permute(0, 3, 1, 2).double(), padding=3)
        dbr += dy.double().sum((0, 1, 2))
        items.append((dy.cuda(), x.cuda(), None))
    wt = torch.zeros(cout, cin, 7, 7).cuda()
    dw = torch.ones(cout, cin, 7, 7).cuda()
    db = torch.ones(cout).cuda()
    fn._concat_gemm_wgrad(items, wt, True, dw, db, acc, 1, 3, 3)
    torch.cuda.synchronize()
    off = 1.0 if acc else 0.0
    _close(dw - off, ref, 1e-5, 1e-4 * np.sqrt(segs * n * h * w), "dw")
    _close(db - off, dbr, 1e-5, 1e-4 * np.sqrt(segs * n * h * w), "db")


@pytest.mark.parametrize("rows,cols,acc", [(16384, 128, False), (16, 1024, True), (524288, 64, True),
                                           (1000, 3, False), (300, 257, True)])
def test_colsum(rows, cols, acc):
    """scflow_colsum (bias gradients) against an fp64 column sum, with a row-major view whose
    row stride exceeds its width; accumulate onto an existing vector."""
    from scflow_amd import ops
    g = torch.Generator().manual_seed(rows + cols)
    base = torch.randn(rows, cols + 5, generator=g)
    x = base[:, 2:2 + cols]
    out0 = torch.randn(cols, generator=g)
    out = out0.clone().cuda()
    ops.colsum(base.cuda()[:, 2:2 + cols], out, accumulate=acc)
    ref = x.double().sum(0) + (out0.double() if acc else 0)
    _close(out, ref, 1e-6, 1e-5 * np.sqrt(rows), "colsum")


def test_corr_pyramid_backward():
    from scflow_amd import ops
    from scflow_amd.train.functions import corr_pyramid
    g = torch.Generator().manual_seed(1)
    n, c, h, w = 2, 32, 16, 16
    f1 = torch.randn(n, c, h, w, generator=g)
    f2 = torch.randn(n, c, h, w, generator=g)
    r1, r2 = f1.double().requires_grad_(), f2.double().requires_grad_()
    levels = orc.corr_pyramid(r1, r2, 4)
    gl = [torch.randn(lv.shape, generator=g, dtype=torch.float64) for lv in levels]
    sum((lv * gg).sum() for lv, gg in zip(levels, gl)).backward()
    a1, a2 = f1.cuda().requires_grad_(), f2.cuda().requires_grad_()
    buf = corr_pyramid(a1, a2, 4)
    gbuf = ops.pyramid_buffer([gg.float().cuda() for gg in gl], n, h, w)
    (buf * gbuf).sum().backward()
    torch.cuda.synchronize()
    _close(a1.grad, r1.grad, 1e-5, 1e-4, "df1")
    _close(a2.grad, r2.grad, 1e-5, 1e-4, "df2")


@pytest.mark.parametrize("radius,flow_kind", [(4, "rand"), (1, "rand"), (4, "grid"), (6, "rand")])
def test_corr_lookup_backward(radius, flow_kind):
    """The adjoint of the lookup: ⟨lookup(pyr), g⟩ differentiated w.r.t. the pyramid, with flow
    in ±6 px (zero padding) — against autograd of the oracle's explicit bilinear gather.  "grid":
    flows on the integer / half / quarter / eighth grid (zero where the reference's flow is
    invalid), the coordinates where the float unnormalisation rounds across a tap boundary."""
    from scflow_amd import ops
    from scflow_amd.train.functions import corr_lookup
    g = torch.Generator().manual_seed(2 + radius)
    n, c, h, w = 2, 16, 16, 16
    f1 = torch.randn(n, c, h, w, generator=g)
    f2 = torch.randn(n, c, h, w, generator=g)
    levels = [lv.double().requires_grad_() for lv in orc.corr_pyramid(f1.double(), f2.double(), 4)]
    flow = (torch.rand(n, 2, h, w, generator=g) - 0.5) * 12
    if flow_kind == "grid":
        d = torch.tensor([1., 2., 4., 8.])[torch.randint(0, 4, (n, 2, h, w), generator=g)]
        flow = torch.round(flow * d) / d
        flow[:, :, ::3] = 0.0
    out = orc.corr_lookup(levels, flow.double(), radius)          # [n, K, h, w]
    gout = torch.randn(out.shape, generator=g, dtype=torch.float64)
    (out * gout).sum().backward()
    pyr = ops.pyramid_buffer([lv.detach().float().cuda() for lv in levels], n, h, w).requires_grad_()
    fl = flow.permute(0, 2, 3, 1).contiguous().cuda()
    o = corr_lookup(pyr, fl, n, h, w, 4, radius)
    _close(o.permute(0, 3, 1, 2), out, 1e-5, 1e-5, "lookup forward")
    (o * gout.float().permute(0, 2, 3, 1).cuda()).sum().backward()
    torch.cuda.synchronize()
    ref = torch.cat([lv.grad.float().reshape(-1) for lv in levels])
    _close(pyr.grad, ref, 1e-5, 1e-5, "lookup backward")


def test_shared_gradient_buffers_across_backward_passes():
    """The lookups' shared pyramid-gradient buffer and the GRU's shared weight-gradient buffers
    are released after each backward pass: a second pass over the same graph (retain_graph, and
    torch.autograd.grad) yields the same gradients, not None and not an accumulation into the
    first pass's buffer."""
    from scflow_amd import ops
    from scflow_amd.train.functions import corr_lookup, corr_pyramid, gru_step
    g = torch.Generator().manual_seed(41)
    n, c, h, w = 2, 16, 16, 16
    f1 = torch.randn(n, c, h, w, generator=g).cuda().requires_grad_()
    f2 = torch.randn(n, c, h, w, generator=g).cuda()
    pyr = corr_pyramid(f1, f2, 4)
    fl = [((torch.rand(n, h, w, 2, generator=g) - 0.5) * 8).cuda() for _ in range(3)]
    loss = sum((corr_lookup(pyr, f, n, h, w, 4, 4) * (i + 1)).sum() for i, f in enumerate(fl))
    loss.backward(retain_graph=True)
    g1 = f1.grad.clone()
    f1.grad = None
    loss.backward(retain_graph=True)
    torch.testing.assert_close(f1.grad, g1, rtol=1e-6, atol=1e-6)
    (g3,) = torch.autograd.grad(loss, f1)
    torch.testing.assert_close(g3, g1, rtol=1e-6, atol=1e-6)
    # GRU weights used by two steps (like the 8 refinement iterations)
    hh = torch.tanh(torch.randn(1, 32, 32, 128, generator=g)).cuda()
    x = torch.randn(1, 32, 32, 128, generator=g).cuda()
    wzr = (torch.randn(256, 256, 1, 5, generator=g) * 0.02).cuda().requires_grad_()
    wq = (torch.randn(128, 256, 1, 5, generator=g) * 0.02).cuda().requires_grad_()
    pzr = torch.zeros(1, 32, 32, 256).cuda()
    pq = torch.zeros(1, 32, 32, 128).cuda()
    y = gru_step(gru_step(hh, x, wzr, wq, pzr, pq, (0, 2)), x, wzr, wq, pzr, pq, (0, 2))
    out = (y * y).sum()
    a = torch.autograd.grad(out, [wzr, wq], retain_graph=True)
    b = torch.autograd.grad(out, [wzr, wq])
    for u, v in zip(a, b):
        assert u is not None and v is not None
        torch.testing.assert_close(u, v, rtol=1e-6, atol=1e-7)


def test_gru_shared_weights_across_cycles_and_short_passes():
    """the same LEAF GRU weights through two separate forward/backward cycles (raw
    leaves and share_weight), and a pass whose loss never reaches the second use, against the
    unfused path (split conv + conv + lerp autograd ops) — no stale use counts, no uninitialised
    gradient memory."""
    from scflow_amd.train.functions import conv2d_nhwc, conv2d_nhwc_split, gru_step, share_weight
    g = torch.Generator().manual_seed(43)
    c = 128
    hh = torch.tanh(torch.randn(1, 32, 32, c, generator=g)).cuda()
    x = torch.randn(1, 32, 32, 128, generator=g).cuda()
    wzr = (torch.randn(2 * c, 256, 1, 5, generator=g) * 0.02).cuda().requires_grad_()
    wq = (torch.randn(c, 256, 1, 5, generator=g) * 0.02).cuda().requires_grad_()
    pzr = (torch.randn(1, 32, 32, 2 * c, generator=g) * 0.1).cuda()
    pq = (torch.randn(1, 32, 32, c, generator=g) * 0.1).cuda()

    def unfused(h):
        z, r = conv2d_nhwc_split(h, wzr, c, None, 1, (0, 2), act="Sigmoid", x1=x, bias_map=pzr)
        q = conv2d_nhwc(r * h, wq, None, 1, (0, 2), act="Tanh", x1=x, bias_map=pq)
        return torch.lerp(h, q, z)

    def grads(loss_fn):
        return [t.detach().clone() for t in torch.autograd.grad(loss_fn(), [wzr, wq])]

    ref2 = grads(lambda: (unfused(unfused(hh)) ** 2).sum())
    ref1 = grads(lambda: (unfused(hh) ** 2).sum())
    for cycle in range(2):  # raw leaves: every call its own node
        got = grads(lambda: (gru_step(gru_step(hh, x, wzr, wq, pzr, pq, (0, 2)), x, wzr, wq, pzr, pq,
                                      (0, 2)) ** 2).sum())
        for u, v, nm in zip(got, ref2, ("wzr", "wq")):
            _close(u, v, 1e-4, 1e-6, f"raw leaves cycle {cycle} d{nm}")

    def shared_two(short):
        sz, sq = share_weight(wzr), share_weight(wq)
        y1 = gru_step(hh, x, sz, sq, pzr, pq, (0, 2))
        y2 = gru_step(y1, x, sz, sq, pzr, pq, (0, 2))
        return ((y1 if short else y2) ** 2).sum()
    for cycle in range(2):
        for short, ref in ((False, ref2), (True, ref1)):
            got = grads(lambda: shared_two(short))
            for u, v, nm in zip(got, ref, ("wzr", "wq")):
                _close(u, v, 1e-4, 1e-6, f"shared cycle {cycle} short={short} d{nm}")


def test_conv_dx_shortcuts_match_conv2d_input():
    """the 1×1 → 1-channel dX shortcut (dY ⊗ w, unpadded only) and the thin large-
    kernel dX (GEMM + col2im) against torch.nn.grad.conv2d_input, plus a PADDED 1×1 → 1 conv,
    which must not take the shortcut, and convs padded by more than k−1 (their
    adjoint's padding k−1−p is negative — the cropped unpadded conv of dY)."""
    from scflow_amd.train.functions import conv2d_nhwc
    g = torch.Generator().manual_seed(44)
    for (cin, cout, k, pad) in ((256, 1, 1, 0), (256, 1, 1, 1), (2, 128, 7, 3), (64, 4, 1, 1),
                                (32, 64, 3, 2), (16, 8, 3, 3)):
        x = torch.randn(2, 32, 32, cin, generator=g)
        wt = torch.randn(cout, cin, k, k, generator=g) / np.sqrt(cin * k * k)
        xg = x.cuda().requires_grad_()
        y = conv2d_nhwc(xg, wt.cuda(), None, 1, pad)
        gy = torch.randn(y.shape, generator=g)
        y.backward(gy.cuda())
        ref = torch.nn.grad.conv2d_input(x.permute(0, 3, 1, 2).shape, wt.double(),
                                         gy.double().permute(0, 3, 1, 2), padding=pad)
        assert xg.grad.shape == x.shape
        _close(xg.grad, ref.permute(0, 2, 3, 1), 1e-5, 1e-6, f"dX {cin}->{cout} {k}x{k} pad {pad}")


@pytest.mark.parametrize("bt,M,N,K,ta,tb", [
    (1, 16, 1024, 2048, False, True),     # pose head FC forward: x · Wᵀ
    (1, 1024, 2048, 16, True, False),     # FC weight grad: dYᵀ · x
    (4, 256, 1024, 1024, False, True),    # corr backward dF1 = F2 · dCᵀ
    (4, 256, 1024, 1024, False, False),   # corr backward dF2 = F1 · dC
    (1, 128, 6272, 4096, True, False),    # 7×7 wgrad dYᵀ · cols
    (1, 64, 147, 32768, True, False),     # stem wgrad: deep K, split over the grid
    (2, 64, 98, 8192, True, False),       # batched + split
    (3, 77, 45, 19, False, False),        # ragged edges, unaligned
    (2, 130, 129, 33, True, True),
])
def test_gemm_f32_strided(bt, M, N, K, ta, tb):
    """scflow_gemm_f32 vs fp64 torch on transposed / batched views (bias, alpha, beta)."""
    from scflow_amd import ops
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = torch.randn(bt, K, M, generator=g).transpose(1, 2) if ta else torch.randn(bt, M, K, generator=g)
    B = torch.randn(bt, N, K, generator=g).transpose(1, 2) if tb else torch.randn(bt, K, N, generator=g)
    C0 = torch.randn(bt, M, N, generator=g)
    bias = torch.randn(N, generator=g)
    ref = 0.5 * torch.matmul(A.double(), B.double()) + 2.0 * C0.double() + bias.double()
    out = C0.cuda()
    ops.gemm(A.cuda(), B.cuda(), out=out, alpha=0.5, beta=2.0, bias=bias.cuda())
    scale = float(ref.abs().max())
    err = float((out.cpu().double() - ref).abs().max())
    assert err <= 2e-6 * scale * max(1.0, K / 256) ** 0.5, err
    if bt == 1:  # 2-D call, fresh output, no bias
        o2 = ops.gemm(A[0].cuda(), B[0].cuda())
        torch.testing.assert_close(o2.cpu().double(), torch.matmul(A[0].double(), B[0].double()),
                                   rtol=1e-5, atol=1e-4 * max(1.0, K / 256) ** 0.5)


@pytest.mark.parametrize("n,h,w,c,relu", [(4, 64, 64, 64, True), (3, 32, 32, 96, False),
                                          (2, 16, 16, 128, True), (2, 8, 12, 4, False)])
def test_instance_norm_nhwc_forward_backward(n, h, w, c, relu):
    """HIP InstanceNorm2d(affine=False) (+ ReLU): output and input gradient against fp64 autograd
    of F.instance_norm on the same channels-last data."""
    from scflow_amd.train.functions import instance_norm_nhwc
    g = torch.Generator().manual_seed(31)
    x = (torch.randn(n, h, w, c, generator=g) * 2 + 0.5)
    dy = torch.randn(n, h, w, c, generator=g)
    xr = x.double().requires_grad_(True)
    yr = F.instance_norm(xr.permute(0, 3, 1, 2), eps=1e-5).permute(0, 2, 3, 1)
    if relu:
        yr = torch.relu(yr)
    (yr * dy.double()).sum().backward()
    xg = x.cuda().requires_grad_(True)
    y = instance_norm_nhwc(xg, 1e-5, relu)
    (y * dy.cuda()).sum().backward()
    _close(y, yr, 1e-5, 1e-5, "instance norm forward")
    _close(xg.grad, xr.grad, 1e-4, 1e-5, "instance norm input gradient")


@pytest.mark.parametrize("n,h,w,c,mode", [(4, 64, 64, 64, "relu"), (3, 32, 32, 96, "plain"),
                                          (2, 16, 16, 128, "res"), (16, 32, 32, 64, "res"),
                                          (2, 8, 12, 4, "relu")])
def test_batch_norm_nhwc_train(n, h, w, c, mode):
    """HIP BatchNorm2d in train mode (the context encoder's norms; + ReLU, or + a residual before
    the ReLU): output, running statistics and the gradients of x, γ, β (and the residual) against
    fp64 autograd of F.batch_norm(training=True) on the same channels-last data."""
    from scflow_amd.train.functions import batch_norm_nhwc
    g = torch.Generator().manual_seed(41 + c)
    x = torch.randn(n, h, w, c, generator=g) * 1.5 + 0.3
    r = torch.randn(n, h, w, c, generator=g)
    dy = torch.randn(n, h, w, c, generator=g)
    bn = torch.nn.BatchNorm2d(c, momentum=0.1, eps=1e-5)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(c, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(c, generator=g) * 0.2)
        bn.running_mean.copy_(torch.randn(c, generator=g) * 0.1)
        bn.running_var.copy_(torch.rand(c, generator=g) + 0.5)
    ref = torch.nn.BatchNorm2d(c, momentum=0.1, eps=1e-5).double()
    ref.load_state_dict(bn.state_dict())
    xr = x.double().requires_grad_(True)
    rr = r.double().requires_grad_(True)
    yr = ref(xr.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    if mode == "res":
        yr = yr + rr
    if mode != "plain":
        yr = torch.relu(yr)
    (yr * dy.double()).sum().backward()
    mod = bn.cuda().train()
    xg = x.cuda().requires_grad_(True)
    rg = r.cuda().requires_grad_(True)
    y = batch_norm_nhwc(xg, mod, relu=mode == "relu", res=rg if mode == "res" else None)
    (y * dy.cuda()).sum().backward()
    torch.cuda.synchronize()
    _close(y, yr, 1e-5, 1e-5, "batch norm forward")
    _close(mod.running_mean, ref.running_mean, 1e-5, 1e-6, "running mean")
    _close(mod.running_var, ref.running_var, 1e-5, 1e-6, "running var")
    assert int(mod.num_batches_tracked) == int(ref.num_batches_tracked) == 1
    m = n * h * w
    _close(xg.grad, xr.grad, 1e-4, 1e-5, "batch norm input gradient")
    _close(mod.weight.grad, ref.weight.grad, 1e-5, 1e-6 * m ** 0.5, "dγ")
    _close(mod.bias.grad, ref.bias.grad, 1e-5, 1e-6 * m ** 0.5, "dβ")
    if mode == "res":
        _close(rg.grad, rr.grad, 1e-6, 1e-6, "residual gradient")


@pytest.mark.parametrize("n,h,w,c", [(4, 64, 64, 64), (3, 32, 32, 96), (2, 16, 16, 128)])
def test_instance_norm_residual_relu(n, h, w, c):
    """relu(InstanceNorm2d(x) + res) — the encoder residual block's tail in one HIP pass each way:
    output and both input gradients against fp64 autograd."""
    from scflow_amd.train.functions import instance_norm_residual_relu_nhwc
    g = torch.Generator().manual_seed(33 + c)
    x = torch.randn(n, h, w, c, generator=g) * 2 + 0.5
    r = torch.randn(n, h, w, c, generator=g)
    dy = torch.randn(n, h, w, c, generator=g)
    xr = x.double().requires_grad_(True)
    rr = r.double().requires_grad_(True)
    yr = torch.relu(F.instance_norm(xr.permute(0, 3, 1, 2), eps=1e-5).permute(0, 2, 3, 1) + rr)
    (yr * dy.double()).sum().backward()
    xg = x.cuda().requires_grad_(True)
    rg = r.cuda().requires_grad_(True)
    y = instance_norm_residual_relu_nhwc(xg, rg, 1e-5)
    (y * dy.cuda()).sum().backward()
    _close(y, yr, 1e-5, 1e-5, "forward")
    _close(xg.grad, xr.grad, 1e-4, 1e-5, "input gradient")
    _close(rg.grad, rr.grad, 0.0, 0.0, "residual gradient")


def test_conv2d_nhwc_split_matches_whole():
    """The split-output conv (GRU z | r) gives the whole conv's outputs and the same gradients,
    including when one half receives no gradient."""
    from scflow_amd.train.functions import conv2d_nhwc, conv2d_nhwc_split
    g = torch.Generator().manual_seed(32)
    x = torch.randn(2, 32, 32, 128, generator=g).cuda()
    x1 = torch.randn(2, 32, 32, 128, generator=g).cuda()
    w = (torch.randn(256, 256, 1, 5, generator=g) * 0.05).cuda()
    for use_r in (True, False):
        ws = w.clone().requires_grad_(True)
        wc = w.clone().requires_grad_(True)
        xs = x.clone().requires_grad_(True)
        xc = x.clone().requires_grad_(True)
        z, r = conv2d_nhwc_split(xs, ws, 128, None, 1, (0, 2), act="Sigmoid", x1=x1)
        y = conv2d_nhwc(xc, wc, None, 1, (0, 2), act="Sigmoid", x1=x1)
        assert torch.equal(z, y[..., :128]) and torch.equal(r, y[..., 128:])
        loss_s = (z * 1.5).sum() + ((r * r).sum() if use_r else 0)
        loss_c = (y[..., :128] * 1.5).sum() + ((y[..., 128:] ** 2).sum() if use_r else 0)
        loss_s.backward()
        loss_c.backward()
        _close(xs.grad, xc.grad, 1e-6, 1e-7, "split conv dX")
        _close(ws.grad, wc.grad, 1e-6, 1e-7, "split conv dW")


@pytest.mark.parametrize("k,pad", [((1, 5), (0, 2)), ((5, 1), (2, 0))])
def test_gru_step_forward_backward(k, pad):
    """One SepConvGRU direction as one autograd node (HIP convs + fused gate kernels) against
    fp64 CPU autograd of the reference's formulation (raft_decoder.py:235-253): h', and the
    gradients of h, x, both weights and both pre-activation maps."""
    from scflow_amd.train.functions import gru_step
    g = torch.Generator().manual_seed(21)
    n, hh, ww, c, cx = 2, 32, 32, 128, 128
    h = torch.tanh(torch.randn(n, hh, ww, c, generator=g))
    x = torch.randn(n, hh, ww, cx, generator=g)
    wzr = torch.randn(2 * c, c + cx, *k, generator=g) / np.sqrt((c + cx) * 5)
    wq = torch.randn(c, c + cx, *k, generator=g) / np.sqrt((c + cx) * 5)
    pzr = torch.randn(n, hh, ww, 2 * c, generator=g) * 0.5
    pq = torch.randn(n, hh, ww, c, generator=g) * 0.5
    leaves = [t.double().requires_grad_() for t in (h, x, wzr, wq, pzr, pq)]
    hr, xr, wzrr, wqr, pzrr, pqr = leaves

    def conv(a, b, w, m):
        y = F.conv2d(torch.cat([a, b], -1).permute(0, 3, 1, 2), w, padding=pad).permute(0, 2, 3, 1)
        return y + m
    zr = torch.sigmoid(conv(hr, xr, wzrr, pzrr))
    z, r = zr[..., :c], zr[..., c:]
    q = torch.tanh(conv(r * hr, xr, wqr, pqr))
    yr = (1 - z) * hr + z * q
    gy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    (yr * gy).sum().backward()
    dev = [t.cuda().requires_grad_() for t in (h, x, wzr, wq, pzr, pq)]
    y = gru_step(*dev, pad)
    (y * gy.float().cuda()).sum().backward()
    torch.cuda.synchronize()
    _close(y, yr.detach(), 1e-5, 1e-5 * np.sqrt(5 * (c + cx)), "h'")
    for name, a_, r_ in zip(("h", "x", "w_zr", "w_q", "pre_zr", "pre_q"), dev, leaves):
        _close(a_.grad, r_.grad, 1e-5, 1e-4 * np.sqrt(n * hh * ww), name)


def test_knn1_matches_argmin():
    """scflow_knn1 (symmetric-class point matching) equals torch's broadcast distances + argmin,
    ties included (duplicated predicted points: the first index wins), Q over one LDS chunk."""
    from scflow_amd import ops
    g = torch.Generator().manual_seed(31)
    B, P, Q = 3, 700, 1500
    gt = torch.randn(B, P, 3, generator=g) * 50
    pred = torch.randn(B, Q, 3, generator=g) * 50
    pred[:, 1100:1200] = pred[:, 100:200]  # exact duplicates later in index order
    gt[:, :50] = pred[:, 150:200]          # exact hits on duplicated points
    ref = ((gt[:, :, None] - pred[:, None]) ** 2).sum(-1).argmin(-1)
    idx = ops.knn1(gt.cuda(), pred.cuda()).cpu()
    assert torch.equal(idx, ref)


@pytest.mark.parametrize("depth,detach_xy", [("exp", True), ("linear", False)])
def test_pose_update6_forward_backward(depth, detach_xy):
    """The HIP ortho6d pose update (forward + hand-written backward) against fp64 autograd of
    the torch formulation (train/model.py:pose_update, pose.py:124-169), gradients of Δrot, Δt,
    R and t."""
    from scflow_amd.train import model as tm
    from scflow_amd.train.functions import pose_update6
    g = torch.Generator().manual_seed(41)
    n = 16
    drot = torch.randn(n, 6, generator=g)
    dt = torch.randn(n, 3, generator=g) * 0.1
    q, _ = torch.linalg.qr(torch.randn(n, 3, 3, generator=g))
    R = q
    t = torch.cat([torch.randn(n, 2, generator=g) * 50, 500 + 200 * torch.rand(n, 1, generator=g)], 1)
    leaves = [v.double().requires_grad_() for v in (drot, dt, R, t)]
    Rr, tr = tm.pose_update(*leaves, depth_transform=depth, detach_depth_for_xy=detach_xy)
    gR = torch.randn(n, 3, 3, generator=g, dtype=torch.float64)
    gt = torch.randn(n, 3, generator=g, dtype=torch.float64)
    ((Rr * gR).sum() + (tr * gt).sum()).backward()
    dev = [v.cuda().requires_grad_() for v in (drot, dt, R, t)]
    Rn, tn = pose_update6(*dev, 10.0, depth == "exp", detach_xy)
    ((Rn * gR.float().cuda()).sum() + (tn * gt.float().cuda()).sum()).backward()
    torch.cuda.synchronize()
    _close(Rn, Rr.detach(), 1e-5, 1e-5, "R_new")
    _close(tn, tr.detach(), 1e-5, 1e-4, "t_new")
    for name, a_, r_ in zip(("drot", "dt", "R", "t"), dev, leaves):
        _close(a_.grad, r_.grad, 1e-4, 1e-5, name)


def test_point_matching_loss_fused():
    """The fused HIP point-matching loss (scflow_pm_loss, symmetric classes matched to the
    nearest predicted point) against the torch formulation in fp64 on the CPU: the loss and its
    gradients w.r.t. the predicted rotation and translation."""
    from scflow_amd.train import losses
    g = torch.Generator().manual_seed(51)
    B, P, C = 8, 1024, 21
    points = [torch.randn(P, 3, generator=g) * 40 for _ in range(C)]
    diam = torch.rand(C, generator=g) * 100 + 50
    labels = torch.tensor([0, 12, 3, 15, 7, 18, 1, 20])
    qr = lambda: torch.linalg.qr(torch.randn(B, 3, 3, generator=g))[0]  # noqa: E731
    gt_r, pr = qr(), qr()
    gt_t = torch.cat([torch.randn(B, 2, generator=g) * 30, 600 + torch.rand(B, 1, generator=g) * 100], 1)
    pt = gt_t + torch.randn(B, 3, generator=g) * 5
    ref_leaves = [pr.double().requires_grad_(), pt.double().requires_grad_()]
    lr = losses.point_matching_loss(ref_leaves[0], ref_leaves[1], gt_r.double(), gt_t.double(), labels,
                                    [p.double() for p in points], diam.double())
    lr.backward()
    dev = [pr.cuda().requires_grad_(), pt.cuda().requires_grad_()]
    l = losses.point_matching_loss(dev[0], dev[1], gt_r.cuda(), gt_t.cuda(), labels.cuda(),
                                   [p.cuda() for p in points], diam.cuda())
    l.backward()
    torch.cuda.synchronize()
    _close(l, lr.detach(), 1e-5, 1e-6, "loss")
    _close(dev[0].grad, ref_leaves[0].grad, 1e-4, 1e-6, "g_pred_r")
    _close(dev[1].grad, ref_leaves[1].grad, 1e-5, 1e-6, "g_pred_t")


@pytest.mark.parametrize("c,use_v,sval", [(2, True, 8.0), (1, False, 1.0)])
def test_up_l1_loss_fused(c, use_v, sval):
    """The fused upsample + L1 loss (flow: valid-masked, ×8 values; mask: plain mean) against
    fp64 torch F.interpolate(align_corners) + L1, value and gradient w.r.t. the low-res input."""
    from scflow_amd.train.functions import up_l1_loss
    g = torch.Generator().manual_seed(61)
    n, h, w, S = 3, 32, 32, 256
    f = torch.randn(n, h, w, c, generator=g) * 2
    tgt = torch.randn(n, c, S, S, generator=g) * 16
    v = (torch.rand(n, S, S, generator=g) > 0.3).float() if use_v else None
    fr = f.double().requires_grad_()
    up = sval * F.interpolate(fr.permute(0, 3, 1, 2), size=(S, S), mode="bilinear", align_corners=True)
    d = (up - tgt.double()).abs()
    if use_v:
        ref = 0.1 * (v.double()[:, None] * d).sum() / (v.double().sum() + 1e-10)
    else:
        ref = 10.0 * d.mean()
    ref.backward()
    fd = f.cuda().requires_grad_()
    if use_v:
        denom = (v.cuda().sum() + 1e-10).reshape(1)
        loss = up_l1_loss(fd, tgt.cuda(), v.cuda(), sval, denom, 0.0, 0.1)
    else:
        loss = up_l1_loss(fd, tgt.cuda(), None, sval, None, float(n * c * S * S), 10.0)
    loss.backward()
    torch.cuda.synchronize()
    _close(loss, ref.detach(), 1e-5, 1e-6, "loss")
    _close(fd.grad, fr.grad, 1e-4, 1e-7, "grad")


@pytest.mark.parametrize("n,h,w,c,relu", [(16, 16, 16, 128, True), (3, 4, 4, 128, True),
                                          (2, 5, 7, 64, False)])
def test_group_norm_nhwc(n, h, w, c, relu):
    """Fused GroupNorm (+ReLU), 4 channels per group, channels-last: forward, dx, dγ, dβ against
    fp64 torch GroupNorm (+ReLU) autograd on NCHW; then the accumulate mode adds onto .grad."""
    from scflow_amd import ops
    from scflow_amd.train.functions import group_norm_nhwc
    g = torch.Generator().manual_seed(n * h + c)
    x = torch.randn(n, h, w, c, generator=g) * 2 + 0.5
    wt = torch.randn(c, generator=g)
    bs = torch.randn(c, generator=g) * 0.3
    dy = torch.randn(n, h, w, c, generator=g)
    xr, wr, br = (t.double().requires_grad_() for t in (x, wt, bs))
    yr = torch.nn.functional.group_norm(xr.permute(0, 3, 1, 2), c // 4, wr, br, 1e-5)
    yr = (torch.relu(yr) if relu else yr).permute(0, 2, 3, 1)
    (yr * dy.double()).sum().backward()
    xc, wc, bc = (t.cuda().requires_grad_() for t in (x, wt, bs))
    y = group_norm_nhwc(xc, wc, bc, c // 4, 1e-5, relu)
    (y * dy.cuda()).sum().backward()
    torch.cuda.synchronize()
    _close(y, yr.detach(), 1e-5, 1e-5, "gn forward")
    _close(xc.grad, xr.grad, 1e-4, 1e-4, "gn dx")
    _close(wc.grad, wr.grad, 1e-4, 1e-4, "gn dgamma")
    _close(bc.grad, br.grad, 1e-4, 1e-4, "gn dbeta")
    # accumulate mode: the partials' sum lands on top of what the buffers hold
    _, stats = ops.group_norm_forward(xc.detach(), wc.detach(), bc.detach(), c // 4, 1e-5, relu)
    dg, db = torch.ones(c, device="cuda"), torch.full((c,), 2.0, device="cuda")
    ops.group_norm_backward(dy.cuda(), xc.detach(), wc.detach(), bc.detach(), stats, c // 4, relu,
                            dg, db, accumulate=True)
    torch.cuda.synchronize()
    _close(dg, wr.grad + 1, 1e-4, 1e-4, "gn dgamma (accumulate)")
    _close(db, br.grad + 2, 1e-4, 1e-4, "gn dbeta (accumulate)")
