"""GPU parity: every C-ABI kernel against the CPU oracle / a plain fp32 PyTorch reference.

Tolerances (fp32 throughout):
* corr pyramid: |Δ| ≤ 2e-5·(1+|ref|) — a K=C fp32 dot product, different summation order;
* lookup: |Δ| ≤ 1e-5 (+ golden fixture from the reference itself);
* convolutions: |Δ| ≤ 2e-5·sqrt(K) relative to the output scale (fp32, K-long sums);
* pose / resampling: ≤ 1e-4 px (float32 projective division).
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tests.helpers import golden, t

pytestmark = pytest.mark.gpu

orc = pytest.importorskip("oracle.scflow_oracle")


@pytest.fixture(scope="module")
def ops():
    from scflow_amd import ops as o
    return o


def close(a, b, atol, rtol=0.0, what=""):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    err = (a - b).abs()
    lim = atol + rtol * b.abs()
    bad = (err > lim)
    assert not bad.any(), f"{what}: max err {err.max().item():.3e} at {bad.nonzero()[0].tolist()}"


# ------------------------------------------------------------------------------ a1
@pytest.mark.parametrize("shape", [(2, 8, 8, 8), (2, 256, 32, 32), (1, 64, 24, 40), (1, 32, 64, 64)])
def test_corr_pyramid(ops, shape):
    g = torch.Generator().manual_seed(1)
    f1 = torch.randn(*shape, generator=g)
    f2 = torch.randn(*shape, generator=g)
    buf, lv = ops.corr_pyramid(f1.cuda(), f2.cuda(), 4)
    ref = orc.corr_pyramid(f1.double(), f2.double(), 4)
    for i, (a, b) in enumerate(zip(lv, ref)):
        close(a, b, 2e-5, 2e-5, f"level {i}")


@pytest.mark.parametrize("n,c,h,w,L", [(2, 256, 32, 32, 4), (1, 64, 64, 64, 4), (3, 16, 16, 24, 2),
                                       (2, 32, 32, 48, 3), (1, 8, 8, 8, 1)])
def test_corr_pyramid_tiled_bit_identical(ops, n, c, h, w, L):
    """The tiled pyramid (4×4 tiles per map, pooling in the GEMM epilogue) holds exactly the
    row-major pyramid's values — the same GEMM sums and AvgPool2d's sum order — at every level,
    and the tiled lookup gives exactly the row-major lookup's output (both align_corners)."""
    g = torch.Generator().manual_seed(5)
    f1 = torch.randn(n, c, h, w, generator=g).cuda()
    f2 = torch.randn(n, c, h, w, generator=g).cuda()
    _, lv = ops.corr_pyramid(f1, f2, L)
    tb = ops.corr_pyramid_tiled(f1, f2, L)
    for i, (a, b) in enumerate(zip(lv, ops.untile_pyramid(tb, n, h, w, L))):
        assert torch.equal(a, b), f"level {i}: max diff {(a - b).abs().max().item():.3e}"
    flow = ((torch.rand(n, 2, h, w, generator=g) - 0.5) * 1.5 * h).cuda()
    flow[:, :, 0, 0] = torch.tensor([0.5, -0.5])
    buf = ops.pyramid_buffer(lv, n, h, w)
    for ac in (True, False):
        if not ops.tiled_lookup_ok(h, w, L, 4, ac):
            continue
        ref = ops.corr_lookup(buf, flow, n, h, w, L, 4, align_corners=ac)
        got = ops.corr_lookup(tb, flow, n, h, w, L, 4, align_corners=ac, tiled=True)
        assert torch.equal(ref, got), f"tiled lookup ac={ac}: {(ref - got).abs().max().item():.3e}"
        # channels-last flow and 16-B aligned channels-last output: the persistent pipelined
        # kernel (corr_lookup_pipe_kernel), both layouts, against the per-batch kernel's NCHW
        K = L * 81
        nhwc = flow.permute(0, 2, 3, 1).contiguous()
        for pyr_buf, til in ((buf, False), (tb, True)):
            o = torch.full((n * h * w, K + 4), 7.0, device="cuda")
            ops.corr_lookup(pyr_buf, nhwc, n, h, w, L, 4, out=ops.Chan(o, 4, K), flow_layout="nhwc",
                            align_corners=ac, tiled=til)
            o2 = o[:, 4:].reshape(n, h, w, K).permute(0, 3, 1, 2)
            assert torch.equal(ref, o2), f"pipelined lookup tiled={til} ac={ac}"
            assert (o[:, :4] == 7).all()


def test_corr_pyramid_golden(ops):
    gd = golden("ops")
    _, lv = ops.corr_pyramid(t(gd["pyr_f1"]).cuda(), t(gd["pyr_f2"]).cuda(), 4)
    for i, a in enumerate(lv):
        close(a, t(gd[f"pyr_l{i}"]), 1e-5, 1e-5, f"golden level {i}")


# ------------------------------------------------------------------------------ a2
@pytest.mark.parametrize("radius", [4, 1])
def test_corr_lookup_golden(ops, radius):
    gd = golden("ops")
    _, lv = ops.corr_pyramid(t(gd["pyr_f1"]).cuda(), t(gd["pyr_f2"]).cuda(), 4)
    buf = ops.pyramid_buffer(lv, 2, 8, 8)
    out = ops.corr_lookup(buf, t(gd["lk_flow"]).cuda(), 2, 8, 8, 4, radius)
    close(out, t(gd[f"lk_r{radius}"]), 2e-5, 2e-5, "lookup vs reference fixture")


def test_corr_lookup_align_corners_false(ops):
    """CorrLookup(align_corners=False) (bilinear_sample's default, corr_lookup.py:35): the fixture from
    the reference's own module, then random flows on the LDS kernel (windowed and whole-map
    levels, 32² and 64²) and on the generic kernel (a windowed level narrower than 2r+1)."""
    from scflow_amd.modules import CorrLookup
    gd = golden("ops")
    _, lv = ops.corr_pyramid(t(gd["pyr_f1"]).cuda(), t(gd["pyr_f2"]).cuda(), 4)
    out = CorrLookup(radius=4, align_corners=False)(lv, t(gd["lk_flow"]).cuda())
    close(out, t(gd["lk_r4_ac0"]), 2e-5, 2e-5, "lookup align_corners=False vs reference fixture")
    g = torch.Generator().manual_seed(23)
    for n, h, w, L, r in ((2, 32, 32, 4, 4), (1, 64, 64, 4, 4), (2, 24, 20, 3, 4), (2, 16, 16, 2, 3)):
        f1 = torch.randn(n, 8, h, w, generator=g)
        f2 = torch.randn(n, 8, h, w, generator=g)
        flow = (torch.rand(n, 2, h, w, generator=g) - 0.5) * h
        flow[:, :, 0, 0] = torch.tensor([0.5, -0.5])
        buf, lv = ops.corr_pyramid(f1.cuda(), f2.cuda(), L)
        ref = orc.corr_lookup([x.cpu() for x in lv], flow, r, align_corners=False)
        got = ops.corr_lookup(buf, flow.cuda(), n, h, w, L, r, align_corners=False)
        close(got, ref, 1e-5, 1e-5, f"lookup align_corners=False {n}x{h}x{w} L{L} r{r}")


@pytest.mark.parametrize("n,h,w", [(2, 32, 32), (1, 64, 64), (3, 20, 28)])
def test_corr_lookup_random(ops, n, h, w):
    g = torch.Generator().manual_seed(2)
    f1 = torch.randn(n, 16, h, w, generator=g)
    f2 = torch.randn(n, 16, h, w, generator=g)
    flow = (torch.rand(n, 2, h, w, generator=g) - 0.5) * 2 * (h / 2)  # hits every padding case
    flow[:, :, 0, 0] = torch.tensor([0.5, -0.25])  # exact half-pixel taps
    buf, lv = ops.corr_pyramid(f1.cuda(), f2.cuda(), 4)
    ref = orc.corr_lookup([x.cpu() for x in lv], flow, 4)
    out = ops.corr_lookup(buf, flow.cuda(), n, h, w, 4, 4)
    close(out, ref, 1e-5, 1e-5, "lookup NCHW")
    # channels-last variant into a wider buffer at an offset
    K = 4 * 81
    wide = torch.full((n * h * w, K + 8), 7.0, device="cuda")
    nhwc_flow = flow.permute(0, 2, 3, 1).contiguous().cuda()
    ops.corr_lookup(buf, nhwc_flow, n, h, w, 4, 4, out=ops.Chan(wide, 4, K), flow_layout="nhwc")
    got = wide[:, 4:4 + K].view(n, h, w, K).permute(0, 3, 1, 2)
    close(got, ref, 1e-5, 1e-5, "lookup NHWC")
    assert (wide[:, :4] == 7).all() and (wide[:, 4 + K:] == 7).all()


@pytest.mark.parametrize("levels,radius,h,w", [(3, 2, 24, 40), (2, 3, 16, 16), (4, 1, 32, 48),
                                               (1, 4, 12, 12)])
def test_corr_lookup_levels_radii(ops, levels, radius, h, w):
    """Other pyramid depths / radii: whole-map LDS regions (maps narrower than the window) next
    to windowed ones, and channel counts L·(2r+1)² that are not a multiple of 4 (the 16-B store
    path's scalar tail), channels-last into a wider buffer."""
    g = torch.Generator().manual_seed(11)
    n = 2
    f1 = torch.randn(n, 8, h, w, generator=g)
    f2 = torch.randn(n, 8, h, w, generator=g)
    flow = (torch.rand(n, 2, h, w, generator=g) - 0.5) * 1.5 * h
    buf, lv = ops.corr_pyramid(f1.cuda(), f2.cuda(), levels)
    ref = orc.corr_lookup([x.cpu() for x in lv], flow, radius)
    K = levels * (2 * radius + 1) ** 2
    for off in (0, 4):
        wide = torch.full((n * h * w, (K + 15) // 4 * 4), 7.0, device="cuda")  # 16-B pixel stride
        ops.corr_lookup(buf, flow.permute(0, 2, 3, 1).contiguous().cuda(), n, h, w, levels, radius,
                        out=ops.Chan(wide, off, K), flow_layout="nhwc")
        got = wide[:, off:off + K].view(n, h, w, K).permute(0, 3, 1, 2)
        close(got, ref, 1e-5, 1e-5, f"lookup L={levels} r={radius} off={off}")
        assert (wide[:, :off] == 7).all() and (wide[:, off + K:] == 7).all()


# ------------------------------------------------------------------------------ convs
def _conv_case(ops, n, h, w, c0, c1, cout, k, pad, act, seed=0, bk=None):
    from scflow_amd.modules import ConvRunner
    g = torch.Generator().manual_seed(seed)
    x0 = torch.randn(n, c0, h, w, generator=g)
    x1 = torch.randn(n, c1, h, w, generator=g) if c1 else None
    conv = torch.nn.Conv2d(c0 + c1, cout, k, padding=pad)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / np.sqrt(conv.weight[0].numel()))
        conv.bias.copy_(torch.randn(cout, generator=g) * 0.1)
    xin = torch.cat([x0, x1], 1) if c1 else x0
    ref = F.conv2d(xin.double(), conv.weight.double(), conv.bias.double(), padding=pad)
    ref = {None: lambda v: v, "ReLU": torch.relu, "Sigmoid": torch.sigmoid, "Tanh": torch.tanh}[act](ref)
    convc = conv.cuda()
    M = n * h * w
    # inputs as channel slices of wider buffers (exercises pixel strides and offsets)
    b0 = torch.zeros(M, c0 + 4, device="cuda")
    ops.nchw_into(x0.cuda(), ops.Chan(b0, 4, c0))
    src1 = None
    if c1:
        b1 = torch.zeros(M, c1 + 8, device="cuda")
        ops.nchw_into(x1.cuda(), ops.Chan(b1, 8, c1))
        src1 = ops.Chan(b1, 8, c1)
    out = torch.full((M, cout + 3), -5.0, device="cuda")
    runner = ConvRunner([convc], act)
    if bk is not None:  # force the K-stage depth (otherwise the library's pick for the shape)
        runner._bk_shape, runner._bk = (n, h, w, c0, c1), bk
    runner.run(ops.Chan(b0, 4, c0), ops.Chan(out, 3, cout), n, h, w, src1=src1)
    got = ops.chan_to_nchw(ops.Chan(out, 3, cout), n, h, w)
    assert (out[:, :3] == -5).all()
    return got, ref


@pytest.mark.parametrize("case", [
    # (n, h, w, c0, c1, cout, k, pad, act)          variant
    (2, 32, 32, 324, 0, 256, 1, 0, "ReLU"),        # mfma 1×1 (corr_net.0, cin not a multiple of 16)
    (2, 32, 32, 256, 0, 192, 3, 1, "ReLU"),        # mfma 3×3 (corr_net.1)
    (2, 32, 32, 128, 256, 128, (1, 5), (0, 2), "Tanh"),  # mfma 1×5, two sources (GRU q)
    (2, 32, 32, 384, 0, 256, (5, 1), (2, 0), "Sigmoid"),  # mfma 5×1 (GRU z|r)
    (2, 32, 32, 192, 64, 126, 3, 1, "ReLU"),       # mfma, cout not a multiple of 64 (out_net)
    (2, 32, 32, 64, 0, 32, 3, 1, None),            # mfma, cout 32
    (1, 64, 64, 128, 0, 64, 3, 1, "ReLU"),         # mfma at the 512² feature size
    (2, 32, 32, 2, 0, 128, 7, 3, "ReLU"),          # small-cin 7×7
    (2, 32, 32, 1, 0, 64, 3, 1, "ReLU"),           # small-cin 3×3, 1 channel
    (2, 32, 32, 256, 0, 2, 3, 1, None),            # thin 3×3 → 2
    (2, 32, 32, 256, 0, 1, 1, 0, "Sigmoid"),       # thin 1×1 → 1
    (1, 64, 64, 256, 0, 2, 3, 1, None),            # thin 3×3 → 2 at the 512² feature size (32-column tiles)
    (2, 64, 64, 128, 0, 1, 3, 1, "Sigmoid"),       # thin 3×3 → 1, 64-wide
    (16, 32, 32, 324, 0, 256, 1, 0, "ReLU"),       # 1×1 kernel (128-row tiles: corr_net.0 at B=16)
    (13, 32, 32, 196, 60, 320, 1, 0, "Tanh"),      # 1×1 kernel, two sources, 5 channel blocks
    (2, 17, 15, 324, 0, 256, 1, 0, "ReLU"),        # wide 1×1: pixels not a multiple of 64
    (3, 32, 32, 256, 0, 192, 1, 0, None),          # wide 1×1: K 256, three channel blocks of 64
    (2, 32, 32, 128, 0, 100, 1, 0, "Tanh"),        # wide 1×1: K 128, cout not a multiple of 32
])
def test_conv2d_variants(ops, case):
    n, h, w, c0, c1, cout, k, pad, act = case
    got, ref = _conv_case(ops, n, h, w, c0, c1, cout, k, pad, act)
    kk = (c0 + c1) * (np.prod(k) if isinstance(k, tuple) else k * k)
    close(got, ref, 2e-6 * np.sqrt(kk) * 4, 1e-5, f"conv {case}")


@pytest.mark.parametrize("wgs", ["0", "1"])
@pytest.mark.parametrize("case", [
    (12, 64, 64, 2, 0, 128, 7, 3, "ReLU"),   # 768 tiles > 2 per CU: workgroups walk 2-3 tiles
    (9, 64, 64, 1, 0, 64, 3, 1, "ReLU"),     # mask encoder.0 shape, a ragged last round
    (17, 32, 32, 2, 0, 128, 7, 3, None),     # 272 tiles at W = 32
    (3, 64, 64, 2, 0, 100, 3, 1, "Tanh"),    # cout not a multiple of 32 (masked columns)
])
def test_conv2d_smallcin_tile_walk(ops, case, wgs, monkeypatch):
    """The small-cin MFMA conv with workgroups walking several tiles (round 6: the grid capped at
    SCFLOW_SMALLCIN_WGS per CU, 2 by default; 1 forces ≥ 3 tiles per workgroup here), the next
    tile's halo double-buffered in LDS — against the fp64 conv."""
    from scflow_amd._lib import reload_switches
    if wgs != "0":
        monkeypatch.setenv("SCFLOW_SMALLCIN_WGS", wgs)
    reload_switches()
    try:
        n, h, w, c0, c1, cout, k, pad, act = case
        got, ref = _conv_case(ops, n, h, w, c0, c1, cout, k, pad, act, seed=3)
    finally:
        monkeypatch.delenv("SCFLOW_SMALLCIN_WGS", raising=False)
        reload_switches()
    close(got, ref, 2e-6 * np.sqrt(c0 * k * k) * 4, 1e-5, f"small-cin conv {case} wgs={wgs}")


@pytest.mark.parametrize("thinz", ["1", "0"])
@pytest.mark.parametrize("case", [
    (16, 32, 32, 256, 0, 2, 3, 1, None),      # XHead flow predictor, configs[1]
    (3, 64, 64, 256, 0, 2, 3, 1, None),       # configs[4] width (4-row workgroups)
    (2, 64, 64, 256, 0, 1, 3, 1, "Sigmoid"),  # one output
    (5, 32, 32, 256, 0, 1, 3, 1, "Tanh"),
    (16, 32, 32, 256, 0, 1, 1, 0, "Sigmoid"),  # XHead mask predictor 1×1, configs[1]
    (3, 64, 64, 256, 0, 1, 1, 0, "Sigmoid"),   # and at configs[4] width
])
def test_conv2d_thin_contraction(ops, case, thinz, monkeypatch):
    """The thin 3×3 conv as a channel contraction on MFMA (round 6, conv_thinz.h: Z = X·W per input
    pixel, then the taps summed over Z) and the LDS kernels it replaces (SCFLOW_THINZ=0), against
    the fp64 conv (image borders: zero padding in both directions)."""
    from scflow_amd._lib import reload_switches
    monkeypatch.setenv("SCFLOW_THINZ", thinz)
    reload_switches()
    try:
        n, h, w, c0, c1, cout, k, pad, act = case
        got, ref = _conv_case(ops, n, h, w, c0, c1, cout, k, pad, act, seed=11)
    finally:
        monkeypatch.delenv("SCFLOW_THINZ")
        reload_switches()
    close(got, ref, 2e-6 * np.sqrt(c0 * k * k) * 4, 1e-5, f"thin conv {case} thinz={thinz}")


@pytest.mark.parametrize("bk", [8, 16])
@pytest.mark.parametrize("case", [
    (2, 32, 32, 324, 0, 256, 1, 0, "ReLU"),
    (2, 32, 32, 256, 0, 192, 3, 1, "ReLU"),
    (2, 32, 32, 128, 256, 128, (1, 5), (0, 2), "Tanh"),
    (2, 32, 32, 200, 56, 126, 3, 1, "ReLU"),        # source boundary inside an 8-deep stage pair
    (1, 64, 64, 128, 0, 64, 3, 1, "ReLU"),
])
def test_conv2d_mfma_stage_depths(ops, case, bk):
    """Both K-stage depths (weights packed for 8- and 16-channel stages) give the conv."""
    n, h, w, c0, c1, cout, k, pad, act = case
    got, ref = _conv_case(ops, n, h, w, c0, c1, cout, k, pad, act, bk=bk)
    kk = (c0 + c1) * (np.prod(k) if isinstance(k, tuple) else k * k)
    close(got, ref, 2e-6 * np.sqrt(kk) * 4, 1e-5, f"conv {case} bk={bk}")


def test_conv_pick_bk_prefers_resident_grids(ops, monkeypatch):
    """Host query: 3×3 / 1×5 / 5×1 stride-1 convs take the Winograd kernels (F(4×4,3×3) for the wide
    3×3 ones); the 1×1 corr_net.0
    conv the wide 1×1 kernel up to two workgroups per CU; a two-source 1×1 conv 16-deep stages
    of the direct conv."""
    from scflow_amd._lib import CONV_WINO, CONV_WINO4
    # the wide 3×3 convs (≥ 160 output channels) take F(4×4,3×3), narrower ones F(2×2,3×3)
    assert ops.conv_pick_bk(16, 32, 32, 256, 0, 192, 3, 3, 1, 1) == CONV_WINO4  # corr_net.1
    assert ops.conv_pick_bk(16, 32, 32, 128, 0, 512, 3, 3, 1, 1) == CONV_WINO4  # XHead hidden
    assert ops.conv_pick_bk(16, 32, 32, 192, 64, 126, 3, 3, 1, 1) == CONV_WINO  # out_net
    # configs[4] (64×64 maps, multi-round grids): out_net on F(4×4,3×3), the 64-wide ones not
    assert ops.conv_pick_bk(32, 64, 64, 192, 64, 126, 3, 3, 1, 1) == CONV_WINO4
    assert ops.conv_pick_bk(32, 64, 64, 128, 0, 64, 3, 3, 1, 1) == CONV_WINO
    assert ops.conv_pick_bk(16, 32, 32, 128, 128, 256, 1, 5, 0, 2) == CONV_WINO
    assert ops.conv_pick_bk(16, 32, 32, 128, 128, 256, 5, 1, 2, 0) == CONV_WINO
    from scflow_amd._lib import CONV_1X1W
    assert ops.conv_pick_bk(16, 32, 32, 324, 0, 256, 1, 1, 0, 0) == CONV_1X1W  # corr_net.0
    # configs[4]'s corr_net.0 (2048 workgroups) stays on conv1x1_kernel (measured faster there)
    assert ops.conv_pick_bk(32, 64, 64, 324, 0, 256, 1, 1, 0, 0) not in (CONV_1X1W, CONV_WINO)
    assert ops.conv_pick_bk(16, 32, 32, 196, 60, 256, 1, 1, 0, 0) == 16  # two sources: direct
    assert ops.conv_pick_bk(2, 20, 20, 64, 0, 64, 3, 3, 1, 1) != CONV_WINO  # width not tileable


@pytest.mark.parametrize("case", [
    # (n, h, w, c0, c1, cout, k, pad, act)
    (2, 32, 32, 256, 0, 192, 3, 1, "ReLU"),        # corr_net.1
    (2, 32, 32, 192, 64, 126, 3, 1, "ReLU"),       # out_net: two sources, cout not /32
    (2, 32, 32, 128, 0, 512, 3, 1, "ReLU"),        # XHead hidden convs (flow ‖ mask)
    (2, 32, 32, 64, 0, 32, 3, 1, None),            # mask_encoder.1
    (3, 32, 32, 12, 20, 40, 3, 1, "Tanh"),         # channels not /8 per source, cout 40
    (1, 64, 64, 128, 0, 64, 3, 1, "ReLU"),         # 512² feature size
    (2, 64, 64, 36, 4, 100, 3, 1, None),           # W=64, ragged channels
    (16, 32, 32, 128, 0, 512, 3, 1, "ReLU"),       # B=16 heads: 64-channel workgroups
    (16, 32, 32, 256, 0, 192, 3, 1, "ReLU"),       # B=16 corr_net.1: 96-channel workgroups
    # F(4,5), 1×5 / 5×1
    (2, 32, 32, 384, 0, 256, (1, 5), (0, 2), "Sigmoid"),    # GRU z|r
    (2, 32, 32, 128, 256, 128, (5, 1), (2, 0), "Tanh"),     # GRU q, two sources
    (3, 32, 32, 20, 44, 72, (1, 5), (0, 2), None),          # channels not /16 per source
    (3, 32, 32, 20, 44, 72, (5, 1), (2, 0), None),
    (1, 64, 64, 128, 128, 256, (1, 5), (0, 2), "ReLU"),     # 512² feature size
    (1, 64, 64, 128, 128, 256, (5, 1), (2, 0), "ReLU"),     # two column blocks per row
    (16, 32, 32, 128, 128, 256, (5, 1), (2, 0), None),      # B=16: 64-channel workgroups
])
def test_conv2d_winograd(ops, case):
    """Winograd F(2×2,3×3) / F(4,5) kernels vs an fp64 direct conv (fp32 tolerance of the direct
    kernel; F(4,5)'s fp32 error is ≈2× the direct conv's, within the same bound)."""
    from scflow_amd._lib import CONV_WINO
    n, h, w, c0, c1, cout, k, pad, act = case
    got, ref = _conv_case(ops, n, h, w, c0, c1, cout, k, pad, act, bk=CONV_WINO)
    kk = (c0 + c1) * (np.prod(k) if isinstance(k, tuple) else k * k)
    close(got, ref, 2e-6 * np.sqrt(kk) * 4, 1e-5, f"winograd conv {case}")


@pytest.mark.parametrize("case", [
    # (n, h, w, c0, c1, cout, act)
    (2, 32, 32, 256, 0, 192, "ReLU"),        # corr_net.1
    (2, 32, 32, 192, 64, 126, "ReLU"),       # out_net: two sources, cout not /32
    (16, 32, 32, 128, 0, 512, "ReLU"),       # B=16 XHead hidden convs (flow ‖ mask)
    (3, 32, 32, 12, 20, 40, "Tanh"),         # channels not /8 per source, cout 40
    (1, 64, 64, 128, 0, 64, None),           # 512² feature size
    (1, 20, 12, 36, 4, 100, "Sigmoid"),      # 15 tiles: a partial tile block, ragged channels
    (2, 128, 128, 64, 0, 64, "ReLU"),        # encoder width
])
@pytest.mark.parametrize("xcd", ["0", "2"])
@pytest.mark.parametrize("depth", ["1", "2"])
def test_conv2d_winograd_f4x4(ops, case, depth, xcd, monkeypatch):
    """Winograd F(4×4,3×3) (SCFLOW_CONV_WINO4: input transform launch + point GEMMs with the
    output transform in the epilogue) vs an fp64 direct conv, with one and two sub-steps of the
    GEMM's operands in flight (SCFLOW_WINO4_DEPTH; two needs an even sub-step count, else one).
    Tolerance: its fp32 error is ≈ 10× the direct conv's (points {0, ±1, 2, −½, ∞}; 1.3e-5 of
    outputs ≈ 4 at 256 channels in a numpy restatement) — 5e-5·√(K/256) absolute on unit-scale
    outputs.  Both GEMM block orders (SCFLOW_WINO4_XCD: 0 linear, 2 XCD-blocked at every size)."""
    from scflow_amd._lib import CONV_WINO4
    from scflow_amd._lib import reload_switches
    monkeypatch.setenv("SCFLOW_WINO4_DEPTH", depth)
    monkeypatch.setenv("SCFLOW_WINO4_XCD", xcd)
    reload_switches()
    n, h, w, c0, c1, cout, act = case
    try:
        got, ref = _conv_case(ops, n, h, w, c0, c1, cout, 3, 1, act, bk=CONV_WINO4)
    finally:
        monkeypatch.delenv("SCFLOW_WINO4_DEPTH")
        monkeypatch.delenv("SCFLOW_WINO4_XCD")
        reload_switches()
    kk = (c0 + c1) * 9
    close(got, ref, 5e-5 * np.sqrt(kk / 256 / 9) * 3 + 1e-6, 1e-5, f"F(4x4,3x3) conv {case}")


def test_conv2d_winograd_f4x4_fused_epilogue(ops):
    """F(4×4,3×3) with the encoder's fused forms: input InstanceNorm + ReLU on load, eval-BN
    affine, residual and bias map, against fp64 (and the workspace query)."""
    from scflow_amd import _lib
    from scflow_amd.modules import ConvRunner
    g = torch.Generator().manual_seed(23)
    n, h, w, c, cout = 2, 32, 32, 64, 96
    x = torch.randn(n, h, w, c, generator=g)
    isc, ish = torch.rand(n, c, generator=g) + 0.5, torch.randn(n, c, generator=g) * 0.2
    osc, osh = torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g) * 0.2
    res = torch.randn(n, h, w, cout, generator=g)
    bm = torch.randn(n, h, w, cout, generator=g)
    conv = torch.nn.Conv2d(c, cout, 3, padding=1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / np.sqrt(9 * c))
        conv.bias.copy_(torch.randn(cout, generator=g) * 0.1)
    xa = torch.relu(x.double() * isc.double()[:, None, None] + ish.double()[:, None, None])
    ref = F.conv2d(xa.permute(0, 3, 1, 2), conv.weight.double(), conv.bias.double(), padding=1)
    ref = ref.permute(0, 2, 3, 1) * osc.double() + osh.double() + res.double() + bm.double()
    ref = torch.relu(ref)
    r = ConvRunner([conv.cuda()], "ReLU")
    packed, bias = r.packed(c, 0, w, _lib.CONV_WINO4)
    out = torch.empty(n * h * w, cout, device="cuda")
    a = ops.conv2d_args(ops.Chan.whole(x.cuda().reshape(-1, c)), packed, bias, n, h, w, cout, 3, 3,
                        1, 1, "ReLU", out=ops.Chan.whole(out), bias_map=ops.Chan.whole(bm.cuda().reshape(-1, cout)),
                        bk=_lib.CONV_WINO4, in_scale=isc.cuda(), in_shift=ish.cuda(),
                        out_scale=osc.cuda(), out_shift=osh.cuda(),
                        res=ops.Chan.whole(res.cuda().reshape(-1, cout)))
    assert a.ws_bytes == -(-n * h * w // 16 // 32) * 8 * 36 * 1024
    ops.check(_lib.load().scflow_conv2d(ctypes.byref(a), ops.raw_stream(0)), "scflow_conv2d")
    torch.cuda.synchronize()
    close(out.view(n, h, w, cout), ref, 2e-4, 1e-5, "F(4x4,3x3) fused epilogue")
    # a workspace that is too small is refused
    a.ws_bytes -= 16
    assert _lib.load().scflow_conv2d(ctypes.byref(a), ops.raw_stream(0)) != 0


@pytest.mark.parametrize("k,pad", [((1, 5), (0, 2)), ((5, 1), (2, 0))])
@pytest.mark.parametrize("bk", [16, 2])
@pytest.mark.parametrize("n", [2, 16])
def test_conv_gru_epilogues(ops, k, pad, bk, n):
    """GRU z|r and q epilogues (with a bias map) on the direct (bk 16) and F(4,5) Winograd
    (bk 2) kernels vs fp64: z = σ(.), r·h, then h ← (1−z)h + z·tanh(q).  n=16 is BASELINE
    configs[1]'s batch: the Winograd launch there takes 64-channel workgroups
    (conv_wino5_kernel<·,32,2,GRU_ZR/GRU_Q>, the instantiation bench.py times)."""
    from scflow_amd._lib import EPI_GRU_Q, EPI_GRU_ZR
    from scflow_amd.modules import ConvRunner
    h, w, hc = 32, 32, 128
    g = torch.Generator().manual_seed(11)
    hid = torch.tanh(torch.randn(n * h * w, hc, generator=g))
    x = torch.randn(n * h * w, 128, generator=g)
    bmap = torch.randn(n * h * w, 3 * hc, generator=g) * 0.3
    czr = torch.nn.Conv2d(2 * hc, 2 * hc, k, padding=pad)
    cq = torch.nn.Conv2d(2 * hc, hc, k, padding=pad)
    for c in (czr, cq):
        with torch.no_grad():
            c.weight.copy_(torch.randn(c.weight.shape, generator=g) / np.sqrt(c.weight[0].numel()))
            c.bias.copy_(torch.randn(c.bias.shape, generator=g) * 0.1)

    def nchw(t):
        return t.view(n, h, w, -1).permute(0, 3, 1, 2).double()
    hx = torch.cat([nchw(hid), nchw(x)], 1)
    pre = F.conv2d(hx, czr.weight.double(), czr.bias.double(), padding=pad) + nchw(bmap[:, :2 * hc])
    z, r = torch.sigmoid(pre[:, :hc]), torch.sigmoid(pre[:, hc:])
    q = torch.tanh(F.conv2d(torch.cat([r * nchw(hid), nchw(x)], 1), cq.weight.double(), cq.bias.double(),
                            padding=pad) + nchw(bmap[:, 2 * hc:]))
    href = (1 - z) * nchw(hid) + z * q

    dh, dx, db = hid.cuda(), x.cuda(), bmap.cuda()
    gate = torch.empty(n * h * w, hc, device="cuda")
    rh = torch.empty(n * h * w, hc, device="cuda")
    rz, rq = ConvRunner([czr.cuda()], None), ConvRunner([cq.cuda()], None)
    for r_ in (rz, rq):
        r_._bk_shape, r_._bk = (n, h, w, hc, 128), bk
    rz.run(ops.Chan.whole(dh), None, n, h, w, src1=ops.Chan.whole(dx), epilogue=EPI_GRU_ZR,
           gate=ops.Chan.whole(gate), rh=ops.Chan.whole(rh), hid=ops.Chan.whole(dh),
           bias_map=ops.Chan(db, 0, 2 * hc))
    close(ops.chan_to_nchw(ops.Chan.whole(gate), n, h, w), z, 2e-5, 1e-5, "z")
    close(ops.chan_to_nchw(ops.Chan.whole(rh), n, h, w), r * nchw(hid), 2e-5, 1e-5, "r·h")
    rq.run(ops.Chan.whole(rh), None, n, h, w, src1=ops.Chan.whole(dx), epilogue=EPI_GRU_Q,
           gate=ops.Chan.whole(gate), hid=ops.Chan.whole(dh), bias_map=ops.Chan(db, 2 * hc, hc))
    close(ops.chan_to_nchw(ops.Chan.whole(dh), n, h, w), href, 3e-5, 1e-5, "h")


def test_conv_gru_module(ops):
    """ConvGRU (SeqConv, 128 hidden, 256 input) through the fused z|r and q launches."""
    from scflow_amd import synthetic
    from scflow_amd.modules import ConvGRU
    gru = ConvGRU(128, 256, "SeqConv")
    synthetic.fill_module_(gru, seed=4)
    g = torch.Generator().manual_seed(5)
    h = torch.tanh(torch.randn(2, 128, 32, 32, generator=g))
    x = torch.randn(2, 256, 32, 32, generator=g)
    sd = {k: v for k, v in gru.state_dict().items()}
    ref = orc.conv_gru({k: v.double() for k, v in sd.items()}, h.double(), x.double(), prefix="")
    out = gru.cuda()(h.cuda(), x.cuda())
    close(out, ref, 5e-5, 1e-5, "ConvGRU")


def test_conv_unsupported_shape_raises(ops):
    from scflow_amd._lib import ScflowError
    from scflow_amd.modules import ConvRunner
    conv = torch.nn.Conv2d(64, 64, 3, padding=1).cuda()
    b = torch.zeros(1 * 20 * 20, 64, device="cuda")
    with pytest.raises(ScflowError):
        ConvRunner([conv], None).run(ops.Chan.whole(b), ops.Chan.whole(b.clone()), 1, 20, 20)


# ------------------------------------------------------------------------------ pose / resampling
def test_pose_golden(ops):
    gd = golden("ops")
    R0, t0, K = (t(gd["pose_ref_rotation"]), t(gd["pose_ref_translation"]), t(gd["pose_internel_k"]))
    depth = t(gd["pose_depth"])
    Ro, to = ops.pose_update(t(gd["pose_drot"]).cuda(), t(gd["pose_dt"]).cuda(), R0.cuda(), t0.cuda())
    close(Ro, t(gd["pose_R1"]), 1e-6, 1e-6, "R")
    close(to, t(gd["pose_t1"]), 1e-4, 1e-6, "t")
    pts = ops.lift_points(depth.cuda(), K.cuda(), R0.cuda(), t0.cuda())
    for inv in (0, 400):
        fl = ops.pose_flow(Ro, to, K.cuda(), pts, float(inv))
        close(fl, t(gd[f"pose_flow_inv{inv}"]), 2e-3, 1e-4, f"pose flow inv={inv}")
    # fused update + flow
    Rf, tf = torch.empty_like(Ro), torch.empty_like(to)
    flf = torch.empty(3, 2, 64, 64, device="cuda")
    ops.pose_update_flow(t(gd["pose_drot"]).cuda(), t(gd["pose_dt"]).cuda(), R0.cuda(), t0.cuda(),
                         K.cuda(), pts, Rf, tf, flf, 400.0)
    close(Rf, Ro, 0, 0, "fused R")
    close(flf, t(gd["pose_flow_inv400"]), 2e-3, 1e-4, "fused flow")


def test_pose_full_res_vs_oracle(ops):
    from scflow_amd import synthetic
    sc = synthetic.make_scene(4, 256, seed=9)
    R0, t0, K, depth = (t(sc[k]) for k in ("ref_rotation", "ref_translation", "internel_k", "depth"))
    g = torch.Generator().manual_seed(3)
    drot = torch.tensor([[1.0, 0, 0, 0, 1.0, 0]]).repeat(4, 1) + 0.03 * torch.randn(4, 6, generator=g)
    dt = 0.05 * torch.randn(4, 3, generator=g)
    Rr, tr = orc.pose_update(drot.double(), dt.double(), R0.double(), t0.double())
    pts_r, valid = orc.lift_points(depth.double(), K.double(), R0.double(), t0.double())
    ref = orc.pose_flow(Rr, tr, K.double(), pts_r, valid, 0.0)
    pts = ops.lift_points(depth.cuda(), K.cuda(), R0.cuda(), t0.cuda())
    Ro, to = torch.empty(4, 3, 3, device="cuda"), torch.empty(4, 3, device="cuda")
    fl = torch.empty(4, 2, 256, 256, device="cuda")
    ops.pose_update_flow(drot.cuda(), dt.cuda(), R0.cuda(), t0.cuda(), K.cuda(), pts, Ro, to, fl, 0.0)
    close(Ro, Rr, 2e-6, 0, "R")
    close(fl, ref, 5e-3, 1e-5, "flow")
    assert ((fl.cpu() == 0) == ~valid[:, None].expand(-1, 2, -1, -1)).all()


def test_pose_update_quaternion(ops):
    """Quaternion (x, y, z, w) delta rotations through pose_update, pose_update_flow and the
    fused pose_step, against the oracle (pose.py:132-133; kornia absent → parity unpinned
    against the reference, the oracle's convention is checked against scipy)."""
    from scflow_amd import synthetic
    sc = synthetic.make_scene(3, 64, seed=4)
    R0, t0, K, depth = (t(sc[k]).cuda() for k in ("ref_rotation", "ref_translation", "internel_k", "depth"))
    g = torch.Generator().manual_seed(8)
    q = torch.tensor([[0.0, 0, 0, 1.0]]).repeat(3, 1) + 0.1 * torch.randn(3, 4, generator=g)
    q[2] *= 3.0  # un-normalised
    dt = 0.05 * torch.randn(3, 3, generator=g)
    Rr, tr = orc.pose_update(q.double(), dt.double(), R0.cpu().double(), t0.cpu().double())
    Ro, to = ops.pose_update(q.cuda(), dt.cuda(), R0, t0)
    close(Ro, Rr, 2e-6, 0, "R quaternion")
    close(to, tr, 1e-5, 1e-6, "t quaternion")
    pts = ops.lift_points(depth, K, R0, t0)
    Rf, tf = torch.empty_like(Ro), torch.empty_like(to)
    fl = torch.empty(3, 2, 64, 64, device="cuda")
    ops.pose_update_flow(q.cuda(), dt.cuda(), R0, t0, K, pts, Rf, tf, fl, 0.0)
    close(Rf, Ro, 0, 0, "fused R quaternion")
    pts_r, valid = orc.lift_points(depth.cpu().double(), K.cpu().double(), R0.cpu().double(),
                                   t0.cpu().double())
    close(fl, orc.pose_flow(Rr, tr, K.cpu().double(), pts_r, valid, 0.0), 5e-3, 1e-5, "flow quaternion")


@pytest.mark.parametrize("S,s,nxt", [(256, 32, True), (256, 32, False), (128, 16, True)])
def test_pose_step_matches_separate_launches(ops, S, s, nxt):
    """scflow_pose_step (the decoder's fused iteration tail) is bit-identical to
    pose_update_flow + flow_upsample + flow_downsample of the new flow."""
    from scflow_amd import synthetic
    n = 3
    sc = synthetic.make_scene(n, S, seed=5)
    R0, t0, K, depth = (t(sc[k]).cuda() for k in ("ref_rotation", "ref_translation", "internel_k",
                                                   "depth"))
    g = torch.Generator().manual_seed(8)
    drot = (torch.tensor([[1.0, 0, 0, 0, 1.0, 0]]).repeat(n, 1) +
            0.03 * torch.randn(n, 6, generator=g)).cuda()
    dt = (0.05 * torch.randn(n, 3, generator=g)).cuda()
    pts = ops.lift_points(depth, K, R0, t0)
    lr = torch.randn(n * s * s, 2, generator=g).cuda()
    delta = torch.randn(n * s * s, 2, generator=g).cuda()
    mask = torch.rand(n * s * s, 1, generator=g).cuda()
    scale = S // s
    # separate launches
    Ra, ta = torch.empty(n, 3, 3, device="cuda"), torch.empty(n, 3, device="cuda")
    fa = torch.empty(n, 2, S, S, device="cuda")
    ops.pose_update_flow(drot, dt, R0, t0, K, pts, Ra, ta, fa, 400.0)
    upa, ma = torch.empty(n, 2, S, S, device="cuda"), torch.empty(n, 1, S, S, device="cuda")
    ops.flow_upsample(lr, delta, mask, n, s, s, S, S, float(scale), upa, ma)
    nxa, hxa = torch.empty(n * s * s, 2, device="cuda"), torch.zeros(n * s * s, 6, device="cuda")
    ops.flow_downsample(fa, ops.Chan.whole(nxa), s, s, 1.0 / scale, out1=ops.Chan(hxa, 4, 2))
    # one launch
    Rb, tb = torch.empty_like(Ra), torch.empty_like(ta)
    fb, upb, mb = torch.empty_like(fa), torch.empty_like(upa), torch.empty_like(ma)
    nxb, hxb = torch.full_like(nxa, 7.0), torch.zeros_like(hxa)
    ops.pose_step(drot, dt, R0, t0, K, pts, Rb, tb, fb, 400.0, lr, delta, mask, upb, mb, s, s,
                  float(scale), lr_next=ops.Chan.whole(nxb) if nxt else None,
                  hx_next=ops.Chan(hxb, 4, 2) if nxt else None)
    torch.cuda.synchronize()
    for a, b, nm in ((Ra, Rb, "R"), (ta, tb, "t"), (fa, fb, "flow"), (upa, upb, "flow ×8"),
                     (ma, mb, "mask ×8")):
        assert torch.equal(a, b), nm
    if nxt:
        assert torch.equal(nxa, nxb), "next ↓8 flow"
        assert torch.equal(hxa, hxb), "next ↓8 flow (second output)"
    else:
        assert (nxb == 7.0).all()
    with pytest.raises(ValueError):
        ops.pose_step(drot, dt, R0, t0, K, pts, Rb, tb, fb, 400.0, lr, delta, mask, upb, mb, s, s,
                      float(scale), lr_next=ops.Chan.whole(lr))
    # the decoder's deferred full-resolution part from the updated pose (no update, 4 pixels per
    # thread): the same outputs bit for bit
    fc, upc, mc = torch.empty_like(fa), torch.empty_like(upa), torch.empty_like(ma)
    ops.pose_step_given(Rb, tb, K, pts, fc, 400.0, lr, delta, mask, upc, mc, s, s, float(scale))
    torch.cuda.synchronize()
    for a, b, nm in ((fa, fc, "flow (given pose)"), (upa, upc, "flow ×8 (given pose)"),
                     (ma, mc, "mask ×8 (given pose)")):
        assert torch.equal(a, b), nm


@pytest.mark.parametrize("rch,parts", [(6, 2), (6, 3), (4, 3)])
def test_pose_step_heads_fused(ops, rch, parts):
    """scflow_pose_step_heads (the pose head's label[0] rotation / translation heads computed in
    the pose step's launch, from the last FC's K-split partial sums) against the heads in fp64
    (relu(Σ partials + bias) · W_cls + b_cls) within 1e-5, and the pose step's outputs against
    scflow_pose_step on those deltas (the same update arithmetic: within fp32 rounding of the
    deltas)."""
    from scflow_amd import synthetic
    n, S, s, k, ncls, split = 3, 256, 32, 256, 21, 4
    sc = synthetic.make_scene(n, S, seed=6)
    R0, t0, K, depth = (t(sc[key]).cuda() for key in ("ref_rotation", "ref_translation",
                                                      "internel_k", "depth"))
    g = torch.Generator().manual_seed(9)
    x = (0.1 * torch.randn(split, n, k, generator=g)).cuda()
    xb = (0.05 * torch.randn(k, generator=g)).cuda()
    Wr = (0.01 * torch.randn(rch * ncls, k, generator=g)).cuda()
    br = torch.tensor(([1.0, 0, 0, 0, 1.0, 0] if rch == 6 else [0, 0, 0, 1.0]) * ncls).cuda()
    Wt = (0.01 * torch.randn(3 * ncls, k, generator=g)).cuda()
    bt = (0.01 * torch.randn(3 * ncls, generator=g)).cuda()
    label = torch.tensor([7, 3, 12], dtype=torch.int64).cuda()  # label[0] = 7 for every sample
    mode = "exp"  # (the quaternion flag comes from drot's width)
    pts = ops.lift_points(depth, K, R0, t0)
    lr = torch.randn(n * s * s, 2, generator=g).cuda()
    delta = torch.randn(n * s * s, 2, generator=g).cuda()
    mask = torch.rand(n * s * s, 1, generator=g).cuda()
    drot = torch.full((n, rch), 5.0, device="cuda")
    dt = torch.full((n, 3), 5.0, device="cuda")
    Rb, tb = torch.empty(n, 3, 3, device="cuda"), torch.empty(n, 3, device="cuda")
    fb, upb = torch.empty(n, 2, S, S, device="cuda"), torch.empty(n, 2, S, S, device="cuda")
    mb = torch.empty(n, 1, S, S, device="cuda")
    nxb = torch.empty(n * s * s, 2, device="cuda")
    ops.pose_step(drot, dt, R0, t0, K, pts, Rb, tb, fb, 400.0, lr, delta, mask, upb, mb, s, s, 8.0,
                  lr_next=ops.Chan.whole(nxb), depth_transform=mode, parts=parts,
                  heads=(x, split, xb, k, Wr, br, rch, Wt, bt, label, ncls))
    torch.cuda.synchronize()
    xr = torch.relu(x.double().sum(0) + xb.double())
    c = 7
    ref_r = xr @ Wr.double()[c * rch:(c + 1) * rch].T + br.double()[c * rch:(c + 1) * rch]
    ref_t = xr @ Wt.double()[c * 3:(c + 1) * 3].T + bt.double()[c * 3:(c + 1) * 3]
    np.testing.assert_allclose(drot.cpu().double().numpy(), ref_r.cpu().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(dt.cpu().double().numpy(), ref_t.cpu().numpy(), rtol=1e-5, atol=1e-6)
    # the rest of the launch: scflow_pose_step on the deltas it wrote
    Ra, ta = torch.empty_like(Rb), torch.empty_like(tb)
    fa, upa, ma = torch.empty_like(fb), torch.empty_like(upb), torch.empty_like(mb)
    nxa = torch.empty_like(nxb)
    ops.pose_step(drot, dt, R0, t0, K, pts, Ra, ta, fa, 400.0, lr, delta, mask, upa, ma, s, s, 8.0,
                  lr_next=ops.Chan.whole(nxa), depth_transform=mode, parts=parts)
    torch.cuda.synchronize()
    assert torch.equal(Ra, Rb) and torch.equal(ta, tb)
    assert torch.equal(nxa, nxb)
    if parts & 1:
        assert torch.equal(fa, fb) and torch.equal(upa, upb) and torch.equal(ma, mb)
    from scflow_amd._lib import ScflowError
    with pytest.raises(ScflowError):  # rch must match the rotation mode
        ops.pose_step(drot, dt, R0, t0, K, pts, Rb, tb, fb, 400.0, lr, delta, mask, upb, mb, s, s,
                      8.0, depth_transform=mode, parts=1,
                      heads=(x, split, xb, k, Wr, br, 5, Wt, bt, label, ncls))


@pytest.mark.parametrize("S,s", [(256, 32), (512, 64), (100, 13)])
def test_flow_resampling(ops, S, s):
    g = torch.Generator().manual_seed(4)
    flow = torch.randn(2, 2, S, S, generator=g) * 5
    F2 = torch.empty(2 * s * s, 2, device="cuda")
    wide = torch.zeros(2 * s * s, 10, device="cuda")
    ops.flow_downsample(flow.cuda(), ops.Chan.whole(F2), s, s, 0.125, out1=ops.Chan(wide, 8, 2))
    # fp32 reference: ATen computes the align_corners source index (in-1)/(out-1)·dst in fp32 too
    ref = 0.125 * F.interpolate(flow, size=(s, s), mode="bilinear", align_corners=True)
    close(F2.view(2, s, s, 2).permute(0, 3, 1, 2), ref, 2e-6, 2e-6, "downsample")
    close(wide[:, 8:], F2, 0, 0, "downsample second output")
    if S == 8 * s:  # the decoder's own call form: 1/8 · interpolate(scale_factor=1/8)
        close(F2.view(2, s, s, 2).permute(0, 3, 1, 2), orc.downsample_flow(flow, 8), 2e-6,
              2e-6, "downsample (scale form)")
    delta = torch.randn(2 * s * s, 2, generator=g).cuda()
    mask = torch.rand(2 * s * s, 1, generator=g).cuda()
    fo = torch.empty(2, 2, S, S, device="cuda")
    mo = torch.empty(2, 1, S, S, device="cuda")
    ops.flow_upsample(F2, delta, mask, 2, s, s, S, S, 8.0, fo, mo)
    lr = (F2 + delta).view(2, s, s, 2).permute(0, 3, 1, 2).cpu()
    ref_up = 8 * F.interpolate(lr, size=(S, S), mode="bilinear", align_corners=True)
    close(fo, ref_up, 2e-5, 2e-6, "upsample flow")
    ref_m = F.interpolate(mask.view(2, s, s, 1).permute(0, 3, 1, 2).cpu(), size=(S, S),
                          mode="bilinear", align_corners=True)
    close(mo, ref_m, 1e-6, 1e-6, "upsample mask")


def test_transpose_roundtrip(ops):
    x = torch.randn(3, 37, 9, 11, device="cuda")
    buf = torch.zeros(3 * 9 * 11, 50, device="cuda")
    ops.nchw_into(x, ops.Chan(buf, 5, 37))
    back = ops.chan_to_nchw(ops.Chan(buf, 5, 37), 3, 9, 11)
    close(back, x, 0, 0, "roundtrip")
    close(buf[:, 5:42].view(3, 9, 11, 37).permute(0, 3, 1, 2), x, 0, 0, "nhwc")


def test_cpu_tensor_rejected(ops):
    from scflow_amd._lib import ScflowError
    with pytest.raises(ScflowError):
        ops.corr_pyramid(torch.randn(1, 8, 8, 8), torch.randn(1, 8, 8, 8), 4)


# ------------------------------------------------------------------------------ a7 pose head
@pytest.mark.parametrize("n,feat", [(16, 32), (32, 32), (3, 64)])
def test_pose_head_hip_vs_oracle(ops, n, feat):
    from scflow_amd import synthetic
    from scflow_amd.modules import MultiClassPoseHead
    head = MultiClassPoseHead(21, 224, "Basic", dict(type="GN", num_groups=32),
                              dict(type="ReLU"), feat_size=(feat, feat), rotation_mode="ortho6d")
    synthetic.fill_module_(head, seed=7)
    g = torch.Generator().manual_seed(8)
    x = torch.relu(torch.randn(n, 224, feat, feat, generator=g))
    label = torch.randint(0, 21, (n,), generator=g)
    sd = {f"pose_pred.{k}": v.double() for k, v in head.state_dict().items()}
    r_ref, t_ref = orc.pose_head(sd, x.double(), label, 21)
    head = head.cuda()
    # two-source form (h | features) as the decoder calls it
    hbuf = torch.zeros(n * feat * feat, 384, device="cuda")
    fbuf = torch.zeros(n * feat * feat, 96, device="cuda")
    ops.nchw_into(x[:, :128].contiguous().cuda(), ops.Chan(hbuf, 0, 128))
    ops.nchw_into(x[:, 128:].contiguous().cuda(), ops.Chan.whole(fbuf))
    r, tt = head.forward_hip(ops.Chan(hbuf, 0, 128), ops.Chan.whole(fbuf), n, feat, feat,
                             label.cuda())
    close(r, r_ref, 2e-5, 1e-5, "pose head rotation")
    close(tt, t_ref, 2e-5, 1e-5, "pose head translation")
    # NCHW module API
    r2, t2 = head(x.cuda(), label.cuda())
    close(r2, r, 1e-6, 1e-6, "pose head NCHW api")


def test_corr_lookup_far_out_of_bounds(ops):
    """Flows that push every window off the map (and half-pixel / integer edge cases) give the
    reference's zero padding, not garbage."""
    g = torch.Generator().manual_seed(9)
    f1 = torch.randn(1, 8, 16, 16, generator=g)
    f2 = torch.randn(1, 8, 16, 16, generator=g)
    buf, lv = ops.corr_pyramid(f1.cuda(), f2.cuda(), 4)
    flow = torch.zeros(1, 2, 16, 16)
    flow[0, 0, :4] = 1e4
    flow[0, 1, 4:8] = -1e4
    flow[0, :, 8:12] = torch.arange(4 * 16 * 2, dtype=torch.float32).view(2, 4, 16) * 0.25 - 8
    flow[0, :, 12:] = 15.0
    ref = orc.corr_lookup([x.cpu() for x in lv], flow, 4)
    out = ops.corr_lookup(buf, flow.cuda(), 1, 16, 16, 4, 4)
    close(out, ref, 1e-5, 1e-5, "lookup far / edge flows")
    assert (out[0, :, :8].abs().max() == 0)


@pytest.mark.parametrize("h,w", [(32, 32), (64, 64), (64, 32)])
def test_corr_lookup_tiled_far_out_of_bounds(ops, h, w):
    """The tiled lookup — 16×16 tile-aligned regions (maps ≤ 32²) or 12×12 regions filled from
    the tile rows of the taps' exact extent (larger maps) — on flows that push windows off the
    map, straddle its edges at every tile phase, sit on integers (zero flow: the coordinate round
    trip moves floors), or are not finite: exactly the row-major lookup's output (the same taps
    and arithmetic, only staged differently)."""
    g = torch.Generator().manual_seed(19)
    n, L = 2, 4
    f1 = torch.randn(n, 16, h, w, generator=g).cuda()
    f2 = torch.randn(n, 16, h, w, generator=g).cuda()
    _, lv = ops.corr_pyramid(f1, f2, L)
    buf = ops.pyramid_buffer(lv, n, h, w)
    tb = ops.corr_pyramid_tiled(f1, f2, L)
    flow = torch.zeros(n, 2, h, w)
    flow[0, 0, :4] = 1e4
    flow[0, 1, 4:8] = -1e4
    flow[0, :, 8:16] = torch.arange(8 * w * 2, dtype=torch.float32).view(2, 8, w) * 0.125 - 32
    flow[0, :, 22:] = 0.0
    flow[0, :, 16:20] = float(h) - 0.5
    flow[0, 0, 20, :8] = float("nan")
    flow[0, 1, 20, 8:16] = float("inf")
    flow[1] = (torch.rand(2, h, w, generator=g) - 0.5) * 3 * h
    flow = flow.cuda()
    for ac in (True, False):
        if not ops.tiled_lookup_ok(h, w, L, 4, ac):
            continue
        ref = ops.corr_lookup(buf, flow, n, h, w, L, 4, align_corners=ac)
        got = ops.corr_lookup(tb, flow, n, h, w, L, 4, align_corners=ac, tiled=True)
        assert torch.equal(torch.nan_to_num(ref, nan=123.0), torch.nan_to_num(got, nan=123.0)), \
            f"ac={ac}: {(ref - got).abs().nan_to_num().max().item():.3e}"


@pytest.mark.parametrize("n,h,w,seed,far", [(2, 32, 32, 61, False), (3, 32, 64, 62, True),
                                            (1, 64, 64, 63, False)])
def test_corr_lookup_conv1x1_fused_bit_identical(ops, n, h, w, seed, far):
    """scflow_corr_lookup_conv1x1 (lookup + corr_net.0 in one launch, features in LDS) equals the
    tiled lookup followed by the wide 1×1 conv bit for bit — random, far off-map, edge and
    non-finite flows included — and the conv against fp64 (the lookup against the oracle is
    pinned by the other lookup tests)."""
    from scflow_amd import _lib
    from scflow_amd.modules import ConvRunner
    g = torch.Generator().manual_seed(seed)
    f1 = torch.randn(n, 32, h, w, generator=g)
    f2 = torch.randn(n, 32, h, w, generator=g)
    flow = (torch.rand(n, h, w, 2, generator=g) - 0.5) * (4 * h if far else 0.6 * h)
    flow[0, 0, 0] = torch.tensor([float("nan"), 1.0])
    flow[0, 0, 1] = torch.tensor([float("inf"), -2.0])
    flow[0, 1, 0] = torch.tensor([-0.5, -0.5])
    flow[-1, -1, -1] = torch.tensor([1e9, -1e9])
    pyr = ops.corr_pyramid_tiled(f1.cuda(), f2.cuda(), 4)
    fl = flow.reshape(-1, 2).contiguous().cuda()
    M = n * h * w
    conv = torch.nn.Conv2d(324, 256, 1).cuda()
    with torch.no_grad():
        conv.weight.copy_((torch.randn(256, 324, 1, 1, generator=g) / 18).cuda())
        conv.bias.copy_((torch.randn(256, generator=g) * 0.1).cuda())
    r = ConvRunner([conv], "ReLU")
    packed, bias = r.packed(324, 0, w, _lib.CONV_1X1W)
    corr = torch.empty(M, 324, device="cuda")
    ops.corr_lookup(pyr, fl, n, h, w, 4, 4, out=ops.Chan.whole(corr), flow_layout="nhwc", tiled=True)
    sep = torch.full((M, 260), -3.0, device="cuda")
    ops.conv2d(ops.Chan.whole(corr), packed, bias, n, h, w, 256, 1, 1, 0, 0, "ReLU",
               out=ops.Chan(sep, 4, 256), bk=_lib.CONV_1X1W)
    fused = torch.full((M, 260), -3.0, device="cuda")
    ops.corr_lookup_conv1x1(pyr, fl, packed, bias, ops.Chan(fused, 4, 256), n, h, w, 4, 4, 256)
    torch.cuda.synchronize()
    assert torch.equal(fused, sep)
    assert (fused[:, :4] == -3).all()
    ref = torch.relu(corr.double().cpu() @ conv.weight.detach().double().cpu().view(256, 324).T +
                     conv.bias.detach().double().cpu())
    close(fused[:, 4:], ref, 1e-4, 1e-5, "fused lookup + conv vs fp64")


@pytest.mark.parametrize("size", [32, 64])
def test_conv2d_pair_bit_identical(ops, size, monkeypatch):
    """scflow_conv2d_pair (round 6: the decoder tail's flow-predictor / mask-predictor branches as
    grouped launches) equals the two separate scflow_conv2d launches bit for bit, for each paired
    kernel (thin 3×3 256→2 ‖ 1×1 256→1, small-cin 7×7 2→128 ‖ 3×3 1→64, F(2×2,3×3) 128→64 ‖
    64→32), in both argument orders, and with pairing off (SCFLOW_CONV_PAIR=0)."""
    from scflow_amd._lib import reload_switches
    from scflow_amd.modules import ConvRunner
    g = torch.Generator().manual_seed(17)
    n, h, w = (6, size, size)
    M = n * h * w

    def conv(cin, cout, k, act):
        c = torch.nn.Conv2d(cin, cout, k, padding=k // 2)
        with torch.no_grad():
            c.weight.copy_(torch.randn(c.weight.shape, generator=g) / np.sqrt(c.weight[0].numel()))
            c.bias.copy_(torch.randn(cout, generator=g) * 0.1)
        return ConvRunner([c.cuda()], act)

    head = torch.randn(M, 512, generator=g).cuda()
    cases = [  # (runner a, src a, cout a), (runner b, src b, cout b)
        ((conv(256, 2, 3, None), ops.Chan(head, 0, 256), 2),
         (conv(256, 1, 1, "Sigmoid"), ops.Chan(head, 256, 256), 1)),
        ((conv(2, 128, 7, "ReLU"), ops.Chan.whole(torch.randn(M, 2, generator=g).cuda()), 128),
         (conv(1, 64, 3, "ReLU"), ops.Chan.whole(torch.randn(M, 1, generator=g).cuda()), 64)),
        ((conv(128, 64, 3, "ReLU"), ops.Chan.whole(torch.randn(M, 128, generator=g).cuda()), 64),
         (conv(64, 32, 3, "ReLU"), ops.Chan.whole(torch.randn(M, 64, generator=g).cuda()), 32)),
    ]
    for (ra, sa, ca), (rb, sb, cb) in cases:
        ref_a = torch.full((M, ca), 7.0, device="cuda")
        ref_b = torch.full((M, cb), 7.0, device="cuda")
        ra.run(sa, ops.Chan.whole(ref_a), n, h, w)
        rb.run(sb, ops.Chan.whole(ref_b), n, h, w)
        for order in (0, 1):
            for pair in ("1", "0"):
                monkeypatch.setenv("SCFLOW_CONV_PAIR", pair)
                reload_switches()
                out_a = torch.full((M, ca), 7.0, device="cuda")
                out_b = torch.full((M, cb), 7.0, device="cuda")
                aa = ra.args(sa, ops.Chan.whole(out_a), n, h, w)
                ab = rb.args(sb, ops.Chan.whole(out_b), n, h, w)
                if order:
                    ops.conv2d_pair(ab, aa, head)
                else:
                    ops.conv2d_pair(aa, ab, head)
                torch.cuda.synchronize()
                assert torch.equal(out_a, ref_a), (ca, cb, order, pair)
                assert torch.equal(out_b, ref_b), (ca, cb, order, pair)
    monkeypatch.delenv("SCFLOW_CONV_PAIR")
    reload_switches()


@pytest.mark.parametrize("n,size", [(3, 32), (2, 64), (1, 16)])
def test_xhead_pred_fused(ops, n, size):
    """scflow_xhead_pred (round 6): the XHeads' 3×3 128 → 2·256 hidden conv (F(4×4,3×3), ReLU)
    with both predictors contracted in its epilogue + the block / tap sum, against an fp64
    reference of raft_decoder.py:256-294 (flow: 3×3 256 → 2, mask: 1×1 256 → 1 + sigmoid) and
    against the unfused launches (hidden conv → HEAD → predictor convs).  Width 16 is outside the
    fused kernel's shapes: SCFLOW_EUNSUPPORTED."""
    from scflow_amd._lib import CONV_WINO4, ScflowError
    from scflow_amd.modules import ConvRunner
    g = torch.Generator().manual_seed(23)
    h = w = size
    M = n * h * w

    def conv(cin, cout, k):
        c = torch.nn.Conv2d(cin, cout, k, padding=k // 2)
        with torch.no_grad():
            c.weight.copy_(torch.randn(c.weight.shape, generator=g) / np.sqrt(c.weight[0].numel()))
            c.bias.copy_(torch.randn(cout, generator=g) * 0.1)
        return c.cuda()

    fh1, mh1, fp, mp = conv(128, 256, 3), conv(128, 256, 3), conv(256, 2, 3), conv(256, 1, 1)
    x = torch.randn(M, 128, generator=g).cuda()
    hr = ConvRunner([fh1, mh1], "ReLU")
    head = torch.empty(M, 512, device="cuda")
    hargs = hr.args(ops.Chan.whole(x), ops.Chan.whole(head), n, h, w)
    pw = ops.xhead_pred_pack(fp.weight, mp.weight)
    d2 = torch.full((M, 2), 7.0, device="cuda")
    mk = torch.full((M, 1), 7.0, device="cuda")
    if size not in (32, 64):
        ws = torch.empty(16, device="cuda")
        with pytest.raises(ScflowError):
            ops.xhead_pred(hargs, 256, pw, ws, fp.bias, mp.bias, None, "Sigmoid", ops.Chan.whole(d2),
                           ops.Chan.whole(mk))
        return
    assert hargs.bk == CONV_WINO4
    ws = ops.xhead_pred_workspace(n, h, w, 256, 512, "cuda")
    ops.xhead_pred(hargs, 256, pw, ws, fp.bias, mp.bias, None, "Sigmoid", ops.Chan.whole(d2),
                   ops.Chan.whole(mk))
    torch.cuda.synchronize()
    # fp64 reference
    xn = x.double().reshape(n, h, w, 128).permute(0, 3, 1, 2)
    hf = F.relu(F.conv2d(xn, fh1.weight.double(), fh1.bias.double(), padding=1))
    hm = F.relu(F.conv2d(xn, mh1.weight.double(), mh1.bias.double(), padding=1))
    rf = F.conv2d(hf, fp.weight.double(), fp.bias.double(), padding=1).permute(0, 2, 3, 1).reshape(M, 2)
    rm = torch.sigmoid(F.conv2d(hm, mp.weight.double(), mp.bias.double())).permute(0, 2, 3, 1).reshape(M, 1)
    scale = rf.abs().max().item()
    close(d2, rf, 1e-4 * scale, what="flow predictor")  # F(4×4) hidden conv: ≈ 1e-5 relative
    close(mk, rm, 2e-5, what="mask predictor")
    # the unfused launches agree to fp32 summation order
    fr, mr = ConvRunner.of(fp, None), ConvRunner.of(mp, "Sigmoid")
    hr.run(ops.Chan.whole(x), ops.Chan.whole(head), n, h, w)
    d2u = torch.empty(M, 2, device="cuda")
    mku = torch.empty(M, 1, device="cuda")
    fr.run(ops.Chan(head, 0, 256), ops.Chan.whole(d2u), n, h, w)
    mr.run(ops.Chan(head, 256, 256), ops.Chan.whole(mku), n, h, w)
    torch.cuda.synchronize()
    close(d2, d2u, 1e-4 * scale, what="fused vs unfused flow")
    close(mk, mku, 1e-5, what="fused vs unfused mask")
