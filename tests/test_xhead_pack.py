"""CPU check of scflow_xhead_pred's predictor packing and its two-phase sum (round 6): the
per-pixel channel contraction Z[q][tap·2 + o] = Σ_c Y[q][c]·pw[c][tap·2 + o] followed by
out[p][o] = b[o] + Σ_tap Z[p + off(tap)][tap·2 + o] (the arithmetic w4_pred_round and
xhead_pred_sum_kernel run, restated in float64 torch) equals the reference's XHead predictors —
a 3×3 conv 256 → 2 and a 1×1 conv 256 → 1 + sigmoid (raft_decoder.py:256-294) — on the same
hidden features."""
import torch
import torch.nn.functional as F

from scflow_amd import ops


def test_xhead_pred_pack_and_tap_sum():
    g = torch.Generator().manual_seed(5)
    n, h, w, cf, cm = 2, 8, 12, 256, 256
    yf = torch.relu(torch.randn(n, cf, h, w, generator=g, dtype=torch.float64))
    ym = torch.relu(torch.randn(n, cm, h, w, generator=g, dtype=torch.float64))
    fw = torch.randn(2, cf, 3, 3, generator=g, dtype=torch.float64) / 48
    mw = torch.randn(1, cm, 1, 1, generator=g, dtype=torch.float64) / 16
    fb = torch.randn(2, generator=g, dtype=torch.float64)
    mb = torch.randn(1, generator=g, dtype=torch.float64)
    pw = ops.xhead_pred_pack(fw.float(), mw.float()).double()
    assert pw.shape == (cf + cm, 20)
    assert torch.equal(pw[:cf, 18:], torch.zeros(cf, 2, dtype=torch.float64))
    assert torch.equal(pw[cf:, 1:], torch.zeros(cm, 19, dtype=torch.float64))
    # phase 1: per-pixel contraction (channels-last), summed over the 32-channel blocks
    Yf = yf.permute(0, 2, 3, 1)  # [n, h, w, cf]
    Z = sum(Yf[..., b:b + 32] @ pw[b:b + 32, :18] for b in range(0, cf, 32))  # [n, h, w, 18]
    Zp = F.pad(Z.permute(0, 3, 1, 2), (1, 1, 1, 1)).permute(0, 2, 3, 1)  # zero halo
    out = fb.expand(n, h, w, 2).clone()
    for ty in range(3):
        for tx in range(3):
            t = ty * 3 + tx
            out += Zp[:, ty:ty + h, tx:tx + w, 2 * t:2 * t + 2]
    ref = F.conv2d(yf, fw, fb, padding=1).permute(0, 2, 3, 1)
    torch.testing.assert_close(out, ref, rtol=1e-6, atol=1e-6)  # packing rounded to fp32
    # the mask head: one column per hidden channel, sigmoid after the block sum
    Ym = ym.permute(0, 2, 3, 1)
    zm = sum(Ym[..., b:b + 32] @ pw[cf + b:cf + b + 32, :1] for b in range(0, cm, 32))
    mref = torch.sigmoid(F.conv2d(ym, mw, mb)).permute(0, 2, 3, 1)
    torch.testing.assert_close(torch.sigmoid(zm + mb), mref, rtol=1e-6, atol=1e-6)
