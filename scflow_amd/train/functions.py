"""Autograd Functions for the training step — HIP forward AND backward.

Activations are channels-last [N, H, W, C] contiguous fp32 tensors on the ROCm device.

* ``conv2d_nhwc`` — forward on the HIP conv variants (MFMA implicit GEMM for the decoder's
  shapes, the encoder MFMA conv for strided / wide ones, the gather conv otherwise).  Backward:
  dX = the same HIP conv of the output gradient with the flipped, in/out-transposed weights
  (for stride s > 1 over the gradient zero-inserted to the input grid — a transposed conv as a
  'same' convolution); dW = HIP im2col of the input + one plain GEMM dYᵀ·cols (hipBLASLt via
  ``torch.matmul``: the "plain library GEMM" case); db = Σ dY.
* ``corr_pyramid`` — forward ``scflow_corr_pyramid``; backward: average-pool adjoints (¼ to each
  of the 4 children) down to level 0, then dF1 = dC·F2ᵀ/√C, dF2 = dCᵀ·F1/√C as batched GEMMs
  (hipBLASLt).  (raft_decoder.py:35-58)
* ``corr_lookup`` — forward ``scflow_corr_lookup``; backward ``scflow_corr_lookup_backward``
  (scatter-add into the pyramid gradient; the flow input is detached in SCFlow,
  scflow_decoder.py:193-194).

Pointwise operations (activations, GRU gate algebra, losses) stay torch ops on the device.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from .. import ops
from .._lib import EPI_PLAIN, ScflowError
from ..ops import Chan

Tensor = torch.Tensor


# ------------------------------------------------------------------------------- conv dispatch
def _flip_t(w: Tensor) -> Tensor:
    """[cout, cin, kh, kw] → [cin, cout, kh, kw] flipped in space (the dgrad weights)."""
    return w.flip(2, 3).transpose(0, 1).contiguous()


def _conv_forward(x: Tensor, w: Tensor, b: Optional[Tensor], stride: int, pad: Tuple[int, int]) -> Tensor:
    """HIP conv of a channels-last input, choosing the variant that supports the shape."""
    n, h, wd, cin = x.shape
    cout, _, kh, kw = w.shape
    ph, pw = pad
    oh, ow = (h + 2 * ph - kh) // stride + 1, (wd + 2 * pw - kw) // stride + 1
    out = torch.empty(n, oh, ow, cout, device=x.device)
    same = stride == 1 and oh == h and ow == wd
    lib_ok = same and (
        (cin <= 4) or (cout <= 4 and cin % 8 == 0) or
        (cin % 4 == 0 and wd in (32, 64) and (kh, kw) in ((1, 1), (3, 3), (1, 5), (5, 1))
         and oh % (128 // wd if wd <= 128 else 1) == 0))
    if lib_ok:
        bk = ops.conv_pick_bk(n, h, wd, cin, 0, cout, kh, kw, ph, pw, 1)
        try:
            packed = ops.pack_conv_weight(w.float(), cin, 0, wd, 1, bk)
            ops.conv2d(Chan.whole(x.view(-1, cin)), packed, b, n, h, wd, cout, kh, kw, ph, pw, None,
                       out=Chan.whole(out.view(-1, cout)), bk=bk)
            return out
        except ScflowError:
            pass
    if cin % 16 == 0 and kh == kw and kh in (1, 3) and ph == pw == kh // 2 and stride in (1, 2):
        try:
            ops.enc_conv(x, ops.enc_conv_pack(w), b, n, h, wd, cin, cout, kh, stride, ph, out)
            return out
        except ScflowError:
            pass
    if ph != pw or kh != kw:
        raise ScflowError(f"no HIP conv for kernel {kh}x{kw} pad {pad} stride {stride}")
    if cin == 3 and kh == 7 and stride in (1, 2) and cout <= 256 and cout != 192:
        # the encoder stem kernel (NCHW image in, channels-last out)
        ops.enc_stem(x.permute(0, 3, 1, 2).contiguous(), ops.enc_stem_pack(w), b, cout, 7, stride,
                     ph, out)
        return out
    if cin % 4:  # the gather conv reads float4 channel groups: zero-pad the channels
        pad4 = 4 - cin % 4
        x = F.pad(x, (0, pad4))
        w = F.pad(w, (0, 0, 0, 0, 0, pad4))
        cin += pad4
    ops.ph_conv(Chan.whole(x.reshape(-1, cin)), None, ops.ph_conv_pack(w.contiguous()), b, n, h, wd,
                cout, kh, stride, ph, out.view(-1, cout))
    return out


class _Conv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, ph, pw):
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.pad, ctx.has_b = stride, (ph, pw), b is not None
        return _conv_forward(x.contiguous(), w.detach().contiguous(),
                             None if b is None else b.detach().contiguous(), stride, (ph, pw))

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        s, (ph, pw) = ctx.stride, ctx.pad
        dy = dy.contiguous()
        n, h, wd, cin = x.shape
        cout, _, kh, kw = w.shape
        _, oh, ow, _ = dy.shape
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if s == 1:
                z = dy
            else:  # zero-insert onto the input grid: a transposed conv as a 'same' conv
                z = torch.zeros(n, h, wd, cout, device=dy.device)
                z[:, 0:(oh - 1) * s + 1:s, 0:(ow - 1) * s + 1:s] = dy
            qh, qw = kh - 1 - ph, kw - 1 - pw  # dgrad padding
            if s > 1:
                qh, qw = (kh - 1) // 2, (kw - 1) // 2
                if (kh - 1 - ph) != qh or (kw - 1 - pw) != qw:
                    raise ScflowError("strided dgrad needs pad == (k-1)/2")
            dx = _conv_forward(z, _flip_t(w.detach()), None, 1, (qh, qw))
        if ctx.needs_input_grad[1]:
            cols = ops.im2col(x.contiguous(), n, h, wd, cin, kh, kw, s, ph, pw)
            dwm = torch.matmul(dy.view(-1, cout).t(), cols)  # [cout, kh·kw·cin] (hipBLASLt)
            dw = dwm.view(cout, kh, kw, cin).permute(0, 3, 1, 2).contiguous()
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = dy.view(-1, cout).sum(0)
        return dx, dw, db, None, None, None


def conv2d_nhwc(x: Tensor, weight: Tensor, bias: Optional[Tensor] = None, stride: int = 1,
                padding=0) -> Tensor:
    """nn.Conv2d (cross-correlation) on channels-last tensors, HIP forward and backward."""
    ph, pw = (padding, padding) if isinstance(padding, int) else padding
    return _Conv2dNHWC.apply(x, weight, bias, stride, ph, pw)


# ------------------------------------------------------------------------------- correlation
class _CorrPyramid(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f1, f2, num_levels):
        """f1, f2 [N, C, h, w] (NCHW, like the reference) → flat pyramid buffer."""
        f1 = f1.contiguous()
        f2 = f2.contiguous()
        ctx.save_for_backward(f1, f2)
        ctx.num_levels = num_levels
        buf, _ = ops.corr_pyramid(f1, f2, num_levels)
        return buf

    @staticmethod
    def backward(ctx, dbuf):
        f1, f2 = ctx.saved_tensors
        n, c, h, w = f1.shape
        P = h * w
        levels = ops.pyramid_views(dbuf.contiguous(), n, h, w, ctx.num_levels)
        g = levels[-1].view(n * P, 1, *levels[-1].shape[-2:])
        for lv in reversed(levels[:-1]):  # AvgPool2d(2,2) adjoint: ¼ to each child (floors)
            hl, wl = lv.shape[-2:]
            up = torch.zeros(n * P, 1, hl, wl, device=dbuf.device)
            up[..., : (hl // 2) * 2, : (wl // 2) * 2] = g.repeat_interleave(2, -2).repeat_interleave(2, -1) * 0.25
            g = lv.view(n * P, 1, hl, wl) + up
        dC = g.view(n, P, P) / (c ** 0.5)                 # dC[n][p][q]
        F1 = f1.view(n, c, P)
        F2 = f2.view(n, c, P)
        df1 = torch.bmm(F2, dC.transpose(1, 2))            # [n][c][p] = Σ_q F2[c][q] dC[p][q]
        df2 = torch.bmm(F1, dC)                           # [n][c][q] = Σ_p F1[c][p] dC[p][q]
        return df1.view_as(f1), df2.view_as(f2), None


def corr_pyramid(f1: Tensor, f2: Tensor, num_levels: int = 4) -> Tensor:
    return _CorrPyramid.apply(f1, f2, num_levels)


class _CorrLookup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pyr, flow_nhwc, n, h, w, num_levels, radius):
        flow_nhwc = flow_nhwc.contiguous()
        ctx.save_for_backward(flow_nhwc)
        ctx.dims = (n, h, w, num_levels, radius, pyr.numel())
        out = torch.empty(n * h * w, num_levels * (2 * radius + 1) ** 2, device=pyr.device)
        ops.corr_lookup(pyr, flow_nhwc, n, h, w, num_levels, radius, out=Chan.whole(out),
                        flow_layout="nhwc")
        return out.view(n, h, w, -1)

    @staticmethod
    def backward(ctx, dout):
        (flow,) = ctx.saved_tensors
        n, h, w, L, r, size = ctx.dims
        dpyr = torch.zeros(size, device=dout.device)
        ops.corr_lookup_backward(dout.contiguous().view(n * h * w, -1), flow, dpyr, n, h, w, L, r)
        return dpyr, None, None, None, None, None, None


def corr_lookup(pyr: Tensor, flow_nhwc: Tensor, n: int, h: int, w: int, num_levels: int = 4,
                radius: int = 4) -> Tensor:
    """[n, h, w, L·(2r+1)²] channels-last lookup; differentiable w.r.t. the pyramid only."""
    return _CorrLookup.apply(pyr, flow_nhwc.detach(), n, h, w, num_levels, radius)
