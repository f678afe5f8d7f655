"""Autograd Functions for the training step — HIP forward AND backward.

Activations are channels-last [N, H, W, C] contiguous fp32 tensors on the ROCm device.

* ``conv2d_nhwc`` — forward on the HIP conv variants (MFMA implicit GEMM for the decoder's
  shapes, the encoder MFMA conv for strided / wide ones, the gather conv otherwise), with the
  activation and an optional pre-activation bias map fused into the epilogue, and an optional
  second input source (channel concat without a copy).  Backward: the activation's derivative
  from the saved output; dX = the same HIP conv of the output gradient with the flipped,
  in/out-transposed weights (stride s > 1: cols = dY·Wmat on the HIP GEMM + the col2im gather,
  no zero-inserted grid); dW and db = ``scflow_conv_wgrad`` (MFMA
  implicit GEMM over the pixels, no im2col matrix); 7×7 kernels use HIP im2col + one
  ``scflow_gemm_f32`` dYᵀ·cols.
* ``corr_pyramid`` — forward ``scflow_corr_pyramid``; backward: average-pool adjoints (¼ to each
  of the 4 children) down to level 0, then dF1 = dC·F2ᵀ/√C, dF2 = dCᵀ·F1/√C as batched
  ``scflow_gemm_f32`` launches.  (raft_decoder.py:35-58)
* ``linear`` — F.linear with the forward and both backward products on ``scflow_gemm_f32``
  (the pose head's FC layers, pose_head.py:201-211).

No vendor BLAS kernel runs in the training step, so the whole forward + backward can be captured
into one hipGraph (the vendor GEMM's kernels could not be instantiated in a captured graph).
* ``corr_lookup`` — forward ``scflow_corr_lookup``; backward ``scflow_corr_lookup_backward``
  (scatter-add into the pyramid gradient; the flow input is detached in SCFlow,
  scflow_decoder.py:193-194).

Pointwise operations (activations, GRU gate algebra, losses) stay torch ops on the device.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from .. import _lib, ops
from .._lib import EPI_PLAIN, ScflowError, weights_generation
from ..ops import Chan

Tensor = torch.Tensor


# ------------------------------------------------------------------------------- conv dispatch
_CAPTURE_CACHE: Optional[dict] = None


class capture_cache:
    """Scope of a hipGraph capture of the forward + backward: inside it each derived weight form
    is made once per capture (the first use records the pack kernel, later uses in the same
    replay read its output), never taken from or left in the eager per-version cache — the
    weights move between replays, so a form made outside the graph would be stale in it."""

    def __enter__(self):
        global _CAPTURE_CACHE
        _CAPTURE_CACHE = {}
        return self

    def __exit__(self, *exc):
        global _CAPTURE_CACHE
        _CAPTURE_CACHE = None
        return False


def _cached(w: Tensor, key: tuple, make):
    """A form derived from weight ``w`` (packed for a kernel, flipped for dX), made once per
    version of ``w`` and kept on the tensor object: a decoder weight is used in every refinement
    iteration (8 forward and 8 dX launches per step) but changes only at the optimizer step (its
    version counter moves).  Tensors made per step (the GRU's concatenated weights) carry their
    cache with them and drop it when they die.  While a hipGraph is being captured the forms
    live in the capture's own cache (``capture_cache``), or are re-made per use outside one."""
    if not w.is_cuda:
        return make()
    if torch.cuda.is_current_stream_capturing():
        if _CAPTURE_CACHE is None:
            return make()
        k = (id(w), w._version) + key
        hit = _CAPTURE_CACHE.get(k)
        if hit is None:
            hit = _CAPTURE_CACHE[k] = (w, make())  # w kept alive so its id stays unique
        return hit[1]
    ver = (w._version, weights_generation())
    cache = getattr(w, "_scflow_cache", None)
    if cache is None or cache[0] != ver:
        cache = (ver, {})
        try:
            w._scflow_cache = cache
        except (AttributeError, RuntimeError):
            return make()
    v = cache[1].get(key)
    if v is None:
        v = cache[1][key] = make()
    return v


def _flip_t(w: Tensor, pad_co: int = 0) -> Tensor:
    """[cout, cin, kh, kw] → [cin, cout (+ pad_co zero channels), kh, kw] flipped in space (the
    dgrad weights), cached per version of ``w``."""
    def make():
        f = w.detach().flip(2, 3).transpose(0, 1)
        return (F.pad(f, (0, 0, 0, 0, 0, pad_co)) if pad_co else f).contiguous()
    return _cached(w, ("flip_t", pad_co), make)


_DIRECT_WGRAD = False


class direct_weight_grads:
    """Scope in which a conv's backward adds its weight / bias gradient straight into the leaf
    parameters' existing ``.grad`` buffers (scflow_conv_wgrad accumulate = 1) and hands autograd
    no gradient for them — instead of a fresh dW per use, autograd summing a decoder weight's 8
    per-iteration gradients and AccumulateGrad adding the sum.  Only for parameters whose
    ``.grad`` is already allocated (GradBuckets' flat views) and when nothing observes their
    accumulation (no post-accumulate-grad hooks: TrainStep without ``overlap``).

    Leaving the scope sums the recorded uses a backward pass never reached
    (``flush_pending_wgrads``), so the gradients are complete once it exits."""

    def __enter__(self):
        global _DIRECT_WGRAD
        self._prev, _DIRECT_WGRAD = _DIRECT_WGRAD, True
        return self

    def __exit__(self, *exc):
        global _DIRECT_WGRAD
        _DIRECT_WGRAD = self._prev
        if exc[0] is None:
            flush_pending_wgrads()
        return False


def _grad_sink(t: Optional[Tensor]) -> Optional[Tensor]:
    """t.grad when gradients of leaf ``t`` may be added into it directly, else None."""
    if t is None or not _DIRECT_WGRAD or not t.is_leaf or not t.requires_grad:
        return None
    gr = t.grad
    if gr is None or not gr.is_contiguous() or gr.dtype != torch.float32:
        return None
    return gr


# A/B switches (tools/train_bench.py runs): SCFLOW_DEFER_LINEAR=0 / SCFLOW_THIN_DX_GEMM=0
_DEFER_LINEAR = os.environ.get("SCFLOW_DEFER_LINEAR", "1") != "0"
_THIN_DX_GEMM = os.environ.get("SCFLOW_THIN_DX_GEMM", "1") != "0"

_ACT_FN = {None: lambda v: v, "ReLU": torch.relu, "Sigmoid": torch.sigmoid, "Tanh": torch.tanh}


def _act_backward(dy: Tensor, y: Tensor, act: Optional[str]) -> Tensor:
    """Gradient through act given its OUTPUT y (ReLU: y > 0; sigmoid: y(1−y); tanh: 1−y²)."""
    if act is None:
        return dy
    if act == "ReLU":
        return torch.ops.aten.threshold_backward(dy, y, 0.0)
    if act == "Sigmoid":
        return torch.ops.aten.sigmoid_backward(dy, y)
    if act == "Tanh":
        return torch.ops.aten.tanh_backward(dy, y)
    raise ValueError(act)


def _chan_view(t: Tensor) -> Optional[Chan]:
    """``t`` [..., c] as a Chan when it is a channel slice [off, off + c) of a channels-last
    buffer with rows of C ≥ c floats (pixel dims packed at stride C; a view whose ``_base`` gives
    the row origin), else None."""
    b = t._base
    if b is None or not b.is_contiguous() or t.dim() < 2 or t.stride(-1) != 1:
        return None
    c = t.shape[-1]
    C = expect = None
    for i in range(t.dim() - 2, -1, -1):  # pixel dims packed at stride C
        if t.shape[i] == 1:
            continue
        if C is None:
            C = expect = t.stride(i)
        elif t.stride(i) != expect:
            return None
        expect *= t.shape[i]
    if C is None:
        C = c
    off = (t.storage_offset() - b.storage_offset()) % C
    if C < c or off + c > C:
        return None
    m = t.numel() // c
    p0 = t.storage_offset() - off
    if p0 < 0 or (p0 + m * C) * t.element_size() > t.untyped_storage().nbytes():
        return None
    return Chan(torch.as_strided(t, (m, C), (C, 1), p0), off, c)


def _chan(t: Tensor) -> Chan:
    """The Chan a conv kernel reads ``t`` (contiguous, or a channel slice read in place) through."""
    if t.is_contiguous():
        return Chan.whole(t.view(-1, t.shape[-1]))
    c = _chan_view(t)
    if c is None:
        raise ValueError("conv source: contiguous or a channel slice of a channels-last buffer")
    return c


def _chan_or_contiguous(t: Tensor) -> Tensor:
    return t if t.is_contiguous() or _chan_view(t) is not None else t.contiguous()


def _src(t: Optional[Tensor]):
    """A weight-gradient source: the tensor itself when contiguous, its Chan when a slice."""
    if t is None or t.is_contiguous():
        return t
    return _chan(t)


def _conv_forward(x0: Tensor, x1: Optional[Tensor], w: Tensor, b: Optional[Tensor], stride: int,
                  pad: Tuple[int, int], act: Optional[str] = None,
                  bias_map: Optional[Tensor] = None, wkey: Optional[Tensor] = None) -> Tensor:
    """act(conv(cat[x0, x1]) + b + bias_map) of channels-last inputs on the HIP conv variant
    that supports the shape; act and bias_map are fused into the epilogue where the variant has
    one, applied after it otherwise.  ``wkey``: the weight tensor object whose version keys the
    cached packed forms (default ``w``)."""
    wkey = w if wkey is None else wkey
    n, h, wd, c0 = x0.shape
    c1 = 0 if x1 is None else x1.shape[-1]
    cin = c0 + c1
    cout, _, kh, kw = w.shape
    ph, pw = pad
    oh, ow = (h + 2 * ph - kh) // stride + 1, (wd + 2 * pw - kw) // stride + 1
    out = torch.empty(n, oh, ow, cout, device=x0.device)
    same = stride == 1 and oh == h and ow == wd
    lib_ok = same and (
        (cin <= 4 and x1 is None) or (cout <= 4 and cin % 8 == 0) or
        (c0 % 4 == 0 and c1 % 4 == 0 and wd in (32, 64) and (kh, kw) in ((1, 1), (3, 3), (1, 5), (5, 1))
         and oh % (128 // wd if wd <= 128 else 1) == 0) or
        # the encoders' 128-wide 3×3 convs (and their dX): Winograd, two output rows per block
        (c0 % 4 == 0 and c1 % 4 == 0 and wd == 128 and (kh, kw) == (3, 3) and oh % 2 == 0))
    if lib_ok:
        bk = ops.conv_pick_bk(n, h, wd, c0, c1, cout, kh, kw, ph, pw, 1)
        try:
            packed = _cached(wkey, ("conv", c0, c1, wd, bk),
                             lambda: ops.pack_conv_weight(w.float(), c0, c1, wd, 1, bk))
            ops.conv2d(_chan(x0), packed, b, n, h, wd, cout, kh, kw, ph, pw, act,
                       out=Chan.whole(out.view(-1, cout)), bk=bk,
                       src1=None if x1 is None else _chan(x1),
                       bias_map=None if bias_map is None else Chan.whole(bias_map.reshape(-1, cout)))
            return out
        except ScflowError:
            pass
    post = True  # act / bias_map still to apply
    if (c0 % 16 == 0 and c1 % 16 == 0 and kh == kw and kh in (1, 3) and ph == pw == kh // 2
            and stride in (1, 2)):
        try:
            fuse = bias_map is None
            ops.enc_conv(_chan(x0), _cached(wkey, ("enc",), lambda: ops.enc_conv_pack(w)),
                         b, n, h, wd, c0, cout, kh,
                         stride, ph, out, act=act if fuse else None,
                         src1=None if x1 is None else _chan(x1))
            post = not fuse
            x0 = None
        except ScflowError:
            pass
    if x0 is not None:
        x = x0 if x1 is None else torch.cat([x0, x1], -1)
        if ph != pw or kh != kw:
            raise ScflowError(f"no HIP conv for kernel {kh}x{kw} pad {pad} stride {stride}")
        if cin == 3 and kh == 7 and stride in (1, 2) and cout <= 256 and cout != 192:
            # the encoder stem kernel (NCHW image in, channels-last out)
            ops.enc_stem(x.permute(0, 3, 1, 2).contiguous(),
                         _cached(wkey, ("stem",), lambda: ops.enc_stem_pack(w)), b, cout, 7, stride,
                         ph, out)
        else:
            pad4 = (4 - cin % 4) % 4
            if pad4:  # the gather conv reads float4 channel groups: zero-pad the channels
                x = F.pad(x, (0, pad4))
                cin += pad4
            packed = _cached(wkey, ("ph", pad4), lambda: ops.ph_conv_pack(
                (F.pad(w, (0, 0, 0, 0, 0, pad4)) if pad4 else w).contiguous()))
            ops.ph_conv(Chan.whole(x.reshape(-1, cin)), None, packed, b, n, h,
                        wd, cout, kh, stride, ph, out.view(-1, cout))
    if post:
        if bias_map is not None:
            out += bias_map
        out = _ACT_FN[act](out)
    return out


def _weight_grad(g: Tensor, x0: Tensor, x1: Optional[Tensor], w: Tensor, s: int, ph: int, pw: int,
                 with_bias: bool, dw: Optional[Tensor] = None,
                 db: Optional[Tensor] = None) -> Tuple[Tensor, Optional[Tensor]]:
    """(dW, db) of the conv; given ``dw`` (and ``db`` when with_bias) the gradients are ADDED
    into them (and returned)."""
    n, h, wd, c0 = x0.shape
    cout, cin, kh, kw = w.shape
    accumulate = dw is not None
    if not accumulate:
        dw = torch.empty(cout, cin, kh, kw, device=g.device)
        db = torch.empty(cout, device=g.device) if with_bias else None
    g2 = g.reshape(-1, g.shape[-1])
    if g.shape[-1] != cout:  # output channels zero-padded to a multiple of 4 (see _conv_backward)
        dwp = torch.empty(g.shape[-1], cin, kh, kw, device=g.device)
        dbp = torch.empty(g.shape[-1], device=g.device) if with_bias else None
        ops.conv_wgrad(g2, _src(x0), _src(x1), dwp, dbp, n, h, wd, kh, kw, s, ph, pw)
        if accumulate:
            dw += dwp[:cout]
            if with_bias:
                db += dbp[:cout]
            return dw, db
        return dwp[:cout], (dbp[:cout] if with_bias else None)
    try:
        ops.conv_wgrad(g2, _src(x0), _src(x1), dw, db, n, h, wd, kh, kw, s, ph, pw,
                       accumulate=accumulate)
        return dw, db
    except ScflowError:
        pass
    # shapes outside the wgrad kernels (7×7): HIP im2col in the weight's own column order + one
    # HIP GEMM written (or accumulated) straight into dW.  (The bias sum as a ones-row GEMM ran
    # 44 µs against torch's 19 µs column sum: kept on torch.)
    x = x0 if x1 is None else torch.cat([x0, x1], -1)
    cols = ops.im2col(x.contiguous(), n, h, wd, cin, kh, kw, s, ph, pw, channel_major=True)
    beta = 1.0 if accumulate else 0.0
    ops.gemm(g2.t(), cols, out=dw.view(cout, cin * kh * kw), beta=beta)
    if with_bias:
        ops.colsum(g2, db, accumulate=accumulate)
    return dw, db


# ------------------------------------------------------------------ batched weight gradients
# A decoder conv runs once per refinement iteration: its weight gradient is the sum of 8 per-use
# weight gradients.  Instead of 8 launches (each with its own split reduction, and short per-use
# pixel walks at B = 16), the uses' (dY, input) pairs are collected as their backward runs and
# summed by ONE scflow_conv_wgrad_batched launch when the last use's backward arrives (autograd
# consumes a weight's gradient only after every use has produced its part).
_FWD_ID = 0


def begin_forward() -> None:
    """Start of a training forward pass: per-weight use counts restart (refiner_train_forward)."""
    global _FWD_ID
    _FWD_ID += 1


def _batchable(kh: int, kw: int, s: int, ph: int, pw: int) -> bool:
    """Shapes whose uses' weight gradients are summed at the last use: scflow_conv_wgrad_batched's
    (Winograd, 1×1, implicit-GEMM, thin) and 7×7 (one concatenated GEMM, _concat_gemm_wgrad);
    shapes a batched call refuses fall back to one launch per use."""
    return (kh, kw) in ((1, 1), (3, 3), (1, 5), (5, 1), (7, 7)) and s in (1, 2)


def _use_holder(w: Tensor) -> dict:
    """The per-forward-pass use record of weight ``w`` (module parameters persist across steps:
    the record restarts with each forward pass, begin_forward)."""
    hold = getattr(w, "_scflow_uses", None)
    if hold is None or hold["fwd"] != _FWD_ID:
        hold = {"fwd": _FWD_ID, "uses": 0, "seen": 0, "items": [], "buf": None}
        try:
            w._scflow_uses = hold
        except (AttributeError, RuntimeError):
            return None
    hold["uses"] += 1
    return hold


def _flush_wgrad(items, w: Tensor, with_bias: bool, dw: Tensor, db: Optional[Tensor],
                 accumulate: bool, s: int, ph: int, pw: int) -> None:
    """dw (db) (+)= Σ over items (g, x0, x1) of the conv weight (bias) gradient.  Uses of one
    weight at different shapes (a shared encoder on differently sized inputs) are summed group by
    group: the batched kernels take one (g, x0, x1) shape per call."""
    groups: dict = {}
    for it in items:
        key = tuple(None if t is None else tuple(t.shape) for t in it)
        groups.setdefault(key, []).append(it)
    for i, grp in enumerate(groups.values()):
        _flush_wgrad_same(grp, w, with_bias, dw, db, accumulate or i > 0, s, ph, pw)


def _flush_wgrad_same(items, w: Tensor, with_bias: bool, dw: Tensor, db: Optional[Tensor],
                      accumulate: bool, s: int, ph: int, pw: int) -> None:
    """_flush_wgrad over items of one shape: batched launches of ≤ 8 segments, per-item launches
    where the batched kernel does not take the shape."""
    g0, x00, x10 = items[0]
    n, h, wd, _ = x00.shape
    cout, cin, kh, kw = w.shape
    padded = g0.shape[-1] != cout  # out_net's 126 output channels, padded to 128 in dY
    if kh * kw > 25 and not padded and len(items) > 1:
        _concat_gemm_wgrad(items, w, with_bias, dw, db, accumulate, s, ph, pw)
        return
    if padded:
        tw = torch.empty(g0.shape[-1], cin, kh, kw, device=g0.device)
        tb = torch.empty(g0.shape[-1], device=g0.device) if with_bias else None
    else:
        tw, tb = dw, db
    try:
        for i in range(0, len(items), 8):
            part = items[i:i + 8]
            ops.conv_wgrad_batched([g.reshape(-1, g.shape[-1]) for g, _, _ in part],
                                   [_src(x0) for _, x0, _ in part],
                                   None if x10 is None else [_src(x1) for _, _, x1 in part],
                                   tw, tb, n, h, wd, kh, kw, s, ph, pw,
                                   accumulate=(accumulate and not padded) or i > 0)
    except ScflowError:  # shapes outside the batched kernels: one launch per use
        if not accumulate:
            dw.zero_()
            if with_bias:
                db.zero_()
        for g, x0, x1 in items:
            _weight_grad(g, x0, x1, w, s, ph, pw, with_bias, dw=dw, db=db)
        return
    if padded:
        if accumulate:
            dw += tw[:cout]
            if with_bias:
                db += tb[:cout]
        else:
            dw.copy_(tw[:cout])
            if with_bias:
                db.copy_(tb[:cout])


def _concat_gemm_wgrad(items, w: Tensor, with_bias: bool, dw: Tensor, db: Optional[Tensor],
                       accumulate: bool, s: int, ph: int, pw: int) -> None:
    """The uses' weight gradient of a large kernel (the flow encoders' 7×7 2 → 128, outside the
    wgrad kernels) as ONE GEMM: every use's patch matrix into one buffer (HIP im2col in the
    weight's column order), the dY's concatenated, dW (+)= Σ dYᵀ·cols over all pixels at once
    (8 accumulating GEMMs over 16k pixels each ran at ≈ 20 TF)."""
    g0, x00, _ = items[0]
    n, h, wd, _ = x00.shape
    cout, cin, kh, kw = w.shape
    m = g0.reshape(-1, g0.shape[-1]).shape[0]
    cols = torch.empty(len(items) * m, cin * kh * kw, device=g0.device)
    for i, (_, x0, x1) in enumerate(items):
        x = x0 if x1 is None else torch.cat([x0, x1], -1)
        ops.im2col(x.contiguous(), n, h, wd, cin, kh, kw, s, ph, pw, out=cols[i * m:(i + 1) * m],
                   channel_major=True)
    gall = torch.cat([g.reshape(-1, cout) for g, _, _ in items])
    ops.gemm(gall.t(), cols, out=dw.view(cout, cin * kh * kw), beta=1.0 if accumulate else 0.0)
    if with_bias:
        ops.colsum(gall, db, accumulate=accumulate)


_PENDING: dict = {}  # id(holder) → holder with recorded uses not yet summed


def _defer(hold: dict, item, flush) -> None:
    """Record this use's item; at the last use of the pass, ``flush(items)`` adds the summed weight
    gradient into the parameter's gradient sinks (direct_weight_grads)."""
    if not hold["items"]:
        hold["flush"] = flush
        _PENDING[id(hold)] = hold
    hold["items"].append(item)
    hold["seen"] += 1
    if hold["seen"] >= hold["uses"]:
        _flush_holder(hold)


def _deferred_wgrad(hold: dict, w: Tensor, item, with_bias: bool, s: int, ph: int, pw: int,
                    sink_w: Tensor, sink_b: Optional[Tensor]) -> None:
    """Record this conv use's (g, x0, x1); on the last use, one batched weight gradient over all
    of them, added into the sinks."""
    _defer(hold, item, lambda items: _flush_wgrad(items, w, with_bias, sink_w, sink_b, True, s,
                                                  ph, pw))


def _flush_holder(hold: dict) -> None:
    items = hold["items"]
    if items:
        hold["flush"](items)
    hold["items"] = []
    hold["seen"] = 0
    hold["buf"] = None
    _PENDING.pop(id(hold), None)


def flush_pending_wgrads() -> None:
    """Sum the weight gradients of uses a backward pass recorded but whose last use it never
    reached (a conv output that does not reach the loss): call after backward, before the
    gradients are read (TrainStep does)."""
    for hold in list(_PENDING.values()):
        _flush_holder(hold)


class ResidualGrad:
    """Hand-over of a residual block's identity gradient (encoder BasicBlock without downsample):
    the block tail's backward (instance_norm_residual_relu_nhwc) leaves dres here instead of
    returning it, and the block's first conv — the identity's other consumer — adds it in its dX
    conv's epilogue (bias map), so the input's two gradients never meet in an autograd add.
    Autograd runs the tail's backward before the first conv's (the conv's output gradient comes
    through the tail), so the hand-over is always complete when it is taken."""
    __slots__ = ("d",)

    def __init__(self):
        self.d = None


class _Conv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x0, x1, w, b, bias_map, stride, ph, pw, act, res_grad=None):
        x0 = _chan_or_contiguous(x0)  # channel slices of a wider buffer are read in place
        x1 = None if x1 is None else _chan_or_contiguous(x1)
        y = _conv_forward(x0, x1, w.detach().contiguous(), None if b is None else b.detach().contiguous(),
                          stride, (ph, pw), act, None if bias_map is None else bias_map.detach().contiguous(),
                          wkey=w)
        ctx.save_for_backward(x0, x1, w, y if act is not None else None)
        ctx.stride, ctx.pad, ctx.has_b, ctx.act = stride, (ph, pw), b is not None, act
        ctx.bias = b  # the leaf itself (direct gradient accumulation), not saved data
        kh, kw = w.shape[2], w.shape[3]
        ctx.uses = _use_holder(w) if _batchable(kh, kw, stride, ph, pw) and w.requires_grad else None
        ctx.res_grad = res_grad
        return y

    @staticmethod
    def backward(ctx, dy):
        return _conv_backward(ctx, dy) + (None,)


class _Conv2dNHWCSplit(torch.autograd.Function):
    """``_Conv2dNHWC`` whose output channels come back as two tensors [..., :split], [..., split:]
    (the GRU's z | r): their gradients are concatenated once in backward, instead of autograd
    zero-filling a full-width buffer per slice and adding the two."""

    @staticmethod
    def forward(ctx, x0, x1, w, b, bias_map, stride, ph, pw, act, split):
        y = _Conv2dNHWC.forward(ctx, x0, x1, w, b, bias_map, stride, ph, pw, act)
        ctx.split = split
        ctx.cout = y.shape[-1]
        return y[..., :split], y[..., split:]

    @staticmethod
    def backward(ctx, da, db_):
        shape = list((da if da is not None else db_).shape)
        parts = []
        for g, c in ((da, ctx.split), (db_, ctx.cout - ctx.split)):
            shape[-1] = c
            parts.append(g.contiguous() if g is not None else
                         torch.zeros(shape, device=(da if da is not None else db_).device))
        return _conv_backward(ctx, torch.cat(parts, -1)) + (None,)


def _conv_backward(ctx, dy):
    """dX (the forward kernels on the flipped weights), dW / db (wgrad) and the bias-map gradient."""
    x0, x1, w, y = ctx.saved_tensors
    s, (ph, pw) = ctx.stride, ctx.pad
    g = _act_backward(dy.contiguous(), y, ctx.act).contiguous()
    n, h, wd, c0 = x0.shape
    cout, cin, kh, kw = w.shape
    _, oh, ow, _ = g.shape
    dx0 = dx1 = dw = db = None
    dbm = g if ctx.needs_input_grad[4] else None
    hold = getattr(ctx, "res_grad", None)
    dres = None if hold is None else hold.d  # the identity's gradient, added into dX (ResidualGrad)
    if hold is not None:
        hold.d = None
    # output channels not a multiple of 4 (out_net's 126): zero-pad dY so dgrad reads whole float4
    # channel groups (the Winograd / MFMA variants) and wgrad stays on its vector path
    pad_co = (-cout) % 4 if cout > 4 else 0
    gp = F.pad(g, (0, pad_co)) if pad_co else g
    if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
        if s == 1 and kh == kw == 1 and cout == 1 and ph == pw == 0:
            # 1×1 to one channel (the mask predictor): dX = dY ⊗ w, one broadcast multiply
            # (a 1 → cin conv launch took 27 µs for the 16 MB it writes)
            dx = g * w.detach().reshape(1, 1, 1, cin)
        elif s == 1 and cin <= 4 and kh * kw > 25 and _THIN_DX_GEMM:
            # a large kernel onto ≤ 4 channels (the Δflow encoder's 7×7 128 → 2 adjoint): the
            # products as one GEMM cols = dY·Wmat, then the col2im gather (the thin conv ran
            # at 11 TF: 37 µs per use)
            wm = _cached(w, ("wmat",), lambda: w.detach().permute(0, 2, 3, 1).reshape(cout, -1).contiguous())
            cols = ops.gemm(g.view(-1, cout), wm)
            dx = ops.col2im(cols, n, h, wd, cin, kh, kw, 1, ph, pw)
        elif s == 1:  # a 'same' conv of dY with the flipped, transposed weights
            # its padding is k−1−p; a conv padded by more than k−1 (p = k−1+e) has an adjoint
            # with padding −e, i.e. the unpadded conv of dY cropped by e on each side
            ey, ex = max(0, ph - (kh - 1)), max(0, pw - (kw - 1))
            gin = gp if ey == ex == 0 else gp[:, ey:oh - ey, ex:ow - ex].contiguous()
            dx = _conv_forward(gin, None, _flip_t(w, pad_co), None, 1,
                               (max(0, kh - 1 - ph), max(0, kw - 1 - pw)),
                               bias_map=dres)
            dres = None
        else:
            # strided: cols = dY·Wmat (exactly the products the transposed conv needs, no
            # zero-inserted grid) and the col2im gather onto the input grid
            wm = _cached(w, ("wmat",), lambda: w.detach().permute(0, 2, 3, 1).reshape(cout, -1).contiguous())
            cols = ops.gemm(g.view(-1, cout), wm)
            dx = ops.col2im(cols, n, h, wd, cin, kh, kw, s, ph, pw)
        if dres is not None:
            dx = dx + dres
        dx0 = dx if x1 is None else dx[..., :c0]
        dx1 = None if x1 is None else dx[..., c0:]
    want_b = ctx.has_b and ctx.needs_input_grad[3]
    hold = getattr(ctx, "uses", None)
    sw = _grad_sink(w) if ctx.needs_input_grad[2] else None
    sb = _grad_sink(ctx.bias) if want_b else None
    if (hold is not None and hold["uses"] > 1 and sw is not None and (sb is not None or not want_b)
            and (want_b or not ctx.has_b)):
        # a weight used by several convs of this pass (the decoder's 8 iterations), gradients
        # added straight into the parameters: one batched weight gradient at the last use
        _deferred_wgrad(hold, w, (gp, x0, x1), want_b, s, ph, pw, sw, sb)
    elif ctx.needs_input_grad[2] or want_b:
        sw = _grad_sink(w) if ctx.needs_input_grad[2] else None
        sb = _grad_sink(ctx.bias) if want_b else None
        if sw is not None and (sb is not None or not want_b):
            _weight_grad(gp, x0, x1, w, s, ph, pw, want_b, dw=sw, db=sb)  # added in place
        else:
            dw, db = _weight_grad(gp, x0, x1, w, s, ph, pw, want_b)
    return dx0, dx1, dw, db, dbm, None, None, None, None


class _DualConv2dNHWC(torch.autograd.Function):
    """Two convs of the same input with the same kernel shape (the XHeads' hidden convs,
    flow_pred.layers[0] and mask_pred.layers[0] on h, raft_decoder.py XHead) as one launch each
    way: the forward on the two weights stacked along cout (cached per weight version) returns
    channel views of one output buffer (the predictors read them in place); the backward runs ONE
    dX conv over both output gradients — the input's two gradients summed by the GEMM instead of
    two launches and an autograd add — and one batched weight gradient over the pass's uses,
    split into the two parameters' gradient sinks."""

    @staticmethod
    def forward(ctx, x, wa, ba, wb, bb, ph, pw, act):
        x = _chan_or_contiguous(x)
        ca = wa.shape[0]
        wcat = _cached(wa, ("dual_w", id(wb), wb._version),
                       lambda: torch.cat([wa.detach(), wb.detach()], 0).contiguous())
        bcat = None
        if ba is not None:
            bcat = _cached(wa, ("dual_b", id(ba), ba._version, id(bb), bb._version),
                           lambda: torch.cat([ba.detach(), bb.detach()], 0).contiguous())
        y = _conv_forward(x, None, wcat, bcat, 1, (ph, pw), act, wkey=wcat)
        ctx.save_for_backward(x, y if act is not None else None)
        ctx.wcat, ctx.params = wcat, (wa, ba, wb, bb)
        ctx.pad, ctx.act, ctx.ca = (ph, pw), act, ca
        ctx.uses = _use_holder(wa) if wa.requires_grad else None
        return y[..., :ca], y[..., ca:]

    @staticmethod
    def backward(ctx, da, db_):
        x, y = ctx.saved_tensors
        wa, ba, wb, bb = ctx.params
        wcat = ctx.wcat
        ph, pw = ctx.pad
        ca = ctx.ca
        ref = da if da is not None else db_
        shape = list(ref.shape)
        parts = []
        for g, c in ((da, ca), (db_, wcat.shape[0] - ca)):
            shape[-1] = c
            parts.append(g if g is not None else torch.zeros(shape, device=ref.device))
        g = _act_backward(torch.cat(parts, -1), y, ctx.act).contiguous()
        _, cin, kh, kw = wcat.shape
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _conv_forward(g, None, _flip_t(wcat), None, 1, (kh - 1 - ph, kw - 1 - pw))
        sinks = [_grad_sink(t) if t is not None and t.requires_grad else None for t in ctx.params]
        want = [t is not None and t.requires_grad for t in ctx.params]
        direct = all(s_ is not None or not w_ for s_, w_ in zip(sinks, want))
        with_bias = ba is not None
        hold = ctx.uses

        def flush(items, into_sinks=True):
            tw = torch.empty_like(wcat)
            tb = torch.empty(wcat.shape[0], device=wcat.device) if with_bias else None
            _flush_wgrad(items, wcat, with_bias, tw, tb, False, 1, ph, pw)
            return tw, tb

        if direct and hold is not None and hold["uses"] > 1:
            def flush_sinks(items):
                tw, tb = flush(items)
                sw_a, sb_a, sw_b, sb_b = sinks
                if sw_a is not None:
                    sw_a += tw[:ca]
                if sw_b is not None:
                    sw_b += tw[ca:]
                if with_bias and sb_a is not None:
                    sb_a += tb[:ca]
                if with_bias and sb_b is not None:
                    sb_b += tb[ca:]
            _defer(hold, (g, x, None), flush_sinks)
            return dx, None, None, None, None, None, None, None
        tw, tb = flush([(g, x, None)])
        grads = [tw[:ca], tb[:ca] if with_bias else None, tw[ca:], tb[ca:] if with_bias else None]
        if direct:
            for s_, gr in zip(sinks, grads):
                if s_ is not None and gr is not None:
                    s_ += gr
            grads = [None] * 4
        return (dx, *grads, None, None, None)


def dual_conv2d_nhwc(x: Tensor, wa: Tensor, ba: Optional[Tensor], wb: Tensor, bb: Optional[Tensor],
                     padding=0, act: Optional[str] = None) -> Tuple[Tensor, Tensor]:
    """(act(conv(x; wa, ba)), act(conv(x; wb, bb))) of channels-last x as one conv each way
    (stride 1, same kernel shape and padding): channel views of one output buffer."""
    ph, pw = (padding, padding) if isinstance(padding, int) else padding
    return _DualConv2dNHWC.apply(x, wa, ba, wb, bb, ph, pw, act)


def conv2d_nhwc_split(x: Tensor, weight: Tensor, split: int, bias: Optional[Tensor] = None,
                      stride: int = 1, padding=0, act: Optional[str] = None,
                      x1: Optional[Tensor] = None, bias_map: Optional[Tensor] = None):
    """``conv2d_nhwc`` returning (out[..., :split], out[..., split:])."""
    ph, pw = (padding, padding) if isinstance(padding, int) else padding
    return _Conv2dNHWCSplit.apply(x, x1, weight, bias, bias_map, stride, ph, pw, act, split)


def conv2d_nhwc(x: Tensor, weight: Tensor, bias: Optional[Tensor] = None, stride: int = 1,
                padding=0, act: Optional[str] = None, x1: Optional[Tensor] = None,
                bias_map: Optional[Tensor] = None, res_grad: Optional[ResidualGrad] = None) -> Tensor:
    """act(nn.Conv2d(cat[x, x1]) + bias_map) (cross-correlation) on channels-last tensors, HIP
    forward and backward.  ``x1``: optional second input (a channel concat without the copy);
    ``bias_map``: an [N, OH, OW, cout] tensor added before the activation; ``res_grad``: a
    ResidualGrad whose identity gradient this conv's dX adds (x is a residual block's input)."""
    ph, pw = (padding, padding) if isinstance(padding, int) else padding
    return _Conv2dNHWC.apply(x, x1, weight, bias, bias_map, stride, ph, pw, act, res_grad)


# ------------------------------------------------------------------------------- ConvGRU step
class _SharedWeight(torch.autograd.Function):
    """Identity node in front of a weight that several GRU steps of one forward pass use (the
    SepConvGRU's concatenated weights, 8 iterations).  The uses' backwards record their (dY, x0,
    x1) here and hand autograd no weight gradient; autograd runs THIS node's backward only after
    every use the pass reached, and it sums exactly the recorded ones in ONE batched weight
    gradient (scflow_conv_wgrad_batched).  The node belongs to one forward pass, so nothing is
    carried between passes, uses a pass never reaches contribute nothing, and a second backward
    over the same graph (retain_graph) records and sums afresh."""

    @staticmethod
    def forward(ctx, w):
        ctx.set_materialize_grads(False)
        ctx.items = []
        ctx.pad = None
        ctx.wmeta = w.detach()
        return w.view_as(w)

    @staticmethod
    def backward(ctx, g):
        items, ctx.items = ctx.items, []
        if not items:
            return g
        ph, pw = ctx.pad
        buf = torch.empty_like(ctx.wmeta)
        _flush_wgrad(items, ctx.wmeta, False, buf, None, False, 1, ph, pw)
        return buf if g is None else g + buf


def share_weight(w: Tensor) -> Tensor:
    """``w`` behind a _SharedWeight node: pass the result to every gru_step of a forward pass that
    uses this weight, so its weight gradient is one batched launch over all the uses."""
    return _SharedWeight.apply(w)


def _shared_node(w: Tensor):
    node = w.grad_fn
    return node if isinstance(node, _SharedWeight._backward_cls) else None


def _record_shared(node, item, ph: int, pw: int) -> None:
    if node.pad is None:
        node.pad = (ph, pw)
    node.items.append(item)


def _channel_rows(t: Tensor) -> bool:
    """``t`` [..., c] is a channel slice of a channels-last buffer (one pixel stride)."""
    if t.stride(-1) != 1 or t.stride(-2) < t.shape[-1] or t.stride(-2) % 4:
        return False
    return all(t.shape[i] == 1 or t.stride(i) == t.stride(i + 1) * t.shape[i + 1]
               for i in range(t.dim() - 2))


class _GruStep(torch.autograd.Function):
    """One SepConvGRU direction (raft_decoder.py:235-253) as one autograd node:
        zr = σ(conv([h, x]; w_zr) + pre_zr)      (z | r from one launch)
        q  = tanh(conv([r·h, x]; w_q) + pre_q)
        h' = h + z·(q − h)
    forward: the two HIP convs (activation and the hoisted context map fused) and two HIP gate
    kernels; backward: the gate / activation derivatives in two HIP kernels, the two convs' dX
    (the second adds the first's in its epilogue) and dW — instead of ~17 separate autograd kernels
    (lerp, mul, the activation backwards, slice concatenation, gradient accumulation)."""

    @staticmethod
    def forward(ctx, h, x, w_zr, w_q, pre_zr, pre_q, pad):
        h = h.contiguous()
        x = x.contiguous()
        zr = _conv_forward(h, x, w_zr.detach(), None, 1, pad, "Sigmoid", pre_zr.detach().contiguous(),
                           wkey=w_zr)
        rh = ops.gru_gate_forward(zr, h, torch.empty_like(h))
        q = _conv_forward(rh, x, w_q.detach(), None, 1, pad, "Tanh", pre_q.detach().contiguous(),
                          wkey=w_q)
        h2 = ops.gru_gate_forward(zr, h, torch.empty_like(h), q=q)
        ctx.save_for_backward(h, x, zr, rh, q, w_zr, w_q)
        ctx.pad = pad
        ctx.acc = (_shared_node(w_zr), _shared_node(w_q))  # gru_step puts both behind one
        return h2

    @staticmethod
    def backward(ctx, dh2):
        h, x, zr, rh, q, w_zr, w_q = ctx.saved_tensors
        ph, pw = ctx.pad
        c = h.shape[-1]
        _, _, kh, kw = w_q.shape
        dq = torch.empty_like(h)
        dzr = torch.empty_like(zr)
        dha = torch.empty_like(h)
        if not _channel_rows(dh2):
            dh2 = dh2.contiguous()
        ops.gru_gate_backward_q(dh2, zr, h, q, dq, dzr, dha)
        dxq = _conv_forward(dq, None, _flip_t(w_q), None, 1, (kh - 1 - ph, kw - 1 - pw))
        _record_shared(ctx.acc[1], (dq, rh, x), ph, pw)
        # dh = dha + drh·r written over drh = dxq[..., :c] itself, so that dxq becomes [dh | dx_q]
        # and the z | r conv's dX, with dxq as its added map, yields both sums in its epilogue:
        # T = [dh + dxz_h | dx_q + dxz_x] (no separate adds; dh and dx leave as channel views)
        ops.gru_gate_backward_r(dxq[..., :c], zr, h, dha, dzr, dxq[..., :c])
        t = _conv_forward(dzr, None, _flip_t(w_zr), None, 1, (kh - 1 - ph, kw - 1 - pw), bias_map=dxq)
        _record_shared(ctx.acc[0], (dzr, h, x), ph, pw)
        return t[..., :c], t[..., c:], None, None, dzr, dq, None


def gru_step(h: Tensor, x: Tensor, w_zr: Tensor, w_q: Tensor, pre_zr: Tensor, pre_q: Tensor,
             padding) -> Tensor:
    """h' of one SepConvGRU direction; channels-last h [.., c], x [.., cx]; w_zr [2c, c + cx, ..],
    w_q [c, c + cx, ..]; pre_zr / pre_q: the pre-activation maps added before σ / tanh.  Weights
    used by several steps of one pass should come through ``share_weight`` (one batched weight
    gradient for all the uses); any other tensor gets a node of its own (one use)."""
    pad = (padding, padding) if isinstance(padding, int) else tuple(padding)
    if _shared_node(w_zr) is None:
        w_zr = share_weight(w_zr)
    if _shared_node(w_q) is None:
        w_q = share_weight(w_q)
    return _GruStep.apply(h, x, w_zr, w_q, pre_zr, pre_q, pad)


# ------------------------------------------------------------------------------- pose update
class _PoseUpdate6(torch.autograd.Function):
    """get_pose_from_delta_pose with the ortho6d rotation (pose.py:124-169) as one HIP kernel
    forward and one backward (chain rule by hand) instead of ~90 tiny autograd kernels."""

    @staticmethod
    def forward(ctx, drot, dt, R, t, weight, depth_exp, detach_xy):
        drot, dt, R, t = (v.contiguous().float() for v in (drot, dt, R, t))
        ctx.save_for_backward(drot, dt, R, t)
        ctx.cfg = (weight, depth_exp, detach_xy)
        return ops.pose_update6_train(drot, dt, R, t, weight, depth_exp, detach_xy)

    @staticmethod
    def backward(ctx, gRn, gtn):
        drot, dt, R, t = ctx.saved_tensors
        gRn = torch.zeros_like(R) if gRn is None else gRn.contiguous()
        gtn = torch.zeros_like(t) if gtn is None else gtn.contiguous()
        gd, gdt, gR, gt = ops.pose_update6_train(drot, dt, R, t, *ctx.cfg, grads=(gRn, gtn))
        return gd, gdt, gR, gt, None, None, None


def pose_update6(drot: Tensor, dt: Tensor, R: Tensor, t: Tensor, weight: float = 10.0,
                 depth_exp: bool = True, detach_xy: bool = True):
    """(R_new [n,3,3], t_new [n,3]) from an ortho6d Δrotation [n,6] and Δt [n,3] (HIP fwd + bwd)."""
    return _PoseUpdate6.apply(drot, dt, R, t, float(weight), bool(depth_exp), bool(detach_xy))


# ------------------------------------------------------------------------------- norms
class _InstanceNormNHWC(torch.autograd.Function):
    """InstanceNorm2d(affine=False) (+ ReLU) of a channels-last [N, H, W, C] tensor on HIP kernels:
    fp64 statistics (scflow_enc_stats), one apply pass, and a three-launch backward
    (scflow_in_backward) — instead of torch's strided mean / var reductions and their autograd
    graph over the channels-last layout."""

    @staticmethod
    def forward(ctx, x, eps, relu):
        x = x.contiguous()
        n, h, w, c = x.shape
        scale = torch.empty(n, c, device=x.device)
        shift = torch.empty(n, c, device=x.device)
        ops.enc_instance_norm_stats(x, n, h * w, c, scale, shift, eps)
        y = torch.empty_like(x)
        ops.in_apply(x, scale, shift, y, n, h * w, c, relu)
        ctx.save_for_backward(x, scale, shift)
        ctx.relu = relu
        return y

    @staticmethod
    def backward(ctx, dy):
        x, scale, shift = ctx.saved_tensors
        n, h, w, c = x.shape
        dx = torch.empty_like(x)
        ops.in_backward(dy.contiguous(), x, scale, shift, dx, n, h * w, c, ctx.relu)
        return dx, None, None


class _InstanceNormResidualNHWC(torch.autograd.Function):
    """relu(InstanceNorm2d(x) + res): a residual block's tail (raft_encoder.py BasicBlock) as one
    HIP pass forward (statistics + scflow_in_apply_residual) and a three-launch backward that
    also writes the identity branch's gradient — instead of the norm's apply, the add, the ReLU
    and the ReLU's backward as separate kernels."""

    @staticmethod
    def forward(ctx, x, res, eps, res_grad=None):
        x = x.contiguous()
        res = res.contiguous()
        n, h, w, c = x.shape
        scale = torch.empty(n, c, device=x.device)
        shift = torch.empty(n, c, device=x.device)
        ops.enc_instance_norm_stats(x, n, h * w, c, scale, shift, eps)
        y = torch.empty_like(x)
        ops.in_apply_residual(x, scale, shift, res, y, n, h * w, c)
        ctx.save_for_backward(x, scale, shift, y)
        ctx.res_grad = res_grad
        return y

    @staticmethod
    def backward(ctx, dy):
        x, scale, shift, y = ctx.saved_tensors
        n, h, w, c = x.shape
        dx = torch.empty_like(x)
        dres = torch.empty_like(x)
        ops.in_backward_residual(dy.contiguous(), x, scale, shift, y, dx, dres, n, h * w, c)
        if ctx.res_grad is not None:  # handed to the block's first conv (ResidualGrad)
            ctx.res_grad.d = dres
            return dx, None, None, None
        return dx, dres, None, None


def instance_norm_residual_relu_nhwc(x: Tensor, res: Tensor, eps: float = 1e-5,
                                     res_grad: Optional[ResidualGrad] = None) -> Tensor:
    """relu(InstanceNorm2d(affine=False)(x) + res) of channels-last tensors (HIP fwd + bwd).
    ``res_grad``: hand res's gradient to the conv given the same ResidualGrad instead of
    returning it (res must be that conv's input)."""
    return _InstanceNormResidualNHWC.apply(x, res, float(eps), res_grad)


class _BatchNormNHWC(torch.autograd.Function):
    """BatchNorm2d in train mode (+ ReLU, + a residual identity before the ReLU) of a
    channels-last tensor: batch statistics in fp64, running statistics updated in the same
    launch sequence, one apply pass (scflow_bn_forward); backward in three launches that also
    give dγ / dβ (added straight into the parameters' gradients when they are direct sinks) and,
    in the residual form, the identity's gradient (scflow_bn_backward) — instead of MIOpen's
    batch norm on permuted views plus the ReLU, the add and their backwards as separate kernels
    (the context encoder, resnet.py BasicBlock with norm_fn 'batch')."""

    @staticmethod
    def forward(ctx, x, weight, bias, res, running_mean, running_var, momentum, eps, relu, res_grad):
        x = x.contiguous()
        res = None if res is None else res.contiguous()
        y = torch.empty_like(x)
        w = None if weight is None else weight.detach()
        b = None if bias is None else bias.detach()
        rstd, shift = ops.bn_forward(x, w, b, y, running_mean, running_var, eps, momentum, relu, res)
        ctx.save_for_backward(x, rstd, shift, y if res is not None else None)
        ctx.wb = (weight, bias)  # the leaves themselves (direct gradient accumulation)
        ctx.relu, ctx.has_res, ctx.res_grad = relu, res is not None, res_grad
        return y

    @staticmethod
    def backward(ctx, dy):
        x, rstd, shift, y = ctx.saved_tensors
        weight, bias = ctx.wb
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if ctx.has_res else None
        dw = db = None
        want_w = weight is not None and ctx.needs_input_grad[1]
        want_b = bias is not None and ctx.needs_input_grad[2]
        sw = _grad_sink(weight) if want_w else None
        sb = _grad_sink(bias) if want_b else None
        direct = (sw is not None or not want_w) and (sb is not None or not want_b)
        if direct:
            gw, gb = sw, sb
        else:
            gw = torch.empty_like(weight) if want_w else None
            gb = torch.empty_like(bias) if want_b else None
        ops.bn_backward(dy.contiguous(), x, rstd, shift,
                        None if weight is None else weight.detach(),
                        None if bias is None else bias.detach(), dx, gw, gb, ctx.relu,
                        y=y, dres=dres, accumulate=direct)
        if not direct:
            dw, db = gw, gb
        if dres is not None and ctx.res_grad is not None:  # handed to the block's first conv
            ctx.res_grad.d = dres
            dres = None
        return dx, dw, db, dres, None, None, None, None, None, None


def batch_norm_nhwc(x: Tensor, mod, relu: bool = False, res: Optional[Tensor] = None,
                    res_grad: Optional[ResidualGrad] = None) -> Tensor:
    """``mod`` (BatchNorm2d, train mode, float momentum) of channels-last x, then + res and ReLU
    (res given: relu(bn(x) + res), the residual block's tail) — HIP forward and backward, the
    running statistics and num_batches_tracked updated as F.batch_norm(training=True) does."""
    y = _BatchNormNHWC.apply(x, mod.weight, mod.bias, res, mod.running_mean, mod.running_var,
                             float(mod.momentum), float(mod.eps), bool(relu or res is not None),
                             res_grad)
    if mod.num_batches_tracked is not None:
        mod.num_batches_tracked.add_(1)
    return y


def bn_fusable(mod, x: Tensor) -> bool:
    """BatchNorm2d modules batch_norm_nhwc takes: train mode with running statistics and a float
    momentum (SCFlow's context encoder), channels a multiple of 4, at most 256, on the GPU."""
    return (isinstance(mod, torch.nn.BatchNorm2d) and mod.training and mod.track_running_stats
            and mod.momentum is not None and x.is_cuda and x.shape[-1] % 4 == 0
            and x.shape[-1] <= 256 and (mod.weight is None) == (mod.bias is None))


def instance_norm_nhwc(x: Tensor, eps: float = 1e-5, relu: bool = False) -> Tensor:
    """InstanceNorm2d(affine=False) (then ReLU if ``relu``) of channels-last x, HIP fwd + bwd
    (channels a multiple of 4, at most 256)."""
    return _InstanceNormNHWC.apply(x, float(eps), bool(relu))


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
        ctx.holder = _dpyr_holder(buf)
        return buf

    @staticmethod
    def backward(ctx, dbuf):
        # the lookups' shared gradient buffer is consumed: the next backward pass over this graph
        # (retain_graph, torch.autograd.grad) starts from a fresh one
        ctx.holder["buf"] = None
        ctx.holder["seen"] = 0
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
        df1 = ops.gemm(F2, dC.transpose(1, 2))  # [n][c][p] = Σ_q F2[c][q] dC[p][q]
        df2 = ops.gemm(F1, dC)                  # [n][c][q] = Σ_p F1[c][p] dC[p][q]
        return df1.view_as(f1), df2.view_as(f2), None


def corr_pyramid(f1: Tensor, f2: Tensor, num_levels: int = 4) -> Tensor:
    return _CorrPyramid.apply(f1, f2, num_levels)


def _dpyr_holder(pyr: Tensor) -> dict:
    """The lookups' shared pyramid-gradient accumulator, kept on the pyramid tensor: ``uses`` =
    lookups recorded on it, ``seen`` = lookup backwards run in the current backward pass; the
    buffer is released when a pass has seen every use or when the pyramid's backward consumes it."""
    holder = getattr(pyr, "_scflow_dpyr", None)
    if holder is None:
        holder = {"buf": None, "uses": 0, "seen": 0}
        try:
            pyr._scflow_dpyr = holder
        except (AttributeError, RuntimeError):
            pass
    return holder


class _CorrLookup(torch.autograd.Function):
    """The pyramid is looked up once per refinement iteration; every iteration's backward
    scatters into ONE gradient buffer shared through the pyramid tensor (zeroed once per step):
    the first backward call hands that buffer to autograd, the later ones add into it in place
    and hand over nothing — autograd runs the pyramid's backward only after all of them, so it
    sees the complete sum, without a zeroed buffer and a full-size add per iteration."""

    @staticmethod
    def forward(ctx, pyr, flow_nhwc, n, h, w, num_levels, radius):
        flow_nhwc = flow_nhwc.contiguous()
        ctx.save_for_backward(flow_nhwc)
        holder = ctx.holder = _dpyr_holder(pyr)
        holder["uses"] += 1
        ctx.dims = (n, h, w, num_levels, radius, pyr.numel())
        out = torch.empty(n * h * w, num_levels * (2 * radius + 1) ** 2, device=pyr.device)
        ops.corr_lookup(pyr, flow_nhwc, n, h, w, num_levels, radius, out=Chan.whole(out),
                        flow_layout="nhwc")
        return out.view(n, h, w, -1)

    @staticmethod
    def backward(ctx, dout):
        (flow,) = ctx.saved_tensors
        n, h, w, L, r, size = ctx.dims
        hd = ctx.holder
        first = hd["buf"] is None
        if first:
            hd["buf"] = torch.zeros(size, device=dout.device)
        dpyr = hd["buf"]
        ops.corr_lookup_backward(dout.contiguous().view(n * h * w, -1), flow, dpyr, n, h, w, L, r)
        hd["seen"] += 1
        if hd["seen"] >= hd["uses"]:  # every lookup of this pass added its share: release it
            hd["buf"] = None
            hd["seen"] = 0
        return (dpyr if first else None), None, None, None, None, None, None


def corr_lookup(pyr: Tensor, flow_nhwc: Tensor, n: int, h: int, w: int, num_levels: int = 4,
                radius: int = 4) -> Tensor:
    """[n, h, w, L·(2r+1)²] channels-last lookup; differentiable w.r.t. the pyramid only."""
    return _CorrLookup.apply(pyr, flow_nhwc.detach(), n, h, w, num_levels, radius)


# ------------------------------------------------------------------------------- upsampling
_INTERP = {}


def _interp_matrix(n_in: int, n_out: int, device) -> Tensor:
    """[n_out, n_in] bilinear weights of align_corners=True resampling along one axis (source
    coordinate o·(n_in−1)/(n_out−1), as ATen's upsample_bilinear2d)."""
    key = (n_in, n_out, str(device))
    m = _INTERP.get(key)
    if m is None:
        scale = (n_in - 1) / (n_out - 1) if n_out > 1 else 0.0
        src = torch.arange(n_out, dtype=torch.float32) * torch.tensor(scale, dtype=torch.float32)
        i0 = src.floor().long().clamp(max=n_in - 1)
        lam = src - i0.float()
        i1 = (i0 + 1).clamp(max=n_in - 1)
        m = torch.zeros(n_out, n_in)
        m.index_put_((torch.arange(n_out), i0), 1.0 - lam, accumulate=True)
        m.index_put_((torch.arange(n_out), i1), lam, accumulate=True)
        m = _INTERP[key] = m.to(device)
    return m


class _UpsampleAC(torch.autograd.Function):
    """F.interpolate(x, scale_factor=s, mode="bilinear", align_corners=True) on NCHW x; the
    backward is the separable adjoint Ayᵀ·g·Ax as two GEMMs on the HIP fp32 MFMA GEMM instead of
    ATen's atomic scatter (75 µs per 16×2×256² gradient; the full-resolution flow / mask of
    every refinement iteration, scflow_decoder.py:223-228)."""

    @staticmethod
    def forward(ctx, x, s):
        ctx.hw = x.shape[-2:]
        return F.interpolate(x, scale_factor=(s, s), mode="bilinear", align_corners=True)

    @staticmethod
    def backward(ctx, g):
        h, w = ctx.hw
        n, c, H, W = g.shape
        ax = _interp_matrix(w, W, g.device)   # [W, w]
        ayt = _interp_matrix(h, H, g.device).t()  # [h, H]
        t = ops.gemm(g.contiguous().view(n * c * H, W), ax)  # [n·c·H, w]
        dx = ops.gemm(ayt.unsqueeze(0).expand(n * c, h, H), t.view(n * c, H, w))
        return dx.view(n, c, h, w), None


class _UpL1Loss(torch.autograd.Function):
    """weight·Σ v·|sval·up(f) − target| / denom with the ×(H/h) align_corners upsampling of the
    channels-last low-resolution f fused into the loss (scflow_up_l1_loss: one pass over the
    full-resolution target, no upsampled tensor); backward = the upsampling's GEMM adjoint of
    the saved v·sgn map, scaled by g·weight·sval/denom."""

    @staticmethod
    def forward(ctx, f, target, vmask, sval, denom, cdenom, weight):
        f = f.contiguous()
        loss, sgn = ops.up_l1_loss(f, target.contiguous(), None if vmask is None else vmask.contiguous(),
                                   sval, denom, cdenom, weight)
        ctx.save_for_backward(sgn, denom if denom is not None else torch.empty(0))
        ctx.cfg = (f.shape, sval, cdenom, weight, denom is not None)
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        sgn, denom = ctx.saved_tensors
        (n, h, w, c), sval, cdenom, weight, has_denom = ctx.cfg
        H, W = sgn.shape[-2:]
        ax = _interp_matrix(w, W, sgn.device)
        ayt = _interp_matrix(h, H, sgn.device).t()
        t = ops.gemm(sgn.view(n * c * H, W), ax)
        dx = ops.gemm(ayt.unsqueeze(0).expand(n * c, h, H), t.view(n * c, H, w)).view(n, c, h, w)
        coef = g * (weight * sval) / (denom[0] if has_denom else cdenom)
        return (dx * coef).permute(0, 2, 3, 1), None, None, None, None, None, None


def up_l1_loss(f_nhwc: Tensor, target: Tensor, vmask: Optional[Tensor], sval: float,
               denom: Optional[Tensor], cdenom: float, weight: float) -> Tensor:
    """Fused upsample + masked L1 loss (see _UpL1Loss); target NCHW at full resolution."""
    return _UpL1Loss.apply(f_nhwc, target, vmask, float(sval), denom, float(cdenom), float(weight))


def upsample_bilinear_ac(x: Tensor, scale: int) -> Tensor:
    """Bilinear ×scale upsampling with align_corners=True of NCHW x (torch forward, GEMM backward)."""
    return _UpsampleAC.apply(x, scale)


# ------------------------------------------------------------------------------- group norm
class _GroupNormNHWC(torch.autograd.Function):
    """GroupNorm (+ReLU) on channels-last data, 4 channels per group (the pose head's GN(32) on
    128 channels): one HIP launch forward, two backward (dx + per-image γ/β partials, then their
    ordered sum — added straight into the parameters' .grad under direct_weight_grads) instead of
    the NCHW copies, native_group_norm(_backward), the ReLU and its backward and the
    AccumulateGrad adds."""

    @staticmethod
    def forward(ctx, x, w, b, groups, eps, relu):
        x = x.contiguous()
        y, stats = ops.group_norm_forward(x, w.detach().contiguous(), b.detach().contiguous(),
                                          groups, eps, relu)
        ctx.save_for_backward(x, w, b, stats)
        ctx.groups, ctx.relu = groups, relu
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, stats = ctx.saved_tensors
        sw, sb = _grad_sink(w), _grad_sink(b)
        direct = sw is not None and sb is not None
        dw = sw if direct else torch.empty_like(w)
        db = sb if direct else torch.empty_like(b)
        dx = ops.group_norm_backward(dy.contiguous(), x, w.detach().contiguous(), b.detach().contiguous(),
                                     stats, ctx.groups, ctx.relu, dw, db, accumulate=direct)
        return dx, (None if direct else dw), (None if direct else db), None, None, None


def group_norm_nhwc(x: Tensor, weight: Tensor, bias: Tensor, groups: int, eps: float,
                    relu: bool = False) -> Tensor:
    """F.group_norm (+ReLU) of a channels-last tensor with 4 channels per group (HIP)."""
    return _GroupNormNHWC.apply(x, weight, bias, groups, eps, relu)


# ------------------------------------------------------------------------------- linear
def _flush_linear(items, sink_w: Tensor, sink_b: Optional[Tensor]) -> None:
    """dW += Σ_uses dYᵀ·X as ONE GEMM over the uses' rows (the pose head's FC layers: 8 uses of
    16 rows each — a 16-deep GEMM per use is all launch latency), db += the column sum."""
    dys = torch.cat([d for d, _ in items])
    xs = torch.cat([x for _, x in items])
    ops.gemm(dys.t(), xs, out=sink_w, beta=1.0)
    if sink_b is not None:
        ops.colsum(dys, sink_b, accumulate=True)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        x = x.contiguous()
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        ctx.bias = b
        ctx.uses = _use_holder(w) if w.requires_grad else None
        return ops.gemm(x, w.detach().t(), bias=None if b is None else b.detach().contiguous())

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        dx = ops.gemm(dy, w.detach()) if ctx.needs_input_grad[0] else None
        dw = db = None
        want_b = ctx.has_b and ctx.needs_input_grad[2]
        hold = getattr(ctx, "uses", None)
        sw = _grad_sink(w) if ctx.needs_input_grad[1] else None
        sb = _grad_sink(ctx.bias) if want_b else None
        if (_DEFER_LINEAR and hold is not None and hold["uses"] > 1 and sw is not None
                and (sb is not None or not want_b) and (want_b or not ctx.has_b)):
            # a layer run once per refinement iteration: its uses' weight gradients as one GEMM
            # at the last use, added straight into the parameters
            _defer(hold, (dy, x), lambda items: _flush_linear(items, sw, sb))
            return dx, None, None
        if ctx.needs_input_grad[1]:
            sw = _grad_sink(w)
            if sw is not None:  # dW added in place: beta = 1 onto the parameter's .grad
                ops.gemm(dy.t(), x, out=sw, beta=1.0)
            else:
                dw = ops.gemm(dy.t(), x)
        if ctx.has_b and ctx.needs_input_grad[2]:
            sb = _grad_sink(ctx.bias)
            if sb is not None:
                ops.colsum(dy, sb, accumulate=True)
            else:
                db = ops.colsum(dy, torch.empty(dy.shape[1], device=dy.device))
        return dx, dw, db


def linear(x: Tensor, weight: Tensor, bias: Optional[Tensor] = None) -> Tensor:
    """F.linear(x, weight, bias) for 2-D x on the HIP GEMM, forward and backward."""
    return _Linear.apply(x, weight, bias)
