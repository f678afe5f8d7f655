"""Drop-in modules of SCFlow's update block, backed by the gfx950 HIP kernels.

Same class names, constructor arguments, forward signatures and state-dict keys as the
reference, so configs, checkpoints and callers work unchanged:

=====================  =====================================================================
module                 reference
=====================  =====================================================================
ConvModule             mmcv ConvModule (conv → norm → act; ``bias = norm is None``)
CorrelationPyramid     models/decoder/raft_decoder.py:19-58
CorrLookup             models/utils/corr_lookup.py:71-136
MotionEncoder          models/decoder/raft_decoder.py:61-166
ConvGRU                models/decoder/raft_decoder.py:168-253
XHead                  models/decoder/raft_decoder.py:256-294
MultiClassPoseHead     models/head/pose_head.py:110-211
=====================  =====================================================================

The NCHW ``forward`` of each module is the reference API (it converts to channels-last,
runs the HIP kernels, converts back).  ``SCFlowDecoder`` (decoder.py) does not go through
these per-module forwards: it keeps every activation channels-last in a few shared buffers
and calls the kernels directly (``ConvRunner``), so no NCHW round trips happen in the loop.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib, library, ops
from ._lib import EPI_GRU_Q, EPI_GRU_ZR, EPI_PLAIN, ScflowError
from .ops import Chan
from .registry import MODELS

Tensor = torch.Tensor


def _pair(v) -> Tuple[int, int]:
    return (v, v) if isinstance(v, int) else (int(v[0]), int(v[1]))


class ConvModule(nn.Module):
    """mmcv ``ConvModule`` as SCFlow uses it: conv (+GroupNorm) (+act), key layout
    ``conv.weight``/``conv.bias``/``gn.weight``/``gn.bias``; ``act_cfg=None`` → identity."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size, stride=1, padding=0,
                 conv_cfg: Optional[dict] = None, norm_cfg: Optional[dict] = None,
                 act_cfg: Optional[dict] = dict(type="ReLU"), **kwargs):
        super().__init__()
        if conv_cfg is not None and conv_cfg.get("type", "Conv2d") != "Conv2d":
            raise NotImplementedError(f"conv_cfg {conv_cfg} is not supported")
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                              bias=norm_cfg is None)
        self.norm_type = None
        if norm_cfg is not None:
            if norm_cfg["type"] != "GN":
                raise NotImplementedError(f"norm {norm_cfg['type']} is not on the SCFlow decoder path")
            self.norm_type = "GN"
            self.gn = nn.GroupNorm(norm_cfg["num_groups"], out_channels)
        self.act_type = None if act_cfg is None else act_cfg["type"]
        if self.act_type not in (None, "ReLU", "Sigmoid", "Tanh"):
            raise NotImplementedError(f"activation {self.act_type}")

    @property
    def kernel_size(self) -> Tuple[int, int]:
        return _pair(self.conv.kernel_size)

    @property
    def padding(self) -> Tuple[int, int]:
        return _pair(self.conv.padding)

    def forward_torch(self, x: Tensor) -> Tensor:
        """Stock PyTorch-ROCm path (MIOpen conv + GN) — used only by the pose head."""
        y = self.conv(x)
        if self.norm_type == "GN":
            y = self.gn(y)
        if self.act_type == "ReLU":
            y = torch.relu(y)
        elif self.act_type == "Sigmoid":
            y = torch.sigmoid(y)
        elif self.act_type == "Tanh":
            y = torch.tanh(y)
        return y

    def forward(self, x: Tensor) -> Tensor:
        if self.norm_type is not None or self.conv.stride != (1, 1):
            return self.forward_torch(x)
        n, c, h, w = x.shape
        r = ConvRunner.of(self.conv, self.act_type)
        src = torch.empty(n * h * w, c, device=x.device)
        ops.nchw_into(x.contiguous(), Chan.whole(src))
        dst = torch.empty(n * h * w, self.conv.out_channels, device=x.device)
        r.run(Chan.whole(src), Chan.whole(dst), n, h, w)
        return ops.chan_to_nchw(Chan.whole(dst), n, h, w)


class ConvRunner:
    """Packs one (or several cout-concatenated) nn.Conv2d weights for scflow_conv2d and runs it.

    The packed copy is cached and re-packed whenever a weight's data pointer or version
    changes (optimizer step, load_state_dict, .to())."""
    force_bk = 0  # 8 / 16 overrides the library's per-launch K-stage depth (tuning only)

    def __init__(self, convs: Sequence[nn.Conv2d], act: Optional[str], split: Optional[int] = None,
                 in_select: Optional[Sequence[Tuple[int, int]]] = None, with_bias: bool = True):
        """``in_select``: keep only these [start, end) input-channel ranges of the weights (the
        rest of the input is accounted for elsewhere, e.g. by a bias map); ``with_bias=False``
        drops the bias (folded into that bias map)."""
        self.convs = list(convs)
        c0 = self.convs[0]
        self.kh, self.kw = _pair(c0.kernel_size)
        self.ph, self.pw = _pair(c0.padding)
        self.stride = _pair(c0.stride)[0]
        self.cout = sum(c.out_channels for c in self.convs)
        self.in_select = None if in_select is None else [tuple(r) for r in in_select]
        self.cin = c0.in_channels if in_select is None else sum(b - a for a, b in self.in_select)
        self.with_bias = with_bias
        self.act = act
        self.split = split
        self._key = None
        self._packed = None
        self._bias = None

    @staticmethod
    def of(conv: nn.Conv2d, act: Optional[str]) -> "ConvRunner":
        r = getattr(conv, "_scflow_runner", None)
        if r is None or r.act != act:
            r = ConvRunner([conv], act)
            conv._scflow_runner = r
        return r

    def packed(self, c0: int, c1: int, w: int, bk: int = 16) -> Tuple[Tensor, Optional[Tensor]]:
        key = (c0, c1, w, bk, _lib.weights_generation()) + tuple((c.weight.data_ptr(), c.weight._version,
                                   None if c.bias is None else (c.bias.data_ptr(), c.bias._version))
                                  for c in self.convs)
        if key != self._key:
            wt = torch.cat([c.weight.detach() for c in self.convs], 0) if len(self.convs) > 1 \
                else self.convs[0].weight.detach()
            if self.in_select is not None:
                wt = torch.cat([wt[:, a:b] for a, b in self.in_select], 1).contiguous()
            self._packed = ops.pack_conv_weight(wt.float(), c0, c1, w, self.stride, bk)
            if not self.with_bias:
                self._bias = None
            elif all(c.bias is not None for c in self.convs):
                self._bias = torch.cat([c.bias.detach().float() for c in self.convs]).contiguous()
            elif any(c.bias is not None for c in self.convs):
                raise ValueError("cannot fuse convs with and without bias")
            else:
                self._bias = None
            self._key = key
        return self._packed, self._bias

    def args(self, src0: Chan, out: Optional[Chan], n: int, h: int, w: int,
             src1: Optional[Chan] = None, epilogue: int = EPI_PLAIN, gate: Optional[Chan] = None,
             rh: Optional[Chan] = None, hid: Optional[Chan] = None,
             bias_map: Optional[Chan] = None):
        """``run``'s scflow_conv_args (weights packed now; the runner keeps them) without
        launching — for ``ops.conv2d_pair``."""
        return self.bind(src0, out, n, h, w, src1, epilogue, gate, rh, hid, bias_map).args

    def bind(self, src0: Chan, out: Optional[Chan], n: int, h: int, w: int,
             src1: Optional[Chan] = None, epilogue: int = EPI_PLAIN, gate: Optional[Chan] = None,
             rh: Optional[Chan] = None, hid: Optional[Chan] = None,
             bias_map: Optional[Chan] = None) -> "ops.BoundLaunch":
        """``run``'s launch with its arguments fixed (weights packed now, buffers persistent):
        calling the result launches it on the current stream.  Re-bind after the weights or
        buffers change."""
        c1 = 0 if src1 is None else src1.c
        if src0.c + c1 != self.cin:
            raise ValueError(f"conv expects {self.cin} input channels, got {src0.c}+{c1}")
        shape = (n, h, w, src0.c, c1)
        if ConvRunner.force_bk:
            self._bk_shape, self._bk = shape, ConvRunner.force_bk
        if getattr(self, "_bk_shape", None) != shape:
            self._bk = ops.conv_pick_bk(n, h, w, src0.c, c1, self.cout, self.kh, self.kw, self.ph,
                                        self.pw, self.stride)
            self._bk_shape = shape
        packed, bias = self.packed(src0.c, c1, w, self._bk)
        args = ops.conv2d_args(src0, packed, bias, n, h, w, self.cout, self.kh, self.kw, self.ph,
                               self.pw, self.act, out=out, src1=src1, epilogue=epilogue, gate=gate,
                               rh=rh, hid=hid, stride=self.stride, bias_map=bias_map, bk=self._bk)
        bl = ops.BoundLaunch(_lib.load().scflow_conv2d, args, src0.buf.device.index, "scflow_conv2d")
        bl.keep = (packed, bias)  # the launch holds the packed weights alive
        return bl

    def run(self, src0: Chan, out: Optional[Chan], n: int, h: int, w: int,
            src1: Optional[Chan] = None, epilogue: int = EPI_PLAIN, gate: Optional[Chan] = None,
            rh: Optional[Chan] = None, hid: Optional[Chan] = None,
            bias_map: Optional[Chan] = None) -> None:
        c1 = 0 if src1 is None else src1.c
        if src0.c + c1 != self.cin:
            raise ValueError(f"conv expects {self.cin} input channels, got {src0.c}+{c1}")
        shape = (n, h, w, src0.c, c1)
        if ConvRunner.force_bk:  # tuning / A-B only
            self._bk_shape, self._bk = shape, ConvRunner.force_bk
        if getattr(self, "_bk_shape", None) != shape:  # host-only query, once per launch shape
            self._bk = ops.conv_pick_bk(n, h, w, src0.c, c1, self.cout, self.kh, self.kw, self.ph,
                                        self.pw, self.stride)
            self._bk_shape = shape
        packed, bias = self.packed(src0.c, c1, w, self._bk)
        ops.conv2d(src0, packed, bias, n, h, w, self.cout, self.kh, self.kw, self.ph, self.pw,
                   self.act, out=out, src1=src1, epilogue=epilogue, gate=gate, rh=rh, hid=hid,
                   stride=self.stride, bias_map=bias_map, bk=self._bk)

    def flops(self, m: int) -> float:
        """Algorithmic FLOPs of one launch over m output pixels (2·m·cout·taps·cin)."""
        return 2.0 * m * self.cout * self.kh * self.kw * self.cin

    @property
    def winograd(self) -> bool:
        """True once a launch picked the Winograd kernel (F(2×2,3×3) or F(4,5))."""
        return getattr(self, "_bk", None) in (_lib.CONV_WINO, _lib.CONV_WINO4)

    @property
    def wino4(self) -> bool:
        """True once a launch picked F(4×4,3×3) (transform launch + point-GEMM launch)."""
        return getattr(self, "_bk", None) == _lib.CONV_WINO4

    def mfma_flops(self, m: int, c0: int, c1: int = 0) -> float:
        """FLOPs the matrix cores execute for one launch over m output pixels with the inputs
        split c0 + c1: the Winograd kernels multiply per transform point (16 per 2×2 tile for
        3×3, 8 per 4-pixel tile for 1×5 / 5×1) over channels padded to 32 per source and output
        channels padded to 32; the direct kernel does the algorithmic work on padded channels."""
        ru = lambda v, q: (v + q - 1) // q * q  # noqa: E731
        kpad, npad = ru(c0, 32) + ru(c1, 32), ru(self.cout, 32)
        if getattr(self, "_bk", None) == _lib.CONV_WINO4:  # 36 points per 4×4 tile, K padded to 8
            return 2.0 * 36 * (m / 16) * (ru(c0, 8) + ru(c1, 8)) * npad
        if self.winograd:
            pts, tile = (16, 4) if self.kh * self.kw == 9 else (8, 4)
            return 2.0 * pts * (m / tile) * kpad * npad
        if getattr(self, "_bk", None) == _lib.CONV_1X1W:  # K padded to 8, N to 64
            return 2.0 * m * ru(self.cout, 64) * ru(c0, 8)
        return 2.0 * m * npad * self.kh * self.kw * (ru(c0, 16) + ru(c1, 16))


# ---------------------------------------------------------------------------------- a1 / a2
class CorrelationPyramid(nn.Module):
    """raft_decoder.py:19-58; returns the levels as views of one HIP-built buffer."""

    def __init__(self, num_levels: int = 4) -> None:
        super().__init__()
        self.num_levels = num_levels

    def forward(self, feat1: Tensor, feat2: Tensor) -> List[Tensor]:
        n, _, h, w = feat1.shape
        buf = library.corr_pyramid(feat1, feat2, self.num_levels)  # torch.ops.scflow.corr_pyramid
        return ops.pyramid_views(buf, n, h, w, self.num_levels)


class CorrLookup(nn.Module):
    """corr_lookup.py:71-136: bilinear, zero padding, align_corners True (SCFlow's config) or
    False (bilinear_sample's default, corr_lookup.py:35)."""

    def __init__(self, radius: int = 4, mode: str = "bilinear", padding_mode: str = "zeros",
                 align_corners: bool = True) -> None:
        super().__init__()
        if mode != "bilinear" or padding_mode != "zeros":
            raise NotImplementedError("CorrLookup kernel: bilinear sampling with zero padding only")
        self.r = radius
        self.mode = mode
        self.padding_mode = padding_mode
        self.align_corners = align_corners

    def forward(self, corr_pyramid: Sequence[Tensor], flow: Tensor) -> Tensor:
        B, _, H, W = flow.shape
        base = corr_pyramid[0]._base
        if torch.compiler.is_compiling():  # (storage offsets are not traceable)
            buf = torch.cat([lv.reshape(-1) for lv in corr_pyramid])
        elif (base is not None and base.dim() == 1 and
                base.numel() == library.pyramid_numel(B, H, W, len(corr_pyramid)) and
                all(lv._base is base for lv in corr_pyramid) and
                [lv.storage_offset() - base.storage_offset() for lv in corr_pyramid] ==
                [sum(B * H * W * (H >> k) * (W >> k) for k in range(l)) for l in range(len(corr_pyramid))]):
            buf = base  # CorrelationPyramid's flat buffer itself: autograd reaches every level
        elif any(lv.requires_grad for lv in corr_pyramid):
            buf = torch.cat([lv.reshape(-1) for lv in corr_pyramid])  # (no aliasing view: autograd)
        else:
            buf = ops.pyramid_buffer(corr_pyramid, B, H, W)
        # torch.ops.scflow.corr_lookup
        return library.corr_lookup(buf, flow.float(), len(corr_pyramid), self.r, self.align_corners)


# ---------------------------------------------------------------------------------- a3
class MotionEncoder(nn.Module):
    """raft_decoder.py:61-166 (same channel tables)."""
    _corr_channels = {"Basic": (256, 192), "Small": 96, "Large": (256, 192)}
    _corr_kernel = {"Basic": (1, 3), "Small": 1, "Large": (1, 3)}
    _corr_padding = {"Basic": (0, 1), "Small": 0, "Large": (0, 1)}
    _flow_channels = {"Basic": (128, 64), "Small": (64, 32), "Large": (128, 64)}
    _flow_kernel = {"Basic": (7, 3), "Small": (7, 3), "Large": (7, 3)}
    _flow_padding = {"Basic": (3, 1), "Small": (3, 1), "Large": (3, 1)}
    _out_channels = {"Basic": 126, "Small": 80, "Large": 126}
    _out_kernel = {"Basic": 3, "Small": 3, "Large": 3}
    _out_padding = {"Basic": 1, "Small": 1, "Large": 1}

    def __init__(self, num_levels: int = 4, radius: int = 4, net_type: str = "Basic",
                 conv_cfg=None, norm_cfg=None, act_cfg=None, **kwargs) -> None:
        super().__init__()
        assert net_type in ["Basic", "Small", "Large"]

        def lst(v):
            return list(v) if isinstance(v, (tuple, list)) else [v]

        corr_ch, corr_k, corr_p = (lst(self._corr_channels[net_type]), lst(self._corr_kernel[net_type]),
                                   lst(self._corr_padding[net_type]))
        self.out_channels = lst(self._out_channels[net_type])
        self.act_cfg = act_cfg
        mk = dict(conv_cfg=conv_cfg, norm_cfg=norm_cfg, act_cfg=act_cfg)
        self.corr_net = nn.Sequential(*self._make(num_levels * (2 * radius + 1) ** 2, corr_ch, corr_k,
                                                  corr_p, mk))
        self.flow_net = nn.Sequential(*self._make(2, lst(self._flow_channels[net_type]),
                                                  lst(self._flow_kernel[net_type]),
                                                  lst(self._flow_padding[net_type]), mk))
        self.out_net = nn.Sequential(*self._make(corr_ch[-1] + lst(self._flow_channels[net_type])[-1],
                                                 self.out_channels, lst(self._out_kernel[net_type]),
                                                 lst(self._out_padding[net_type]), mk))

    @staticmethod
    def _make(cin, chans, kernels, pads, mk):
        layers = []
        for ch, k, p in zip(chans, kernels, pads):
            layers.append(ConvModule(cin, ch, k, padding=p, **mk))
            cin = ch
        return layers

    def forward(self, corr: Tensor, flow: Tensor) -> Tensor:
        n, _, h, w = corr.shape
        dev = corr.device
        M = n * h * w
        cc = self.corr_net[-1].conv.out_channels
        cf = self.flow_net[-1].conv.out_channels
        co = self.out_channels[0]
        cbuf = torch.empty(M, corr.shape[1], device=dev)
        ops.nchw_into(corr.contiguous(), Chan.whole(cbuf))
        fbuf = torch.empty(M, 2, device=dev)
        ops.nchw_into(flow.contiguous(), Chan.whole(fbuf))
        mf = torch.empty(M, cc + cf, device=dev)
        run_chain(self.corr_net, Chan.whole(cbuf), Chan(mf, 0, cc), n, h, w)
        run_chain(self.flow_net, Chan.whole(fbuf), Chan(mf, cc, cf), n, h, w)
        out = torch.empty(M, co + 2, device=dev)
        run_chain(self.out_net, Chan.whole(mf), Chan(out, 0, co), n, h, w)
        out[:, co:].copy_(fbuf)
        return ops.chan_to_nchw(Chan.whole(out), n, h, w)


def bind_chain(layers: Sequence[ConvModule], src: Chan, dst: Chan, n: int, h: int, w: int,
               scratch: List[Tensor]) -> List["ops.BoundLaunch"]:
    """run_chain's launches bound once (see ConvRunner.bind)."""
    out_l, cur = [], src
    for i, m in enumerate(layers):
        out = dst if i == len(layers) - 1 else Chan.whole(scratch[i])
        out_l.append(ConvRunner.of(m.conv, m.act_type).bind(cur, out, n, h, w))
        cur = out
    return out_l


def run_chain(layers: Sequence[ConvModule], src: Chan, dst: Chan, n: int, h: int, w: int,
              scratch: Optional[List[Tensor]] = None, hooks: Optional[Sequence] = None) -> None:
    """Run a Sequential of stride-1 ConvModules channels-last; the last one writes ``dst``.
    ``hooks[i]``: optional callable(start: bool) bracketing layer i's launch (kernel timers)."""
    cur = src
    for i, m in enumerate(layers):
        hk = hooks[i] if hooks is not None and i < len(hooks) else None
        if hk is not None:
            ops.host_call(lambda hk=hk: hk(True))
        r = ConvRunner.of(m.conv, m.act_type)
        if i == len(layers) - 1:
            out = dst
        else:
            buf = scratch[i] if scratch is not None else torch.empty(n * h * w, m.conv.out_channels,
                                                                      device=src.buf.device)
            out = Chan.whole(buf)
        r.run(cur, out, n, h, w)
        if hk is not None:
            ops.host_call(lambda hk=hk: hk(False))
        cur = out


def run_chain_pair(chain_a: Sequence[ConvModule], src_a: Chan, dst_a: Chan,
                   chain_b: Sequence[ConvModule], src_b: Chan, dst_b: Chan, n: int, h: int, w: int,
                   scratch_a: Sequence[Tensor], scratch_b: Sequence[Tensor]) -> None:
    """Two independent ``run_chain``s of equal length, layer i of both as one
    ``ops.conv2d_pair`` launch (a grouped kernel where one covers the pair, else two launches):
    the decoder's flow-predictor and mask-predictor branches on one stream, no events."""
    if len(chain_a) != len(chain_b):
        raise ValueError("run_chain_pair: chains of different lengths")
    cur_a, cur_b = src_a, src_b
    for i, (ma, mb) in enumerate(zip(chain_a, chain_b)):
        last = i == len(chain_a) - 1
        out_a = dst_a if last else Chan.whole(scratch_a[i])
        out_b = dst_b if last else Chan.whole(scratch_b[i])
        ra = ConvRunner.of(ma.conv, ma.act_type)
        rb = ConvRunner.of(mb.conv, mb.act_type)
        ops.conv2d_pair(ra.args(cur_a, out_a, n, h, w), rb.args(cur_b, out_b, n, h, w), cur_a.buf)
        cur_a, cur_b = out_a, out_b


# ---------------------------------------------------------------------------------- a4
class ConvGRU(nn.Module):
    """raft_decoder.py:168-253.  z and r share one conv launch (cout = 2·h_channels) whose
    epilogue writes z and r·h; the q launch's epilogue applies h ← (1−z)h + z·tanh(q)."""
    _kernel = {"Conv": 3, "SeqConv": ((1, 5), (5, 1))}
    _padding = {"Conv": 1, "SeqConv": ((0, 2), (2, 0))}

    def __init__(self, h_channels: int, x_channels: int, net_type: str = "SeqConv") -> None:
        super().__init__()
        assert net_type in ["Conv", "SeqConv"]
        ks = self._kernel[net_type] if isinstance(self._kernel[net_type], (tuple, list)) \
            else [self._kernel[net_type]]
        ps = self._padding[net_type] if isinstance(self._padding[net_type], (tuple, list)) \
            else [self._padding[net_type]]
        cz, cr, cq = [], [], []
        for k, p in zip(ks, ps):
            for lst_, act in ((cz, "Sigmoid"), (cr, "Sigmoid"), (cq, "Tanh")):
                lst_.append(ConvModule(h_channels + x_channels, h_channels, k, padding=p,
                                       act_cfg=dict(type=act)))
        self.conv_z = nn.ModuleList(cz)
        self.conv_r = nn.ModuleList(cr)
        self.conv_q = nn.ModuleList(cq)
        self.h_channels = h_channels
        self.x_channels = x_channels
        self._runners = None

    def init_weights(self) -> None:
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.orthogonal_(m.weight)

    def runners(self):
        if self._runners is None:
            self._runners = [(ConvRunner([z.conv, r.conv], "Sigmoid"), ConvRunner([q.conv], "Tanh"))
                             for z, r, q in zip(self.conv_z, self.conv_r, self.conv_q)]
        return self._runners

    # -------------------------------------------------------------- loop-invariant context
    # x = cat[cxt, motion]: the context part is the same in every refinement iteration, so its
    # share of the z|r and q pre-activations (a linear map, + the biases) is computed once per
    # forward into a per-pixel map, and the per-iteration convs contract only h (or r·h) and
    # the motion features — 1/3 fewer GRU FLOPs per iteration at SCFlow's 128|128|128 split.
    def _ctx_runners(self, cxt_channels: int):
        key = cxt_channels
        if getattr(self, "_ctx_key", None) != key:
            hc = self.h_channels
            keep = [(0, hc), (hc + cxt_channels, hc + self.x_channels)]
            ctx = [(hc, hc + cxt_channels)]
            self._ctx = [(ConvRunner([z.conv, r.conv], "Sigmoid", in_select=keep, with_bias=False),
                          ConvRunner([q.conv], "Tanh", in_select=keep, with_bias=False),
                          ConvRunner([z.conv, r.conv, q.conv], None, in_select=ctx))
                         for z, r, q in zip(self.conv_z, self.conv_r, self.conv_q)]
            self._ctx_key = key
        return self._ctx

    def context_map(self, cxt: Chan, n: int, h: int, w: int) -> Tensor:
        """[n·h·w, stages·3·hc] map: per SeqConv stage, [z|r|q] pre-activation contribution of
        the context channels plus the biases."""
        hc = self.h_channels
        runners = self._ctx_runners(cxt.c)
        bm = torch.empty(n * h * w, len(runners) * 3 * hc, device=cxt.buf.device)
        for i, (_, _, rc) in enumerate(runners):
            rc.run(cxt, Chan(bm, i * 3 * hc, 3 * hc), n, h, w)
        return bm

    def bind_step(self, hx: Chan, z: Chan, rh: Chan, n: int, h: int, w: int,
                  ctx_map: Optional[Tensor] = None, cxt_channels: int = 0):
        """``step``'s launches bound once; returns step(hooks=None) replaying them."""
        hc = self.h_channels
        hid = Chan(hx.buf, hx.off, hc)
        x = Chan(hx.buf, hx.off + hc, hx.c - hc)
        launches = []
        if ctx_map is not None:
            mot = Chan(hx.buf, hx.off + hc + cxt_channels, hx.c - hc - cxt_channels)
            for i, (rzr, rq, _) in enumerate(self._ctx_runners(cxt_channels)):
                bzr = Chan(ctx_map, i * 3 * hc, 2 * hc)
                bq = Chan(ctx_map, i * 3 * hc + 2 * hc, hc)
                launches.append((rzr.bind(hid, None, n, h, w, src1=mot, epilogue=EPI_GRU_ZR, gate=z,
                                          rh=rh, hid=hid, bias_map=bzr),
                                 rq.bind(rh, None, n, h, w, src1=mot, epilogue=EPI_GRU_Q, gate=z,
                                         hid=hid, bias_map=bq)))
        else:
            for rzr, rq in self.runners():
                launches.append((rzr.bind(hx, None, n, h, w, epilogue=EPI_GRU_ZR, gate=z, rh=rh,
                                          hid=hid),
                                 rq.bind(rh, None, n, h, w, src1=x, epilogue=EPI_GRU_Q, gate=z,
                                         hid=hid)))

        def step(hooks=None) -> None:
            hzr = hooks.get("gru_zr") if hooks else None
            hq = hooks.get("gru_q") if hooks else None
            for lzr, lq in launches:
                if hzr:
                    hzr(True)
                lzr()
                if hzr:
                    hzr(False)
                if hq:
                    hq(True)
                lq()
                if hq:
                    hq(False)
        return step

    def step(self, hx: Chan, z: Chan, rh: Chan, n: int, h: int, w: int, hooks=None,
             ctx_map: Optional[Tensor] = None, cxt_channels: int = 0) -> None:
        """In-place GRU update of channels [0, hc) of ``hx`` (= cat[h, x] channels-last).

        ``ctx_map`` (from ``context_map``): the first ``cxt_channels`` of x are the loop-invariant
        context whose contribution is in the map; the convs then skip those channels.
        ``hooks`` (optional dict name -> callable(start)) brackets the z|r and q launches."""
        hc = self.h_channels
        hid = Chan(hx.buf, hx.off, hc)
        x = Chan(hx.buf, hx.off + hc, hx.c - hc)
        hzr = hooks.get("gru_zr") if hooks else None
        hq = hooks.get("gru_q") if hooks else None
        if ctx_map is not None:
            mot = Chan(hx.buf, hx.off + hc + cxt_channels, hx.c - hc - cxt_channels)
            stages = [(rzr, rq, mot, Chan(ctx_map, i * 3 * hc, 2 * hc), Chan(ctx_map, i * 3 * hc + 2 * hc, hc))
                      for i, (rzr, rq, _) in enumerate(self._ctx_runners(cxt_channels))]
        else:
            stages = [(rzr, rq, None, None, None) for rzr, rq in self.runners()]
        for rzr, rq, mot, bzr, bq in stages:
            if hzr:
                hzr(True)
            if mot is None:
                rzr.run(hx, None, n, h, w, epilogue=EPI_GRU_ZR, gate=z, rh=rh, hid=hid)
            else:
                rzr.run(hid, None, n, h, w, src1=mot, epilogue=EPI_GRU_ZR, gate=z, rh=rh, hid=hid,
                        bias_map=bzr)
            if hzr:
                hzr(False)
            if hq:
                hq(True)
            if mot is None:
                rq.run(rh, None, n, h, w, src1=x, epilogue=EPI_GRU_Q, gate=z, hid=hid)
            else:
                rq.run(rh, None, n, h, w, src1=mot, epilogue=EPI_GRU_Q, gate=z, hid=hid, bias_map=bq)
            if hq:
                hq(False)

    def zr_runner(self, cxt_channels: int = 0) -> "ConvRunner":
        """The first SeqConv stage's fused z|r conv (context hoisted if cxt_channels > 0)."""
        return self._ctx_runners(cxt_channels)[0][0] if cxt_channels else self.runners()[0][0]

    def q_runner(self, cxt_channels: int = 0) -> "ConvRunner":
        """The first SeqConv stage's q conv (context hoisted if cxt_channels > 0)."""
        return self._ctx_runners(cxt_channels)[0][1] if cxt_channels else self.runners()[0][1]

    def zr_flops(self, m: int, cxt_channels: int = 0) -> float:
        """Algorithmic FLOPs of one z|r launch over m pixels (with the context hoisted if
        cxt_channels > 0)."""
        return self.zr_runner(cxt_channels).flops(m)

    def forward(self, h: Tensor, x: Tensor) -> Tensor:
        n, hc, hh, ww = h.shape
        xc = x.shape[1]
        dev = h.device
        M = n * hh * ww
        hx = torch.empty(M, hc + xc, device=dev)
        ops.nchw_into(h.contiguous(), Chan(hx, 0, hc))
        ops.nchw_into(x.contiguous(), Chan(hx, hc, xc))
        z = torch.empty(M, hc, device=dev)
        rh = torch.empty(M, hc, device=dev)
        self.step(Chan.whole(hx), Chan.whole(z), Chan.whole(rh), n, hh, ww)
        return ops.chan_to_nchw(Chan(hx, 0, hc), n, hh, ww)


# ---------------------------------------------------------------------------------- a5
class XHead(nn.Module):
    """raft_decoder.py:256-294."""

    def __init__(self, in_channels: int, feat_channels: Sequence[int], x_channels: int, x: str) -> None:
        super().__init__()
        layers = []
        for ch in feat_channels:
            layers.append(ConvModule(in_channels, ch, 3, padding=1))
            in_channels = ch
        self.layers = nn.Sequential(*layers)
        if x in ("flow", "tradeoff"):
            self.predict_layer = nn.Conv2d(feat_channels[-1], x_channels, kernel_size=3, padding=1)
        elif x == "mask":
            self.predict_layer = nn.Conv2d(feat_channels[-1], x_channels, kernel_size=1, padding=0)
        else:
            raise ValueError(f"x must be 'flow' or 'mask', but got {x}")
        self.x = x

    def forward(self, x: Tensor) -> Tensor:
        n, c, h, w = x.shape
        src = torch.empty(n * h * w, c, device=x.device)
        ops.nchw_into(x.contiguous(), Chan.whole(src))
        hid = torch.empty(n * h * w, self.layers[-1].conv.out_channels, device=x.device)
        run_chain(self.layers, Chan.whole(src), Chan.whole(hid), n, h, w)
        out = torch.empty(n * h * w, self.predict_layer.out_channels, device=x.device)
        ConvRunner.of(self.predict_layer, None).run(Chan.whole(hid), Chan.whole(out), n, h, w)
        return ops.chan_to_nchw(Chan.whole(out), n, h, w)


# ---------------------------------------------------------------------------------- a7
@MODELS.register_module()
class MultiClassPoseHead(nn.Module):
    """pose_head.py:110-211.  Three stride-2 3×3 conv + GroupNorm + ReLU layers, two FCs and the
    per-class rotation / translation heads (label[0] quirk kept); forward_hip / trunk_hip run them
    on the HIP kernels (MFMA halo conv and gather conv with K splits, GroupNorm-statistics
    reduce, K-split FCs), 0.16 GFLOP per pair-iteration."""
    # workgroups the K splits aim for: the MFMA halo convs (conv1, conv2) and the gather conv
    # (conv3) — tuning attributes (tools/ab_bench.py; conv3 at B = 16: 128 → 4 K slices, 5.220 vs
    # 5.240 ms/forward for 256 → 8, median of 9)
    conv_wg_target = 512
    gather_wg_target = 128
    fc_ksplit = 4  # K slices of the split FCs (workgroups = ⌈out/16⌉ · fc_ksplit)
    _conv_feat_channels = {"Basic": [128, 128, 128], "Large": [128, 128, 128]}
    _conv_strides = {"Basic": [2, 2, 2], "Large": [2, 2, 2]}
    _conv_paddings = {"Basic": [1, 1, 1], "Large": [1, 1, 1]}
    _conv_kernel_sizes = {"Basic": [3, 3, 3], "Large": [3, 3, 3]}
    _fc_feat_channels = {"Basic": [1024, 256], "Large": [1024, 256]}
    _feat_size = {"Basic": (32, 32), "Large": (64, 64)}

    def __init__(self, num_class: int, in_channels: int, net_type: str, norm_cfg: dict,
                 act_cfg: dict, feat_size: tuple = None, rotation_mode: str = "quaternion",
                 init_cfg=None):
        super().__init__()
        self.num_class = num_class
        assert net_type in ["Basic", "Small", "Large"]
        if feat_size is None:
            feat_size = self._feat_size.get(net_type)
        conv_layers = []
        conv_out_size = feat_size[0] * feat_size[1]
        for ch, k, s, p in zip(self._conv_feat_channels[net_type], self._conv_kernel_sizes[net_type],
                               self._conv_strides[net_type], self._conv_paddings[net_type]):
            conv_layers.append(ConvModule(in_channels, ch, k, stride=s, padding=p, norm_cfg=norm_cfg,
                                          act_cfg=act_cfg))
            in_channels = ch
            conv_out_size = int(conv_out_size / (s ** 2))
        self.conv_layers = nn.Sequential(*conv_layers)
        fc_in = in_channels * conv_out_size
        fcs = []
        for ch in self._fc_feat_channels[net_type]:
            fcs.append(nn.Sequential(nn.Linear(fc_in, ch), nn.ReLU()))
            fc_in = ch
        self.flatten_op = nn.Flatten(start_dim=1, end_dim=-1)
        self.fc_layers = nn.Sequential(*fcs)
        if rotation_mode == "quaternion":
            self.rotation_out_channels = 4
        elif rotation_mode == "ortho6d":
            self.rotation_out_channels = 6
        else:
            raise RuntimeError(f"Not supported rotation mode:{rotation_mode}")
        self.rotation_mode = rotation_mode
        self.rotation_pred = nn.Linear(fc_in, self.rotation_out_channels * num_class)
        self.translation_pred = nn.Linear(fc_in, 3 * num_class)
        self.init_weights()

    def init_weights(self):
        nn.init.zeros_(self.translation_pred.weight)
        nn.init.zeros_(self.translation_pred.bias)
        nn.init.zeros_(self.rotation_pred.weight)
        with torch.no_grad():
            base = [0.0, 0.0, 0.0, 1.0] if self.rotation_mode == "quaternion" else [1.0, 0, 0, 0, 1.0, 0]
            self.rotation_pred.bias.copy_(torch.tensor(base * self.num_class))

    # ------------------------------------------------------------------ HIP path
    def _packs(self, c_last: int, hw_last: int):
        w1 = self.fc_layers[0][0].weight
        key = tuple((m.conv.weight.data_ptr(), m.conv.weight._version) for m in self.conv_layers) + (
            w1.data_ptr(), w1._version, c_last, hw_last, _lib.weights_generation())
        if getattr(self, "_pack_key", None) != key:
            self._packed = [ops.ph_conv_pack(m.conv.weight) for m in self.conv_layers]
            self._fc1_perm = ops.ph_fc_permute(w1, c_last, hw_last)
            self._pack_key = key
        return self._packed, self._fc1_perm

    def _conv_mfma(self, i: int, src0: Chan, src1: Optional[Chan], n: int, h: int, w: int,
                   scale: Optional[Tensor], shift: Optional[Tensor], keep: Optional[list] = None):
        """conv_layers[i] on the MFMA halo conv (scflow_enc_conv; the previous GroupNorm + ReLU
        applied on load) with a K split over grid.z so that ≥ 512 workgroups run, when the shape
        allows it: returns (partial slabs [ksplit·n·oh·ow, cout], ksplit) or None."""
        conv = self.conv_layers[i].conv
        c1 = 0 if src1 is None else src1.c
        if conv.kernel_size != (3, 3) or conv.padding[0] != 1 or conv.stride[0] not in (1, 2) \
                or src0.c % 16 or c1 % 16 or conv.bias is not None:
            return None
        s = conv.stride[0]
        oh, ow = (h - 1) // s + 1, (w - 1) // s + 1
        tm = 128 if s == 1 else 64
        tc = min(ow, tm)
        if tc < 8 or tm % tc or ow % tc or oh % (tm // tc):
            return None
        wt = conv.weight
        packs = getattr(self, "_mfma_packs", None)
        if packs is None:
            packs = self._mfma_packs = {}
        key = (wt.data_ptr(), wt._version, _lib.weights_generation())
        if packs.get(i, (None,))[0] != key:
            packs[i] = (key, ops.enc_conv_pack(wt))
        tiles = n * (oh // (tm // tc)) * (ow // tc) * ((conv.out_channels + 63) // 64)
        nst = (src0.c + c1) // 16
        ksplit = max(1, min(nst, -(-self.conv_wg_target // tiles)))
        parts = torch.empty(ksplit * n * oh * ow, conv.out_channels, device=src0.buf.device)
        if keep is not None:
            keep.append(parts)
        ops.enc_conv(src0, packs[i][1], None, n, h, w, src0.c, conv.out_channels, 3, s, 1, parts,
                     src1=src1, ksplit=ksplit, in_scale=scale, in_shift=shift)
        return parts, ksplit

    def forward_hip(self, src0: Chan, src1: Optional[Chan], n: int, h: int, w: int,
                    label: Tensor) -> Tuple[Tensor, Tensor]:
        """Channels-last input cat[src0, src1] of n samples at h×w → (Δrot, Δt)."""
        dev = src0.buf.device
        x = self.trunk_hip(src0, src1, n, h, w)
        drot = torch.empty(n, self.rotation_out_channels, device=dev)
        dt = torch.empty(n, 3, device=dev)
        self.heads_hip(x, label, drot, dt)
        return drot, dt

    def trunk_hip(self, src0: Chan, src1: Optional[Chan], n: int, h: int, w: int,
                  ws: Optional[list] = None) -> Tensor:
        """Convs + FCs of forward_hip → the last FC's output [n, 256].  Every buffer it allocates
        is appended to ``ws`` (the decoder keeps them alive while replaying these launches).

        Each conv runs on the MFMA halo conv with a K split into partial slabs when its shape
        allows (conv1 and conv2 at SCFlow's sizes; summed by the GroupNorm-statistics kernel),
        else on the gather conv (conv3's 4×4 output)."""
        if any(m.norm_type != "GN" or m.act_type != "ReLU" for m in self.conv_layers):
            raise NotImplementedError("HIP pose head: conv + GroupNorm + ReLU layers only")
        dev = src0.buf.device
        keep = ws if ws is not None else []

        def empty(*shape):
            t = torch.empty(*shape, device=dev)
            keep.append(t)
            return t
        hl, wl = h, w
        for m in self.conv_layers:
            k, st, p = m.conv.kernel_size[0], m.conv.stride[0], m.conv.padding[0]
            hl, wl = (hl + 2 * p - k) // st + 1, (wl + 2 * p - k) // st + 1
        packs, fc1_w = self._packs(self.conv_layers[-1].conv.out_channels, hl * wl)
        cur0, cur1, hh, ww = src0, src1, h, w
        scale = shift = None
        for i, m in enumerate(self.conv_layers):
            conv = m.conv
            k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
            oh, ow = (hh + 2 * p - k) // s + 1, (ww + 2 * p - k) // s + 1
            cout = conv.out_channels
            y = empty(n * oh * ow, cout)
            split = self._conv_mfma(i, cur0, cur1, n, hh, ww, scale, shift, keep)
            if split is None and conv.bias is None:
                # gather conv with its K split over enough slices to fill the CUs (conv3 at B=16:
                # 32 output tiles → 4 slices), summed by the GroupNorm-statistics kernel
                tiles = -(-n * oh * ow // 32) * -(-cout // 32)
                nk = k * k * -(-(cur0.c + (0 if cur1 is None else cur1.c)) // 16)
                ks = max(1, min(nk // 16, -(-self.gather_wg_target // tiles)))
                parts = empty(ks * n * oh * ow, cout)
                ops.ph_conv(cur0, cur1, packs[i], None, n, hh, ww, cout, k, s, p, parts, scale, shift,
                            ksplit=ks)
                split = (parts, ks)
            elif split is None:
                ops.ph_conv(cur0, cur1, packs[i], None if conv.bias is None else conv.bias.detach(), n,
                            hh, ww, cout, k, s, p, y, scale, shift)
            scale = empty(n, cout)
            shift = empty(n, cout)
            if split is not None:
                ops.ph_gn_reduce(split[0], split[1], y, n, oh * ow, cout, m.gn.num_groups,
                                 m.gn.weight.detach(), m.gn.bias.detach(), m.gn.eps, scale, shift)
            else:
                ops.ph_gn_stats(y, n, oh * ow, cout, m.gn.num_groups, m.gn.weight.detach(),
                                m.gn.bias.detach(), m.gn.eps, scale, shift)
            cur0, cur1, hh, ww = Chan.whole(y), None, oh, ow
        c = cur0.c
        x = cur0.buf
        k_in = c * hh * ww
        # The FCs (M = n ≤ 32 rows) are weight-streaming: each runs with its K split over 4
        # workgroup slices (FC1 64 → 256 workgroups) into partial sums that the next layer adds,
        # biases and ReLUs on load; the trunk returns (partials, split, bias) for the heads.
        self._split_fc = n <= 32 and all(fc[0].in_features % 64 == 0 for fc in self.fc_layers)
        if not self._split_fc:
            for i, fc in enumerate(self.fc_layers):
                lin = fc[0]
                y = empty(n, lin.out_features)
                if i == 0:
                    ops.ph_fc(x, k_in, n, k_in, fc1_w, lin.bias.detach(), y, lin.out_features, True,
                              gn_c=c, scale=scale, shift=shift)
                else:
                    ops.ph_fc(x, x.shape[1], n, x.shape[1], lin.weight.detach(), lin.bias.detach(),
                              y, lin.out_features, True)
                x = y
            return x
        ks, xsplit, xbias, ldx = self.fc_ksplit, 0, None, k_in
        for i, fc in enumerate(self.fc_layers):
            lin = fc[0]
            y = empty(ks, n, lin.out_features)
            if i == 0:
                ops.ph_fc_split(x, k_in, n, k_in, fc1_w, y, lin.out_features, ks, gn_c=c, scale=scale,
                                shift=shift)
            else:
                ops.ph_fc_split(x, ldx, n, ldx, lin.weight.detach(), y, lin.out_features, ks,
                                xsplit=xsplit, xbias=xbias)
            x, xsplit, xbias, ldx = y, ks, lin.bias.detach(), lin.out_features
        return x

    def heads_args(self, x, label: Tensor) -> Optional[tuple]:
        """The heads' operands for ``ops.pose_step(heads=...)`` (the heads computed inside the
        pose step's launch), or None when the trunk's output is not the split FC's partial sums."""
        if x.dim() != 3:
            return None
        return (x, x.shape[0], self.fc_layers[-1][0].bias.detach(), x.shape[2],
                self.rotation_pred.weight.detach(), self.rotation_pred.bias.detach(),
                self.rotation_out_channels, self.translation_pred.weight.detach(),
                self.translation_pred.bias.detach(), label.long(), self.num_class)

    def heads_hip(self, x, label: Tensor, drot: Tensor, dt: Tensor) -> None:
        """Rotation / translation heads of label[0]'s class on the trunk output x → drot, dt
        (x: [n, 256] or the last FC's split partial sums [split, n, 256])."""
        if x.dim() == 3:
            n, k = x.shape[1], x.shape[2]
            ops.ph_heads(x, n, k, self.rotation_pred.weight.detach(),
                         self.rotation_pred.bias.detach(), self.rotation_out_channels,
                         self.translation_pred.weight.detach(), self.translation_pred.bias.detach(),
                         label.long(), self.num_class, drot, dt, xsplit=x.shape[0],
                         xbias=self.fc_layers[-1][0].bias.detach())
            return
        n = x.shape[0]
        ops.ph_heads(x, n, x.shape[1], self.rotation_pred.weight.detach(),
                     self.rotation_pred.bias.detach(), self.rotation_out_channels,
                     self.translation_pred.weight.detach(), self.translation_pred.bias.detach(),
                     label.long(), self.num_class, drot, dt)

    def forward(self, x: Tensor, label: Tensor) -> Tuple[Tensor, Tensor]:
        """Reference API (NCHW in).  Runs the HIP kernels (inference; no autograd graph)."""
        n, c, h, w = x.shape
        src = torch.empty(n * h * w, c, device=x.device)
        ops.nchw_into(x.contiguous().float(), Chan.whole(src))
        return self.forward_hip(Chan.whole(src), None, n, h, w, label.to(x.device))

    def forward_torch(self, x: Tensor, label: Tensor) -> Tuple[Tensor, Tensor]:
        """Stock PyTorch-ROCm path (autograd-capable); the reference's own composition."""
        for m in self.conv_layers:
            x = m.forward_torch(x)
        x = self.flatten_op(x)
        x = self.fc_layers(x)
        t = self.translation_pred(x).view(-1, self.num_class, 3)
        r = self.rotation_pred(x).view(-1, self.num_class, self.rotation_out_channels)
        # reference quirk kept (pose_head.py:208-209): index_select over ALL labels then [:, 0],
        # i.e. every sample uses label[0]'s class head
        t = torch.index_select(t, dim=1, index=label)[:, 0, :]
        r = torch.index_select(r, dim=1, index=label)[:, 0, :]
        return r, t
