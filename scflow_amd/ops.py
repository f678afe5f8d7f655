"""Tensor-level wrappers over the C ABI (include/scflow_hip.h).

Each wrapper validates devices/dtypes/contiguity, passes raw device pointers and the current
HIP stream of the tensor's device, and raises ``ScflowError`` on any non-zero status.  Inputs
must live on a ROCm device: there is deliberately no CPU path here.

Channels-last activations are described by ``Chan`` = (buffer, first channel, channel count):
the buffer is a contiguous ``[..., C_total]`` tensor, so a ``Chan`` is a channel slice of an
NHWC image with pixel stride ``C_total`` — how the decoder keeps cat[h, cxt, motion, flow] in
one buffer without ever materialising a concatenation.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import ScflowError, check

Tensor = torch.Tensor


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(t: Tensor) -> int:
    """The current HIP stream of t's device as a raw handle (the C entry points take it)."""
    if _raw_stream is not None:
        return _raw_stream(t.device.index)
    return torch.cuda.current_stream(t.device).cuda_stream


class BoundCall:
    """A recorded C-ABI launch: its arguments (device pointers of persistent buffers, sizes)
    fixed, the stream taken at call time.  See ``binding``."""
    __slots__ = ("fn", "args", "dev", "name")

    def __init__(self, fn, args, dev: int, name: str) -> None:
        self.fn, self.args, self.dev, self.name = fn, args, dev, name

    def __call__(self) -> None:
        rc = self.fn(*self.args, raw_stream(self.dev))
        if rc:
            check(rc, self.name)


_BINDING: Optional[list] = None
_BINDING_RUN = True


class binding:
    """``with ops.binding(calls):`` — the wrappers below record their launch as a ``BoundCall``
    into ``calls`` and ALSO run it (so the first pass computes; later passes replay ``calls``,
    costing one ctypes call per launch instead of the wrapper's Python).  ``run=False`` only
    records (the launches are replayed later; their buffers must outlive the replay)."""

    def __init__(self, calls: list, run: bool = True) -> None:
        self.calls, self.run = calls, run

    def __enter__(self):
        global _BINDING, _BINDING_RUN
        self._prev, _BINDING = _BINDING, self.calls
        self._prev_run, _BINDING_RUN = _BINDING_RUN, self.run
        return self.calls

    def __exit__(self, *exc):
        global _BINDING, _BINDING_RUN
        _BINDING, _BINDING_RUN = self._prev, self._prev_run


def host_call(fn) -> None:
    """Run a host-side callable (a kernel-timer hook) in launch order: inside ``binding`` it is
    recorded with the launches (and replayed with them), else it just runs."""
    if _BINDING is not None:
        _BINDING.append(fn)
        if not _BINDING_RUN:
            return
    fn()


def _launch(name: str, dev_tensor: Tensor, *args) -> None:
    fn = getattr(_lib.load(), name)
    if _BINDING is not None:
        bc = BoundCall(fn, args, dev_tensor.device.index, name)
        _BINDING.append(bc)
        if _BINDING_RUN:
            bc()
        return
    check(fn(*args, _stream(dev_tensor)), name)


def raw_stream(device_index: int) -> int:
    """Current HIP stream of a device by index (no Stream object; for per-launch hot paths)."""
    if _raw_stream is not None:
        return _raw_stream(device_index)
    return torch.cuda.current_stream(device_index).cuda_stream


def _require(t: Tensor, name: str, dtype=torch.float32, contiguous=True) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a tensor")
    if t.device.type != "cuda":
        raise ScflowError(f"{name} is on {t.device}: the SCFlow HIP path only runs on a ROCm GPU "
                          "(no CPU fallback)")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if contiguous and not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _require_rows(t: Tensor, name: str) -> None:
    """``t`` [..., c] is a channel slice of a channels-last buffer: unit channel stride and one
    pixel stride (``t.stride(-2)``, a multiple of 4) over all leading dimensions."""
    _require(t, name, contiguous=False)
    ok = t.stride(-1) == 1 and t.stride(-2) >= t.shape[-1] and t.stride(-2) % 4 == 0
    for i in range(t.dim() - 3, -1, -1):
        ok = ok and (t.shape[i] == 1 or t.stride(i) == t.stride(i + 1) * t.shape[i + 1])
    if not ok:
        raise ValueError(f"{name} must be channels-last rows with one pixel stride, got strides "
                         f"{tuple(t.stride())} for shape {tuple(t.shape)}")


def _p(t: Optional[Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


@dataclass
class Chan:
    """A channel slice [off, off+c) of a contiguous channels-last buffer ``buf[..., C_total]``."""
    buf: Tensor
    off: int
    c: int

    @property
    def stride(self) -> int:
        return self.buf.shape[-1]

    @property
    def ptr(self) -> int:
        return self.buf.data_ptr() + 4 * self.off

    @staticmethod
    def whole(buf: Tensor) -> "Chan":
        return Chan(buf, 0, buf.shape[-1])


# ------------------------------------------------------------------------------- a1 pyramid
def pyramid_level_shapes(h: int, w: int, num_levels: int) -> List[Tuple[int, int]]:
    return [(h >> l, w >> l) for l in range(num_levels)]


def corr_pyramid(feat1: Tensor, feat2: Tensor, num_levels: int = 4) -> Tuple[Tensor, List[Tensor]]:
    """Returns (one flat buffer, list of level views ``[N·H·W,1,H_l,W_l]``) — the reference's
    CorrelationPyramid output (raft_decoder.py:35-58) as views of one allocation."""
    _require(feat1, "feat1")
    _require(feat2, "feat2")
    if feat1.shape != feat2.shape or feat1.dim() != 4:
        raise ValueError(f"feature shapes differ or are not 4-D: {feat1.shape} {feat2.shape}")
    n, c, h, w = feat1.shape
    lib = _lib.load()
    size = lib.scflow_corr_pyramid_size(n, h, w, num_levels)
    if size <= 0:
        raise ScflowError(f"bad pyramid geometry n={n} h={h} w={w} L={num_levels}")
    buf = torch.empty(size, device=feat1.device, dtype=torch.float32)
    check(lib.scflow_corr_pyramid(_p(feat1), _p(feat2), _p(buf), n, c, h, w, num_levels,
                                  _stream(feat1)), "scflow_corr_pyramid")
    return buf, pyramid_views(buf, n, h, w, num_levels)


def tiled_pyramid_ok(h: int, w: int, num_levels: int) -> bool:
    """Whether scflow_corr_pyramid_tiled supports this geometry."""
    g = 4 << (num_levels - 1)
    return 1 <= num_levels <= 4 and h % 8 == 0 and w % 8 == 0 and h % g == 0 and w % g == 0


def tiled_lookup_ok(h: int, w: int, num_levels: int, radius: int, align_corners: bool) -> bool:
    """Whether scflow_corr_lookup_tiled supports this geometry (its LDS kernel: r in 1..4, and
    without align_corners every windowed level at least 2r+1 wide and tall)."""
    if not tiled_pyramid_ok(h, w, num_levels) or not 1 <= radius <= 4:
        return False
    if not align_corners:
        win = 2 * radius + 4
        for l in range(num_levels):
            hl, wl = h >> l, w >> l
            whole = hl + 2 <= win and wl + 2 <= win
            if not whole and (hl < 2 * radius + 1 or wl < 2 * radius + 1):
                return False
    return True


def corr_pyramid_tiled(feat1: Tensor, feat2: Tensor, num_levels: int = 4) -> Tensor:
    """The pyramid in the TILED layout (scflow_corr_pyramid_tiled: every map in 4×4 tiles of 16
    floats, pooling fused into the GEMM epilogue) as one flat buffer — for ``corr_lookup(...,
    tiled=True)``; ``untile_pyramid`` turns it back into the reference's level views."""
    _require(feat1, "feat1")
    _require(feat2, "feat2")
    if feat1.shape != feat2.shape or feat1.dim() != 4:
        raise ValueError(f"feature shapes differ or are not 4-D: {feat1.shape} {feat2.shape}")
    n, c, h, w = feat1.shape
    if not tiled_pyramid_ok(h, w, num_levels):
        raise ScflowError(f"tiled pyramid needs L <= 4 and h, w multiples of 8 and 4*2^(L-1): "
                          f"h={h} w={w} L={num_levels}")
    lib = _lib.load()
    buf = torch.empty(lib.scflow_corr_pyramid_size(n, h, w, num_levels), device=feat1.device,
                      dtype=torch.float32)
    _launch("scflow_corr_pyramid_tiled", feat1, _p(feat1), _p(feat2), _p(buf), n, c, h, w,
            num_levels)
    return buf


def untile_pyramid(buf: Tensor, n: int, h: int, w: int, num_levels: int) -> List[Tensor]:
    """Level views ``[N·H·W, 1, H_l, W_l]`` (row-major copies) of a tiled pyramid buffer."""
    out, off, P = [], 0, h * w
    for hl, wl in pyramid_level_shapes(h, w, num_levels):
        t = buf[off: off + n * P * hl * wl].view(n * P, hl // 4, wl // 4, 4, 4)
        out.append(t.permute(0, 1, 3, 2, 4).reshape(n * P, 1, hl, wl))
        off += n * P * hl * wl
    return out


def pyramid_views(buf: Tensor, n: int, h: int, w: int, num_levels: int) -> List[Tensor]:
    views, off, P = [], 0, h * w
    for hl, wl in pyramid_level_shapes(h, w, num_levels):
        views.append(buf[off: off + n * P * hl * wl].view(n * P, 1, hl, wl))
        off += n * P * hl * wl
    return views


def pyramid_buffer(levels: Sequence[Tensor], n: int, h: int, w: int) -> Tensor:
    """The flat buffer behind ``levels``; copies on device if they are not views of one."""
    L = len(levels)
    base = levels[0]
    if base.device.type == "cuda" and base.dtype == torch.float32:
        st = base.untyped_storage()
        ok = all(lv.is_contiguous() and lv.untyped_storage().data_ptr() == st.data_ptr()
                 for lv in levels)
        if ok:
            sizes = [n * h * w * hl * wl for hl, wl in pyramid_level_shapes(h, w, L)]
            off0 = base.storage_offset()
            offs = [off0 + sum(sizes[:i]) for i in range(L)]
            if all(lv.storage_offset() == o for lv, o in zip(levels, offs)):
                total = sum(sizes)
                return torch.as_strided(base, (total,), (1,), off0)
    for i, lv in enumerate(levels):
        _require(lv, f"pyramid level {i}", contiguous=False)
    return torch.cat([lv.reshape(-1) for lv in levels])


# ------------------------------------------------------------------------------- a2 lookup
def corr_lookup(pyr: Tensor, flow: Tensor, n: int, h: int, w: int, num_levels: int, radius: int,
                out: Optional[Chan] = None, flow_layout: str = "nchw",
                align_corners: bool = True, tiled: bool = False) -> Tensor:
    """Window lookup.  ``out=None`` → NCHW ``[n, L(2r+1)², h, w]`` (the reference's layout,
    corr_lookup.py:135-136); otherwise written channels-last into ``out``.  ``align_corners``:
    grid_sample's (SCFlow's config True; False: bilinear_sample's default, corr_lookup.py:35).
    ``tiled``: ``pyr`` is a ``corr_pyramid_tiled`` buffer."""
    _require(pyr, "pyramid")
    _require(flow, "flow")
    K = num_levels * (2 * radius + 1) ** 2
    lay = _lib.LAYOUT_NCHW if flow_layout == "nchw" else _lib.LAYOUT_NHWC
    if out is None:
        res = torch.empty(n, K, h, w, device=flow.device, dtype=torch.float32)
        ptr, olay, ostride = res.data_ptr(), _lib.LAYOUT_NCHW, K
    else:
        res = out.buf
        ptr, olay, ostride = out.ptr, _lib.LAYOUT_NHWC, out.stride
    if tiled:
        _launch("scflow_corr_lookup_tiled", flow, _p(pyr), _p(flow), lay, ptr, olay, ostride, n, h,
                w, num_levels, radius, int(bool(align_corners)))
    elif align_corners:
        _launch("scflow_corr_lookup", flow, _p(pyr), _p(flow), lay, ptr, olay, ostride, n, h, w,
                num_levels, radius)
    else:
        _launch("scflow_corr_lookup_ex", flow, _p(pyr), _p(flow), lay, ptr, olay, ostride, n, h, w,
                num_levels, radius, 0)
    return res


def corr_lookup_conv1x1(pyr: Tensor, flow: Tensor, packed: Tensor, bias: Optional[Tensor], out: Chan,
                        n: int, h: int, w: int, num_levels: int, radius: int, cout: int,
                        act: Optional[str] = "ReLU", align_corners: bool = True) -> None:
    """The tiled lookup and corr_net.0 (1×1, weights packed with ``_lib.CONV_1X1W``) in one launch
    (scflow_corr_lookup_conv1x1): ``out`` ← act(W·lookup + bias); ``flow`` [n·h·w, 2] (NHWC)."""
    _require(pyr, "pyramid")
    _require(flow, "flow", contiguous=False)
    _require(packed, "packed weight")
    if bias is not None:
        _require(bias, "bias")
    if out.c != cout:
        raise ValueError(f"out has {out.c} channels, expected {cout}")
    _launch("scflow_corr_lookup_conv1x1", flow, _p(pyr), _p(flow), _p(packed), _p(bias), out.ptr,
            out.stride, n, h, w, num_levels, radius, cout, _lib.SCFLOW_ACT[act], int(bool(align_corners)))


def lookup_conv1x1_ok(h: int, w: int, num_levels: int, radius: int, cin: int, cout: int) -> bool:
    """Whether scflow_corr_lookup_conv1x1 supports this geometry."""
    return (num_levels == 4 and radius == 4 and h % 32 == 0 and w % 32 == 0 and cout <= 256 and
            cin == num_levels * (2 * radius + 1) ** 2)


# ------------------------------------------------------------------------------- convolutions
def pack_conv_weight(weight: Tensor, c0: int, c1: int, w: int, stride: int = 1, bk: int = 16) -> Tensor:
    """Pack an nn.Conv2d weight ``[cout, c0+c1, kh, kw]`` for scflow_conv2d (packing format bk:
    K-stage depth 8/16 of the direct conv, or ``_lib.CONV_WINO`` for the Winograd kernel)."""
    _require(weight, "conv weight", contiguous=False)
    weight = weight.detach().contiguous()
    cout, cin, kh, kw = weight.shape
    if cin != c0 + c1:
        raise ValueError(f"weight has {cin} input channels, expected {c0}+{c1}")
    lib = _lib.load()
    size = lib.scflow_conv_packed_size_bk(cout, c0, c1, kh, kw, stride, w, bk)
    if size < 0:
        raise ScflowError(f"no conv kernel for cout={cout} cin={c0}+{c1} k={kh}x{kw} w={w}")
    packed = torch.empty(size, device=weight.device, dtype=torch.float32)
    check(lib.scflow_conv_pack_weights(_p(weight), _p(packed), cout, c0, c1, kh, kw, stride, w, bk,
                                       _stream(weight)), "scflow_conv_pack_weights")
    return packed


def conv_pick_bk(n: int, h: int, w: int, c0: int, c1: int, cout: int, kh: int, kw: int, ph: int,
                 pw: int, stride: int = 1) -> int:
    """The library's preferred packing format for this launch shape (host-only query): the
    direct conv's K-stage depth (8 or 16), ``_lib.CONV_WINO`` or ``_lib.CONV_1X1W``."""
    a = _lib.ConvArgs()
    a.c0, a.c1, a.n, a.h, a.w = c0, c1, n, h, w
    a.cout, a.kh, a.kw, a.ph, a.pw, a.stride = cout, kh, kw, ph, pw, stride
    bk = _lib.load().scflow_conv_pick_bk(ctypes.byref(a))
    if bk not in (8, 16, _lib.CONV_WINO, _lib.CONV_1X1W, _lib.CONV_WINO4):
        check(bk if bk < 0 else -2, "scflow_conv_pick_bk")
    return bk


def conv2d(src0: Chan, packed: Tensor, bias: Optional[Tensor], n: int, h: int, w: int, cout: int,
           kh: int, kw: int, ph: int, pw: int, act: Optional[str] = None, out: Optional[Chan] = None,
           src1: Optional[Chan] = None, epilogue: int = _lib.EPI_PLAIN, gate: Optional[Chan] = None,
           rh: Optional[Chan] = None, hid: Optional[Chan] = None, stride: int = 1,
           bias_map: Optional[Chan] = None, bk: int = 16, **fused) -> None:
    """One scflow_conv2d launch; ``fused``: in_scale / in_shift / out_scale / out_shift / res
    (Winograd 3×3 only, see conv2d_args)."""
    a = conv2d_args(src0, packed, bias, n, h, w, cout, kh, kw, ph, pw, act, out, src1, epilogue,
                    gate, rh, hid, stride, bias_map, bk, **fused)
    _launch("scflow_conv2d", src0.buf,ctypes.byref(a))


def conv2d_pair(args_a, args_b, dev_tensor: Tensor) -> None:
    """scflow_conv2d_pair: two independent convs (argument structs from ``ConvRunner.args``; the
    runners keep their packed weights) as one grouped launch where a paired kernel covers them,
    else two launches in order — bit-identical to the separate launches."""
    _launch("scflow_conv2d_pair", dev_tensor, ctypes.byref(args_a), ctypes.byref(args_b))


def xhead_pred_pack(flow_w: Tensor, mask_w: Tensor) -> Tensor:
    """scflow_xhead_pred's predictor weights: flow predictor [2, cf, 3, 3] and mask predictor
    [1, cm, 1, 1] → [cf + cm, 20] (row c < cf: W[o][c][ty][tx] at column (3·ty + tx)·2 + o; row
    cf + c: the mask weight at column 0)."""
    cf, cm = flow_w.shape[1], mask_w.shape[1]
    pw = torch.zeros(cf + cm, 20, device=flow_w.device, dtype=torch.float32)
    pw[:cf, :18] = flow_w.detach().float().permute(1, 2, 3, 0).reshape(cf, 18)
    pw[cf:, 0] = mask_w.detach().float().reshape(cm)
    return pw


def xhead_pred_workspace(n: int, h: int, w: int, flow_channels: int, hidden_channels: int,
                         device) -> Tensor:
    """The partial-sum workspace of scflow_xhead_pred (float32, 16-byte aligned)."""
    nb = int(_lib.load().scflow_xhead_pred_workspace_bytes(n, h, w, flow_channels, hidden_channels))
    if nb < 0:
        check(nb, "scflow_xhead_pred_workspace_bytes")
    return torch.empty(max(nb // 4, 1), device=device)


def xhead_pred(hidden_args, flow_channels: int, pred_w: Tensor, ws: Tensor,
               flow_bias: Optional[Tensor], mask_bias: Optional[Tensor], flow_act, mask_act,
               flow_out: Chan, mask_out: Chan) -> None:
    """scflow_xhead_pred: the XHeads' hidden conv (argument struct from ``ConvRunner.args``, the
    runner keeps its packed weights) with both predictors contracted in its epilogue, then the
    block / tap sum → flow_out (2 channels), mask_out (1 channel)."""
    _require(pred_w, "pred_w")
    _launch("scflow_xhead_pred", ws, ctypes.byref(hidden_args), flow_channels, _p(pred_w), _p(ws),
            ws.numel() * 4, _p(flow_bias), _p(mask_bias), _lib.SCFLOW_ACT[flow_act], _lib.SCFLOW_ACT[mask_act],
            _p(flow_out.buf) + 4 * flow_out.off, flow_out.buf.shape[1],
            _p(mask_out.buf) + 4 * mask_out.off, mask_out.buf.shape[1])


class BoundLaunch:
    """A C-ABI launch whose argument struct is built once (pointers of persistent buffers):
    calling it costs one ctypes call on the caller's current stream.  The decoder binds every
    convolution of its refinement loop once per forward and replays them every iteration."""
    __slots__ = ("fn", "args", "ref", "dev", "name", "keep")

    def __init__(self, fn, args, dev: int, name: str) -> None:
        self.fn, self.args, self.dev, self.name = fn, args, dev, name
        self.ref = ctypes.byref(args)

    def __call__(self) -> None:
        rc = self.fn(self.ref, raw_stream(self.dev))
        if rc:
            check(rc, self.name)


class SyncEvent:
    """A device-scope cross-stream event (scflow_sync_event_*): ``record(stream)`` then
    ``wait(stream)`` orders the second stream after the first without the system-scope cache
    writeback of a default HIP event.  ``timing=True``: a timing event (``elapsed_ms``)."""

    def __init__(self, timing: bool = False) -> None:
        lib = _lib.load()
        h = ctypes.c_void_p()
        if timing:
            check(lib.scflow_timing_event_create(ctypes.byref(h)), "scflow_timing_event_create")
        else:
            check(lib.scflow_sync_event_create(ctypes.byref(h)), "scflow_sync_event_create")
        self._h, self._lib = h, lib

    def elapsed_ms(self, end: "SyncEvent") -> float:
        """Milliseconds from this (timing) event to ``end`` (waits for ``end``)."""
        ms = ctypes.c_float()
        check(self._lib.scflow_event_elapsed_ms(self._h, end._h, ctypes.byref(ms)),
              "scflow_event_elapsed_ms")
        return float(ms.value)

    def record(self, stream: int) -> None:
        rc = self._lib.scflow_sync_event_record(self._h, stream)
        if rc:
            check(rc, "scflow_sync_event_record")

    def wait(self, stream: int) -> None:
        rc = self._lib.scflow_stream_wait_event(stream, self._h)
        if rc:
            check(rc, "scflow_stream_wait_event")

    def __del__(self) -> None:
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                self._lib.scflow_sync_event_destroy(h)
            except Exception:
                pass


def conv2d_args(src0: Chan, packed: Tensor, bias: Optional[Tensor], n: int, h: int, w: int,
                cout: int, kh: int, kw: int, ph: int, pw: int, act: Optional[str] = None,
                out: Optional[Chan] = None, src1: Optional[Chan] = None,
                epilogue: int = _lib.EPI_PLAIN, gate: Optional[Chan] = None,
                rh: Optional[Chan] = None, hid: Optional[Chan] = None, stride: int = 1,
                bias_map: Optional[Chan] = None, bk: int = 16, in_scale: Optional[Tensor] = None,
                in_shift: Optional[Tensor] = None, out_scale: Optional[Tensor] = None,
                out_shift: Optional[Tensor] = None, res: Optional[Chan] = None) -> "_lib.ConvArgs":
    """The validated scflow_conv_args of one launch (see conv2d).  in_/out_scale/shift and res
    (Winograd 3×3 only): relu(x·in_scale + in_shift) on load, (conv + b)·out_scale + out_shift,
    + res before the activation."""
    for nm, ch in (("src0", src0), ("src1", src1), ("out", out), ("gate", gate), ("rh", rh),
                   ("hid", hid), ("bias_map", bias_map)):
        if ch is not None:
            _require(ch.buf, nm)
    _require(packed, "packed weight")
    if bias is not None:
        _require(bias, "bias")
    a = _lib.ConvArgs()
    a.src0, a.c0, a.s0 = src0.ptr, src0.c, src0.stride
    if src1 is not None:
        a.src1, a.c1, a.s1 = src1.ptr, src1.c, src1.stride
    a.weight = packed.data_ptr()
    a.bias = None if bias is None else bias.data_ptr()
    if out is not None:
        a.out, a.so = out.ptr, out.stride
    a.n, a.h, a.w = n, h, w
    a.cout, a.kh, a.kw, a.ph, a.pw, a.stride = cout, kh, kw, ph, pw, stride
    a.act = _lib.SCFLOW_ACT[act]
    a.epilogue = epilogue
    if gate is not None:
        a.gate, a.sg = gate.ptr, gate.stride
    if rh is not None:
        a.rh, a.srh = rh.ptr, rh.stride
    if hid is not None:
        a.hid, a.sh = hid.ptr, hid.stride
    if bias_map is not None:
        a.bias_map, a.sbm = bias_map.ptr, bias_map.stride
    a.bk = bk
    for nm, t in (("in_scale", in_scale), ("in_shift", in_shift), ("out_scale", out_scale),
                  ("out_shift", out_shift)):
        if t is not None:
            _require(t, nm)
            setattr(a, nm, t.data_ptr())
    if res is not None:
        _require(res.buf, "res")
        a.res, a.sres = res.ptr, res.stride
    if bk == _lib.CONV_WINO4:
        # the transformed-input workspace, private to this launch (a bound launch keeps it with
        # its arguments; an eager one returns it to the stream-ordered caching allocator)
        nb = int(_lib.load().scflow_conv_workspace_bytes(ctypes.byref(a)))
        check(nb if nb < 0 else 0, "scflow_conv_workspace_bytes")
        ws = torch.empty(max(nb // 4, 1), device=src0.buf.device)
        a.ws, a.ws_bytes = ws.data_ptr(), nb
        a._ws = ws
    return a


# ------------------------------------------------------------------------------- pose
def lift_points(depth: Tensor, K: Tensor, R: Tensor, t: Tensor) -> Tensor:
    """[N,H,W,4] float32: object-frame point + validity (pose.py:26-64, dense)."""
    for nm, x in (("depth", depth), ("K", K), ("R", R), ("t", t)):
        _require(x, nm)
    n, h, w = depth.shape
    pts = torch.empty(n, h, w, 4, device=depth.device, dtype=torch.float32)
    _launch("scflow_lift_points", depth,_p(depth), _p(K), _p(R), _p(t), _p(pts), n, h, w)
    return pts


POSE_QUAT_XYZW = 16  # SCFLOW_POSE_QUAT_XYZW


def pose_mode(drot: Tensor, depth_transform: str) -> int:
    """The C-ABI pose-update mode word: depth transform bit | quaternion flag (drot [n, 4])."""
    if drot.dim() != 2 or drot.shape[1] not in (4, 6):
        raise ValueError(f"delta rotation must be [n, 6] (ortho6d) or [n, 4] (quaternion x, y, z, w), "
                         f"got {tuple(drot.shape)}")
    return (0 if depth_transform == "exp" else 1) | (POSE_QUAT_XYZW if drot.shape[1] == 4 else 0)


def pose_update(drot: Tensor, dt: Tensor, R: Tensor, t: Tensor, weight: float = 10.0,
                depth_transform: str = "exp") -> Tuple[Tensor, Tensor]:
    """get_pose_from_delta_pose (pose.py:124-149): drot ortho6d [n, 6] or quaternion [n, 4]."""
    for nm, x in (("drot", drot), ("dt", dt), ("R", R), ("t", t)):
        _require(x, nm)
    mode = pose_mode(drot, depth_transform)
    n = drot.shape[0]
    Ro, to = torch.empty_like(R), torch.empty_like(t)
    _launch("scflow_pose_update", drot, _p(drot), _p(dt), _p(R), _p(t), _p(Ro), _p(to), n,
            float(weight), mode)
    return Ro, to


def pose_flow(R: Tensor, t: Tensor, K: Tensor, points: Tensor, invalid_num: float,
              out: Optional[Tensor] = None) -> Tensor:
    for nm, x in (("R", R), ("t", t), ("K", K), ("points", points)):
        _require(x, nm)
    n, h, w, _ = points.shape
    flow = out if out is not None else torch.empty(n, 2, h, w, device=R.device, dtype=torch.float32)
    _launch("scflow_pose_flow", R,_p(R), _p(t), _p(K), _p(points), _p(flow), n, h, w,
                                       float(invalid_num))
    return flow


def pose_update_flow(drot: Tensor, dt: Tensor, R: Tensor, t: Tensor, K: Tensor, points: Tensor,
                     R_out: Tensor, t_out: Tensor, flow_out: Tensor, invalid_num: float,
                     weight: float = 10.0, depth_transform: str = "exp") -> None:
    for nm, x in (("drot", drot), ("dt", dt), ("R", R), ("t", t), ("K", K), ("points", points),
                  ("R_out", R_out), ("t_out", t_out), ("flow_out", flow_out)):
        _require(x, nm)
    n, h, w, _ = points.shape
    _launch("scflow_pose_update_flow", drot,
        _p(drot), _p(dt), _p(R), _p(t), _p(K), _p(points), _p(R_out), _p(t_out), _p(flow_out), n, h,
        w, float(weight), pose_mode(drot, depth_transform), float(invalid_num))


def pose_step(drot: Tensor, dt: Tensor, R: Tensor, t: Tensor, K: Tensor, points: Tensor,
              R_out: Tensor, t_out: Tensor, flow_out: Tensor, invalid_num: float,
              lr: Tensor, delta: Optional[Tensor], mask: Optional[Tensor], flow_up: Tensor,
              mask_up: Optional[Tensor], h: int, w: int, up_scale: float,
              lr_next: Optional[Chan] = None, hx_next: Optional[Chan] = None,
              weight: float = 10.0, depth_transform: str = "exp", parts: int = 3,
              heads: Optional[tuple] = None) -> None:
    """One launch: ``pose_update_flow`` + ``flow_upsample(lr, delta, mask → flow_up, mask_up)``
    + (if ``lr_next``) the next iteration's ``flow_downsample`` of the new pose flow into
    ``lr_next`` / ``hx_next``, computed from the pose directly (scflow_pose_step).  ``parts``
    (scflow_pose_step_part): 1 = only the full-resolution outputs, 2 = only the ↓8 flow.
    ``heads`` (``MultiClassPoseHead.heads_args``): the pose head's rotation / translation heads
    in the same launch (scflow_pose_step_heads) — ``drot`` / ``dt`` are then written, not read."""
    for nm, x in (("drot", drot), ("dt", dt), ("R", R), ("t", t), ("K", K), ("points", points),
                  ("R_out", R_out), ("t_out", t_out), ("flow_out", flow_out), ("lr", lr),
                  ("flow_up", flow_up)):
        _require(x, nm)
    n, H, W, _ = points.shape
    if lr_next is not None and lr_next.buf.data_ptr() == lr.data_ptr():
        raise ValueError("pose_step: lr_next must not alias lr")
    args = (_p(drot), _p(dt), _p(R), _p(t), _p(K), _p(points), _p(R_out), _p(t_out), _p(flow_out), n,
            H, W, float(weight), pose_mode(drot, depth_transform), float(invalid_num), _p(lr),
            _p(delta), _p(mask), _p(flow_up), _p(mask_up),
            None if lr_next is None else lr_next.ptr, 0 if lr_next is None else lr_next.stride,
            None if hx_next is None else hx_next.ptr, 0 if hx_next is None else hx_next.stride,
            h, w, float(up_scale), 1.0 / float(up_scale))
    if heads is not None:
        x, xsplit, xbias, k, Wr, br, rch, Wt, bt, label, num_class = heads
        if label.dtype != torch.int64 or label.device != x.device:
            raise TypeError("label must be an int64 tensor on the same device")
        _launch("scflow_pose_step_heads", drot, _p(x), int(xsplit), _p(xbias), int(k), _p(Wr), _p(br),
                int(rch), _p(Wt), _p(bt), _p(label), int(num_class), *args, int(parts))
    elif parts == 3:
        _launch("scflow_pose_step", drot, *args)
    else:
        _launch("scflow_pose_step_part", drot, *args, int(parts))


def pose_step_given(R: Tensor, t: Tensor, K: Tensor, points: Tensor, flow_out: Tensor,
                    invalid_num: float, lr: Tensor, delta: Optional[Tensor], mask: Optional[Tensor],
                    flow_up: Tensor, mask_up: Optional[Tensor], h: int, w: int,
                    up_scale: float) -> None:
    """``pose_step``'s full-resolution part (parts = 1) from an already updated pose R, t (the ↓8
    part's R_out / t_out): pose flow, ×8 flow prediction and mask, no pose update
    (scflow_pose_step_part with drot6 = NULL)."""
    for nm, x in (("R", R), ("t", t), ("K", K), ("points", points), ("flow_out", flow_out),
                  ("lr", lr), ("flow_up", flow_up)):
        _require(x, nm)
    n, H, W, _ = points.shape
    _launch("scflow_pose_step_part", R, None, None, _p(R), _p(t), _p(K), _p(points), None, None,
            _p(flow_out), n, H, W, 10.0, 0, float(invalid_num), _p(lr), _p(delta), _p(mask),
            _p(flow_up), _p(mask_up), None, 0, None, 0, h, w, float(up_scale),
            1.0 / float(up_scale), 1)


# ------------------------------------------------------------------------------- resampling
def flow_downsample(flow: Tensor, out0: Chan, h: int, w: int, value_scale: float,
                    out1: Optional[Chan] = None) -> None:
    _require(flow, "flow")
    n, _, H, W = flow.shape
    _launch("scflow_flow_downsample", flow,
        _p(flow), out0.ptr, out0.stride, None if out1 is None else out1.ptr,
        0 if out1 is None else out1.stride, n, H, W, h, w, float(value_scale))


def flow_upsample(lr: Tensor, delta: Optional[Tensor], mask: Optional[Tensor], n: int, h: int,
                  w: int, H: int, W: int, value_scale: float, flow_out: Tensor,
                  mask_out: Optional[Tensor]) -> None:
    _require(lr, "lr flow")
    _launch("scflow_flow_upsample", lr,_p(lr), _p(delta), _p(mask), _p(flow_out), _p(mask_out),
                                           n, h, w, H, W, float(value_scale))


# ------------------------------------------------------------------------------- layout
def nchw_into(x: Tensor, dst: Chan) -> None:
    """x [N,C,H,W] → channels [off, off+C) of channels-last ``dst.buf`` ([N,H,W,Ct] or [NHW,Ct])."""
    _require(x, "x")
    n, c, h, w = x.shape
    if c != dst.c:
        raise ValueError(f"channel mismatch {c} vs {dst.c}")
    st = dst.stride
    _launch("scflow_transpose", x,_p(x), dst.ptr, n, c, h * w, c * h * w, h * w,
                                       h * w * st, st)


def chan_to_nchw(src: Chan, n: int, h: int, w: int, out: Optional[Tensor] = None) -> Tensor:
    res = out if out is not None else torch.empty(n, src.c, h, w, device=src.buf.device,
                                                   dtype=torch.float32)
    st = src.stride
    _launch("scflow_transpose", src.buf,src.ptr, _p(res), n, h * w, src.c, h * w * st, st,
                                       src.c * h * w, h * w)
    return res


# ------------------------------------------------------------------------------- a7 pose head
def ph_conv_pack(weight: Tensor) -> Tensor:
    _require(weight, "pose conv weight", contiguous=False)
    w = weight.detach().contiguous().float()
    cout, cin, kh, kw = w.shape
    lib = _lib.load()
    packed = torch.empty(lib.scflow_ph_conv_packed_size(cout, cin, kh, kw), device=w.device)
    check(lib.scflow_ph_conv_pack(_p(w), _p(packed), cout, cin, kh, kw, _stream(w)),
          "scflow_ph_conv_pack")
    return packed


def ph_conv(src0: Chan, src1: Optional[Chan], packed: Tensor, bias: Optional[Tensor], n: int, h: int,
            w: int, cout: int, k: int, stride: int, pad: int, out: Tensor,
            scale: Optional[Tensor] = None, shift: Optional[Tensor] = None, ksplit: int = 1) -> None:
    """ksplit > 1: ``out`` holds ksplit partial slabs [ksplit, n·oh·ow, cout] (bias None)."""
    _launch("scflow_ph_conv_split", out,
        src0.ptr, src0.c, src0.stride, None if src1 is None else src1.ptr,
        0 if src1 is None else src1.c, 0 if src1 is None else src1.stride, _p(scale), _p(shift),
        _p(packed), _p(bias), _p(out), n, h, w, cout, k, k, stride, pad, ksplit)


def ph_gn_stats(x: Tensor, n: int, hw: int, c: int, groups: int, gamma: Tensor, beta: Tensor,
                eps: float, scale: Tensor, shift: Tensor) -> None:
    _launch("scflow_ph_gn_stats", x,_p(x), n, hw, c, groups, _p(gamma), _p(beta), float(eps),
                                         _p(scale), _p(shift))


def ph_gn_reduce(parts: Tensor, nsplit: int, y: Tensor, n: int, hw: int, c: int, groups: int,
                 gamma: Tensor, beta: Tensor, eps: float, scale: Tensor, shift: Tensor) -> None:
    """y = sum of the nsplit partial slabs of ``parts`` [nsplit, n·hw, c]; GN scale/shift of y."""
    _launch("scflow_ph_gn_reduce", parts,_p(parts), nsplit, n * hw * c, _p(y), n, hw, c, groups,
                                          _p(gamma), _p(beta), float(eps), _p(scale), _p(shift))


def ph_fc_permute(W: Tensor, c: int, hw: int) -> Tensor:
    """nn.Linear weight with NCHW-flatten columns → channels-last column order."""
    _require(W, "fc weight", contiguous=False)
    W = W.detach().contiguous().float()
    Wp = torch.empty_like(W)
    _launch("scflow_ph_fc_permute", W,_p(W), _p(Wp), W.shape[0], c, hw)
    return Wp


def ph_fc(x: Tensor, ldx: int, m: int, k: int, W: Tensor, bias: Optional[Tensor], y: Tensor, n: int,
          relu: bool, gn_c: int = 0, scale: Optional[Tensor] = None,
          shift: Optional[Tensor] = None) -> None:
    _launch("scflow_ph_fc", x,_p(x), ldx, m, k, _p(W), _p(bias), _p(y), n, int(relu), gn_c,
                                   _p(scale), _p(shift))


def ph_fc_split(x: Tensor, ldx: int, m: int, k: int, W: Tensor, parts: Tensor, n: int, ksplit: int,
                gn_c: int = 0, scale: Optional[Tensor] = None, shift: Optional[Tensor] = None,
                xsplit: int = 0, xbias: Optional[Tensor] = None) -> None:
    """parts [ksplit, m, n] = K-split partial sums of x·Wᵀ (no bias / activation); xsplit > 0:
    x is [xsplit, m, ldx] partial sums read as relu(Σ + xbias)."""
    _launch("scflow_ph_fc_split", x, _p(x), ldx, m, k, _p(W), _p(parts), n, ksplit, gn_c,
            _p(scale), _p(shift), xsplit, _p(xbias))


def ph_fc_sum(parts: Tensor, nsplit: int, m: int, k: int, xbias: Tensor, W: Tensor,
              bias: Optional[Tensor], y: Tensor, n: int, relu: bool) -> None:
    """y = act(relu(Σ parts + xbias)·Wᵀ + bias)."""
    _launch("scflow_ph_fc_sum", parts,_p(parts), nsplit, m, k, _p(xbias), _p(W), _p(bias), _p(y), n,
                                       int(relu))


def ph_heads(x: Tensor, m: int, k: int, Wr: Tensor, br: Tensor, rch: int, Wt: Tensor, bt: Tensor,
             label: Tensor, num_class: int, drot: Tensor, dt: Tensor, xsplit: int = 0,
             xbias: Optional[Tensor] = None) -> None:
    """xsplit > 0: x is [xsplit, m, k] partial sums of the previous FC, read as relu(Σ + xbias)."""
    if label.dtype != torch.int64 or label.device != x.device:
        raise TypeError("label must be an int64 tensor on the same device")
    _launch("scflow_ph_heads_sum", x, _p(x), xsplit, _p(xbias), m, k, _p(Wr), _p(br), rch, _p(Wt),
            _p(bt), _p(label), num_class, _p(drot), _p(dt))


# ------------------------------------------------------------------------------- §8(f)-1 encoder
def enc_conv_pack(weight: Tensor) -> Tensor:
    _require(weight, "encoder conv weight", contiguous=False)
    w = weight.detach().contiguous().float()
    cout, cin, kh, kw = w.shape
    lib = _lib.load()
    size = lib.scflow_enc_conv_packed_size(cout, cin, kh, kw)
    if size < 0:
        check(int(size), "scflow_enc_conv_packed_size")
    packed = torch.empty(size, device=w.device)
    check(lib.scflow_enc_conv_pack(_p(w), _p(packed), cout, cin, kh, kw, _stream(w)),
          "scflow_enc_conv_pack")
    return packed


def enc_stem_pack(weight: Tensor) -> Tensor:
    _require(weight, "encoder stem weight", contiguous=False)
    w = weight.detach().contiguous().float()
    cout, cin, kh, kw = w.shape
    lib = _lib.load()
    packed = torch.empty(lib.scflow_enc_stem_packed_size(cout, cin, kh, kw), device=w.device)
    check(lib.scflow_enc_stem_pack(_p(w), _p(packed), cout, cin, kh, kw, _stream(w)),
          "scflow_enc_stem_pack")
    return packed


def enc_conv(src, packed: Tensor, bias: Optional[Tensor], n: int, h: int, w: int, cin: int,
             cout: int, k: int, stride: int, pad: int, out: Tensor,
             in_scale: Optional[Tensor] = None, in_shift: Optional[Tensor] = None,
             out_scale: Optional[Tensor] = None, out_shift: Optional[Tensor] = None,
             res: Optional[Tensor] = None, act: Optional[str] = None, act2: Optional[str] = None,
             act_split: Optional[int] = None, src1: Optional[Chan] = None, ksplit: int = 1) -> None:
    """One channels-last MFMA conv (see scflow_enc_conv in include/scflow_hip.h); ``src`` is a
    contiguous channels-last tensor or a ``Chan`` (channel slice with its pixel stride)."""
    if isinstance(src, Chan):
        _require(src.buf, "src")
        sptr, sstride = src.ptr, src.stride
    else:
        _require(src, "src")
        sptr, sstride = src.data_ptr(), src.shape[-1]
    _require(out, "out")
    a = _lib.EncConvArgs()
    a.src, a.cin, a.s_in = sptr, cin, sstride
    if src1 is not None:
        _require(src1.buf, "src1")
        a.src1, a.cin1, a.s_in1 = src1.ptr, src1.c, src1.stride
    a.ksplit = ksplit
    a.in_scale, a.in_shift = _p(in_scale), _p(in_shift)
    a.weight, a.bias = packed.data_ptr(), _p(bias)
    a.out_scale, a.out_shift = _p(out_scale), _p(out_shift)
    a.res, a.s_res = _p(res), (res.shape[-1] if res is not None else 0)
    a.out, a.s_out = out.data_ptr(), out.shape[-1]
    a.n, a.h, a.w, a.cout, a.kh, a.kw, a.stride, a.pad = n, h, w, cout, k, k, stride, pad
    a.act = _lib.SCFLOW_ACT[act]
    a.act2 = _lib.SCFLOW_ACT[act2 if act2 is not None else act]
    a.act_split = cout if act_split is None else act_split
    _launch("scflow_enc_conv", out,ctypes.byref(a))


def enc_stem(img: Tensor, packed: Tensor, bias: Optional[Tensor], cout: int, k: int, stride: int,
             pad: int, out: Tensor, out_scale: Optional[Tensor] = None,
             out_shift: Optional[Tensor] = None, act: Optional[str] = None) -> None:
    _require(img, "image")
    n, cin, h, w = img.shape
    _launch("scflow_enc_stem", img,_p(img), _p(packed), _p(bias), _p(out_scale), _p(out_shift),
                                      _p(out), n, cin, h, w, cout, k, k, stride, pad,
                                      _lib.SCFLOW_ACT[act])


def enc_instance_norm_stats(x: Tensor, n: int, hw: int, c: int, scale: Tensor, shift: Tensor,
                            eps: float = 1e-5, partial: Optional[Tensor] = None) -> None:
    """InstanceNorm2d(affine=False) statistics of channels-last x → per (image, channel) affine."""
    chunks = max(1, min(64, hw // 256))
    need = n * chunks * 2 * c
    if partial is None or partial.numel() < need:
        partial = torch.empty(need, dtype=torch.float64, device=x.device)
    lib = _lib.load()
    check(lib.scflow_enc_stats(_p(x), n, hw, c, chunks, _p(partial), _stream(x)), "scflow_enc_stats")
    check(lib.scflow_enc_norm_finalize(_p(partial), n, chunks, c, hw, float(eps), _p(scale),
                                       _p(shift), _stream(x)), "scflow_enc_norm_finalize")


def in_apply(x: Tensor, scale: Tensor, shift: Tensor, y: Tensor, n: int, hw: int, c: int,
             relu: bool) -> None:
    """y = act(x·scale + shift) per (image, channel) of channels-last x (scflow_in_apply)."""
    _launch("scflow_in_apply", x, _p(x), _p(scale), _p(shift), _p(y), n, hw, c, int(bool(relu)))


def in_backward(dy: Tensor, x: Tensor, scale: Tensor, shift: Tensor, dx: Tensor, n: int, hw: int,
                c: int, relu: bool) -> None:
    """InstanceNorm(+ReLU) backward (scflow_in_backward): dx from dy, the input x and its
    scale/shift (rstd, −mean·rstd)."""
    chunks = max(1, min(64, hw // 256))
    partial = torch.empty(n * chunks * 2 * c, dtype=torch.float64, device=x.device)
    mm = torch.empty(n * 2 * c, device=x.device)
    _launch("scflow_in_backward", x, _p(dy), _p(x), _p(scale), _p(shift), _p(dx), _p(partial),
            _p(mm), n, hw, c, chunks, int(bool(relu)))


def _bn_chunks(m: int) -> int:
    return max(1, min(1024, m // 256))


def bn_forward(x: Tensor, gamma: Optional[Tensor], beta: Optional[Tensor], y: Tensor,
               running_mean: Optional[Tensor], running_var: Optional[Tensor], eps: float,
               momentum: float, relu: bool, res: Optional[Tensor] = None
               ) -> Tuple[Tensor, Tensor]:
    """BatchNorm2d (train mode) of channels-last x [..., c] (+ReLU, + res before the ReLU) into y,
    running statistics updated in place (scflow_bn_forward).  Returns (rstd, shift) per channel
    (x̂ = x·rstd + shift) for the backward."""
    c = x.shape[-1]
    m = x.numel() // c
    chunks = _bn_chunks(m)
    dev = x.device
    rstd, shift = torch.empty(c, device=dev), torch.empty(c, device=dev)
    sc, sh = torch.empty(c, device=dev), torch.empty(c, device=dev)
    partial = torch.empty(chunks * 2 * c, dtype=torch.float64, device=dev)
    _launch("scflow_bn_forward", x, _p(x), _p(gamma), _p(beta), _p(res), _p(y), _p(running_mean),
            _p(running_var), _p(rstd), _p(shift), _p(sc), _p(sh), _p(partial), m, c, chunks,
            float(eps), float(momentum), int(bool(relu)))
    return rstd, shift


def bn_backward(dy: Tensor, x: Tensor, rstd: Tensor, shift: Tensor, gamma: Optional[Tensor],
                beta: Optional[Tensor], dx: Tensor, dgamma: Optional[Tensor],
                dbeta: Optional[Tensor], relu: bool, y: Optional[Tensor] = None,
                dres: Optional[Tensor] = None, accumulate: bool = False) -> None:
    """BatchNorm2d (train mode) backward (scflow_bn_backward); y / dres: the residual form (ReLU
    mask from the block output, the identity's gradient written to dres)."""
    c = x.shape[-1]
    m = x.numel() // c
    chunks = _bn_chunks(m)
    partial = torch.empty(chunks * 2 * c, dtype=torch.float64, device=x.device)
    mm = torch.empty(2 * c, device=x.device)
    _launch("scflow_bn_backward", x, _p(dy), _p(x), _p(rstd), _p(shift), _p(gamma), _p(beta), _p(y),
            _p(dx), _p(dres), _p(dgamma), _p(dbeta), _p(partial), _p(mm), m, c, chunks,
            int(bool(relu)), int(bool(accumulate)))


def colsum(x: Tensor, out: Tensor, accumulate: bool = False) -> Tensor:
    """out (+)= x.sum(0) of a 2-D row-major x with unit column stride (scflow_colsum)."""
    _require(out, "out")
    _require(x, "x", contiguous=False)
    if x.dim() != 2 or x.stride(1) != 1 or out.numel() != x.shape[1]:
        raise ValueError(f"colsum: 2-D row-major x and a [{x.shape[-1]}] out expected")
    rows, cols = x.shape
    lib = _lib.load()
    nws = int(lib.scflow_colsum_workspace(rows, cols))
    ws = torch.empty(max(1, nws), device=x.device) if nws > 0 else None
    check(lib.scflow_colsum(_p(x), rows, cols, x.stride(0), _p(out), int(accumulate), _p(ws),
                            _stream(x)), "scflow_colsum")
    return out


def in_apply_residual(x: Tensor, scale: Tensor, shift: Tensor, res: Tensor, y: Tensor, n: int,
                      hw: int, c: int) -> None:
    """y = relu(x·scale + shift + res) (scflow_in_apply_residual: a residual block's tail)."""
    _require(res, "res")
    _launch("scflow_in_apply_residual", x, _p(x), _p(scale), _p(shift), _p(res), _p(y), n, hw, c)


def in_backward_residual(dy: Tensor, x: Tensor, scale: Tensor, shift: Tensor, y: Tensor,
                         dx: Tensor, dres: Tensor, n: int, hw: int, c: int) -> None:
    """Backward of y = relu(IN(x) + res) (scflow_in_backward_residual): dres = dy·(y > 0), dx
    the InstanceNorm backward of it."""
    chunks = max(1, min(64, hw // 256))
    partial = torch.empty(n * chunks * 2 * c, dtype=torch.float64, device=x.device)
    mm = torch.empty(n * 2 * c, device=x.device)
    _launch("scflow_in_backward_residual", x, _p(dy), _p(x), _p(scale), _p(shift), _p(y), _p(dx),
            _p(dres), _p(partial), _p(mm), n, hw, c, chunks)


def enc_apply(x: Tensor, scale: Tensor, shift: Tensor, out: Tensor, n: int, hw: int, c: int,
              id: Optional[Tensor] = None, id_scale: Optional[Tensor] = None,
              id_shift: Optional[Tensor] = None) -> None:
    _launch("scflow_enc_apply", x,_p(x), _p(scale), _p(shift), _p(id), _p(id_scale),
                                       _p(id_shift), _p(out), n, hw, c)


# ------------------------------------------------------------------------------- §8(f)-2 training
def conv_wgrad(dy: Tensor, src0, src1: Optional[Chan], dw: Tensor, db: Optional[Tensor], n: int,
               h: int, w: int, kh: int, kw: int, stride: int, ph: int, pw: int,
               accumulate: bool = False) -> None:
    """dw [cout, cin0+cin1, kh, kw] (+)= conv weight gradient; db [cout] (+)= Σ dy (optional).
    dy: [n·oh·ow, cout] contiguous; src0 / src1: channels-last tensors or ``Chan`` slices.
    Raises ScflowError(SCFLOW_EUNSUPPORTED) for shapes outside the kernel's set."""
    _require(dy, "dy")
    _require(dw, "dw")
    srcs = []
    for nm, x in (("src0", src0), ("src1", src1)):
        if x is None:
            srcs.append((None, 0, 0))
        elif isinstance(x, Chan):
            _require(x.buf, nm)
            srcs.append((x.ptr, x.c, x.stride))
        else:
            _require(x, nm)
            srcs.append((x.data_ptr(), x.shape[-1], x.shape[-1]))
    a = _lib.WgradArgs()
    a.dy, a.sdy = dy.data_ptr(), dy.shape[-1]
    (a.src0, a.cin0, a.s0), (a.src1, a.cin1, a.s1) = srcs
    a.dw, a.db = dw.data_ptr(), _p(db)
    a.n, a.h, a.w, a.cout, a.kh, a.kw = n, h, w, dy.shape[-1], kh, kw
    a.stride, a.ph, a.pw, a.accumulate = stride, ph, pw, int(accumulate)
    lib = _lib.load()
    need = ctypes.c_longlong(0)
    check(lib.scflow_conv_wgrad_workspace(ctypes.byref(a), ctypes.byref(need)),
          "scflow_conv_wgrad_workspace")
    ws = torch.empty(max(1, need.value), device=dy.device)
    a.workspace, a.workspace_floats = ws.data_ptr(), need.value
    check(lib.scflow_conv_wgrad(ctypes.byref(a), _stream(dy)), "scflow_conv_wgrad")


def conv_wgrad_batched(dys: List[Tensor], src0s: list, src1s: Optional[list], dw: Tensor,
                       db: Optional[Tensor], n: int, h: int, w: int, kh: int, kw: int, stride: int,
                       ph: int, pw: int, accumulate: bool = False) -> None:
    """dw (+)= Σ_i weight gradient of segment i (dys[i] with src0s[i] / src1s[i], each n images
    of h×w) in one launch (scflow_conv_wgrad_batched; ≤ 8 equally shaped segments; the Winograd,
    1×1, implicit-GEMM and thin kernels — ScflowError(SCFLOW_EUNSUPPORTED) otherwise)."""
    segs = len(dys)
    if not 1 <= segs <= 8 or len(src0s) != segs or (src1s is not None and len(src1s) != segs):
        raise ValueError(f"conv_wgrad_batched: 1..8 segments with matching sources, got {segs}")
    _require(dw, "dw")

    def desc(x, nm):
        if isinstance(x, Chan):
            _require(x.buf, nm)
            return x.ptr, x.c, x.stride
        _require(x, nm)
        return x.data_ptr(), x.shape[-1], x.shape[-1]

    d0 = [desc(x, "src0") for x in src0s]
    d1 = [desc(x, "src1") for x in src1s] if src1s is not None else None
    for t in dys:
        _require(t, "dy")
        if t.shape != dys[0].shape:
            raise ValueError("conv_wgrad_batched: segments differ in dY shape")
    if len({d[1:] for d in d0}) != 1 or (d1 is not None and len({d[1:] for d in d1}) != 1):
        raise ValueError("conv_wgrad_batched: segments differ in source channels / strides")
    a = _lib.WgradArgs()
    a.dy, a.sdy = dys[0].data_ptr(), dys[0].shape[-1]
    a.src0, a.cin0, a.s0 = d0[0]
    a.src1, a.cin1, a.s1 = d1[0] if d1 is not None else (None, 0, 0)
    a.dw, a.db = dw.data_ptr(), _p(db)
    a.n, a.h, a.w, a.cout, a.kh, a.kw = n * segs, h, w, dys[0].shape[-1], kh, kw
    a.stride, a.ph, a.pw, a.accumulate = stride, ph, pw, int(accumulate)
    lib = _lib.load()
    need = ctypes.c_longlong(0)
    check(lib.scflow_conv_wgrad_workspace(ctypes.byref(a), ctypes.byref(need)),
          "scflow_conv_wgrad_workspace")
    ws = torch.empty(max(1, need.value), device=dw.device)
    a.workspace, a.workspace_floats = ws.data_ptr(), need.value
    a.n = n
    arr = ctypes.c_void_p * segs
    p_dy = arr(*[t.data_ptr() for t in dys])
    p_s0 = arr(*[d[0] for d in d0])
    p_s1 = arr(*[d[0] for d in d1]) if d1 is not None else None
    check(lib.scflow_conv_wgrad_batched(ctypes.byref(a), segs, p_dy, p_s0, p_s1, _stream(dw)),
          "scflow_conv_wgrad_batched")


def im2col(x, n: int, h: int, w: int, cin: int, kh: int, kw: int, stride: int, ph: int, pw: int,
           out: Optional[Tensor] = None, channel_major: bool = False) -> Tensor:
    """Patch matrix [n·oh·ow, kh·kw·cin] of a channels-last input (tensor or Chan); columns in
    (ty, tx, c) order, or (c, ty, tx) with channel_major (a conv weight's own order)."""
    if isinstance(x, Chan):
        _require(x.buf, "x")
        ptr, sx, dev = x.ptr, x.stride, x.buf.device
    else:
        _require(x, "x")
        ptr, sx, dev = x.data_ptr(), x.shape[-1], x.device
    oh, ow = (h + 2 * ph - kh) // stride + 1, (w + 2 * pw - kw) // stride + 1
    if out is None:
        out = torch.empty(n * oh * ow, kh * kw * cin, device=dev)
    check(_lib.load().scflow_im2col_ex(ptr, sx, _p(out), n, h, w, cin, kh, kw, stride, ph, pw,
                                       int(channel_major), torch.cuda.current_stream(dev).cuda_stream),
          "scflow_im2col_ex")
    return out


def pose_update6_train(drot: Tensor, dt: Tensor, R: Tensor, t: Tensor, weight: float, depth_exp: bool,
                       detach_xy: bool, grads: Optional[Tuple[Tensor, Tensor]] = None):
    """Forward (Rn, tn) or, given grads = (gRn, gtn), the backward (g drot, g dt, g R, g t) of the
    training step's ortho6d pose update (scflow_pose_update6_train)."""
    for nm, x in (("drot", drot), ("dt", dt), ("R", R), ("t", t)):
        _require(x, nm)
    n = drot.shape[0]
    if grads is None:
        Rn = torch.empty(n, 3, 3, device=drot.device)
        tn = torch.empty(n, 3, device=drot.device)
        _launch("scflow_pose_update6_train", drot, _p(drot), _p(dt), _p(R), _p(t), None, None, _p(Rn),
                _p(tn), None, None, n, float(weight), int(depth_exp), int(detach_xy), 0)
        return Rn, tn
    gRn, gtn = grads
    out = [torch.empty(n, 6, device=drot.device), torch.empty(n, 3, device=drot.device),
           torch.empty(n, 3, 3, device=drot.device), torch.empty(n, 3, device=drot.device)]
    _launch("scflow_pose_update6_train", drot, _p(drot), _p(dt), _p(R), _p(t), _p(gRn), _p(gtn),
            *[_p(o) for o in out], n, float(weight), int(depth_exp), int(detach_xy), 1)
    return tuple(out)


def pm_loss(pts: Tensor, gt_r: Tensor, gt_t: Tensor, pred_r: Tensor, pred_t: Tensor,
            sym: Optional[Tensor], diam: Tensor, weight: float):
    """Fused point-matching loss of one iteration (scflow_pm_loss): (loss [1], workspace) where
    workspace = (gt_rt, pred_rot, idx) feeds pm_loss_backward."""
    B, P, _ = pts.shape
    for nm, x in (("pts", pts), ("gt_r", gt_r), ("gt_t", gt_t), ("pred_r", pred_r), ("pred_t", pred_t),
                  ("diam", diam)):
        _require(x, nm)
    gt_rt = torch.empty(B, P, 3, device=pts.device)
    pred_rot = torch.empty(B, P, 3, device=pts.device)
    idx = torch.empty(B, P, dtype=torch.int64, device=pts.device) if sym is not None else None
    loss = torch.empty(1, device=pts.device)
    _launch("scflow_pm_loss", pts, _p(pts), _p(gt_r), _p(gt_t), _p(pred_r), _p(pred_t), _p(sym), _p(diam),
            _p(gt_rt), _p(pred_rot), _p(idx), _p(loss), B, P, float(weight))
    return loss, (gt_rt, pred_rot, idx)


def pm_loss_backward(gloss: Tensor, pts: Tensor, ws, sym: Optional[Tensor], pred_t: Tensor,
                     gt_t: Tensor, diam: Tensor, weight: float) -> Tuple[Tensor, Tensor]:
    gt_rt, pred_rot, idx = ws
    B, P, _ = pts.shape
    g_r = torch.empty(B, 3, 3, device=pts.device)
    g_t = torch.empty(B, 3, device=pts.device)
    _launch("scflow_pm_loss_backward", pts, _p(gloss), _p(pts), _p(gt_rt), _p(pred_rot), _p(idx), _p(sym),
            _p(pred_t), _p(gt_t), _p(diam), _p(g_r), _p(g_t), B, P, float(weight))
    return g_r, g_t


def up_l1_loss(f: Tensor, target: Tensor, vmask: Optional[Tensor], sval: float,
               denom: Optional[Tensor], cdenom: float, weight: float) -> Tuple[Tensor, Tensor]:
    """(loss [1], sgn [N, C, H, W]) of scflow_up_l1_loss; f channels-last [N, h, w, C]."""
    _require(f, "f")
    _require(target, "target")
    N, h, w, C = f.shape
    H, W = target.shape[-2:]
    sgn = torch.empty(N, C, H, W, device=f.device)
    partial = torch.empty((N * H * W + 255) // 256, device=f.device)
    loss = torch.empty(1, device=f.device)
    _launch("scflow_up_l1_loss", f, _p(f), C, h, w, _p(target), _p(vmask), N, H, W, float(sval),
            _p(denom), float(cdenom), float(weight), _p(sgn), _p(partial), _p(loss))
    return loss, sgn


def knn1(gt: Tensor, pred: Tensor) -> Tensor:
    """[B, P] int64 index of the nearest ``pred`` point ([B, Q, 3]) of every ``gt`` point ([B, P, 3])."""
    _require(gt, "gt")
    _require(pred, "pred")
    B, P, _ = gt.shape
    idx = torch.empty(B, P, dtype=torch.int64, device=gt.device)
    _launch("scflow_knn1", gt, _p(gt), _p(pred), _p(idx), B, P, pred.shape[1])
    return idx


def group_norm_forward(x: Tensor, gamma: Tensor, beta: Tensor, groups: int, eps: float,
                       relu: bool) -> Tuple[Tensor, Tensor]:
    """GroupNorm (+ReLU) of channels-last x [n, h, w, c] (c == 4·groups) → (y, stats [n·groups, 2]
    = (mean, rstd))."""
    for nm, t in (("x", x), ("gamma", gamma), ("beta", beta)):
        _require(t, nm)
    n, c = x.shape[0], x.shape[-1]
    hw = x.numel() // (n * c)
    y = torch.empty_like(x)
    stats = torch.empty(n * groups, 2, device=x.device, dtype=torch.float32)
    _launch("scflow_group_norm_forward", x, _p(x), _p(gamma), _p(beta), _p(y), _p(stats), n, hw, c,
            groups, float(eps), int(relu))
    return y, stats


def group_norm_backward(dy: Tensor, x: Tensor, gamma: Tensor, beta: Tensor, stats: Tensor,
                        groups: int, relu: bool, dgamma: Tensor, dbeta: Tensor,
                        accumulate: bool) -> Tensor:
    """dx of group_norm_forward; dγ / dβ written to (or, accumulate, added onto) dgamma / dbeta."""
    for nm, t in (("dy", dy), ("x", x), ("gamma", gamma), ("beta", beta), ("stats", stats),
                  ("dgamma", dgamma), ("dbeta", dbeta)):
        _require(t, nm)
    n, c = x.shape[0], x.shape[-1]
    hw = x.numel() // (n * c)
    dx = torch.empty_like(x)
    part = torch.empty(n * c * 2, device=x.device, dtype=torch.float32)
    _launch("scflow_group_norm_backward", x, _p(dy), _p(x), _p(gamma), _p(beta), _p(stats), _p(dx),
            _p(part), _p(dgamma), _p(dbeta), n, hw, c, groups, int(relu), int(accumulate))
    return dx


def gru_gate_forward(zr: Tensor, h: Tensor, out: Tensor, q: Optional[Tensor] = None) -> Tensor:
    """SepConvGRU gate (training): out = r·h (q None) or h + z·(q − h); zr [..., 2c], h / q / out
    [..., c], channels-last contiguous."""
    for nm, t in (("zr", zr), ("h", h), ("out", out)) + ((("q", q),) if q is not None else ()):
        _require(t, nm)
    c = h.shape[-1]
    _launch("scflow_gru_gate_forward", h, _p(zr), _p(h), _p(q), _p(out), h.numel() // c, c,
            0 if q is None else 1)
    return out


def gru_gate_backward_q(dh2: Tensor, zr: Tensor, h: Tensor, q: Tensor, dq: Tensor, dzr: Tensor,
                        dha: Tensor) -> None:
    """dq = dh2·z·(1 − q²), dzr[..., :c] = dh2·(q − h)·z(1 − z), dha = dh2·(1 − z); dh2 may be
    a channel slice (pixel stride ≥ c)."""
    for nm, t in (("zr", zr), ("h", h), ("q", q), ("dq", dq), ("dzr", dzr), ("dha", dha)):
        _require(t, nm)
    _require_rows(dh2, "dh2")
    c = h.shape[-1]
    _launch("scflow_gru_gate_backward_q", h, _p(dh2), dh2.stride(-2), _p(zr), _p(h), _p(q), _p(dq),
            _p(dzr), _p(dha), h.numel() // c, c)


def gru_gate_backward_r(drh: Tensor, zr: Tensor, h: Tensor, dha: Tensor, dzr: Tensor,
                        dh: Tensor) -> None:
    """dzr[..., c:] = drh·h·r(1 − r), dh = dha + drh·r; drh and dh may be channel slices (pixel
    stride ≥ c), and dh may be drh itself (overwritten in place)."""
    for nm, t in (("zr", zr), ("h", h), ("dha", dha), ("dzr", dzr)):
        _require(t, nm)
    _require_rows(drh, "drh")
    _require_rows(dh, "dh")
    c = h.shape[-1]
    _launch("scflow_gru_gate_backward_r", h, _p(drh), drh.stride(-2), _p(zr), _p(h), _p(dha),
            _p(dzr), _p(dh), dh.stride(-2), h.numel() // c, c)


def col2im(cols: Tensor, n: int, h: int, w: int, cin: int, kh: int, kw: int, stride: int, ph: int,
           pw: int, out: Optional[Tensor] = None) -> Tensor:
    """Adjoint of im2col: [n·oh·ow, kh·kw·cin] patch gradients → channels-last [n, h, w, cin]."""
    _require(cols, "cols")
    if out is None:
        out = torch.empty(n, h, w, cin, device=cols.device)
    _require(out, "out", contiguous=False)
    _launch("scflow_col2im", cols, _p(cols), _p(out), out.stride(-2), n, h, w, cin, kh, kw, stride,
            ph, pw)
    return out


def corr_lookup_backward(dout: Tensor, flow: Tensor, dpyr: Tensor, n: int, h: int, w: int,
                         num_levels: int, radius: int, out_layout: str = "nhwc",
                         flow_layout: str = "nhwc") -> None:
    """dpyr (zeroed, pyramid layout) += adjoint of corr_lookup applied to dout."""
    for nm, t in (("dout", dout), ("flow", flow), ("dpyr", dpyr)):
        _require(t, nm)
    lay = {"nchw": _lib.LAYOUT_NCHW, "nhwc": _lib.LAYOUT_NHWC}
    stride = dout.shape[-1] if out_layout == "nhwc" else 0
    _launch("scflow_corr_lookup_backward", dout,_p(dout), lay[out_layout], stride, _p(flow),
                                                  lay[flow_layout], _p(dpyr), n, h, w, num_levels,
                                                  radius)


def gemm(a: Tensor, b: Tensor, out: Optional[Tensor] = None, alpha: float = 1.0, beta: float = 0.0,
         bias: Optional[Tensor] = None, bias_dim: str = "n") -> Tensor:
    """``alpha·(a @ b) [+ beta·out] [+ bias]`` on the HIP fp32 MFMA GEMM (scflow_gemm_f32).
    ``a`` [M, K] or [Bt, M, K], ``b`` [K, N] or [Bt, K, N] — any strides (transposed views are
    free); ``out`` [M, N] / [Bt, M, N] (any strides; allocated contiguous if None; read when
    beta ≠ 0).  ``bias`` [N] (bias_dim "n") or [M] ("m")."""
    for t, nm in ((a, "a"), (b, "b")):
        _require(t, nm, contiguous=False)
    batched = a.dim() == 3
    if a.dim() != b.dim() or a.dim() not in (2, 3):
        raise ValueError(f"gemm: a {tuple(a.shape)} and b {tuple(b.shape)} must both be 2-D or 3-D")
    A = a if batched else a.unsqueeze(0)
    B = b if batched else b.unsqueeze(0)
    bt, M, K = A.shape
    if B.shape[0] != bt or B.shape[1] != K:
        raise ValueError(f"gemm: shapes {tuple(a.shape)} x {tuple(b.shape)} do not contract")
    N = B.shape[2]
    if out is None:
        if beta != 0.0:
            raise ValueError("gemm: beta != 0 needs out")
        out = torch.empty((bt, M, N) if batched else (M, N), device=a.device)
    _require(out, "out", contiguous=False)
    C = out if batched else out.unsqueeze(0)
    if tuple(C.shape) != (bt, M, N):
        raise ValueError(f"gemm: out {tuple(out.shape)} is not {(bt, M, N)}")
    mode = 0
    if bias is not None:
        _require(bias, "bias")
        mode = 1 if bias_dim == "n" else 2
        if bias.numel() != (N if mode == 1 else M):
            raise ValueError("gemm: bias size")
    sa, sb, sc = A.stride(), B.stride(), C.stride()
    splits = int(_lib.load().scflow_gemm_f32_splits(bt, M, N, K))
    ws = torch.empty(splits * bt * M * N, device=a.device) if splits > 1 else None
    _launch("scflow_gemm_f32", a, _p(a), _p(b), _p(out), _p(bias), bt, M, N, K,
            sa[0], sa[1], sa[2], sb[0], sb[1], sb[2], sc[0], sc[1], sc[2], float(alpha), float(beta), mode,
            splits, _p(ws))
    return out
