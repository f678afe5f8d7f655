"""RAFTEncoder ('Basic') on the gfx950 kernels of csrc/encoder.hip — SURVEY.md §8(f) rank 1.

Drop-in for ``models/encoder/raft_encoder.py:RAFTEncoder`` (registered under the same name):
same constructor arguments, the same sub-module names and therefore the same state-dict keys
(``conv1``, ``in1``/``bn1``, ``res_layer{1,2,3}.{0,1}.{conv1,in1|bn1,conv2,in2|bn2}``,
``res_layer{2,3}.0.downsample.{0,1}``, ``conv2``), and ``forward(x) -> NCHW features``.

Data flow (channels-last between layers; reference lines in brackets):

* stem conv1 7×7/2 [raft_encoder.py:297-299] — ``enc_stem`` reads the NCHW image directly.
* BasicBlock [resnet.py:65-92] with InstanceNorm (feature encoder): conv1 writes its raw
  output, its statistics are reduced in fp64, and conv2 applies that IN + ReLU to the input
  halo it stages (the normalised tensor is never written); the block output
  ``relu(IN(conv2) + identity)`` — identity = the block input or ``IN(downsample conv)`` — is
  materialised once by ``enc_apply`` because the next block needs it twice.
* with BatchNorm in eval mode (context encoder): BN folds into a per-channel affine in the conv
  epilogue, together with the residual add and ReLU — three launches per block, no extra pass.
* conv2 1×1 [raft_encoder.py:313] — optionally with a split activation, which is how
  ``SCFlowRefiner.extract_feat`` (scflow_refiner.py:101-104) turns the context output into
  ``tanh(h) | relu(cxt)`` in the same launch.

Inference only: BatchNorm in training mode (batch statistics + running-stat update) raises.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple, Union

import torch
import torch.nn as nn

from . import _lib, ops
from .registry import MODELS

Tensor = torch.Tensor


def build_norm_layer(cfg: dict, num_features: int, postfix: Union[int, str] = "") -> Tuple[str, nn.Module]:
    """mmcv ``build_norm_layer`` for the norms the encoder uses: IN → ``in<postfix>``
    (InstanceNorm2d, affine=False unless asked), BN → ``bn<postfix>`` (BatchNorm2d)."""
    cfg = dict(cfg)
    typ = cfg.pop("type")
    cfg.pop("requires_grad", None)
    cfg.setdefault("eps", 1e-5)
    if typ == "IN":
        return f"in{postfix}", nn.InstanceNorm2d(num_features, **cfg)
    if typ in ("BN", "BN2d", "SyncBN"):
        return f"bn{postfix}", nn.BatchNorm2d(num_features, **cfg)
    raise NotImplementedError(f"norm {typ} is not supported by the HIP encoder")


class BasicBlock(nn.Module):
    """models/backbone/resnet.py:12-92 (conv3×3 → norm → ReLU → conv3×3 → norm, + identity)."""
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, dilation: int = 1,
                 downsample: Optional[nn.Module] = None, style: str = "pytorch", with_cp: bool = False,
                 conv_cfg: Optional[dict] = None, norm_cfg: dict = dict(type="BN"), dcn=None,
                 plugins=None, init_cfg=None):
        super().__init__()
        if dcn is not None or plugins is not None or dilation != 1:
            raise NotImplementedError("BasicBlock: dcn / plugins / dilation are not supported")
        self.norm1_name, norm1 = build_norm_layer(norm_cfg, planes, postfix=1)
        self.norm2_name, norm2 = build_norm_layer(norm_cfg, planes, postfix=2)
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride=stride, padding=dilation, bias=True)
        self.add_module(self.norm1_name, norm1)
        self.conv2 = nn.Conv2d(planes, planes, 3, padding=1, bias=True)
        self.add_module(self.norm2_name, norm2)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    @property
    def norm1(self) -> nn.Module:
        return getattr(self, self.norm1_name)

    @property
    def norm2(self) -> nn.Module:
        return getattr(self, self.norm2_name)


class ResLayer(nn.Sequential):
    """models/backbone/resnet.py:676-771 (downsample = 1×1/stride conv + norm when the shape changes)."""

    def __init__(self, block, inplanes: int, planes: int, num_blocks: int, stride: int = 1,
                 avg_down: bool = False, conv_cfg: Optional[dict] = None,
                 norm_cfg: dict = dict(type="BN"), downsample_first: bool = True, **kwargs):
        if avg_down or not downsample_first:
            raise NotImplementedError("ResLayer: avg_down / downsample_first=False are not supported")
        downsample = None
        if stride != 1 or inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(inplanes, planes * block.expansion, 1, stride=stride, bias=True),
                build_norm_layer(norm_cfg, planes * block.expansion)[1])
        layers = [block(inplanes=inplanes, planes=planes, stride=stride, downsample=downsample,
                        conv_cfg=conv_cfg, norm_cfg=norm_cfg, **kwargs)]
        inplanes = planes * block.expansion
        for _ in range(1, num_blocks):
            layers.append(block(inplanes=inplanes, planes=planes, stride=1, conv_cfg=conv_cfg,
                                norm_cfg=norm_cfg, **kwargs))
        super().__init__(*layers)


def _bn_affine(bn: nn.BatchNorm2d) -> Tuple[Tensor, Tensor]:
    """Eval BatchNorm as y = x·scale + shift (per channel), cached per parameter version."""
    key = tuple((t.data_ptr(), t._version) for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var)
                if t is not None) + (_lib.weights_generation(),)
    if getattr(bn, "_scflow_key", None) != key:
        with torch.no_grad():
            inv = torch.rsqrt(bn.running_var.float() + bn.eps)
            sc = inv * bn.weight.float() if bn.weight is not None else inv
            sh = -bn.running_mean.float() * sc
            if bn.bias is not None:
                sh = sh + bn.bias.float()
        bn._scflow_affine = (sc.contiguous(), sh.contiguous())
        bn._scflow_key = key
    return bn._scflow_affine


def _packed(conv: nn.Conv2d, stem: bool = False) -> Tensor:
    w = conv.weight
    key = (w.data_ptr(), w._version, stem, _lib.weights_generation())
    if getattr(conv, "_scflow_enc_key", None) != key:
        conv._scflow_enc_packed = ops.enc_stem_pack(w) if stem else ops.enc_conv_pack(w)
        conv._scflow_enc_key = key
    return conv._scflow_enc_packed


def _wino_ok(conv: nn.Conv2d, h: int, w: int, cin: int) -> bool:
    """3×3 stride-1 pad-1 convs at widths 32/64/128 run on the Winograd F(2×2,3×3) kernel with
    the block's normalisation fused (scflow_conv2d, SCFLOW_CONV_WINO)."""
    return (conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1) and
            w in (32, 64, 128) and h % (4 if w == 32 else 2) == 0 and cin % 4 == 0 and
            conv.groups == 1 and conv.dilation == (1, 1))


def _wino_conv(conv: nn.Conv2d, x: Tensor, out: Tensor, n: int, h: int, w: int, cin: int,
               in_scale: Optional[Tensor] = None, in_shift: Optional[Tensor] = None,
               out_scale: Optional[Tensor] = None, out_shift: Optional[Tensor] = None,
               res: Optional[Tensor] = None, act: Optional[str] = None) -> None:
    wt = conv.weight
    key = (wt.data_ptr(), wt._version, cin, w, _lib.weights_generation())
    cache = getattr(conv, "_scflow_wino", None)
    if cache is None or cache[0] != key:
        cache = (key, ops.pack_conv_weight(wt.detach().float(), cin, 0, w, 1, _lib.CONV_WINO))
        conv._scflow_wino = cache
    cout = conv.out_channels
    ops.conv2d(ops.Chan.whole(x.view(-1, cin)), cache[1], _bias(conv), n, h, w, cout, 3, 3, 1, 1,
               act, out=ops.Chan.whole(out.view(-1, cout)), bk=_lib.CONV_WINO, in_scale=in_scale,
               in_shift=in_shift, out_scale=out_scale, out_shift=out_shift,
               res=None if res is None else ops.Chan.whole(res.view(-1, res.shape[-1])))


def _bias(conv: nn.Conv2d) -> Optional[Tensor]:
    return None if conv.bias is None else conv.bias.detach().float().contiguous()


@MODELS.register_module()
class RAFTEncoder(nn.Module):
    """models/encoder/raft_encoder.py:13-314, 'Basic' / 'Large' (BasicBlock) variants."""
    _arch_settings = {"Basic": (BasicBlock, (2, 2, 2)), "Large": (BasicBlock, (2, 2))}
    _stem_channels = {"Basic": 64, "Small": 32, "Large": 64}
    _base_channels = {"Basic": (64, 96, 128), "Small": (8, 16, 24), "Large": (64, 96)}
    _strides = {"Basic": (1, 2, 2), "Small": (1, 2, 2), "Large": (1, 2)}
    _dilations = {"Basic": (1, 1, 1), "Small": (1, 1, 1), "Large": (1, 1)}

    def __init__(self, in_channels: int, out_channels: int, scale: float = 1 / 8,
                 net_type: str = "Basic", stem_channels: Optional[int] = None,
                 base_channels: Optional[Sequence[int]] = None, num_stages: Optional[int] = None,
                 strides: Optional[Sequence[int]] = None, dilations: Optional[Sequence[int]] = None,
                 deep_stem: bool = False, avg_down: bool = False, frozen_stages: int = -1,
                 conv_cfg: Optional[dict] = None, norm_cfg: dict = dict(type="BN", requires_grad=True),
                 norm_eval: bool = False, plugins=None, with_cp: bool = False, init_cfg=None) -> None:
        super().__init__()
        if net_type not in self._stem_channels:
            raise KeyError(f"invalid net type {net_type} for RAFT")
        if net_type not in self._arch_settings:
            raise NotImplementedError(f"net_type {net_type} (Bottleneck) is not supported by the HIP encoder")
        if deep_stem or plugins is not None:
            raise NotImplementedError("deep_stem / plugins are not supported by the HIP encoder")
        if conv_cfg is not None and conv_cfg.get("type", "Conv2d") != "Conv2d":
            raise NotImplementedError(f"conv_cfg {conv_cfg} is not supported")
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.scale = scale
        self.net_type = net_type
        self.stem_channels = stem_channels if stem_channels is not None else self._stem_channels[net_type]
        self.base_channels = tuple(base_channels if base_channels is not None else self._base_channels[net_type])
        self.num_stages = num_stages if num_stages is not None else len(self.base_channels)
        assert 1 <= self.num_stages <= 3
        self.strides = tuple(strides if strides is not None else self._strides[net_type])
        self.dilations = tuple(dilations if dilations is not None else self._dilations[net_type])
        assert len(self.strides) == len(self.dilations) == self.num_stages
        self.deep_stem, self.avg_down = deep_stem, avg_down
        self.frozen_stages, self.norm_cfg, self.norm_eval = frozen_stages, norm_cfg, norm_eval
        self.norm_type = "IN" if norm_cfg["type"] == "IN" else "BN"
        block, stage_blocks = self._arch_settings[net_type]
        self.stage_blocks = stage_blocks[:self.num_stages]
        stem_stride = 1 if scale == 1 / 4 else 2
        self.conv1 = nn.Conv2d(in_channels, self.stem_channels, kernel_size=7, stride=stem_stride,
                               padding=3, bias=True)
        self.norm1_name, norm1 = build_norm_layer(norm_cfg, self.stem_channels, postfix=1)
        self.add_module(self.norm1_name, norm1)
        self.relu = nn.ReLU(inplace=True)
        self.res_layers = []
        inplanes = self.stem_channels
        for i, num_blocks in enumerate(self.stage_blocks):
            planes = self.base_channels[i]
            layer = ResLayer(block=block, inplanes=inplanes, planes=planes, num_blocks=num_blocks,
                             stride=self.strides[i], dilation=self.dilations[i], conv_cfg=conv_cfg,
                             norm_cfg=norm_cfg)
            inplanes = planes
            name = f"res_layer{i + 1}"
            self.add_module(name, layer)
            self.res_layers.append(name)
        self.conv2 = nn.Conv2d(self.base_channels[-1], out_channels, kernel_size=1)
        if self.norm_type == "IN" and getattr(norm1, "affine", False):
            raise NotImplementedError("affine InstanceNorm is not supported by the HIP encoder")

    @property
    def norm1(self) -> nn.Module:
        return getattr(self, self.norm1_name)

    def train(self, mode: bool = True):
        super().train(mode)
        if mode and self.norm_eval:
            for m in self.modules():
                if isinstance(m, nn.BatchNorm2d):
                    m.eval()
        return self

    # ------------------------------------------------------------------ HIP path
    def _check_bn(self) -> None:
        if self.norm_type == "BN" and any(m.training for m in self.modules() if isinstance(m, nn.BatchNorm2d)):
            raise NotImplementedError("HIP RAFTEncoder: BatchNorm in training mode (batch statistics) "
                                      "is not supported; call .eval()")

    def forward_cl(self, x: Tensor, out: Optional[Tensor] = None, act: Optional[str] = None,
                   act2: Optional[str] = None, act_split: Optional[int] = None) -> Tensor:
        """NCHW image batch → channels-last features [n, h/8, w/8, out_channels] (written to
        ``out`` if given; ``act``/``act2``/``act_split`` optionally activate the output)."""
        ops._require(x, "image")
        self._check_bn()
        n, _, H, W = x.shape
        dev = x.device
        IN = self.norm_type == "IN"
        c0 = self.stem_channels
        s = self.conv1.stride[0]
        h, w = (H + 6 - 7) // s + 1, (W + 6 - 7) // s + 1
        stem = torch.empty(n, h, w, c0, device=dev)
        if IN:
            ops.enc_stem(x, _packed(self.conv1, stem=True), _bias(self.conv1), c0, 7, s, 3, stem)
            sc = torch.empty(n, c0, device=dev)
            sh = torch.empty(n, c0, device=dev)
            ops.enc_instance_norm_stats(stem, n, h * w, c0, sc, sh, eps=self.norm1.eps)
            cur = torch.empty_like(stem)
            ops.enc_apply(stem, sc, sh, cur, n, h * w, c0)
        else:
            bsc, bsh = _bn_affine(self.norm1)
            ops.enc_stem(x, _packed(self.conv1, stem=True), _bias(self.conv1), c0, 7, s, 3, stem,
                         out_scale=bsc, out_shift=bsh, act="ReLU")
            cur = stem
        cin = c0
        for name in self.res_layers:
            for blk in getattr(self, name):
                cur, h, w, cin = self._block(blk, cur, n, h, w, cin, IN)
        cout = self.out_channels
        if out is None:
            out = torch.empty(n, h, w, cout, device=dev)
        ops.enc_conv(cur, _packed(self.conv2), _bias(self.conv2), n, h, w, cin, cout, 1, 1, 0, out,
                     act=act, act2=act2, act_split=act_split)
        return out

    def _block(self, blk: BasicBlock, x: Tensor, n: int, h: int, w: int, cin: int, IN: bool):
        planes = blk.conv1.out_channels
        st = blk.stride
        oh, ow = (h + 2 - 3) // st + 1, (w + 2 - 3) // st + 1
        dev = x.device
        y1 = torch.empty(n, oh, ow, planes, device=dev)
        out = torch.empty(n, oh, ow, planes, device=dev)
        ds = blk.downsample
        if IN:
            sc1, sh1, sc2, sh2 = (torch.empty(n, planes, device=dev) for _ in range(4))
            if st == 1 and _wino_ok(blk.conv1, h, w, cin):
                _wino_conv(blk.conv1, x, y1, n, h, w, cin)
            else:
                ops.enc_conv(x, _packed(blk.conv1), _bias(blk.conv1), n, h, w, cin, planes, 3, st, 1,
                             y1)
            ops.enc_instance_norm_stats(y1, n, oh * ow, planes, sc1, sh1, eps=blk.norm1.eps)
            y2 = torch.empty_like(y1)
            if _wino_ok(blk.conv2, oh, ow, planes):
                _wino_conv(blk.conv2, y1, y2, n, oh, ow, planes, in_scale=sc1, in_shift=sh1)
            else:
                ops.enc_conv(y1, _packed(blk.conv2), _bias(blk.conv2), n, oh, ow, planes, planes, 3,
                             1, 1, y2, in_scale=sc1, in_shift=sh1)
            ops.enc_instance_norm_stats(y2, n, oh * ow, planes, sc2, sh2, eps=blk.norm2.eps)
            if ds is not None:
                d = torch.empty_like(y1)
                scd, shd = torch.empty(n, planes, device=dev), torch.empty(n, planes, device=dev)
                ops.enc_conv(x, _packed(ds[0]), _bias(ds[0]), n, h, w, cin, planes, 1, st, 0, d)
                ops.enc_instance_norm_stats(d, n, oh * ow, planes, scd, shd, eps=ds[1].eps)
                ops.enc_apply(y2, sc2, sh2, out, n, oh * ow, planes, id=d, id_scale=scd, id_shift=shd)
            else:
                ops.enc_apply(y2, sc2, sh2, out, n, oh * ow, planes, id=x)
        else:
            b1, b2 = _bn_affine(blk.norm1), _bn_affine(blk.norm2)
            if st == 1 and _wino_ok(blk.conv1, h, w, cin):
                _wino_conv(blk.conv1, x, y1, n, h, w, cin, out_scale=b1[0], out_shift=b1[1],
                           act="ReLU")
            else:
                ops.enc_conv(x, _packed(blk.conv1), _bias(blk.conv1), n, h, w, cin, planes, 3, st, 1,
                             y1, out_scale=b1[0], out_shift=b1[1], act="ReLU")
            res = x
            if ds is not None:
                res = torch.empty_like(y1)
                bd = _bn_affine(ds[1])
                ops.enc_conv(x, _packed(ds[0]), _bias(ds[0]), n, h, w, cin, planes, 1, st, 0, res,
                             out_scale=bd[0], out_shift=bd[1])
            if _wino_ok(blk.conv2, oh, ow, planes):
                _wino_conv(blk.conv2, y1, out, n, oh, ow, planes, out_scale=b2[0], out_shift=b2[1],
                           res=res, act="ReLU")
            else:
                ops.enc_conv(y1, _packed(blk.conv2), _bias(blk.conv2), n, oh, ow, planes, planes, 3,
                             1, 1, out, out_scale=b2[0], out_shift=b2[1], res=res, act="ReLU")
        return out, oh, ow, planes

    def forward(self, x: Tensor, return_middle_result: bool = False) -> Tensor:
        """raft_encoder.py:286-314 — NCHW in, NCHW out."""
        if return_middle_result:
            raise NotImplementedError("return_middle_result is not supported by the HIP encoder")
        cl = self.forward_cl(x)
        n, h, w, c = cl.shape
        return ops.chan_to_nchw(ops.Chan.whole(cl), n, h, w)
