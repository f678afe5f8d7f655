"""SCFlowDecoder — drop-in replacement for the reference decoder, running on gfx950 HIP kernels.

Reference: ``/root/reference/models/decoder/scflow_decoder.py:19-252``.  Same constructor
kwargs (:48-68), same submodules and state-dict keys (so reference checkpoints load), same
``forward`` signature (:151-156) and the same 7-list return (:252).  ``iters`` is re-read on
every call (the refiner overwrites it temporarily, ``scflow_refiner.py:150-158``).

Forward, per call (B pairs, features h×w = image/8, M = B·h·w):

* a1  ``scflow_corr_pyramid``: correlation GEMM (fp32 MFMA) + pooled levels, once;
* a9  ``scflow_lift_points``: dense per-pixel object-frame points, once (no ``nonzero``, no
  host sync);
* then ``iters`` times, with every activation channels-last in a handful of buffers
  (``HX = [h | cxt | motion | flow]`` is exactly the GRU's ``cat[h, x]``):
  a11↓ downsample → a2 lookup → a3 motion encoder (5 convs) → a4 GRU (4 launches: z/r fused,
  q with the state update fused) → a5 heads (hidden convs of both heads in one launch, thin
  predictors) → a6 Δflow/mask encoders → a7 pose head (PyTorch-ROCm) → a11↑ upsample →
  a8+a10 pose update + reprojection (one launch).

No host synchronisation happens inside ``forward``; the whole call can be captured into a
HIP graph (``graph.py``).  There is no CPU path: inputs must be on a ROCm device.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Sequence, Tuple, Union

import torch
import torch.nn as nn

from . import _lib, ops
from ._lib import ScflowError
from .modules import (ConvGRU, ConvModule, ConvRunner, CorrelationPyramid, CorrLookup,
                      MotionEncoder, XHead, run_chain, run_chain_pair)
from .ops import Chan
from .registry import MODELS

Tensor = torch.Tensor


def _record_on(out, stream) -> None:
    """The forward ran on the decoder's priority stream, so the caching allocator ties its
    outputs' blocks to that stream: record the caller's stream on each one (once per storage)
    so a caller reading them there cannot see the blocks reused before its reads finish."""
    seen = set()
    for item in out:
        for t in (item if isinstance(item, (list, tuple)) else (item,)):
            if isinstance(t, Tensor):
                key = t.untyped_storage().data_ptr()
                if key not in seen:
                    seen.add(key)
                    t.record_stream(stream)


@MODELS.register_module()
class SCFlowDecoder(nn.Module):
    _h_channels = {"Basic": 128, "Small": 96}
    _cxt_channels = {"Basic": 128, "Small": 64}

    def __init__(self, net_type: str, num_levels: int, radius: int, iters: int, detach_flow: bool,
                 detach_mask: bool, detach_pose: bool, mask_flow: bool, mask_corr: bool,
                 pose_head_cfg: dict, depth_transform: str = "exp", detach_depth_for_xy: bool = False,
                 corr_lookup_cfg: dict = dict(align_corners=True), gru_type: str = "SeqConv",
                 feat_channels: Union[int, Sequence[int]] = 256, conv_cfg: Optional[dict] = None,
                 norm_cfg: Optional[dict] = None, act_cfg: Optional[dict] = None) -> None:
        super().__init__()
        assert net_type in ["Basic", "Small"]
        assert type(feat_channels) in (int, tuple, list)
        self.corr_block = CorrelationPyramid(num_levels=num_levels)
        feat_channels = list(feat_channels) if isinstance(feat_channels, (tuple, list)) else [feat_channels]
        self.net_type = net_type
        self.num_levels = num_levels
        self.radius = radius
        self.detach_flow = detach_flow
        self.detach_mask = detach_mask
        self.detach_pose = detach_pose
        self.detach_depth_for_xy = detach_depth_for_xy
        self.mask_flow = mask_flow
        self.mask_corr = mask_corr
        self.depth_transform = depth_transform
        self.h_channels = self._h_channels.get(net_type)
        self.cxt_channels = self._cxt_channels.get(net_type)
        self.iters = iters
        corr_lookup_cfg = dict(corr_lookup_cfg)
        corr_lookup_cfg["radius"] = radius
        self.corr_lookup = CorrLookup(**corr_lookup_cfg)
        self.encoder = MotionEncoder(num_levels=num_levels, radius=radius, net_type=net_type,
                                     conv_cfg=conv_cfg, norm_cfg=norm_cfg, act_cfg=act_cfg)
        self.gru_type = gru_type
        self.gru = ConvGRU(self.h_channels, self.encoder.out_channels[0] + 2 + self.cxt_channels,
                           net_type=gru_type)
        self.pose_pred = MODELS.build(pose_head_cfg)
        self.flow_pred = XHead(self.h_channels, feat_channels, 2, x="flow")
        self.mask_pred = XHead(self.h_channels, feat_channels, 1, x="mask")
        mk = dict(conv_cfg=conv_cfg, norm_cfg=norm_cfg, act_cfg=act_cfg)
        self.delta_flow_encoder = nn.Sequential(
            ConvModule(2, 128, 7, padding=3, **mk), ConvModule(128, 64, 3, padding=1, **mk))
        self.mask_encoder = nn.Sequential(
            ConvModule(1, 64, 3, padding=1, **mk), ConvModule(64, 32, 3, padding=1, **mk))
        self._head_runner = None
        # optional per-kernel timing hooks (bench.py): name -> callable(start: bool)
        # name -> callable(start: bool) bracketing one launch (bench.py's live kernel timing):
        # gru_zr, gru_q, corr_pyramid, corr_lookup, pose_flow
        self.kernel_hooks: Dict[str, object] = {}
        # compute the context features' (loop-invariant) GRU contribution once per forward
        self.hoist_context = True
        # independent branches on a second HIP stream (else everything on the current stream)
        self.side_stream = True
        # the tail's flow-predictor / mask-predictor branches as paired launches on the main
        # stream (scflow_conv2d_pair) instead of two streams joined by events (round 6).
        # -1 = automatic: on for maps of at most 32 × 32 (configs[1]: 4.598 vs 4.612 ms per
        # forward, the profiled iteration 550 → 538 µs with 1.9 µs idle), off above (configs[4]:
        # 43.23 vs 43.17 ms) — profiles/r06/g11_*
        self.pair_tail = -1
        # the XHeads' predictors contracted in the hidden conv's epilogue (scflow_xhead_pred:
        # the 512-channel hidden output is never written; round 6) where the shapes allow it
        self.fuse_xhead_pred = os.environ.get("SCFLOW_XHEAD_PRED", "1") != "0"
        self.dbg_skip_fullres = False  # measurement only (tools/ab_bench.py)
        # fork / join with device-scope events (no system-scope cache writeback per record)
        self.device_scope_events = True
        # the iteration's tail (pose update, pose flow, ×8 prediction, next ↓8 flow) as one
        # launch (scflow_pose_step); only without flow/correlation masking
        self.fuse_tail = True
        # the lookup and corr_net.0 (1×1 324→256) as ONE launch (scflow_corr_lookup_conv1x1: the
        # correlation features stay in LDS) when the geometry allows (tiled pyramid, L = 4, r = 4)
        # and the feature map has at most 32×32 pixels: measured 5.112 vs 5.131 ms/forward at
        # configs[1] (round 5, tools/sess_r5d.sh), but 49.2 vs 48.0 ms at configs[4] (64×64),
        # where the separate lookup (tile-row regions) and 1×1 conv win
        self.fuse_lookup_conv = True
        self.fuse_lookup_conv_max_px = 32 * 32
        # a batch of ≥ 2·pingpong_min pairs runs as two interleaved halves (_forward_pingpong).
        # Off: measured slower at B=16 (5.76 vs 5.33 ms/step) — a half's tail kernels do not get
        # CUs while the other half's convolutions hold every CU's LDS, so they serialise anyway
        self.pingpong = False
        self.pingpong_min = 4
        # with fuse_tail: the iteration's pose step runs only its ↓8 part (the next iteration's
        # flow, scflow_pose_step_part) on the critical path; its full-resolution outputs (pose
        # flow, ×8 prediction, mask) run on the side stream during the next iteration's GRU
        # (they only feed the returned lists)
        self.defer_full_res = True
        # with fuse_tail: the pose head's rotation / translation heads computed inside the pose
        # step's launch (scflow_pose_step_heads) instead of a launch of their own;
        # SCFLOW_FUSE_HEADS=0: off (A/B)
        self.fuse_heads = os.environ.get("SCFLOW_FUSE_HEADS", "1") != "0"
        # the deferred full-resolution part reads the pose the ↓8 part wrote instead of
        # recomputing the update per workgroup (ops.pose_step_given); SCFLOW_FULLRES_GIVEN=0: off
        self.fullres_given = os.environ.get("SCFLOW_FULLRES_GIVEN", "1") != "0"
        # correlation pyramid in the tiled layout (4×4 tiles of 16 floats per map, pooling fused
        # into the GEMM epilogue; ops.corr_pyramid_tiled) when the geometry allows it
        self.tiled_pyramid = True
        # 0: every stream at the default priority; 1: the forward's critical stream is a
        # high-priority stream of the decoder's own (the side branches at the default), so the
        # CP dispatches its workgroups first when both queues hold work; 2: the side branches'
        # stream at high priority instead; -1 (default): 1 for feature maps above 32×32, else 0.
        # Measured (round 5, tools/sess_r5ag.sh, in-process A/B): configs[4] 44.64 / 44.90 /
        # 44.99 ms per forward for 1 / 0 / 2; configs[1] 4.926 / 4.841 / 4.909 ms — at 32² the
        # side branches are nearly as long as the critical ones and must not be held back
        self.main_priority = -1
        self._hooks_on = True
        self.hook_batch = 0

    # ------------------------------------------------------------------ helpers
    def _hidden_heads(self):
        """Both XHeads' first hidden conv as one launch when they have the same shape."""
        fl, ml = self.flow_pred.layers, self.mask_pred.layers
        if len(fl) == 1 and len(ml) == 1 and fl[0].conv.kernel_size == ml[0].conv.kernel_size \
                and fl[0].conv.padding == ml[0].conv.padding:
            if self._head_runner is None:
                self._head_runner = ConvRunner([fl[0].conv, ml[0].conv], "ReLU")
            return self._head_runner
        return None

    def _xhead_pred_plan(self, head_runner, hid, HEAD, N, h, w, dev):
        """(hidden conv args, packed predictor weights, workspace, flow bias, mask bias) for
        scflow_xhead_pred, or None when the heads do not have its shape (3×3 two-output flow
        predictor, 1×1 one-output mask predictor, hidden convs on F(4×4,3×3), width 32 / 64)."""
        if not self.fuse_xhead_pred or head_runner is None or w not in (32, 64) or h % 4:
            return None
        fp, mp = self.flow_pred.predict_layer, self.mask_pred.predict_layer
        fh = self.flow_pred.layers[-1].conv.out_channels
        mh = self.mask_pred.layers[-1].conv.out_channels
        if (tuple(fp.kernel_size) != (3, 3) or tuple(fp.padding) != (1, 1) or tuple(fp.stride) != (1, 1)
                or fp.out_channels != 2 or tuple(mp.kernel_size) != (1, 1) or tuple(mp.padding) != (0, 0)
                or mp.out_channels != 1 or fh % 32 or mh % 32 or head_runner.act != "ReLU"):
            return None
        hargs = head_runner.args(hid, Chan.whole(HEAD), N, h, w)
        if hargs.bk != _lib.CONV_WINO4:
            return None
        key = (fp.weight.data_ptr(), fp.weight._version, mp.weight.data_ptr(), mp.weight._version,
               _lib.weights_generation())
        if getattr(self, "_xpred_key", None) != key:
            self._xpred_w = ops.xhead_pred_pack(fp.weight, mp.weight)
            self._xpred_key = key
        ws = ops.xhead_pred_workspace(N, h, w, fh, fh + mh, dev)
        fb = None if fp.bias is None else fp.bias.detach()
        mb = None if mp.bias is None else mp.bias.detach()
        return hargs, self._xpred_w, ws, fb, mb, fh

    @property
    def hx_channels(self) -> int:
        """Channels of the channels-last GRU working buffer: [h | cxt | motion | flow]."""
        return self.h_channels + self.cxt_channels + self.encoder.out_channels[0] + 2

    def _sync_events(self, dev, slot=0):
        """The fork / join events of a side stream (created once per device and slot, on it)."""
        evs = getattr(self, "_sync_evs", None)
        if evs is None:
            evs = self._sync_evs = {}
        if (dev, slot) not in evs:
            with torch.cuda.device(dev):
                evs[(dev, slot)] = (ops.SyncEvent(), ops.SyncEvent())
        return evs[(dev, slot)]

    def _pp_events(self, dev):
        """The two ping-pong events of _forward_pingpong (device scope, once per device)."""
        return self._sync_events(dev, "pingpong")

    def _side_stream(self, dev, slot=0) -> torch.cuda.Stream:
        """An extra HIP stream (created once per device and slot): slot 0 / 1 the side branches
        of each ping-pong half, "main1" the second half's main stream."""
        ss = getattr(self, "_streams", None)
        if ss is None:
            ss = self._streams = {}
        # "priority" (main_priority 1) and the side branches under main_priority 2: the highest
        # priority the device allows (a lower number is a higher priority)
        prio = -8 if slot == "priority" or (self.main_priority == 2 and slot in (0, 1)) else 0
        if (dev, slot, prio) not in ss:
            ss[(dev, slot, prio)] = torch.cuda.Stream(device=dev, priority=prio)
        return ss[(dev, slot, prio)]

    def _hook(self, name: str, start: bool) -> None:
        if not self._hooks_on:
            return
        h = self.kernel_hooks.get(name)
        if h is not None:
            h(start)

    def _hooks_for(self, *names):
        """Per-layer hooks for run_chain (None where no timer is installed); recorded with the
        segment's launches, so replays bracket the same launches."""
        if not self._hooks_on:
            return None
        hs = [self.kernel_hooks.get(n) if n else None for n in names]
        return hs if any(hs) else None

    # ------------------------------------------------------------------ forward
    def forward(self, feat_render: Tensor, feat_real: Tensor, h_feat: Tensor, cxt_feat: Tensor,
                ref_rotation: Tensor, ref_translation: Tensor, depth: Tensor, internel_k: Tensor,
                label: Tensor, init_flow: Tensor, invalid_flow_num: float,
                head_label: Optional[Tensor] = None):
        """``head_label`` (extension, default None = ``label``): the labels whose first entry
        picks the pose head's class for the whole batch (the reference's ``label[0]`` quirk,
        ``pose_head.py:208-209``).  A data-parallel shard passes the GLOBAL batch's ``label[:1]``
        so that sharded output equals the unsharded forward (``dist.shard_batch``)."""
        if feat_render.device.type != "cuda":
            raise ScflowError("SCFlowDecoder runs on the gfx950 HIP kernels only; move inputs to a "
                              "ROCm device (there is no CPU fallback)")
        with torch.no_grad():
            return self._forward(feat_render, feat_real, h_feat, cxt_feat, ref_rotation,
                                 ref_translation, depth, internel_k, label, init_flow,
                                 float(invalid_flow_num), head_label=head_label)

    def _forward(self, feat_render, feat_real, h_feat, cxt_feat, R0, t0, depth, K, label, init_flow,
                 invalid, hx: Optional[Tensor] = None, head_label: Optional[Tensor] = None):
        """``hx``: optional channels-last [N·h·w, ≥ hc+xc+co+2] buffer whose first hc+xc channels
        already hold tanh(h) | relu(cxt) (SCFlowRefiner writes the context encoder's output
        there directly); h_feat / cxt_feat are then ignored.

        With ``self.pingpong`` and a batch of ≥ 2·``pingpong_min`` pairs the batch runs as two
        halves interleaved on two stream pairs (``_forward_pingpong``); else as one."""
        N = feat_render.shape[0]
        if self.pingpong and hx is None and N >= 2 * self.pingpong_min:
            return self._forward_pingpong(feat_render, feat_real, h_feat, cxt_feat, R0, t0, depth, K,
                                          label, init_flow, invalid, head_label)
        mp = self.main_priority
        if mp < 0:
            mp = 1 if feat_render.shape[-2] * feat_render.shape[-1] > 32 * 32 else 0
        if mp == 1:
            dev = feat_render.device
            cur = torch.cuda.current_stream(dev)
            hp = self._side_stream(dev, "priority")
            hp.wait_stream(cur)  # inputs produced on the caller's stream
            with torch.cuda.stream(hp):
                out = self._run_steps(feat_render, feat_real, h_feat, cxt_feat, R0, t0, depth, K,
                                      label, init_flow, invalid, hx, head_label)
            cur.wait_stream(hp)
            _record_on(out, cur)
            return out
        return self._run_steps(feat_render, feat_real, h_feat, cxt_feat, R0, t0, depth, K, label,
                               init_flow, invalid, hx, head_label)

    def _run_steps(self, feat_render, feat_real, h_feat, cxt_feat, R0, t0, depth, K, label,
                   init_flow, invalid, hx, head_label):
        gen = self._forward_steps(feat_render, feat_real, h_feat, cxt_feat, R0, t0, depth, K, label,
                                  init_flow, invalid, hx=hx, head_label=head_label)
        while True:
            try:
                next(gen)
            except StopIteration as e:
                return e.value

    def _forward_pingpong(self, feat_render, feat_real, h_feat, cxt_feat, R0, t0, depth, K, label,
                          init_flow, invalid, head_label):
        """The batch as two halves A | B, each a complete forward on its own (main, side) stream
        pair, with their iterations interleaved so that one half's latency-bound iteration tail
        (Δflow / mask encoders, pose head, pose update: many small launches that leave most CUs
        idle) runs while the other half's convolutions fill the chip.  Two device-scope events
        keep the halves' convolution phases ("heavy": lookup → motion encoder → GRU → heads) in
        strict alternation: A.heavy(i) → B.heavy(i) → A.heavy(i+1) → …, each half's tail
        overlapping the other's heavy phase.  Every sample is independent except the pose head's
        class, which both halves take from the whole batch's label[0] (pose_head.py:208-209), so
        the result equals the unsplit forward.  Outputs are written straight into the full-batch
        tensors (per-half views)."""
        dev = feat_render.device
        N = feat_render.shape[0]
        n0 = N // 2
        iters = int(self.iters)
        _, H, W = depth.shape
        f32 = torch.float32
        outs = dict(flow_pose=torch.empty(iters, N, 2, H, W, device=dev, dtype=f32),
                    flow_pred=torch.empty(iters, N, 2, H, W, device=dev, dtype=f32),
                    mask=torch.empty(iters, N, 1, H, W, device=dev, dtype=f32),
                    R=torch.empty(iters, N, 3, 3, device=dev, dtype=f32),
                    t=torch.empty(iters, N, 3, device=dev, dtype=f32),
                    drot=torch.empty(iters, N, self.pose_pred.rotation_out_channels, device=dev,
                                     dtype=f32),
                    dt=torch.empty(iters, N, 3, device=dev, dtype=f32))
        gl = (label if head_label is None else head_label).to(dev).long()[:1]
        cur = torch.cuda.current_stream(dev)
        mains = [cur, self._side_stream(dev, "main1")]
        ev = self._pp_events(dev)  # (A heavy done, B heavy done)
        h_main = [m.cuda_stream for m in mains]
        mains[1].wait_stream(cur)  # inputs produced on the caller's stream
        halves = [slice(0, n0), slice(n0, N)]

        def pp(k):
            def before(it):
                if k == 1:
                    ev[0].wait(h_main[1])      # B.heavy(i) after A.heavy(i)
                elif it > 0:
                    ev[1].wait(h_main[0])      # A.heavy(i) after B.heavy(i−1)

            def after(it):
                ev[k].record(h_main[k])
            return before, after

        gens = []
        for k, sl in enumerate(halves):
            sub = dict(flow_pose=outs["flow_pose"][:, sl], flow_pred=outs["flow_pred"][:, sl],
                       mask=outs["mask"][:, sl], R=outs["R"][:, sl], t=outs["t"][:, sl],
                       drot=outs["drot"][:, sl], dt=outs["dt"][:, sl])
            with torch.cuda.stream(mains[k]):
                gens.append(self._forward_steps(
                    feat_render[sl], feat_real[sl], h_feat[sl], cxt_feat[sl], R0[sl], t0[sl],
                    depth[sl], K[sl], label[sl], init_flow[sl], invalid, head_label=gl, outs=sub,
                    slot=k, pp=pp(k), hooks=k == 0))
        # host issue order: A.heavy(i), B.heavy(i), A.tail(i), B.tail(i), … (each generator step
        # runs up to its next yield on its own main stream)
        live = [True, True]
        while any(live):
            for k in (0, 1):
                if live[k]:
                    with torch.cuda.stream(mains[k]):
                        try:
                            next(gens[k])
                        except StopIteration:
                            live[k] = False
        cur.wait_stream(mains[1])
        return (list(outs["flow_pose"].unbind(0)), list(outs["flow_pred"].unbind(0)),
                list(outs["R"].unbind(0)), list(outs["t"].unbind(0)), list(outs["mask"].unbind(0)),
                list(outs["drot"].unbind(0)), list(outs["dt"].unbind(0)))

    def _forward_steps(self, feat_render, feat_real, h_feat, cxt_feat, R0, t0, depth, K, label,
                       init_flow, invalid, hx: Optional[Tensor] = None,
                       head_label: Optional[Tensor] = None, outs: Optional[dict] = None,
                       slot: int = 0, pp=None, hooks: bool = True):
        """The forward as a generator on the CURRENT stream (+ this slot's side stream): yields
        after each iteration's heavy phase (through the heads) and after its tail; returns the
        7 lists.  ``outs``: preallocated output tensors (``_forward_pingpong``'s views);
        ``pp``: (before_heavy(it), after_heavy(it)) callables ordering this half against the
        other; ``hooks``: whether the bench's kernel timers bracket this forward's launches."""
        dev = feat_render.device
        self._hooks_on = hooks
        self.hook_batch = feat_render.shape[0]  # pairs per bracketed launch (bench roofline)
        f32 = torch.float32
        feat_render = feat_render.contiguous().float()
        feat_real = feat_real.contiguous().float()
        N, C, h, w = feat_render.shape
        _, H, W = depth.shape
        scale = 2 ** (self.num_levels - 1)
        M = N * h * w
        hc, xc = self.h_channels, self.cxt_channels
        co = self.encoder.out_channels[0]
        hx_c = self.hx_channels
        iters = int(self.iters)

        # a1 + a9 (once per forward)
        tiled = self.tiled_pyramid and ops.tiled_lookup_ok(h, w, self.num_levels, self.radius,
                                                           self.corr_lookup.align_corners)
        self._hook("corr_pyramid", True)
        if tiled:
            pyr = ops.corr_pyramid_tiled(feat_render, feat_real, self.num_levels)
        else:
            pyr, _ = ops.corr_pyramid(feat_render, feat_real, self.num_levels)
        self._hook("corr_pyramid", False)
        depth = depth.contiguous().float()
        K = K.contiguous().float()
        R_prev = R0.contiguous().float()
        t_prev = t0.contiguous().float()
        points = ops.lift_points(depth, K, R_prev, t_prev)

        # channels-last working set
        if hx is not None:
            if hx.shape != (M, hx_c) or hx.dtype != f32 or not hx.is_contiguous():
                raise ValueError(f"hx must be a contiguous float32 [{M}, {hx_c}] buffer")
            HX = hx
        else:
            HX = torch.empty(M, hx_c, device=dev, dtype=f32)
            ops.nchw_into(h_feat.contiguous().float(), Chan(HX, 0, hc))
            ops.nchw_into(cxt_feat.contiguous().float(), Chan(HX, hc, xc))
        # loop-invariant context share of the GRU pre-activations (once per forward)
        ctx_map = self.gru.context_map(Chan(HX, hc, xc), N, h, w) if self.hoist_context else None
        F2 = torch.empty(M, 2, device=dev, dtype=f32)
        K_look = self.num_levels * (2 * self.radius + 1) ** 2
        CORR = torch.empty(M, K_look, device=dev, dtype=f32)
        cc = self.encoder.corr_net[-1].conv.out_channels
        cf = self.encoder.flow_net[-1].conv.out_channels
        MF = torch.empty(M, cc + cf, device=dev, dtype=f32)
        Z = torch.empty(M, hc, device=dev, dtype=f32)
        RH = torch.empty(M, hc, device=dev, dtype=f32)
        fh = self.flow_pred.layers[-1].conv.out_channels
        mh = self.mask_pred.layers[-1].conv.out_channels
        HEAD = torch.empty(M, fh + mh, device=dev, dtype=f32)
        D2 = torch.empty(M, 2, device=dev, dtype=f32)
        MASK = torch.empty(M, 1, device=dev, dtype=f32)
        dfc = self.delta_flow_encoder[-1].conv.out_channels
        mfc = self.mask_encoder[-1].conv.out_channels
        FM = torch.empty(M, dfc + mfc, device=dev, dtype=f32)  # [Δflow feat | mask feat]

        def scratch(mods):
            return [torch.empty(M, m.conv.out_channels, device=dev, dtype=f32) for m in mods[:-1]]

        s_corr = scratch(self.encoder.corr_net)
        s_flow = scratch(self.encoder.flow_net)
        s_out = scratch(self.encoder.out_net)
        s_dfe = scratch(self.delta_flow_encoder)
        s_me = scratch(self.mask_encoder)

        # outputs (stacked; the lists returned are views)
        if outs is not None:
            o_flow_pose, o_flow_pred, o_mask = outs["flow_pose"], outs["flow_pred"], outs["mask"]
            o_R, o_t = outs["R"], outs["t"]
        else:
            o_flow_pose = torch.empty(iters, N, 2, H, W, device=dev, dtype=f32)
            o_flow_pred = torch.empty(iters, N, 2, H, W, device=dev, dtype=f32)
            o_mask = torch.empty(iters, N, 1, H, W, device=dev, dtype=f32)
            o_R = torch.empty(iters, N, 3, 3, device=dev, dtype=f32)
            o_t = torch.empty(iters, N, 3, device=dev, dtype=f32)
        drots, dts = [], []

        head_runner = self._hidden_heads()
        flow_pred_r = ConvRunner.of(self.flow_pred.predict_layer, None)
        mask_pred_r = ConvRunner.of(self.mask_pred.predict_layer, "Sigmoid")
        label = (label if head_label is None else head_label).to(dev).long()
        mask_lr = None
        if self.mask_corr or self.mask_flow:
            mask_lr = torch.ones(M, 1, device=dev, dtype=f32)  # interpolate(ones, 1/8) == ones
        flow_full = init_flow.contiguous().float()
        hx_flow = Chan(HX, hx_c - 2, 2)
        hx_motion = Chan(HX, hc + xc, co)
        hid = Chan(HX, 0, hc)
        # independent branches run concurrently on a second stream, joined with events:
        # flow_net ‖ (lookup, corr_net); mask predictor + mask encoder ‖ flow predictor +
        # Δflow encoder.  Every buffer is allocated above on the main stream and outlives the
        # forward, and the main stream always waits for the side branch before reusing them.
        main = torch.cuda.current_stream(dev)
        two = self.side_stream
        side = self._side_stream(dev, slot) if two else main

        # two events reused every iteration (a wait captures the event's state when issued);
        # device-scope ones (ops.SyncEvent) unless self.device_scope_events is False
        if two and self.device_scope_events:
            ev_fork, ev_join = self._sync_events(dev, slot)
            h_main, h_side = main.cuda_stream, side.cuda_stream

            def fork():
                ev_fork.record(h_main)
                ev_fork.wait(h_side)

            def join():
                ev_join.record(h_side)
                ev_join.wait(h_main)
        else:
            ev_fork, ev_join = (torch.cuda.Event(), torch.cuda.Event()) if two else (None, None)

            def fork():
                if two:
                    ev_fork.record(main)
                    side.wait_event(ev_fork)

            def join():
                if two:
                    ev_join.record(side)
                    main.wait_event(ev_join)

        # Host path: the launches that read and write the same persistent buffers in every
        # iteration are recorded on the first iteration (ops.binding: argument structs built
        # once) and replayed afterwards as one ctypes call each; only the launches whose
        # arguments change per iteration (flow in / out, poses, Δpose) go through the wrappers.
        # This keeps the host well ahead of the GPU (a Python wrapper costs more than several of
        # the pose head's kernels take to run).
        rec = {}
        keep = []  # buffers the recorded pose-head launches write (alive for the forward)

        def segment(name, fn):
            calls = rec.get(name)
            if calls is None:
                calls = rec[name] = []
                with ops.binding(calls):
                    fn()
            else:
                for c in calls:
                    c()

        gru_step = self.gru.bind_step(Chan.whole(HX), Chan.whole(Z), Chan.whole(RH), N, h, w,
                                      ctx_map=ctx_map, cxt_channels=xc)
        if outs is not None:
            o_drot, o_dt = outs["drot"], outs["dt"]
        else:
            o_drot = torch.empty(iters, N, self.pose_pred.rotation_out_channels, device=dev,
                                 dtype=f32)
            o_dt = torch.empty(iters, N, 3, device=dev, dtype=f32)
        # Fused iteration tail (no masking): one launch does the pose update, the pose flow, this
        # iteration's ×8 prediction (from F2) and the next iteration's ↓8 flow (into the other
        # F2 buffer, computed from the new pose).  F2 alternates between two buffers, so the
        # recorded launches that read it (lookup, flow branch) are recorded once per parity.
        fuse_tail = self.fuse_tail and not (self.mask_flow or self.mask_corr)
        F2s = [F2, torch.empty_like(F2)] if fuse_tail else [F2, F2]
        flow_in = F2 * mask_lr if self.mask_flow else F2

        def seg_flow_branch():
            run_chain(self.encoder.flow_net, Chan.whole(flow_in), Chan(MF, cc, cf), N, h, w, s_flow,
                      hooks=self._hooks_for(None, "flow_net1"))

        def seg_lookup():
            ops.corr_lookup(pyr, F2, N, h, w, self.num_levels, self.radius, out=Chan.whole(CORR),
                            flow_layout="nhwc", align_corners=self.corr_lookup.align_corners,
                            tiled=tiled)

        corr_net = self.encoder.corr_net
        c0m = corr_net[0].conv
        fuse_lc = (self.fuse_lookup_conv and h * w <= self.fuse_lookup_conv_max_px and tiled and
                   not self.mask_corr and len(corr_net) == 2 and
                   tuple(c0m.kernel_size) == (1, 1) and tuple(c0m.stride) == (1, 1) and
                   tuple(c0m.padding) == (0, 0) and
                   ops.lookup_conv1x1_ok(h, w, self.num_levels, self.radius, c0m.in_channels,
                                         c0m.out_channels))

        def seg_lookup_conv():  # a2 + corr_net.0 in one launch
            r0 = ConvRunner.of(c0m, corr_net[0].act_type)
            packed, bias = r0.packed(c0m.in_channels, 0, w, _lib.CONV_1X1W)
            ops.corr_lookup_conv1x1(pyr, F2, packed, bias, Chan.whole(s_corr[-1]), N, h, w,
                                    self.num_levels, self.radius, c0m.out_channels,
                                    corr_net[0].act_type, self.corr_lookup.align_corners)

        def seg_corr_hidden():  # corr_net.0 (1×1 324→256)
            if len(corr_net) > 1:
                run_chain(corr_net[:-1], Chan.whole(CORR), Chan.whole(s_corr[-1]), N, h, w,
                          s_corr[:-1])

        def seg_corr_last():  # corr_net.1 (3×3 256→192), bracketed by the "corr_net1" hook
            src = Chan.whole(s_corr[-1]) if len(corr_net) > 1 else Chan.whole(CORR)
            ConvRunner.of(corr_net[-1].conv, corr_net[-1].act_type).run(src, Chan(MF, 0, cc), N, h, w)

        def seg_out():
            run_chain(self.encoder.out_net, Chan.whole(MF), hx_motion, N, h, w, s_out,
                      hooks=self._hooks_for("out_net"))

        xpred = self._xhead_pred_plan(head_runner, hid, HEAD, N, h, w, dev)

        def seg_heads():
            if xpred is not None:  # hidden conv + both predictors → Δflow, mask
                hargs, pw, xws, fb, mb, fh_ = xpred
                ops.xhead_pred(hargs, fh_, pw, xws, fb, mb, None, "Sigmoid",
                               Chan.whole(D2s[cur_par[0]]), Chan.whole(MASKs[cur_par[0]]))
            elif head_runner is not None:
                head_runner.run(hid, Chan.whole(HEAD), N, h, w)
            else:
                run_chain(self.flow_pred.layers, hid, Chan(HEAD, 0, fh), N, h, w)
                run_chain(self.mask_pred.layers, hid, Chan(HEAD, fh, mh), N, h, w)

        def seg_mask_branch():
            MK = MASKs[cur_par[0]]
            if xpred is None:
                mask_pred_r.run(Chan(HEAD, fh, mh), Chan.whole(MK), N, h, w)
            run_chain(self.mask_encoder, Chan.whole(MK), Chan(FM, dfc, mfc), N, h, w, s_me,
                      hooks=self._hooks_for(None, "mask_enc1"))

        def seg_tail_pair():
            # the flow-predictor and mask-predictor branches on the main stream, their k-th
            # launches paired into one grid each (scflow_conv2d_pair): no fork / join events
            D2, MK = D2s[cur_par[0]], MASKs[cur_par[0]]
            if xpred is None:
                ops.conv2d_pair(flow_pred_r.args(Chan(HEAD, 0, fh), Chan.whole(D2), N, h, w),
                                mask_pred_r.args(Chan(HEAD, fh, mh), Chan.whole(MK), N, h, w), HEAD)
            run_chain_pair(self.delta_flow_encoder, Chan.whole(D2), Chan(FM, 0, dfc),
                           self.mask_encoder, Chan.whole(MK), Chan(FM, dfc, mfc), N, h, w, s_dfe,
                           s_me)

        def seg_flow_pred():
            D2 = D2s[cur_par[0]]
            if xpred is None:
                flow_pred_r.run(Chan(HEAD, 0, fh), Chan.whole(D2), N, h, w)
            run_chain(self.delta_flow_encoder, Chan.whole(D2), Chan(FM, 0, dfc), N, h, w, s_dfe,
                      hooks=self._hooks_for(None, "dflow1"))

        pose_x = []
        tail_calls = None  # fused tail: per-iteration (heads, pose_step) launches, built once
        defer = fuse_tail and self.defer_full_res and iters > 1
        # Δflow alternates between two buffers when the full-resolution outputs are deferred: the
        # previous iteration's deferred launch reads its Δflow on the side stream while this
        # iteration's flow predictor writes the other one on the main stream
        D2s = [D2, torch.empty_like(D2)] if defer else [D2, D2]
        # the mask likewise (read by the previous iteration's deferred launch on the side stream
        # while this iteration's mask predictor writes the other one — on the main stream when
        # the tail is paired)
        MASKs = [MASK, torch.empty_like(MASK)] if defer else [MASK, MASK]
        pt = self.pair_tail if self.pair_tail >= 0 else int(h * w <= 32 * 32)
        pair_tail = (bool(pt) and len(self.delta_flow_encoder) == len(self.mask_encoder) and
                     not (self.mask_flow or self.mask_corr))
        cur_par = [0]
        pending = []  # the previous iteration's deferred full-resolution launches
        if defer:  # the deferred launches' pose outputs (duplicates of o_R / o_t: not read)
            R_scr = torch.empty(N, 3, 3, device=dev, dtype=f32)
            t_scr = torch.empty(N, 3, device=dev, dtype=f32)

        def seg_pose_trunk():
            pose_x.append(self.pose_pred.trunk_hip(hid, Chan.whole(FM), N, h, w, ws=keep))

        for it in range(iters):
            par = f"{it % 2}" if fuse_tail else ""
            F2 = F2s[it % 2]
            if not self.mask_flow:
                flow_in = F2
            # a11 ↓: flow at feature resolution → F2 (and the motion-feature flow channels); the
            # fused tail of the previous iteration already wrote it
            if not fuse_tail or it == 0:
                ops.flow_downsample(flow_full, Chan.whole(F2), h, w, 1.0 / scale,
                                    out1=None if self.mask_flow else hx_flow)
            if self.mask_flow:
                torch.mul(F2, mask_lr, out=flow_in)
                HX[:, hx_c - 2:].copy_(flow_in)
            if pp is not None:
                pp[0](it)
            # a3 (flow branch) on the side stream
            fork()
            with torch.cuda.stream(side):
                segment("flow_branch" + par, seg_flow_branch)
            # a2 + a3 (correlation branch)
            if fuse_lc:
                self._hook("corr_lookup_conv", True)
                segment("lookup_conv" + par, seg_lookup_conv)
                self._hook("corr_lookup_conv", False)
            else:
                self._hook("corr_lookup", True)
                segment("lookup" + par, seg_lookup)
                self._hook("corr_lookup", False)
                if self.mask_corr:
                    CORR.mul_(mask_lr)
                segment("corr_hidden", seg_corr_hidden)
            self._hook("corr_net1", True)
            segment("corr_last", seg_corr_last)
            self._hook("corr_net1", False)
            join()
            if pending:
                # the previous iteration's full-resolution outputs on the side stream AFTER the
                # join's record: they overlap out_net and the GRU (MFMA-bound) instead of
                # lengthening a joined branch; the mask branch queued behind them reads MASK after
                # they do, and Δflow / F2 are double-buffered against this iteration's writes
                with torch.cuda.stream(side):
                    self._hook("pose_flow", True)
                    for c in pending:
                        c()
                    self._hook("pose_flow", False)
                pending = []
            segment("out", seg_out)
            # a4 GRU (in place on HX[:, :hc])
            gru_step(self.kernel_hooks)
            # a5 heads (with xpred: the predictors too, into this iteration's Δflow / mask)
            cur_par[0] = it % 2 if defer else 0
            self._hook("heads", True)
            segment("heads" + (par if xpred is not None and defer else ""), seg_heads)
            self._hook("heads", False)
            if pp is not None:
                pp[1](it)
            yield "heavy"
            if pair_tail:
                # flow predictor + Δflow encoder ‖ mask predictor + mask encoder (a5, a6) as
                # paired launches on this stream
                segment("tail_pair" + (par if defer else ""), seg_tail_pair)
            else:
                # mask predictor + mask encoder (a5, a6) on the side stream, after the previous
                # iteration's deferred full-resolution outputs (they read its MASK; the side
                # branch is the shorter one here)
                fork()
                with torch.cuda.stream(side):
                    segment("mask_branch" + (par if defer else ""), seg_mask_branch)
                # flow predictor + Δflow encoder (into this iteration's Δflow buffer)
                segment("flow_pred" + (par if defer else ""), seg_flow_pred)
                join()
            if mask_lr is not None:
                mask_lr = MASKs[cur_par[0]]
            # a7 pose head on cat[h, Δflow feat, mask feat] (two channel sources, no concat)
            segment("pose_trunk", seg_pose_trunk)
            drot, dtr = o_drot[it], o_dt[it]
            if fuse_tail:
                # a8 + a10 + a11 ↑ (+ the next iteration's a11 ↓): one launch.  The heads and
                # this launch take per-iteration pointers; their argument lists for every
                # iteration are built once (after the trunk's first pass) and replayed as one
                # ctypes call each, like the recorded segments
                if tail_calls is None:
                    tail_calls = []
                    Rp, tp = R_prev, t_prev
                    for j in range(iters):
                        last = j == iters - 1
                        hc, pc, fc = [], [], []
                        step = (o_drot[j], o_dt[j], Rp, tp, K, points, o_R[j], o_t[j],
                                o_flow_pose[j], invalid, F2s[j % 2], D2s[j % 2], MASKs[j % 2], o_flow_pred[j],
                                o_mask[j], h, w, float(scale))
                        nxt = dict(lr_next=None if last else Chan.whole(F2s[(j + 1) % 2]),
                                   hx_next=None if last else hx_flow,
                                   depth_transform=self.depth_transform)
                        # the rotation / translation heads inside the pose step's launch
                        # (scflow_pose_step_heads), or as their own launch before it
                        ha = self.pose_pred.heads_args(pose_x[0], label) if self.fuse_heads else None
                        if ha is None:
                            with ops.binding(hc, run=False):
                                self.pose_pred.heads_hip(pose_x[0], label, o_drot[j], o_dt[j])
                        else:
                            nxt["heads"] = ha
                        if defer and not last:
                            with ops.binding(pc, run=False):
                                ops.pose_step(*step, **nxt, parts=2)
                            with ops.binding(fc, run=False):
                                if self.fullres_given:
                                    ops.pose_step_given(o_R[j], o_t[j], *step[4:6], *step[8:])
                                else:  # (reads the deltas the ↓8 launch wrote)
                                    fstep = step[:6] + (R_scr, t_scr) + step[8:]
                                    ops.pose_step(*fstep, **{k: v for k, v in nxt.items() if k != "heads"},
                                                  parts=1)
                        else:
                            with ops.binding(pc, run=False):
                                ops.pose_step(*step, **nxt)
                        tail_calls.append((hc, pc, fc))
                        Rp, tp = o_R[j], o_t[j]
                hc, pc, fc = tail_calls[it]
                for c in hc:
                    c()
                # deferred: this is the critical-path ↓8 launch (its own timer); otherwise the
                # whole pose step
                hook = "pose_step_crit" if fc else "pose_flow"
                self._hook(hook, True)
                for c in pc:
                    c()
                self._hook(hook, False)
                if self.kernel_hooks:  # measurement only: bench.py times a launch alone
                    self._tail_calls = tail_calls
                # (dbg_skip_fullres: measurement only — drops the deferred full-resolution
                # outputs to price their side-stream contention; outputs are then incomplete)
                pending = [] if self.dbg_skip_fullres else fc
            else:
                self.pose_pred.heads_hip(pose_x[0], label, drot, dtr)
                # a11 ↑: flow_pred = 8·up(flow + Δflow), mask ↑
                ops.flow_upsample(F2, D2s[0], MASKs[0], N, h, w, H, W, float(scale), o_flow_pred[it],
                                  o_mask[it])
                # a8 + a10: pose update + pose-induced flow (one launch)
                self._hook("pose_flow", True)
                ops.pose_update_flow(drot, dtr, R_prev, t_prev, K, points, o_R[it], o_t[it],
                                     o_flow_pose[it], invalid, depth_transform=self.depth_transform)
                self._hook("pose_flow", False)
            R_prev, t_prev = o_R[it], o_t[it]
            flow_full = o_flow_pose[it]
            drots.append(drot)
            dts.append(dtr)
            yield "tail"
        if pair_tail:
            # with the tail paired on the main stream the side stream's last work (the deferred
            # full-resolution outputs queued in the last iteration) is not joined inside the loop
            join()

        return (list(o_flow_pose.unbind(0)), list(o_flow_pred.unbind(0)), list(o_R.unbind(0)),
                list(o_t.unbind(0)), list(o_mask.unbind(0)), drots, dts)
