"""Generate golden vectors by running the REFERENCE's own hot-path modules on CPU.

Run in the development container only (needs ``/root/reference``; never on the GPU box):

    python tests/golden/make_golden.py            # writes tests/golden/*.npz
    python tests/golden/make_golden.py train      # only the training-step fixtures
    python tests/golden/make_golden.py metric     # only golden_metric_add.npz (metrics/add.py ADD)

The reference (GiaKhangLuu/SCFlow) is pure Python/PyTorch; its hot-path modules import
mmcv / mmengine / kornia / cv2 / turtle / a registry, none of which are installed here
(SURVEY.md §8(c)).  This script installs minimal test-only stand-ins for those imports
*in this process only*, then loads the reference files straight from ``/root/reference``
by path (bypassing ``models/__init__.py``, which would import pytorch3d):

* ``mmcv.cnn.ConvModule`` — restated as conv → (norm) → act with ``bias = norm is None``
  (mmcv's documented ``bias='auto'`` behaviour; layer names ``conv``/``gn`` so the
  state-dict keys are the reference's);
* ``mmengine.model.BaseModule`` — ``nn.Module`` accepting ``init_cfg``;
* ``registry.MODELS`` — ``register_module()`` / ``build(cfg)``;
* ``kornia``, ``cv2``, ``datasets.pose``, ``turtle`` — empty modules (only used off-path:
  quaternion mode, PnP, ``from turtle import forward`` at raft_decoder.py:3).

Everything arithmetic on the path — CorrelationPyramid, CorrLookup, MotionEncoder,
ConvGRU, XHead, MultiClassPoseHead, pose.py, SCFlowDecoder.forward — is the reference's
own code.  Inputs and weights come from ``scflow_amd.synthetic`` (deterministic), so the
fixtures store outputs (and small inputs); nothing of the reference's source is stored.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from scflow_amd import synthetic  # noqa: E402


# ------------------------------------------------------------------ test-only stand-ins
class _BaseModule(nn.Module):
    def __init__(self, init_cfg=None):
        super().__init__()
        self.init_cfg = init_cfg


class _ConvModule(nn.Module):
    """mmcv ConvModule as used on the path: conv → norm → act, bias iff no norm."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0,
                 conv_cfg=None, norm_cfg=None, act_cfg=dict(type="ReLU"), **kw):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride=stride,
                              padding=padding, bias=norm_cfg is None)
        self.norm_name = None
        if norm_cfg is not None:
            assert norm_cfg["type"] == "GN"
            self.norm_name = "gn"
            self.gn = nn.GroupNorm(norm_cfg["num_groups"], out_channels)
        self.act = None
        if act_cfg is not None:
            self.act = {"ReLU": nn.ReLU, "Sigmoid": nn.Sigmoid, "Tanh": nn.Tanh}[act_cfg["type"]]()

    def forward(self, x):
        x = self.conv(x)
        if self.norm_name:
            x = self.gn(x)
        if self.act is not None:
            x = self.act(x)
        return x


class _Registry:
    def __init__(self):
        self._m = {}

    def register_module(self, name=None, module=None, force=False):
        def deco(cls):
            self._m[cls.__name__] = cls
            return cls
        return deco

    def build(self, cfg):
        cfg = dict(cfg)
        typ = cfg.pop("type")
        cls = self._m[typ] if isinstance(typ, str) else typ
        return cls(**cfg)


def _build_conv_layer(cfg, *args, **kwargs):
    """mmcv build_conv_layer with cfg None / Conv2d → nn.Conv2d."""
    assert cfg is None or cfg.get("type", "Conv2d") == "Conv2d"
    return nn.Conv2d(*args, **kwargs)


def _build_norm_layer(cfg, num_features, postfix=""):
    """mmcv build_norm_layer: (abbr + postfix, layer); IN → InstanceNorm2d, BN → BatchNorm2d,
    GN → GroupNorm; ``requires_grad`` dropped, eps defaults to 1e-5."""
    cfg = dict(cfg)
    typ = cfg.pop("type")
    cfg.pop("requires_grad", None)
    cfg.setdefault("eps", 1e-5)
    if typ == "IN":
        return f"in{postfix}", nn.InstanceNorm2d(num_features, **cfg)
    if typ == "BN":
        return f"bn{postfix}", nn.BatchNorm2d(num_features, **cfg)
    if typ == "GN":
        return f"gn{postfix}", nn.GroupNorm(num_channels=num_features, **cfg)
    raise KeyError(typ)


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def _pkg(name, path):
    m = _stub(name)
    m.__path__ = [path]
    return m


def _load(name, relpath):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, relpath))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    """Import the reference hot-path modules; returns a namespace of them."""
    _stub("mmcv")
    _stub("mmcv.cnn", ConvModule=_ConvModule, build_conv_layer=_build_conv_layer,
          build_norm_layer=_build_norm_layer, build_plugin_layer=None)
    _stub("mmengine")
    _stub("mmengine.model", BaseModule=_BaseModule, Sequential=nn.Sequential)
    MODELS = _Registry()
    _stub("registry", MODELS=MODELS)
    _stub("kornia")
    _stub("cv2")
    _stub("turtle", forward=None)
    _pkg("datasets", os.path.join(REF, "datasets"))
    _stub("datasets.pose", remap_pose=None)
    _pkg("models", os.path.join(REF, "models"))
    utils = _pkg("models.utils", os.path.join(REF, "models/utils"))
    _pkg("models.decoder", os.path.join(REF, "models/decoder"))
    _pkg("models.head", os.path.join(REF, "models/head"))
    cl = _load("models.utils.corr_lookup", "models/utils/corr_lookup.py")
    pose = _load("models.utils.pose", "models/utils/pose.py")
    for k in ("CorrLookup", "coords_grid"):
        setattr(utils, k, getattr(cl, k))
    for k in ("get_flow_from_delta_pose_and_points", "get_pose_from_delta_pose",
              "cal_3d_2d_corr", "get_flow_from_delta_pose_and_depth"):
        setattr(utils, k, getattr(pose, k))
    rd = _load("models.decoder.raft_decoder", "models/decoder/raft_decoder.py")
    sd = _load("models.decoder.scflow_decoder", "models/decoder/scflow_decoder.py")
    ph = _load("models.head.pose_head", "models/head/pose_head.py")
    _pkg("models.backbone", os.path.join(REF, "models/backbone"))
    _pkg("models.encoder", os.path.join(REF, "models/encoder"))
    _load("models.backbone.resnet", "models/backbone/resnet.py")
    enc = _load("models.encoder.raft_encoder", "models/encoder/raft_encoder.py")
    return types.SimpleNamespace(MODELS=MODELS, corr_lookup=cl, pose=pose, raft=rd, scflow=sd,
                                 pose_head=ph, encoder=enc)


# encoder blocks of configs/refine_models/scflow_ycbv_real.py:179-206
def encoder_cfg(norm):
    return dict(in_channels=3, out_channels=256, net_type="Basic", norm_cfg=dict(type=norm))


# decoder block of configs/refine_models/scflow_ycbv_real.py:207-230
def decoder_cfg(ref, iters=4, feat_size=None):
    head = dict(type=ref.pose_head.MultiClassPoseHead, num_class=21, in_channels=224,
                net_type="Basic", rotation_mode="ortho6d",
                norm_cfg=dict(type="GN", num_groups=32, requires_grad=True),
                act_cfg=dict(type="ReLU"))
    if feat_size is not None:
        head["feat_size"] = feat_size
    return dict(net_type="Basic", num_levels=4, radius=4, iters=iters, detach_flow=True,
                detach_mask=True, detach_pose=True, detach_depth_for_xy=True, mask_flow=False,
                mask_corr=False, pose_head_cfg=head, corr_lookup_cfg=dict(align_corners=True),
                gru_type="SeqConv", act_cfg=dict(type="ReLU"))


def t32(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def gen_ops(ref, out):
    rng = np.random.default_rng(123)
    # (1) correlation pyramid, N=2 C=8 H=W=8
    f1 = rng.standard_normal((2, 8, 8, 8)).astype(np.float32)
    f2 = rng.standard_normal((2, 8, 8, 8)).astype(np.float32)
    pyr = ref.raft.CorrelationPyramid(num_levels=4)(t32(f1), t32(f2))
    out["pyr_f1"], out["pyr_f2"] = f1, f2
    for i, p in enumerate(pyr):
        out[f"pyr_l{i}"] = p.numpy()
    # (2) lookup on that pyramid, flow in ±6 px (hits zero padding), r=4 and r=1
    flow = rng.uniform(-6, 6, (2, 2, 8, 8)).astype(np.float32)
    out["lk_flow"] = flow
    for r in (4, 1):
        lk = ref.corr_lookup.CorrLookup(radius=r, align_corners=True)
        out[f"lk_r{r}"] = lk([p.clone() for p in pyr], t32(flow)).numpy()
    # align_corners=False (bilinear_sample's default, corr_lookup.py:35; a CorrLookup option)
    lk = ref.corr_lookup.CorrLookup(radius=4, align_corners=False)
    out["lk_r4_ac0"] = lk([p.clone() for p in pyr], t32(flow)).numpy()
    # (3) one SeqConv GRU step, h/x at 2×8×8 (h 8 ch, x 16 ch)
    gru = ref.raft.ConvGRU(8, 16, net_type="SeqConv")
    synthetic.fill_module_(gru, seed=3)
    h = np.tanh(rng.standard_normal((2, 8, 8, 8))).astype(np.float32)
    x = rng.standard_normal((2, 16, 8, 8)).astype(np.float32)
    with torch.no_grad():
        out["gru_h"], out["gru_x"] = h, x
        out["gru_out"] = gru(t32(h), t32(x)).numpy()
    # (4) pose update + pose-induced flow: B=3 poses, analytic depth 64², f chosen per scene
    scene = synthetic.make_scene(3, 64, seed=5)
    drot = (np.tile([1.0, 0, 0, 0, 1.0, 0], (3, 1)) + 0.05 * rng.standard_normal((3, 6))).astype(np.float32)
    dtr = (np.array([[0.5, -0.3, 0.02]]) * rng.standard_normal((3, 3))).astype(np.float32)
    R1, t1 = ref.pose.get_pose_from_delta_pose(t32(drot), t32(dtr), t32(scene["ref_rotation"]),
                                              t32(scene["ref_translation"]), depth_transform="exp",
                                              detach_depth_for_xy=True)
    p2d, p3d = [], []
    for i in range(3):
        a, b = ref.pose.cal_3d_2d_corr(t32(scene["depth"][i]), t32(scene["internel_k"][i]),
                                       t32(scene["ref_rotation"][i]), t32(scene["ref_translation"][i]))
        p2d.append(a)
        p3d.append(b)
    for k, v in scene.items():
        out[f"pose_{k}"] = v
    out["pose_drot"], out["pose_dt"] = drot, dtr
    out["pose_R1"], out["pose_t1"] = R1.numpy(), t1.numpy()
    for inv in (0.0, 400.0):
        fl = ref.pose.get_flow_from_delta_pose_and_points(R1, t1, t32(scene["internel_k"]), p2d, p3d,
                                                          64, 64, invalid_num=inv)
        out[f"pose_flow_inv{int(inv)}"] = fl.numpy()
    gtf = ref.pose.get_flow_from_delta_pose_and_depth(
        t32(scene["ref_rotation"]), t32(scene["ref_translation"]), R1, t1, t32(scene["depth"]),
        t32(scene["internel_k"]), invalid_num=400)
    out["pose_gtflow"] = gtf.numpy()


def run_decoder(ref, inputs, iters, feat_size=None, dtype=torch.float32, seed=0):
    dec = ref.MODELS.build(dict(type=ref.scflow.SCFlowDecoder, **decoder_cfg(ref, iters, feat_size)))
    synthetic.fill_module_(dec, seed=seed)
    dec = dec.to(dtype).eval()
    t = {k: t32(v) for k, v in inputs.items()}
    for k, v in t.items():
        if v.is_floating_point():
            t[k] = v.to(dtype)
    with torch.no_grad():
        res = dec(t["feat_render"], t["feat_real"], t["h_feat"], t["cxt_feat"], t["ref_rotation"],
                  t["ref_translation"], t["depth"], t["internel_k"], label=t["labels"],
                  init_flow=t["init_flow"], invalid_flow_num=0.0)
    return dec, res


def gen_e2e(ref, out, B=2, S=256, iters=4):
    inputs = synthetic.make_decoder_inputs(B, S, seed=11)
    dec, res = run_decoder(ref, inputs, iters)
    flow_pose, flow_pred, Rs, ts, masks, drs, dts = res
    for k, v in inputs.items():
        if k not in ("feat_render", "feat_real", "h_feat", "cxt_feat", "init_flow"):
            out[f"in_{k}"] = v
    # big inputs regenerated from the seed in the test; store checksums to pin generation
    for k in ("feat_render", "feat_real", "h_feat", "cxt_feat"):
        out[f"sum_{k}"] = np.array([inputs[k].astype(np.float64).sum(),
                                    np.abs(inputs[k]).astype(np.float64).sum()])
    out["flow_pose_last"] = flow_pose[-1].numpy()
    out["flow_pred_last"] = flow_pred[-1].numpy()
    out["mask_last"] = masks[-1].numpy()
    out["R"] = torch.stack(Rs).numpy()
    out["t"] = torch.stack(ts).numpy()
    out["drot"] = torch.stack(drs).numpy()
    out["dt"] = torch.stack(dts).numpy()
    out["flow_pose_absmean"] = np.array([f.abs().double().mean().item() for f in flow_pose])
    out["flow_pred_absmean"] = np.array([f.abs().double().mean().item() for f in flow_pred])
    out["meta"] = np.array([B, S, iters, 11])
    out["state_keys"] = np.array(list(dec.state_dict().keys()))
    out["state_shapes"] = np.array([",".join(map(str, v.shape)) for v in dec.state_dict().values()])


def build_encoder(ref, norm, seed):
    enc = ref.encoder.RAFTEncoder(**encoder_cfg(norm))
    synthetic.fill_module_(enc, seed=seed)
    return enc.eval()


def gen_enc(ref, out, B=1, S=128):
    """Both encoders at 128² (features 16²); images regenerated from the seed in the test."""
    imgs = synthetic.make_images(B, S, seed=5)
    x = t32(imgs["render_images"])
    out["sum_images"] = np.array([imgs["render_images"].astype(np.float64).sum()])
    with torch.no_grad():
        for norm, seed in (("IN", 1), ("BN", 2)):
            enc = build_encoder(ref, norm, seed)
            out[f"enc_{norm}"] = enc(x).numpy()
            out[f"keys_{norm}"] = np.array(list(enc.state_dict().keys()))
            out[f"shapes_{norm}"] = np.array([",".join(map(str, v.shape))
                                              for v in enc.state_dict().values()])
    out["meta"] = np.array([B, S, 5])


def gen_refine(ref, out, B=2, S=256, iters=4):
    """Images → encoders → decoder, the reference's SCFlowRefiner.get_pose data flow
    (scflow_refiner.py:108-138 with extract_feat :84-106; seperate_encoder=False shares one
    feature encoder, base_refiner.py:33-40).  Encoder seed 1, context seed 2, decoder seed 0."""
    imgs = synthetic.make_images(B, S, seed=13)
    scene = synthetic.make_scene(B, S, seed=13)
    enc, ctx = build_encoder(ref, "IN", 1), build_encoder(ref, "BN", 2)
    dec = ref.MODELS.build(dict(type=ref.scflow.SCFlowDecoder, **decoder_cfg(ref, iters)))
    synthetic.fill_module_(dec, seed=0)
    dec.eval()
    render, real = t32(imgs["render_images"]), t32(imgs["real_images"])
    with torch.no_grad():
        real_feat = enc(real)
        render_feat = enc(render)
        cxt = ctx(render)
        h_feat, cxt_feat = torch.split(cxt, [128, 128], dim=1)
        h_feat, cxt_feat = torch.tanh(h_feat), torch.relu(cxt_feat)
        init_flow = torch.zeros(B, 2, S, S)
        res = dec(render_feat, real_feat, h_feat, cxt_feat, t32(scene["ref_rotation"]),
                  t32(scene["ref_translation"]), t32(scene["depth"]), t32(scene["internel_k"]),
                  init_flow=init_flow, label=t32(scene["labels"]), invalid_flow_num=0.)
    flow_pose, flow_pred, Rs, ts, masks, drs, dts = res
    out["sum_images"] = np.array([imgs["render_images"].astype(np.float64).sum(),
                                  imgs["real_images"].astype(np.float64).sum()])
    for k, v in (("render_feat", render_feat), ("real_feat", real_feat), ("h_feat", h_feat),
                 ("cxt_feat", cxt_feat)):
        out[f"stat_{k}"] = np.array([v.double().sum().item(), v.double().abs().sum().item()])
    out["render_feat_s0c0"] = render_feat[0, :8].numpy()
    out["cxt_feat_s1"] = cxt_feat[1, :8].numpy()
    out["flow_pose_last"] = flow_pose[-1].numpy()
    out["flow_pred_last"] = flow_pred[-1].numpy()
    out["R"] = torch.stack(Rs).numpy()
    out["t"] = torch.stack(ts).numpy()
    out["flow_pred_absmean"] = np.array([f.abs().double().mean().item() for f in flow_pred])
    out["meta"] = np.array([B, S, iters, 13])


def _knn_points_standin(p1, p2, K=1, **kw):
    """pytorch3d.ops.knn_points restated for K=1 (absent here): for every point of p1[b] the
    index of its nearest point of p2[b] by squared Euclidean distance.  Only the symmetric-class
    fixture exercises it."""
    assert K == 1
    d = torch.cdist(p1, p2)
    dist, idx = d.min(dim=2)
    return types.SimpleNamespace(dists=(dist ** 2)[..., None], idx=idx[..., None], knn=None)


def load_losses(ref, mesh_points):
    """The reference's loss modules (models/loss/sequence_loss.py, point_matching_loss.py) and
    models/utils/flow.py.  Test-only stand-ins: ``trimesh.load`` returns the synthetic model
    points of the class whose file it is asked for (the reference's own ``_load_mesh`` globs and
    sorts the files); ``pytorch3d.ops.knn_points`` is the brute-force K=1 search above."""
    import tempfile
    mesh_dir = tempfile.mkdtemp(prefix="scflow_meshes_")
    for c in range(len(mesh_points)):
        open(os.path.join(mesh_dir, f"obj_{c + 1:06d}.obj"), "w").close()

    def _trimesh_load(path):
        c = int(os.path.basename(path)[4:10]) - 1
        return types.SimpleNamespace(vertices=np.asarray(mesh_points[c]))
    _stub("trimesh", load=_trimesh_load)
    _stub("pytorch3d")
    _stub("pytorch3d.ops", knn_points=_knn_points_standin)
    _pkg("models.loss", os.path.join(REF, "models/loss"))
    seq = _load("models.loss.sequence_loss", "models/loss/sequence_loss.py")
    pm = _load("models.loss.point_matching_loss", "models/loss/point_matching_loss.py")
    _load("models.utils.warp", "models/utils/warp.py")
    flow = _load("models.utils.flow", "models/utils/flow.py")
    return types.SimpleNamespace(seq=seq, pm=pm, flow=flow, mesh_dir=mesh_dir)


# configs/refine_models/scflow_ycbv_real.py:19-21 (mesh_diameter), :34-40 (symmetry_types)
YCBV_SYMMETRY = {"cls_13": {"z": 0}, "cls_16": {"x": 180, "y": 180, "z": 90}, "cls_19": {"y": 180},
                 "cls_20": {"x": 180}, "cls_21": {"x": 180, "y": 90, "z": 180}}


def gen_train(ref, out, labels, B=2, S=256, iters=2, seed=5):
    """One training-step slice (SURVEY §8(c) fixture 6): SCFlowRefiner.loss's data flow
    (scflow_refiner.py:182-242) on the reference's modules in train mode — shared IN feature
    encoder (seed 1), BN context encoder (seed 2, batch statistics), decoder (seed 0) — the GT
    flow from pose.get_flow_from_delta_pose_and_depth + flow.filter_flow_by_mask, and the three
    configured SequenceLosses (config :231-262).  Stores the losses, the per-iteration loss
    lists and the gradient norm of every parameter (the shared encoder's gradient sums both
    passes, as it does for the reference's shared module)."""
    pts = synthetic.make_model_points(256)
    L = load_losses(ref, pts)
    raw = synthetic.make_train_batch(B, S, seed=seed, labels=list(labels))
    t = {k: t32(v) for k, v in raw.items()}
    enc, ctx = build_encoder(ref, "IN", 1).train(), build_encoder(ref, "BN", 2).train()
    dec = ref.MODELS.build(dict(type=ref.scflow.SCFlowDecoder, **decoder_cfg(ref, iters)))
    synthetic.fill_module_(dec, seed=0)
    dec.train()
    real_feat = enc(t["real_images"])
    render_feat = enc(t["render_images"])
    cxt = ctx(t["render_images"])
    h_feat, cxt_feat = torch.split(cxt, [128, 128], dim=1)
    h_feat, cxt_feat = torch.tanh(h_feat), torch.relu(cxt_feat)
    depth = t["depth"]
    res = dec(render_feat, real_feat, h_feat, cxt_feat, t["ref_rotation"], t["ref_translation"],
              depth, t["internel_k"], init_flow=torch.zeros(B, 2, S, S), label=t["label"],
              invalid_flow_num=0.)
    flow_pose, flow_pred, Rs, ts, masks, _, _ = res
    max_flow = 400.
    gt_flow = ref.pose.get_flow_from_delta_pose_and_depth(
        t["ref_rotation"], t["ref_translation"], t["gt_rotation"], t["gt_translation"], depth,
        t["internel_k"], invalid_num=max_flow)
    gt_flow = L.flow.filter_flow_by_mask(gt_flow, t["gt_masks"], invalid_num=max_flow)
    rendered_masks = (depth > 0).to(torch.float32)  # base_refiner.py:191
    pose_loss = L.seq.SequenceLoss(gamma=0.8, loss_func_cfg=dict(
        type=L.pm.DisentanglePointMatchingLoss, symmetry_types=YCBV_SYMMETRY,
        mesh_diameter=list(synthetic.YCBV_DIAMETERS), mesh_path=L.mesh_dir, loss_type="l1",
        disentangle_z=True, loss_weight=10.0))
    flow_loss = L.seq.SequenceLoss(gamma=0.8, loss_func_cfg=dict(type=L.seq.RAFTLoss, loss_weight=.1,
                                                                 max_flow=400.))
    mask_loss = L.seq.SequenceLoss(gamma=0.8, loss_func_cfg=dict(type=L.seq.L1Loss, loss_weight=10.))
    lp, lp_seq = pose_loss(Rs, ts, gt_r=t["gt_rotation"], gt_t=t["gt_translation"], labels=t["label"],
                           scale_factors=None)
    lf, lf_seq = flow_loss(flow_pred, gt_flow=gt_flow, valid=rendered_masks)
    occ = (torch.sum(gt_flow, dim=1, keepdim=False) < max_flow).to(torch.float32)
    lm, lm_seq = mask_loss([m.squeeze(dim=1) for m in masks], gt_mask=occ, valid=rendered_masks)
    loss = lp + lf + lm
    loss.backward()
    out["losses"] = np.array([loss.item(), lp.item(), lf.item(), lm.item()])
    out["seq_losses"] = np.array([[x.item() for x in s] for s in (lp_seq, lf_seq, lm_seq)])
    out["gt_flow_stats"] = np.array([gt_flow.double().sum().item(), (gt_flow >= max_flow).sum().item(),
                                     gt_flow[gt_flow < max_flow].double().abs().sum().item()])
    out["R"] = torch.stack(Rs).detach().numpy()
    out["t"] = torch.stack(ts).detach().numpy()
    names, norms = [], []
    for prefix, mod in (("encoder.", enc), ("context.", ctx), ("decoder.", dec)):
        for n, p in mod.named_parameters():
            names.append(prefix + n)
            norms.append(np.nan if p.grad is None else p.grad.double().norm().item())
    out["grad_names"] = np.array(names)
    out["grad_norms"] = np.array(norms)
    out["meta"] = np.array([B, S, iters, seed, *labels])


# ------------------------------------------------------------------ §8(f)-4: the ADD metric
def load_metric(ref, mesh_verts):
    """The reference's ``metrics/add.py`` (class ``ADD``) with test-only stand-ins for its absent
    imports: ``mmengine.evaluator.BaseMetric`` (keeps ``results``), ``mmengine.load`` (json),
    ``mmengine.logging.print_log`` and ``terminaltables.AsciiTable`` (printing only),
    ``trimesh.load`` (the synthetic vertices of the class whose ``obj_XXXXXX.ply`` it is asked
    for), ``datasets.Compose``, and cv2 / matplotlib / mmcv for ``datasets/utils.py``'s imports.
    ``datasets/pose.py`` (project_3d_point) and ``datasets/utils.py`` (dumps_json) are the
    reference's own."""
    import json as _json

    class _BaseMetric:
        def __init__(self, collect_device="cpu", prefix=None):
            self.results = []

    def _mm_load(path):
        with open(path) as f:
            return _json.load(f)

    def _trimesh_load(path):
        c = int(os.path.basename(path)[4:10]) - 1
        return types.SimpleNamespace(vertices=np.asarray(mesh_verts[c]))
    mm = sys.modules.get("mmengine") or _stub("mmengine")
    mm.load = _mm_load
    _stub("mmengine.evaluator", BaseMetric=_BaseMetric)
    _stub("mmengine.logging", print_log=lambda *a, **k: None)
    _stub("terminaltables", AsciiTable=lambda data: types.SimpleNamespace(table=""))
    _stub("trimesh", load=_trimesh_load)
    _stub("cv2")
    _stub("matplotlib")
    _stub("matplotlib.pyplot")
    _stub("mmcv", is_str=lambda x: isinstance(x, str))
    ds = _pkg("datasets", os.path.join(REF, "datasets"))
    ds.Compose = None
    _load("datasets.utils", "datasets/utils.py")
    _load("datasets.pose", "datasets/pose.py")
    reg = sys.modules.get("registry") or _stub("registry")
    reg.METRICS = _Registry()
    _pkg("metrics", os.path.join(REF, "metrics"))
    return _load("metrics.add", "metrics/add.py")


def gen_metric(out, seed=11):
    """§8(f)-4 fixture from the reference's own ``ADD`` (metrics/add.py), constructed with its real
    ``__init__`` on a synthetic BOP tree (gt = ref annotations root): ``compute_metrics`` end to
    end (match_results → eval_pose_error → parse_error_to_metric → print_metric's 4-decimal
    rounding → parse_metric_to_tensorboard) under a fixed numpy seed, with the vertex subsamples
    its two ``np.random.choice`` rounds draw (match_results :190, compute_metrics :157) recorded
    as indices; ``match_results`` alone; ``eval_pose_error`` on a direct batch (symmetric classes
    included); ``parse_error_to_metric`` for several metric configurations; and the
    ``format_results`` scene_gt.json text."""
    import copy
    import json as _json
    import tempfile
    root = tempfile.mkdtemp(prefix="scflow_bop_")
    from tests.helpers import _rot_np, make_bop_case
    results, verts, lines = make_bop_case(root, seed)
    add_mod = load_metric(None, verts)
    names = tuple(f"obj_{c + 1:02d}" for c in range(verts.shape[0]))
    diam = list(synthetic.YCBV_DIAMETERS)
    data = os.path.join(root, "data")
    metric = add_mod.ADD(data_root=data, image_list=os.path.join(root, "test.txt"),
                         keypoints_json=os.path.join(root, "bbox.json"), class_names=names,
                         ref_annots_root=data, keypoints_num=8, mesh_symmetry=YCBV_SYMMETRY,
                         meshes_eval=os.path.join(root, "models_eval"), mesh_diameter=diam,
                         metrics={"auc": [], "add": [0.05, 0.10, 0.20, 0.50], "rep": [2, 5, 10]})
    n_cls = verts.shape[0]

    def draws(s, rounds):
        np.random.seed(s)
        return np.stack([np.stack([np.random.choice(verts.shape[1], 1000) for _ in range(n_cls)])
                         for _ in range(rounds)])
    # compute_metrics end to end
    out["cm_seed"] = np.array(1234)
    out["cm_draws"] = draws(1234, 2).astype(np.int16)  # [round (match, eval), class, 1000]
    np.random.seed(1234)
    flat = metric.compute_metrics(copy.deepcopy(results))
    out["cm_flat"] = np.array(_json.dumps(flat))
    # match_results alone
    out["mr_draws"] = draws(99, 1).astype(np.int16)
    np.random.seed(99)
    mr = metric.match_results(copy.deepcopy(results))
    for k, v in zip(("gt_R", "gt_t", "pred_R", "pred_t", "labels", "valid", "K"), mr):
        out["mr_" + k] = v
    # eval_pose_error on a direct batch (every class, symmetric ones included)
    rng = np.random.default_rng(seed + 1)
    n = 48
    labels = np.arange(n) % n_cls
    gR = np.stack([_rot_np(rng) for _ in range(n)])
    gT = np.stack([[rng.normal() * 50, rng.normal() * 50, 700 + 300 * rng.random()] for _ in range(n)]
                  ).astype(np.float32)
    pR = np.stack([gR[i] if i % 3 else _rot_np(rng) for i in range(n)])
    pT = (gT + rng.normal(size=gT.shape) * 10).astype(np.float32)
    K = np.repeat(np.array([[572.4, 0, 325.3], [0, 573.6, 242.0], [0, 0, 1]], np.float32)[None], n, 0)
    vsub = verts[:, :1000]
    e3n, e2, e3 = metric.eval_pose_error(list(vsub), gt_t=gT, gt_r=gR, pred_t=pT, pred_r=pR,
                                         labels=labels, k=K, symmetry_types=YCBV_SYMMETRY,
                                         mesh_diameters=np.array(diam))
    for k, v in (("gR", gR), ("gT", gT), ("pR", pR), ("pT", pT), ("labels", labels), ("K", K),
                 ("add", e3n), ("rep", e2), ("add_mm", e3)):
        out["ep_" + k] = v
    # parse_error_to_metric: thresholds on add / rep, a threshold-free metric, a skipped one,
    # classes absent from the labels
    lab = np.array([0, 0, 3, 3, 3, 12, 12, 15, 20, 20, 20, 20])
    err = dict(add=np.linspace(0.01, 0.6, lab.size), rep=np.linspace(0.5, 12.0, lab.size)[::-1].copy())
    pcs = []
    for m in ({"auc": [], "add": [0.05, 0.10, 0.20, 0.50]}, {"add": [0.1], "rep": [2, 5, 10]},
              {"rep": []}, {"add": [0.05, 0.5], "x": [1]}):
        md, headers = metric.parse_error_to_metric(err, lab, m, classnames=names)
        pcs.append(dict(metrics=m, metric_dict=md, headers=headers))
    out["pe_labels"] = lab
    out["pe_add"] = err["add"]
    out["pe_rep"] = err["rep"]
    out["pe_cases"] = np.array(_json.dumps(pcs))
    # format_results: the BOP scene_gt.json dump (reference formatting, datasets/utils.py dumps_json)
    save = os.path.join(root, "dump")
    metric.format_results(copy.deepcopy(results), save)
    texts = {}
    for seq in sorted(os.listdir(save)):
        with open(os.path.join(save, seq, "scene_gt.json")) as f:
            texts[seq] = f.read()
    out["fr_texts"] = np.array(_json.dumps(texts))
    # the inputs the tests rebuild the tree from
    out["in_seed"] = np.array(seed)
    out["in_verts_sum"] = np.array(float(verts.astype(np.float64).sum()))
    out["in_results"] = np.array(_json.dumps([
        dict(img_path=os.path.relpath(r["img_metas"]["img_path"], data),
             labels=r["pred"]["labels"].tolist(), rotations=r["pred"]["rotations"].tolist(),
             translations=r["pred"]["translations"].tolist()) for r in results]))
    with open(os.path.join(data, "000048", "scene_gt.json")) as f:
        out["in_scene_gt_48"] = np.array(f.read())


# ------------------------------------------------------------------ §8(f)-3: renderer wiring
RENDER_CASES = ((True, True), (True, False), (False, True), (False, False))  # (default, seperate)


def load_rendering(mesh_verts):
    """The reference's ``models/utils/rendering.py`` with RECORDING stand-ins for pytorch3d (absent):
    ``PerspectiveCameras`` / ``PointLights`` / ``RasterizationSettings`` / ``BlendParams`` keep their
    keyword arguments, ``MeshRendererWithFragments`` records the keywords of each call (znear,
    zfar, cameras, lights) and returns placeholders, ``join_meshes_as_batch`` / the PLY reader
    serve the synthetic vertices of the class named by the file (``obj_XXXXXX.ply``).
    ``cameras_from_opencv_projection`` and ``Renderer.__init__`` / ``to`` / ``forward`` run as the
    reference wrote them; nothing is rasterised (the rasteriser stays parity-unpinned)."""
    rec = {"calls": []}

    class _Kw:
        def __init__(self, *args, **kw):
            self.args, self.kw = args, kw

    class _Cameras(_Kw):
        pass

    class _Lights(_Kw):
        pass

    class _MeshRendererWithFragments(_Kw):
        def __call__(self, meshes, **kw):
            rec["calls"].append(kw)
            return None, None

    class _Mesh:
        def __init__(self, verts):
            self.verts = verts

        def to(self, device):
            return _Mesh(self.verts.to(device))

    class _PlyFormat:
        def read(self, path, include_textures=True, device="cpu", path_manager=None):
            c = int(os.path.basename(path).split(".")[0].split("_")[-1]) - 1
            return _Mesh(torch.as_tensor(mesh_verts[c], dtype=torch.float32))

    class _Batch:
        def __init__(self, meshes):
            self.meshes = meshes

        def verts_list(self):
            return [m.verts for m in self.meshes]

    names = ("PointLights", "PerspectiveCameras", "BlendParams", "MeshRasterizer",
             "RasterizationSettings", "HardPhongShader", "SoftPhongShader", "HardGouraudShader",
             "SoftGouraudShader", "SoftSilhouetteShader", "HardFlatShader")
    p3r = {n: type(n, (_Kw,), {}) for n in names}
    p3r["PerspectiveCameras"], p3r["PointLights"] = _Cameras, _Lights
    _stub("iopath")
    _stub("iopath.common")
    _stub("iopath.common.file_io", PathManager=lambda: None)
    _stub("pytorch3d")
    _stub("pytorch3d.structures", join_meshes_as_batch=lambda ms, include_textures=True: _Batch(ms))
    _stub("pytorch3d.renderer", **p3r)
    _stub("pytorch3d.renderer.mesh")
    _stub("pytorch3d.renderer.mesh.renderer", MeshRendererWithFragments=_MeshRendererWithFragments)
    _stub("pytorch3d.io")
    _stub("pytorch3d.io.ply_io", MeshPlyFormat=_PlyFormat)
    _stub("pytorch3d.io.obj_io", MeshObjFormat=_PlyFormat)
    _stub("torchvision")
    _stub("torchvision.utils", save_image=None)
    return _load("models.utils.rendering", "models/utils/rendering.py"), rec


def render_case_inputs(B=4, S=256, seed=31):
    """Poses / intrinsics / labels of the renderer-wiring fixture (synthetic.make_scene, with one
    pose pushed close so that max(z_min − 400, 0) clamps to 0 for it)."""
    sc = synthetic.make_scene(B, S, seed=seed)
    sc["ref_translation"][1, 2] = 380.0
    return sc


def gen_render(out, B=4, S=256):
    """§8(f)-3 fixture: the reference's ``Renderer.forward`` (rendering.py:185-248) for the four
    (default_lights, seperate_lights) settings — the PerspectiveCameras it builds through
    ``cameras_from_opencv_projection`` (:17-60: R, T, focal_length, principal_point, image_size),
    the znear / zfar it rounds to 100 mm (:193-199) and passes to the renderer call, and the
    PointLights keywords (location :210-229, colours)."""
    import tempfile
    verts = [synthetic.ellipsoid_mesh(np.array(synthetic.ELLIPSOID_AXES) * d, 12, 24)[0]
             for d in synthetic.YCBV_DIAMETERS]
    mod, rec = load_rendering(verts)
    sc = render_case_inputs(B, S)
    mesh_dir = tempfile.mkdtemp(prefix="scflow_meshes_")
    for c in range(len(verts)):
        open(os.path.join(mesh_dir, f"obj_{c + 1:06d}.ply"), "w").close()
    R, t, K = (torch.from_numpy(sc[k]) for k in ("ref_rotation", "ref_translation", "internel_k"))
    labels = torch.from_numpy(sc["labels"])
    out["in_R"], out["in_t"], out["in_K"], out["in_labels"] = sc["ref_rotation"], \
        sc["ref_translation"], sc["internel_k"], sc["labels"]
    out["in_S"] = np.array(S)
    for deflt, seps in RENDER_CASES:
        tag = f"d{int(deflt)}s{int(seps)}"
        rend = mod.Renderer(mesh_dir, (S, S), shader_type="Phong", soft_blending=False,
                            render_mask=False, default_lights=deflt, seperate_lights=seps)
        rend.to("cpu")
        rec["calls"].clear()
        rend(R, t, K, labels)
        (call,) = rec["calls"]
        cam, lights = call["cameras"], call["lights"]
        for k in ("R", "T", "focal_length", "principal_point", "image_size"):
            out[f"{tag}_cam_{k}"] = cam.kw[k].detach().numpy()
        out[f"{tag}_znear_zfar"] = np.array([call["znear"], call["zfar"]])
        loc = lights.kw.get("location")
        out[f"{tag}_light_location"] = np.zeros((0, 3), np.float32) if loc is None else \
            loc.detach().numpy()
        for k in ("ambient_color", "diffuse_color", "specular_color"):
            v = lights.kw.get(k)
            out[f"{tag}_light_{k}"] = np.zeros(0, np.float32) if v is None else np.array(v, np.float32)
    out["mesh_verts_sum"] = np.array([float(np.asarray(v, np.float64).sum()) for v in verts])


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    if len(sys.argv) > 1 and sys.argv[1] == "render":  # only the renderer-wiring fixture
        rw = {}
        gen_render(rw)
        np.savez_compressed(os.path.join(HERE, "golden_render_wiring.npz"), **rw)
        print({k: getattr(v, "shape", None) for k, v in rw.items()})
        return
    ref = load_reference()
    if len(sys.argv) > 1 and sys.argv[1] == "ops":  # only golden_ops.npz
        ops = {}
        gen_ops(ref, ops)
        np.savez_compressed(os.path.join(HERE, "golden_ops.npz"), **ops)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "metric":  # only the ADD-metric fixture
        mt = {}
        gen_metric(mt)
        np.savez_compressed(os.path.join(HERE, "golden_metric_add.npz"), **mt)
        print({k: getattr(v, "shape", None) for k, v in mt.items()})
        return
    if len(sys.argv) > 1 and sys.argv[1] == "train":  # only the training fixtures
        for tag, labels in (("", (4, 9)), ("_sym", (15, 20))):
            tr = {}
            gen_train(ref, tr, labels)
            np.savez_compressed(os.path.join(HERE, f"golden_train_b2_s256_it2{tag}.npz"), **tr)
            print(tag, tr["losses"], tr["seq_losses"])
        return
    ops = {}
    gen_ops(ref, ops)
    np.savez_compressed(os.path.join(HERE, "golden_ops.npz"), **ops)
    e2e = {}
    gen_e2e(ref, e2e)
    np.savez_compressed(os.path.join(HERE, "golden_e2e_b2_s256_it4.npz"), **e2e)
    enc = {}
    gen_enc(ref, enc)
    np.savez_compressed(os.path.join(HERE, "golden_enc_b1_s128.npz"), **enc)
    rf = {}
    gen_refine(ref, rf)
    np.savez_compressed(os.path.join(HERE, "golden_refine_b2_s256_it4.npz"), **rf)
    for name, d in (("ops", ops), ("e2e", e2e), ("enc", enc), ("refine", rf)):
        print(name, {k: getattr(v, "shape", None) for k, v in d.items()})


if __name__ == "__main__":
    main()
