"""Time the pose-head (a7) kernels in isolation at B pairs (default 16), 32×32 input features.

usage: python tools/ph_bench.py [--batch 16] [--reps 50]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scflow_amd import ops, synthetic  # noqa: E402
from scflow_amd.ops import Chan  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    n, h, w = a.batch, a.size, a.size
    dev = "cuda"
    from scflow_amd import MODELS
    cfg = dict(type="MultiClassPoseHead", num_class=21, in_channels=224, net_type="Basic",
               rotation_mode="ortho6d", norm_cfg=dict(type="GN", num_groups=32), act_cfg=dict(type="ReLU"))
    if h != 32:
        cfg["feat_size"] = (h, w)
    head = MODELS.build(cfg)
    synthetic.fill_module_(head, seed=3)
    head = head.to(dev).eval()
    x = torch.randn(n * h * w, 224, device=dev)
    label = torch.randint(0, 21, (n,), device=dev)
    res = {}
    res["whole head (forward_hip)"] = timed(lambda: head.forward_hip(Chan.whole(x), None, n, h, w, label), a.reps)
    c1 = head.conv_layers[0].conv
    pk = ops.ph_conv_pack(c1.weight)
    oh, ow = h // 2, w // 2
    y1 = torch.empty(n * oh * ow, 128, device=dev)
    res["conv1 ph_conv"] = timed(lambda: ops.ph_conv(Chan.whole(x), None, pk, None, n, h, w, 128, 3, 2, 1, y1), a.reps)
    epk = ops.enc_conv_pack(c1.weight)
    y1e = torch.empty(n, oh, ow, 128, device=dev)
    res["conv1 enc_conv (MFMA halo)"] = timed(lambda: ops.enc_conv(x, epk, None, n, h, w, 224, 128, 3, 2, 1, y1e), a.reps)
    sc = torch.empty(n, 128, device=dev)
    sh = torch.empty(n, 128, device=dev)
    gn = head.conv_layers[0].gn
    res["gn stats conv1"] = timed(lambda: ops.ph_gn_stats(y1, n, oh * ow, 128, 32, gn.weight, gn.bias, gn.eps, sc, sh), a.reps)
    c2 = head.conv_layers[1].conv
    pk2 = ops.ph_conv_pack(c2.weight)
    y2 = torch.empty(n * (oh // 2) * (ow // 2), 128, device=dev)
    res["conv2 ph_conv"] = timed(lambda: ops.ph_conv(Chan.whole(y1), None, pk2, None, n, oh, ow, 128, 3, 2, 1, y2, sc, sh), a.reps)
    res["gn stats conv2"] = timed(lambda: ops.ph_gn_stats(y2, n, (oh // 2) * (ow // 2), 128, 32, gn.weight, gn.bias, gn.eps, sc, sh), a.reps)
    y3 = torch.empty(n * (oh // 4) * (ow // 4), 128, device=dev)
    res["conv3 ph_conv"] = timed(lambda: ops.ph_conv(Chan.whole(y2), None, pk2, None, n, oh // 2, ow // 2, 128, 3, 2, 1, y3, sc, sh), a.reps)
    k1 = 128 * (oh // 4) * (ow // 4)
    fc1 = head.fc_layers[0][0]
    wp = ops.ph_fc_permute(fc1.weight, 128, (oh // 4) * (ow // 4))
    f1 = torch.empty(n, 1024, device=dev)
    res["fc1 (GN on load)"] = timed(lambda: ops.ph_fc(y3, k1, n, k1, wp, fc1.bias, f1, 1024, True, gn_c=128, scale=sc, shift=sh), a.reps)
    fc2 = head.fc_layers[1][0]
    f2 = torch.empty(n, 256, device=dev)
    res["fc2"] = timed(lambda: ops.ph_fc(f1, 1024, n, 1024, fc2.weight, fc2.bias, f2, 256, True), a.reps)
    dr = torch.empty(n, 6, device=dev)
    dt = torch.empty(n, 3, device=dev)
    res["heads"] = timed(lambda: ops.ph_heads(f2, n, 256, head.rotation_pred.weight, head.rotation_pred.bias, 6,
                                              head.translation_pred.weight, head.translation_pred.bias, label, 21, dr, dt), a.reps)
    for k, v in res.items():
        print(f"{k:32s} {v:8.2f} us", flush=True)


if __name__ == "__main__":
    main()
