"""torch.profiler attribution of one training step (which aten ops own the device time).

usage: python tools/train_torchprof.py [--batch 16] [--rows 45]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


GLUE = ("aten::add_", "aten::add", "aten::copy_", "aten::threshold_backward", "aten::sum",
        "aten::clamp_min", "aten::fill_", "aten::zero_", "aten::cat", "aten::flip", "aten::mul",
        "aten::div", "aten::index", "aten::sub", "aten::mul_", "aten::scatter_add_")


def _glue_sites(prof, depth, rows):
    """Device time of the elementwise glue ops by (op, input shapes, innermost repo frames):
    ops without a Python stack ran inside the autograd engine (gradient accumulation)."""
    agg = {}
    for e in prof.events():
        if e.name not in GLUE:
            continue
        frames = [f for f in (e.stack or []) if "scflow_amd" in f or "tools/" in f or "bench" in f]
        key = (e.name, str(e.input_shapes)[:90], " <- ".join(frames[:depth]) or "(autograd engine)")
        t, n = agg.get(key, (0.0, 0))
        agg[key] = (t + e.self_device_time_total, n + 1)
    tot = sum(t for t, _ in agg.values())
    print(f"glue device time {tot / 1e3:.3f} ms over {sum(n for _, n in agg.values())} ops")
    for (name, shp, where), (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:rows]:
        print(f"{t / 1e3:8.3f} ms {n:5d}  {name:26s} {shp}\n        {where}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--rows", type=int, default=45)
    ap.add_argument("--shapes", action="store_true", help="group by input shapes (record_shapes)")
    ap.add_argument("--stack", type=int, default=0, help="group by the top N Python frames")
    a = ap.parse_args()
    import bench
    from scflow_amd import synthetic
    from scflow_amd.train.step import TrainStep
    dev = torch.device("cuda", 0)
    ref = bench.build_refiner(8, dev).train()
    raw = synthetic.make_train_batch(a.batch, 256, seed=2000)
    batch = {k: torch.from_numpy(v).to(dev) for k, v in raw.items()}
    pts = [torch.from_numpy(p).to(dev) for p in synthetic.make_model_points(1024)]
    step = TrainStep(ref, pts, synthetic.YCBV_DIAMETERS)
    for _ in range(2):
        step(batch)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=a.shapes or a.stack > 0, with_stack=a.stack > 0) as prof:
        step(batch)
        torch.cuda.synchronize()
    if a.stack:
        _glue_sites(prof, a.stack, a.rows)
        return
    print(prof.key_averages(group_by_input_shape=a.shapes, group_by_stack_n=a.stack).table(
        sort_by="self_cuda_time_total", row_limit=a.rows, max_name_column_width=60,
        max_shapes_column_width=90))


if __name__ == "__main__":
    main()
