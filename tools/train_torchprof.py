"""torch.profiler attribution of one training step (which aten ops own the device time).

usage: python tools/train_torchprof.py [--batch 16] [--rows 45]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--rows", type=int, default=45)
    ap.add_argument("--shapes", action="store_true", help="group by input shapes (record_shapes)")
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
                 record_shapes=a.shapes) as prof:
        step(batch)
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=a.shapes).table(
        sort_by="self_cuda_time_total", row_limit=a.rows, max_name_column_width=60,
        max_shapes_column_width=90))


if __name__ == "__main__":
    main()
