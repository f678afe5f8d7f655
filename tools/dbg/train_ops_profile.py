"""Which torch ops (and from which source lines) one eager training step issues at configs[3]:
torch.profiler over one step after warm-up, CPU-side op counts grouped by the innermost
scflow_amd / torch.autograd frames.

    python tools/dbg/train_ops_profile.py [--top 40]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    import bench
    from scflow_amd import synthetic
    from scflow_amd.train.step import TrainStep
    dev = torch.device("cuda", 0)
    ref = bench.build_refiner(8, dev).train()
    raw = synthetic.make_train_batch(16, 256, seed=2000)
    batch = {k: torch.from_numpy(v).to(dev) for k, v in raw.items()}
    pts = [torch.from_numpy(p).to(dev) for p in synthetic.make_model_points(1024)]
    step = TrainStep(ref, pts, synthetic.YCBV_DIAMETERS)
    for _ in range(3):
        step(batch)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        step(batch)
        torch.cuda.synchronize()
    # leaf aten ops that launch kernels, attributed to the nearest repo frame
    cnt = collections.Counter()
    tot = collections.Counter()
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.cpu_children:
            continue
        frame = "?"
        for fr in (ev.stack or []):
            if "scflow_amd" in fr or "torch/autograd" in fr:
                frame = fr.split("/")[-1]
                break
        cnt[(ev.name, frame)] += 1
        tot[ev.name] += 1
    print("leaf aten ops per step:", sum(tot.values()))
    for k, v in tot.most_common(25):
        print(f"  {v:6d}  {k}")
    chains = collections.Counter()
    for ev in prof.events():
        if ev.name != "aten::_local_scalar_dense":
            continue
        c, e = [], ev
        while e is not None and len(c) < 8:
            c.append(e.name + ("@" + e.stack[0].split("/")[-1] if e.stack else ""))
            e = e.cpu_parent
        chains[" <- ".join(c)] += 1
    print("host syncs (_local_scalar_dense) by caller chain:")
    for k, v in chains.most_common(15):
        print(f"  {v:5d}  {k[:300]}")
    print("by op and source frame:")
    for (nm, fr), v in cnt.most_common(a.top):
        print(f"  {v:6d}  {nm:32s} {fr}")


if __name__ == "__main__":
    main()
