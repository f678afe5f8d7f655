"""Where do the end-to-end forward's device copies come from?  torch.profiler over
SCFlowRefiner.get_pose (bench.py's configs[2] leg), listing the ops that issue Memcpy/Memset
activity with their Python stacks.  usage: python tools/dbg/e2e_copies.py [batch]"""
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    dev = torch.device("cuda", 0)
    ref = bench.build_refiner(8, dev)
    rin = bench.make_refine_inputs(batch, 256, seed=1000, device=dev)
    for _ in range(2):
        ref.get_pose(**rin)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        ref.get_pose(**rin)
        torch.cuda.synchronize()
    runtime = Counter()
    stacks = Counter()
    for e in prof.events():
        name = e.name
        if "Memcpy" in name or "memcpy" in name or "copyBuffer" in name or "Memset" in name:
            runtime[name] += 1
            st = [s for s in (e.stack or []) if "scflow_amd" in s or "bench" in s][:3]
            stacks[(name, " <- ".join(st))] += 1
    print("copy-like events:", dict(runtime))
    for (name, st), c in stacks.most_common(25):
        print(f"{c:4d}  {name}  {st}")
    print(prof.key_averages().table(sort_by="count", row_limit=25))


if __name__ == "__main__":
    main()
