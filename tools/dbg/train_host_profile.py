"""Host-side cost of one eager training step at configs[3]: cProfile over 2 steps after warm-up
(GPU work overlaps; the step is host-bound where the Python + launch path is slower than the
kernels it issues).

    python tools/dbg/train_host_profile.py [--top 45]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--main-thread-backward", action="store_true",
                    help="run autograd's backward on the calling thread, so cProfile sees it")
    a = ap.parse_args()
    if a.main_thread_backward:
        torch.autograd.set_multithreading_enabled(False)
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
    t0 = time.perf_counter()
    step(batch)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"one step: host enqueue {1e3 * (t1 - t0):.1f} ms, until GPU done {1e3 * (t2 - t0):.1f} ms")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(2):
        step(batch)
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(a.top)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(a.top)
    print(s.getvalue())


if __name__ == "__main__":
    main()
