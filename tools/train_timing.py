"""Where the training step's time goes: host enqueue vs GPU execution.

For each of K steps after W warm-ups it reports
* ``host_ms``   — time for ``TrainStep.__call__`` to return (no sync), GPU running freely;
* ``gpu_ms``    — device time between events recorded on the step's stream before / after it;
* ``wall_ms``   — pipelined wall time per step (K steps back to back, one sync at the end);
and, in a second pass, ``gpu_pure_ms``: the same step enqueued behind a long ``torch.cuda._sleep``
so the host has finished enqueueing before the GPU starts it — the step's pure GPU time, with no
host starvation.  host_ms ≥ gpu_pure_ms means the step is host-bound.

    python tools/train_timing.py [--steps 12] [--warmup 3] [--graph]
"""
import argparse
import collections
import gc
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _stats(xs):
    return {"median": round(statistics.median(xs), 3), "min": round(min(xs), 3),
            "max": round(max(xs), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--sleep-ms", type=float, default=120.0)
    ap.add_argument("--freeze", action="store_true", help="gc.collect() + gc.freeze() after warm-up")
    a = ap.parse_args()
    import bench
    from scflow_amd import synthetic
    from scflow_amd.train.step import TrainStep
    dev = torch.device("cuda", 0)
    ref = bench.build_refiner(8, dev).train()
    raw = synthetic.make_train_batch(a.batch, 256, seed=2000)
    batch = {k: torch.from_numpy(v).to(dev) for k, v in raw.items()}
    pts = [torch.from_numpy(p).to(dev) for p in synthetic.make_model_points(1024)]
    step = TrainStep(ref, pts, synthetic.YCBV_DIAMETERS, graph=a.graph)
    for _ in range(a.warmup):
        step(batch)
    torch.cuda.synchronize()
    if a.freeze:
        gc.collect()
        gc.freeze()
    gc_log = []

    def on_gc(phase, info):
        if phase == "start":
            gc_log.append([info["generation"], time.perf_counter(), None])
        elif gc_log and gc_log[-1][2] is None:
            gc_log[-1][2] = time.perf_counter()
    gc.callbacks.append(on_gc)

    # pass 1: pipelined, per-step host return time and device time
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(a.steps)]
    host = []
    t0 = time.perf_counter()
    for i in range(a.steps):
        ev[i][0].record(step.stream)
        h0 = time.perf_counter()
        step(batch)
        host.append((time.perf_counter() - h0) * 1e3)
        ev[i][1].record(step.stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / a.steps
    gpu = [s.elapsed_time(e) for s, e in ev]

    # pass 2: each step enqueued behind a sleep kernel → pure GPU time, and the enqueue time
    # of a host that never waits for the GPU
    cyc = int(a.sleep_ms * 1e-3 * 2.1e9)
    pure, host_free = [], []
    for i in range(min(a.steps, 6)):
        torch.cuda.synchronize()
        with torch.cuda.stream(step.stream):
            torch.cuda._sleep(cyc)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(step.stream)
        h0 = time.perf_counter()
        step(batch)
        host_free.append((time.perf_counter() - h0) * 1e3)
        e.record(step.stream)
        torch.cuda.synchronize()
        pure.append(s.elapsed_time(e))
    out = {"steps": a.steps, "graph": a.graph, "wall_ms_per_step": round(wall, 3),
           "host_ms": _stats(host), "gpu_ms": _stats(gpu), "host_ms_gpu_held": _stats(host_free),
           "gpu_pure_ms": _stats(pure), "sleep_ms": a.sleep_ms,
           "per_step_host": [round(x, 2) for x in host], "per_step_gpu": [round(x, 2) for x in gpu],
           "gc_freeze": a.freeze, "gc_collections": collections.Counter(g for g, _, _ in gc_log),
           "gc_ms_by_generation": {g: round(sum(1e3 * (e - s) for gg, s, e in gc_log if gg == g and e), 2)
                                   for g in (0, 1, 2)},
           "gc_max_ms": round(max((1e3 * (e - s) for _, s, e in gc_log if e), default=0.0), 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
