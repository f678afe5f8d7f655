"""Probe: one eager training step (kernel names via rocprofv3) or the hipGraph capture of it."""
import sys
import torch
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_train_host import build_train_refiner, train_batch
from scflow_amd.train.step import TrainStep

mode = sys.argv[1] if len(sys.argv) > 1 else "eager"
batch, points, diam = train_batch(2, 256, seed=7)
gb = {k: v.cuda() for k, v in batch.items()}
r = build_train_refiner(2).cuda()
step = TrainStep(r, [p.cuda() for p in points], diam, lr=0.0, graph=(mode == "graph"))
for i in range(3 if mode == "graph" else 2):
    out = step(gb)
    torch.cuda.synchronize()
    print(i, float(out["loss"]), flush=True)
