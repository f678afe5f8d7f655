"""Host-side submission time of one decoder forward vs its GPU time (is the forward launch-bound?)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import bench
from scflow_amd import synthetic
from scflow_amd.registry import MODELS

dev = torch.device("cuda:0")
dec = MODELS.build(bench.decoder_cfg(8))
synthetic.fill_module_(dec)
dec = dec.to(dev).eval()
inp = bench.make_inputs(16, 256, 0, dev)
for _ in range(3):
    dec(**inp, invalid_flow_num=0.0)
torch.cuda.synchronize()
hs, gs = [], []
for _ in range(10):
    t0 = time.perf_counter()
    dec(**inp, invalid_flow_num=0.0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    hs.append(t1 - t0); gs.append(t2 - t0)
print(f"host submit {1e3*sorted(hs)[5]:.3f} ms, submit+drain {1e3*sorted(gs)[5]:.3f} ms per forward")
import cProfile, pstats
pr = cProfile.Profile(); pr.enable()
for _ in range(5):
    dec(**inp, invalid_flow_num=0.0)
pr.disable(); torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
