"""Time conv kernels vs K to split fixed (prologue/epilogue) and per-stage cost."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from scflow_amd.modules import ConvRunner
from scflow_amd.ops import Chan

n, h, w = 16, 32, 32
M = n * h * w
KS = [((1, 5), (0, 2)), ((5, 1), (2, 0)), ((3, 3), (1, 1))]
if len(sys.argv) > 1:
    KS = [kp for kp in KS if f"{kp[0][0]}x{kp[0][1]}" in sys.argv[1].split(",")]
for k, pad in KS:
    for cout in (128, 256, 512):
        for cin in (128, 256, 512, 1024):
            conv = torch.nn.Conv2d(cin, cout, k, padding=pad).cuda()
            x = torch.randn(M, cin, device="cuda")
            out = torch.empty(M, cout, device="cuda")
            r = ConvRunner([conv], None)
            run = lambda: r.run(Chan.whole(x), Chan.whole(out), n, h, w)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            s.record()
            for _ in range(reps):
                run()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 1e3 / reps
            taps = k[0] * k[1]
            pts = 16 if taps == 9 else 8
            tiles = M / (4 if taps == 9 else 4)
            mf = 2 * pts * tiles * cin * cout
            print(f"k={k} cin={cin:5d} cout={cout:4d} {us:8.2f} us  mfma-TF {mf/us/1e6:7.2f}  alg-TF {2*M*cin*cout*taps/us/1e6:7.2f}", flush=True)
