import torch, sys
sys.path.insert(0, '.')
from scflow_amd import ops
a = torch.randn(16384, 324, device='cuda'); b = torch.randn(324, 256, device='cuda'); bias = torch.randn(256, device='cuda')
out = torch.empty(16384, 256, device='cuda')
for _ in range(5): ops.gemm(a, b, out=out, bias=bias)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda._sleep(2_000_000); e0.record()
for _ in range(20): ops.gemm(a, b, out=out, bias=bias)
e1.record(); torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / 20
print(f"gemm 16384x324x256: {us:.1f} us, {2*16384*324*256/us/1e6:.1f} TF")
bt = b.t().contiguous().t()
for _ in range(3): ops.gemm(a, bt, out=out, bias=bias)
torch.cuda.synchronize(); torch.cuda._sleep(2_000_000); e0.record()
for _ in range(20): ops.gemm(a, bt, out=out, bias=bias)
e1.record(); torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / 20
print(f"gemm (B col-major): {us:.1f} us")
