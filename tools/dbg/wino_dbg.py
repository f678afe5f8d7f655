"""Debug: Winograd vs direct conv on one shape; prints error pattern."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch, torch.nn.functional as F
from scflow_amd import ops
from scflow_amd._lib import CONV_WINO
from scflow_amd.train.functions import _conv_forward

torch.manual_seed(0)
for (n, h, w, c0, cout, k, pad, relu_mask) in [(2, 32, 32, 256, 128, (1, 5), (0, 2), False),
                                               (2, 32, 32, 256, 128, (1, 5), (0, 2), True),
                                               (2, 32, 32, 256, 128, (5, 1), (2, 0), True)]:
    x = torch.randn(n, h, w, c0)
    if relu_mask:
        x = x * (torch.rand_like(x) > 0.5)
    wt = torch.randn(cout, c0, *k) / np.sqrt(c0 * 5)
    ref = F.conv2d(x.permute(0, 3, 1, 2).double(), wt.double(), padding=pad).permute(0, 2, 3, 1)
    for bk in (16, CONV_WINO):
        os.environ["SCFLOW_CONV_WINO"] = "1"
        packed = ops.pack_conv_weight(wt.cuda(), c0, 0, w, 1, bk)
        out = torch.empty(n, h, w, cout, device="cuda")
        ops.conv2d(ops.Chan.whole(x.cuda().view(-1, c0)), packed, None, n, h, w, cout, k[0], k[1], pad[0], pad[1],
                   None, out=ops.Chan.whole(out.view(-1, cout)), bk=bk)
        err = (out.cpu().double() - ref).abs()
        print(k, "mask" if relu_mask else "", "bk", bk, "max err", err.max().item(), "mean", err.mean().item(),
              "worst idx", np.unravel_index(err.argmax().item(), err.shape), "scale", ref.abs().max().item())
    y = _conv_forward(x.cuda(), None, wt.cuda(), None, 1, pad)
    err = (y.cpu().double() - ref).abs()
    print("  _conv_forward max err", err.max().item())
