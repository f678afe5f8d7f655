"""GPU parity at BASELINE.json's own config sizes (the shapes bench.py times), against the CPU
oracle (pinned to the reference by tests/golden): mean flow EPE ≤ 1e-3 px per sample (north_star),
rotations ≤ 1e-5, translations ≤ 1e-3 mm.

* configs[1]: SCFlowDecoder, B=16 pairs, 256², 8 iterations — every sample.  At B=16 the SepConvGRU
  launches take the 64-channel Winograd workgroups (conv_wino5_kernel<·,32,2,GRU_ZR/GRU_Q>), the
  instantiation the bench's roofline line times.
* configs[4]: B=32, 512², 12 iterations, pose head feat_size=(64,64) — the HIP decoder runs the
  whole batch (2.85 GB pyramid); the oracle runs samples {0, 13, 31} with the batch's label[0] as
  the pose head's label (every op is per sample except that quirk, pose_head.py:208-209, so the
  subset is exact).
* configs[2]: SCFlowRefiner.get_pose (images → encoders → decoder), B=32, 256², 8 iterations —
  same sample subset.  The encoders' BatchNorm is in eval mode (per sample).

Reference: models/decoder/scflow_decoder.py:151-252, models/refiner/scflow_refiner.py:108-138.
"""
import numpy as np
import pytest
import torch

from tests.helpers import decoder_inputs, refine_inputs, refiner_state_dict
from tests.test_gpu_decoder import EPE_TOL, build_decoder

orc = pytest.importorskip("oracle.scflow_oracle")

SUBSET = [0, 13, 31]


def _subset(inp, idx):
    out = {k: v[idx] for k, v in inp.items()}
    out["head_label"] = inp["label"][:1]
    return out


def _check(out, ref, idx, iters):
    """out: GPU 7 lists over the full batch; ref: oracle 7 lists over the samples ``idx``."""
    for it in range(iters):
        for k in (0, 1):
            epe = orc.cal_epe_mean(ref[k][it], out[k][it][idx].cpu())
            assert float(epe.max()) <= EPE_TOL, f"iter {it} output {k}: EPE {epe.tolist()}"
    np.testing.assert_allclose(torch.stack([x[idx].cpu() for x in out[2]]).numpy(),
                               torch.stack(ref[2]).numpy(), atol=1e-5)
    np.testing.assert_allclose(torch.stack([x[idx].cpu() for x in out[3]]).numpy(),
                               torch.stack(ref[3]).numpy(), rtol=1e-6, atol=1e-3)


@pytest.mark.gpu
def test_config1_decoder_b16_256_8iters():
    inp = decoder_inputs(16, 256, seed=31)
    inp["label"] = torch.from_numpy(np.arange(16) % 21)  # multi-class batch
    dec = build_decoder(8, seed=3)
    out = dec.cuda()(**{k: v.cuda() for k, v in inp.items()}, invalid_flow_num=0.0)
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
    ref = orc.decoder_forward(sd, **inp, iters=8)
    _check(out, ref, list(range(16)), 8)


@pytest.mark.gpu
def test_config4_decoder_b32_512_12iters():
    inp = decoder_inputs(32, 512, seed=41)
    dec = build_decoder(12, feat_size=(64, 64), seed=5)
    out = dec.cuda()(**{k: v.cuda() for k, v in inp.items()}, invalid_flow_num=0.0)
    torch.cuda.synchronize()
    out = [[x.cpu() for x in lst] for lst in out]
    sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
    ref = orc.decoder_forward(sd, **_subset(inp, SUBSET), iters=12)
    _check(out, ref, SUBSET, 12)


@pytest.mark.gpu
def test_config2_get_pose_b32_256_8iters():
    from tests.test_gpu_encoder import build_refiner
    inp = refine_inputs(32, 256, seed=51)
    r = build_refiner()
    r.decoder.iters = 8
    gi = {k: v.cuda() for k, v in inp.items()}
    out = r.get_pose(gi["render_images"], gi["real_images"], gi["ref_rotation"], gi["ref_translation"],
                     gi["depth"], gi["internel_k"], gi["label"])
    torch.cuda.synchronize()
    out = [[x.cpu() for x in lst] for lst in out]
    sub = _subset(inp, SUBSET)
    sd = refiner_state_dict()
    rf, lf, h, cxt = orc.extract_feat(sd, sub["render_images"], sub["real_images"])
    N, _, H, W = sub["real_images"].shape
    ref = orc.decoder_forward(sd, rf, lf, h, cxt, sub["ref_rotation"], sub["ref_translation"],
                              sub["depth"], sub["internel_k"], sub["label"], torch.zeros(N, 2, H, W),
                              0.0, iters=8, head_label=sub["head_label"])
    _check(out, ref, SUBSET, 8)


@pytest.mark.gpu
def test_sharded_decoder_equals_unsharded_multiclass():
    """dist.shard_batch + head_label: two shards of a mixed-label batch decoded separately give
    the unsharded decoder's outputs (per-sample independence + the global label[0])."""
    from scflow_amd.dist import shard_batch
    inp = {k: v.cuda() for k, v in decoder_inputs(6, 256, seed=61).items()}
    inp["label"] = torch.tensor([4, 9, 17, 2, 4, 20], device="cuda")
    dec = build_decoder(3, seed=6).cuda()
    full = dec(**inp, invalid_flow_num=0.0)
    parts = [dec(**shard_batch(inp, r, 2), invalid_flow_num=0.0) for r in range(2)]
    torch.cuda.synchronize()
    for k in (0, 1):
        got = torch.cat([p[k][-1] for p in parts]).cpu()
        assert float(orc.cal_epe_mean(full[k][-1].cpu(), got).max()) <= 1e-4
    torch.testing.assert_close(torch.cat([p[2][-1] for p in parts]), full[2][-1], rtol=0, atol=1e-6)
    # without the global label the second shard picks class 2's head: outputs differ
    alone = dec(**{k: v for k, v in shard_batch(inp, 1, 2).items() if k != "head_label"},
                invalid_flow_num=0.0)
    assert not torch.allclose(alone[2][-1], full[2][-1][3:], atol=1e-6)
