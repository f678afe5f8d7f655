"""GPU: a captured hipGraph replay of the decoder / refiner forward gives exactly the eager
result (same kernels, same inputs), follows new inputs, and re-captures after a weight update."""
import pytest
import torch

from tests.helpers import decoder_inputs

pytestmark = pytest.mark.gpu


def _eq(a, b):
    for la, lb in zip(a, b):
        for x, y in zip(la, lb):
            assert torch.equal(x, y)


def test_graphed_decoder_matches_eager_and_follows_inputs():
    from scflow_amd.graph import GraphedForward
    from scflow_amd.profiling import KernelTimer
    from tests.test_gpu_decoder import build_decoder
    dec = build_decoder(3, seed=4).cuda()
    a = {k: v.cuda() for k, v in decoder_inputs(2, 256, seed=3).items()}
    b = {k: v.cuda() for k, v in decoder_inputs(2, 256, seed=8).items()}
    timer = KernelTimer()
    timer.enabled = False
    dec.kernel_hooks["gru_zr"] = timer

    def arm():
        timer.enabled = True
    g = GraphedForward(dec, a, before_capture=arm, invalid_flow_num=0.0)
    timer.enabled = False
    out_a = [[x.clone() for x in l] for l in g(**a)]
    eager_a = dec(**a, invalid_flow_num=0.0)
    _eq(out_a, eager_a)
    out_b = [[x.clone() for x in l] for l in g(**b)]
    _eq(out_b, dec(**b, invalid_flow_num=0.0))
    torch.cuda.synchronize()
    assert timer.count() == 6 and timer.mean_ms() > 0  # 3 iters × 2 SeqConv stages, in-graph events
    # a weight update (new version) triggers a re-capture: the replay follows the new weights
    with torch.no_grad():
        dec.flow_pred.predict_layer.bias.add_(0.5)
    dec.kernel_hooks.clear()
    _eq([[x.clone() for x in l] for l in g(**a)], dec(**a, invalid_flow_num=0.0))


def test_graphed_refiner_matches_eager():
    from scflow_amd.graph import GraphedForward
    from tests.helpers import refine_inputs
    from tests.test_gpu_encoder import build_refiner
    r = build_refiner()
    r.decoder.iters = 2
    inp = {k: v.cuda() for k, v in refine_inputs(2, 256, seed=4).items()}
    g = GraphedForward(r, inp, fn=r.get_pose)
    out = [[x.clone() for x in l] for l in g(**inp)]
    _eq(out, r.get_pose(**inp))
