"""GPU: the hot-path ops registered with torch.library (scflow_amd/library.py).

* ``torch.library.opcheck`` on ``scflow::corr_pyramid``, ``scflow::corr_lookup`` and
  ``scflow::pose_update_flow`` (schema, fake-tensor / meta implementation, autograd
  registration, AOT dispatch);
* the reference-signature modules ``CorrelationPyramid(num_levels)(f1, f2)`` and
  ``CorrLookup(radius, mode, padding_mode, align_corners)(pyramid, flow)``
  (raft_decoder.py:35-58, corr_lookup.py:91-136) through the ops, against the fixture generated
  from the reference's own modules (|Δ| ≤ 2e-5);
* their registered backward against fp64 CPU autograd of the oracle (relative 1e-4 of the
  gradient scale);
* a ``torch.compile(fullgraph=True, backend="aot_eager")`` trace of pyramid → lookup equal to eager
  (the ops are no graph breaks).
"""
import numpy as np
import pytest
import torch

from tests.helpers import golden, t

pytestmark = pytest.mark.gpu
orc = pytest.importorskip("oracle.scflow_oracle")


def _close(a, b, rtol, atol, what):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item()
    assert err <= atol + rtol * scale, f"{what}: max err {err:.3e} (scale {scale:.3e})"


def _inputs(n=2, c=16, h=16, w=16, seed=51):
    g = torch.Generator().manual_seed(seed)
    f1 = torch.randn(n, c, h, w, generator=g)
    f2 = torch.randn(n, c, h, w, generator=g)
    flow = (torch.rand(n, 2, h, w, generator=g) - 0.5) * 10
    return f1, f2, flow


def test_opcheck_corr_pyramid_and_lookup():
    from scflow_amd import library
    f1, f2, flow = _inputs()
    torch.library.opcheck(torch.ops.scflow.corr_pyramid.default,
                          (f1.cuda().requires_grad_(), f2.cuda().requires_grad_(), 4))
    pyr = library.corr_pyramid(f1.cuda(), f2.cuda(), 4)
    torch.library.opcheck(torch.ops.scflow.corr_lookup.default,
                          (pyr.detach().clone().requires_grad_(), flow.cuda(), 4, 4, True))
    torch.library.opcheck(torch.ops.scflow.corr_lookup.default, (pyr, flow.cuda(), 4, 1, False))


def test_opcheck_pose_update_flow():
    gd = golden("ops")
    R0, t0, K = (t(gd["pose_ref_rotation"]).cuda(), t(gd["pose_ref_translation"]).cuda(),
                 t(gd["pose_internel_k"]).cuda())
    from scflow_amd import ops
    pts = ops.lift_points(t(gd["pose_depth"]).cuda(), K, R0, t0)
    args = (t(gd["pose_drot"]).cuda(), t(gd["pose_dt"]).cuda(), R0, t0, K, pts, 400.0, 10.0, "exp")
    torch.library.opcheck(torch.ops.scflow.pose_update_flow.default, args)
    R1, t1, flow = torch.ops.scflow.pose_update_flow(*args)
    _close(R1, t(gd["pose_R1"]), 0, 1e-6, "R vs reference fixture")
    _close(t1, t(gd["pose_t1"]), 1e-6, 1e-4, "t vs reference fixture")
    _close(flow, t(gd["pose_flow_inv400"]), 0, 2e-3, "flow vs reference fixture")


def test_modules_through_ops_match_reference_fixture():
    """CorrLookup(radius, mode, padding_mode, align_corners)(pyramid, flow) — the reference's
    constructor and call signature — on the fixture of the reference's own modules."""
    from scflow_amd.modules import CorrelationPyramid, CorrLookup
    gd = golden("ops")
    lv = CorrelationPyramid(num_levels=4)(t(gd["pyr_f1"]).cuda(), t(gd["pyr_f2"]).cuda())
    for i, lvl in enumerate(lv):
        _close(lvl, t(gd[f"pyr_l{i}"]), 0, 2e-5, f"pyramid level {i}")
    for r in (4, 1):
        lk = CorrLookup(radius=r, mode="bilinear", padding_mode="zeros", align_corners=True)
        _close(lk(lv, t(gd["lk_flow"]).cuda()), t(gd[f"lk_r{r}"]), 0, 2e-5, f"lookup r={r}")
    lk0 = CorrLookup(4, "bilinear", "zeros", False)
    _close(lk0(lv, t(gd["lk_flow"]).cuda()), t(gd["lk_r4_ac0"]), 0, 2e-5, "lookup align_corners=False")


def test_registered_backward_matches_fp64_autograd():
    from scflow_amd.modules import CorrelationPyramid, CorrLookup
    f1, f2, flow = _inputs(2, 32, 16, 16, seed=52)
    g = torch.Generator().manual_seed(53)
    gy = torch.randn(2, 4 * 81, 16, 16, generator=g)
    a1 = f1.double().requires_grad_()
    a2 = f2.double().requires_grad_()
    ref = orc.corr_lookup(orc.corr_pyramid(a1, a2, 4), flow.double(), 4)
    (ref * gy.double()).sum().backward()
    d1 = f1.cuda().requires_grad_()
    d2 = f2.cuda().requires_grad_()
    out = CorrLookup(4)(CorrelationPyramid(4)(d1, d2), flow.cuda())
    (out * gy.cuda()).sum().backward()
    _close(out, ref, 1e-5, 1e-5, "lookup forward")
    _close(d1.grad, a1.grad, 1e-4, 1e-6, "dfeat1")
    _close(d2.grad, a2.grad, 1e-4, 1e-6, "dfeat2")


def test_compile_traces_through_ops():
    from scflow_amd.modules import CorrelationPyramid, CorrLookup
    pyr_m, lk_m = CorrelationPyramid(4), CorrLookup(4)

    def fn(a, b, fl):
        return lk_m(pyr_m(a, b), fl) * 2.0
    f1, f2, flow = (x.cuda() for x in _inputs(1, 16, 16, 16, seed=54))
    eager = fn(f1, f2, flow)
    compiled = torch.compile(fn, fullgraph=True, backend="aot_eager")(f1, f2, flow)
    assert torch.equal(eager, compiled)
    assert np.isfinite(compiled.cpu().numpy()).all()
