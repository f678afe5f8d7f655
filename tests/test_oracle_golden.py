"""CPU: the oracle (oracle/scflow_oracle.py) against golden vectors produced by the reference.

Pins the oracle before anything else trusts it (tests/golden/make_golden.py ran the
reference's own modules to produce these fixtures).
"""
import numpy as np
import pytest
import torch

from tests.helpers import GOLDEN, golden, oracle_state_dict, t

orc = pytest.importorskip("oracle.scflow_oracle")


def test_corr_pyramid_matches_reference():
    g = golden("ops")
    pyr = orc.corr_pyramid(t(g["pyr_f1"]), t(g["pyr_f2"]), 4)
    for i, p in enumerate(pyr):
        np.testing.assert_allclose(p.numpy(), g[f"pyr_l{i}"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("radius", [4, 1])
def test_corr_lookup_matches_reference(radius):
    g = golden("ops")
    pyr = [t(g[f"pyr_l{i}"]) for i in range(4)]
    out = orc.corr_lookup(pyr, t(g["lk_flow"]), radius)
    np.testing.assert_allclose(out.numpy(), g[f"lk_r{radius}"], rtol=1e-5, atol=1e-6)


def test_corr_lookup_align_corners_false_matches_reference():
    """CorrLookup(align_corners=False) (grid_sample's other convention; bilinear_sample's own
    default, corr_lookup.py:35)."""
    g = golden("ops")
    pyr = [t(g[f"pyr_l{i}"]) for i in range(4)]
    out = orc.corr_lookup(pyr, t(g["lk_flow"]), 4, align_corners=False)
    np.testing.assert_allclose(out.numpy(), g["lk_r4_ac0"], rtol=1e-5, atol=1e-6)


def test_conv_gru_matches_reference():
    g = golden("ops")
    from scflow_amd import synthetic
    shapes = []
    for gate in "zrq":
        for i, (k, _) in enumerate(orc.GRU_KERNELS["SeqConv"]):
            shapes.append((f"conv_{gate}.{i}.conv.weight", (8, 24) + k))
            shapes.append((f"conv_{gate}.{i}.conv.bias", (8,)))
    sd = {k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(shapes, seed=3).items()}
    out = orc.conv_gru(sd, t(g["gru_h"]), t(g["gru_x"]), prefix="")
    np.testing.assert_allclose(out.numpy(), g["gru_out"], rtol=1e-5, atol=1e-5)


def test_pose_update_and_flow_match_reference():
    g = golden("ops")
    R1, t1 = orc.pose_update(t(g["pose_drot"]), t(g["pose_dt"]), t(g["pose_ref_rotation"]),
                             t(g["pose_ref_translation"]))
    np.testing.assert_allclose(R1.numpy(), g["pose_R1"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(t1.numpy(), g["pose_t1"], rtol=1e-6, atol=1e-4)
    pts, valid = orc.lift_points(t(g["pose_depth"]), t(g["pose_internel_k"]),
                                 t(g["pose_ref_rotation"]), t(g["pose_ref_translation"]))
    assert valid.any() and (~valid).any()
    for inv in (0, 400):
        fl = orc.pose_flow(t(g["pose_R1"]), t(g["pose_t1"]), t(g["pose_internel_k"]), pts, valid,
                           float(inv))
        np.testing.assert_allclose(fl.numpy(), g[f"pose_flow_inv{inv}"], rtol=1e-4, atol=2e-3)
    gt = orc.flow_from_delta_pose_and_depth(t(g["pose_ref_rotation"]), t(g["pose_ref_translation"]),
                                            t(g["pose_R1"]), t(g["pose_t1"]), t(g["pose_depth"]),
                                            t(g["pose_internel_k"]))
    np.testing.assert_allclose(gt.numpy(), g["pose_gtflow"], rtol=1e-4, atol=2e-3)


def test_decoder_e2e_matches_reference():
    """Full SCFlowDecoder forward (B=2, 256², 4 iters): mean EPE ≤ 1e-3 px vs the reference."""
    g = golden("e2e")
    B, S, iters, seed = (int(v) for v in g["meta"])
    from tests.helpers import decoder_inputs
    inp = decoder_inputs(B, S, seed, g)
    sd = oracle_state_dict()
    outs = orc.decoder_forward(sd, **inp, iters=iters)
    fp, fpred, Rs, ts, masks, drs, dts = outs
    epe_pose = orc.cal_epe_mean(t(g["flow_pose_last"]), fp[-1])
    epe_pred = orc.cal_epe_mean(t(g["flow_pred_last"]), fpred[-1])
    assert float(epe_pose.max()) <= 1e-3, epe_pose
    assert float(epe_pred.max()) <= 1e-3, epe_pred
    np.testing.assert_allclose(torch.stack(Rs).numpy(), g["R"], atol=1e-5)
    np.testing.assert_allclose(torch.stack(ts).numpy(), g["t"], rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(torch.stack(drs).numpy(), g["drot"], atol=1e-5)
    np.testing.assert_allclose(torch.stack(dts).numpy(), g["dt"], atol=1e-5)
    np.testing.assert_allclose(masks[-1].numpy(), g["mask_last"], atol=1e-5)
    # the fixture is not degenerate: the pose moves and the flow is non-trivial
    assert g["flow_pose_absmean"][-1] > 0.05


@pytest.mark.parametrize("norm,seed", [("IN", 1), ("BN", 2)])
def test_raft_encoder_matches_reference(norm, seed):
    """RAFTEncoder 'Basic' (feature encoder IN / context encoder BN eval) at 128²."""
    from scflow_amd import synthetic
    from tests.helpers import encoder_state_dict
    g = golden("enc")
    B, S, iseed = (int(v) for v in g["meta"])
    x = t(synthetic.make_images(B, S, seed=iseed)["render_images"])
    assert abs(float(x.double().sum()) - float(g["sum_images"][0])) < 1e-6
    out = orc.raft_encoder(encoder_state_dict(norm, seed), x, norm)
    np.testing.assert_allclose(out.numpy(), g[f"enc_{norm}"], rtol=1e-4, atol=1e-4)


def test_refine_e2e_matches_reference():
    """Images → encoders → decoder (B=2, 256², 4 iters): mean EPE ≤ 1e-3 px vs the reference."""
    from tests.helpers import refine_inputs, refiner_state_dict
    g = golden("refine")
    B, S, iters, seed = (int(v) for v in g["meta"])
    inp = refine_inputs(B, S, seed, g)
    sd = refiner_state_dict()
    render, real, h, c = orc.extract_feat(sd, inp["render_images"], inp["real_images"])
    for k, v in (("render_feat", render), ("real_feat", real), ("h_feat", h), ("cxt_feat", c)):
        got = np.array([v.double().sum().item(), v.double().abs().sum().item()])
        np.testing.assert_allclose(got, g[f"stat_{k}"], rtol=1e-4)
    np.testing.assert_allclose(render[0, :8].numpy(), g["render_feat_s0c0"], rtol=1e-4, atol=1e-4)
    dsd = {k: v for k, v in sd.items() if not k.startswith(("real_encoder.", "render_encoder.", "context."))}
    fp, fpred, Rs, ts, *_ = orc.decoder_forward(
        dsd, render, real, h, c, inp["ref_rotation"], inp["ref_translation"], inp["depth"],
        inp["internel_k"], label=inp["label"], init_flow=torch.zeros(B, 2, S, S), iters=iters)
    assert float(orc.cal_epe_mean(t(g["flow_pose_last"]), fp[-1]).max()) <= 1e-3
    assert float(orc.cal_epe_mean(t(g["flow_pred_last"]), fpred[-1]).max()) <= 1e-3
    np.testing.assert_allclose(torch.stack(ts).numpy(), g["t"], rtol=1e-5, atol=1e-3)


def test_quaternion_delta_rotation_convention():
    """The quaternion branch of get_pose_from_delta_pose (pose.py:132-133) goes through kornia,
    which is absent and unpinned (PARITY UNPINNED against the reference): the oracle's
    restatement is checked against scipy's independent x, y, z, w (scalar-last) rotation, the
    order the pose head's identity bias [0, 0, 0, 1] assumes (pose_head.py:192-194), and the
    identity bias must give ΔR = I."""
    from scipy.spatial.transform import Rotation
    g = torch.Generator().manual_seed(3)
    q = torch.randn(64, 4, generator=g, dtype=torch.float64) * torch.rand(64, 1, generator=g,
                                                                          dtype=torch.float64) * 3
    got = orc.rotation_from_quaternion_xyzw(q)
    ref = torch.from_numpy(Rotation.from_quat(q.numpy()).as_matrix())
    np.testing.assert_allclose(got.numpy(), ref.numpy(), atol=1e-12)
    eye = orc.rotation_from_quaternion_xyzw(torch.tensor([[0.0, 0.0, 0.0, 1.0]], dtype=torch.float64))
    np.testing.assert_allclose(eye[0].numpy(), np.eye(3), atol=0)
    # the update with a quaternion delta equals the ortho6d update with ΔR's first two columns
    R0 = torch.from_numpy(Rotation.random(64, random_state=1).as_matrix())
    t0 = torch.tensor([[10.0, -20.0, 900.0]], dtype=torch.float64).repeat(64, 1)
    dt = torch.randn(64, 3, generator=g, dtype=torch.float64) * 0.1
    Rq, tq = orc.pose_update(q, dt, R0, t0)
    o6 = torch.cat([ref[:, :, 0], ref[:, :, 1]], 1)
    R6, t6 = orc.pose_update(o6, dt, R0, t0)
    np.testing.assert_allclose(Rq.numpy(), R6.numpy(), atol=1e-12)
    np.testing.assert_allclose(tq.numpy(), t6.numpy(), atol=0)
