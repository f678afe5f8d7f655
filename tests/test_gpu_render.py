"""GPU: the HIP renderer (scflow_render) against the oracle restatement of pytorch3d's
rasteriser + hard Phong shader (oracle/render_oracle.py; parity with pytorch3d itself is
UNPINNED — it is absent — the oracle is pinned to closed-form ellipsoid depth in
tests/test_render_host.py), and directly against the closed-form depth at 256².

Tolerances: pix_to_face equal on ≥ 99.7 % of pixels (the rest are fp32 vs fp64 decisions on
pixel centres within rounding of a shared edge), zbuf relative 1e-5 and RGB 2e-3 absolute on the
pixels where both pick the same face (barycentrics 1e-3: fp32 edge functions of small
triangles in NDC cancel); coverage equal to the oracle's on ≥ 99.7 %."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ro = pytest.importorskip("oracle.render_oracle")


def _meshes():
    from scflow_amd import synthetic
    out = {}
    for lab in (3, 7):
        semi = np.array(synthetic.ELLIPSOID_AXES) * synthetic.YCBV_DIAMETERS[lab]
        out[lab] = synthetic.ellipsoid_mesh(semi, 16 + 4 * (lab % 4), 32)
    return out


@pytest.mark.parametrize("S,seps,deflt", [(64, True, True), (128, True, True), (64, False, True),
                                          (64, True, False), (64, False, False)])
def test_render_matches_oracle(S, seps, deflt):
    from scflow_amd import synthetic
    from scflow_amd.renderer import Renderer
    meshes = _meshes()
    sc = synthetic.make_scene(4, S, seed=11)
    labels = np.array([3, 7, 3, 7])
    r = Renderer(image_size=(S, S), soft_blending=False, render_mask=False, seperate_lights=seps,
                 default_lights=deflt, meshes=meshes).to("cuda")
    R, t, K = (torch.from_numpy(sc[k]) for k in ("ref_rotation", "ref_translation", "internel_k"))
    out = r(R.cuda(), t.cuda(), K.cuda(), torch.from_numpy(labels).cuda())
    torch.cuda.synchronize()
    om = {lab: tuple(torch.from_numpy(x).double() if x.dtype != np.int64 else torch.from_numpy(x)
                     for x in m) for lab, m in meshes.items()}
    imgs, zbuf, p2f, bary = ro.render(om, R.double(), t.double(), K.double(), labels.tolist(), S,
                                      light=(seps, deflt))
    g_p2f = out["fragments"].pix_to_face[..., 0].cpu()
    same = g_p2f == p2f
    assert same.float().mean() >= 0.997
    assert ((g_p2f >= 0) == (p2f >= 0)).float().mean() >= 0.997
    hit = same & (p2f >= 0)
    assert hit.sum() > 100
    gz = out["fragments"].zbuf[..., 0].cpu().double()
    np.testing.assert_allclose(gz[hit].numpy(), zbuf[hit].numpy(), rtol=1e-5)
    assert (gz[p2f < 0][g_p2f[p2f < 0] < 0] == -1).all()
    gb = out["fragments"].bary_coords[..., 0, :].cpu().double()
    np.testing.assert_allclose(gb[hit].numpy(), bary[hit].numpy(), atol=1e-3)
    gi = out["images"].cpu().double()
    np.testing.assert_allclose(gi[hit].numpy(), imgs[hit].numpy(), atol=2e-3)
    bg = (p2f < 0) & (g_p2f < 0)
    np.testing.assert_allclose(gi[bg].numpy(), imgs[bg].numpy(), atol=0)


def test_render_depth_matches_closed_form_256():
    """Finely tessellated stand-in object at the bench resolution: the HIP z-buffer against the
    ray/ellipsoid depth at pytorch3d's sample positions (faceting error only)."""
    from scflow_amd import synthetic
    from scflow_amd.renderer import Renderer
    from tests.test_render_host import analytic_depth
    S = 256
    sc = synthetic.make_scene(2, S, seed=5)
    meshes, refs = {}, []
    for i, lab in enumerate(sc["labels"].tolist()):
        semi = np.array(synthetic.ELLIPSOID_AXES) * synthetic.YCBV_DIAMETERS[lab]
        meshes[lab] = synthetic.ellipsoid_mesh(semi, 128, 256)
        refs.append(analytic_depth(sc["ref_rotation"][i].astype(np.float64),
                                   sc["ref_translation"][i].astype(np.float64),
                                   sc["internel_k"][i].astype(np.float64), S, semi))
    r = Renderer(image_size=(S, S), soft_blending=False, render_mask=False, seperate_lights=True,
                 meshes=meshes).to("cuda")
    out = r(*(torch.from_numpy(sc[k]).cuda() for k in ("ref_rotation", "ref_translation",
                                                       "internel_k", "labels")))
    z = out["fragments"].zbuf[..., 0].cpu().numpy()
    for i, (zr, hit) in enumerate(refs):
        cov = z[i] > 0
        assert (cov != hit).mean() < 0.01
        both = cov & hit
        rel = np.abs(z[i][both] - zr[both]) / zr[both]
        assert np.median(rel) < 1e-4 and rel.max() < 2e-3


def test_refiner_render_and_refine_cycles():
    """SCFlowRefiner with a renderer config: ``render`` = the Renderer's image / zbuf / mask
    (format_data_test's render step), and ``refine`` (render → get_pose per cycle) with one
    cycle equals get_pose on the rendered inputs; two cycles re-render at the refined pose."""
    from scflow_amd import MODELS, synthetic
    from tests.test_gpu_decoder import decoder_cfg
    from tests.test_gpu_encoder import encoder_state_dict  # noqa: F401  (same weights as the e2e tests)
    from tests.helpers import refiner_state_dict
    S, B = 256, 2
    sc = synthetic.make_scene(B, S, seed=21)
    meshes = {}
    for lab in set(sc["labels"].tolist()):
        semi = np.array(synthetic.ELLIPSOID_AXES) * synthetic.YCBV_DIAMETERS[lab]
        meshes[lab] = synthetic.ellipsoid_mesh(semi, 24, 48)
    enc = dict(type="RAFTEncoder", in_channels=3, out_channels=256, net_type="Basic", norm_cfg=dict(type="IN"))
    ctx = dict(type="RAFTEncoder", in_channels=3, out_channels=256, net_type="Basic", norm_cfg=dict(type="BN"))
    r = MODELS.build(dict(type="SCFlowRefiner", cxt_channels=128, h_channels=128, seperate_encoder=False,
                          encoder=enc, cxt_encoder=ctx, decoder=dict(type="SCFlowDecoder", **decoder_cfg(2)),
                          renderer=dict(mesh_dir=None, image_size=(S, S), soft_blending=False,
                                        render_mask=False, seperate_lights=True, meshes=meshes),
                          test_cfg=dict(iters=2, cycles=2)))
    r.load_state_dict({("decoder." + k if not k.startswith(("real_encoder.", "render_encoder.", "context."))
                        else k): v for k, v in refiner_state_dict().items()}, strict=False)
    r = r.eval().cuda()
    R, t, K, lab = (torch.from_numpy(sc[k]).cuda() for k in ("ref_rotation", "ref_translation",
                                                             "internel_k", "labels"))
    tgt = synthetic.make_train_targets(sc, S, seed=21)
    real, _, _ = r.render(torch.from_numpy(tgt["gt_rotation"]).cuda(),
                          torch.from_numpy(tgt["gt_translation"]).cuda(), K, lab)
    img, depth, mask = r.render(R, t, K, lab)
    direct = r.renderer(R, t, K, lab)
    torch.testing.assert_close(img, direct["images"][..., :3].permute(0, 3, 1, 2))
    torch.testing.assert_close(depth, direct["fragments"].zbuf[..., 0])
    assert ((depth > 0) == (mask > 0)).all() and mask.sum() > 1000
    R1, t1, out1 = r.refine(real, R, t, K, lab, cycles=1)
    ref_out = r.get_pose(img, real, R, t, depth, K, lab)
    torch.testing.assert_close(R1, ref_out[2][-1])
    torch.testing.assert_close(t1, ref_out[3][-1])
    R2, t2, _ = r.refine(real, R, t, K, lab)  # test_cfg cycles = 2
    torch.cuda.synchronize()
    assert torch.isfinite(R2).all() and torch.isfinite(t2).all()
    assert not torch.equal(R2, R1)


@pytest.mark.parametrize("deflt,seps", [(True, True), (True, False), (False, True), (False, False)])
def test_kernel_light_location_matches_reference_fixture(deflt, seps):
    """The light each image is shaded with (scflow_render's light_out) against the PointLights
    location the reference's own Renderer.forward builds (golden_render_wiring.npz, rendering.py:
    209-230; tests/test_render_wiring.py pins the rest of the wiring on the CPU)."""
    from scflow_amd import synthetic
    from scflow_amd.renderer import Renderer
    from tests.helpers import golden
    gd = golden("render_wiring")
    labels = gd["in_labels"]
    meshes = {int(l): synthetic.ellipsoid_mesh(np.array(synthetic.ELLIPSOID_AXES) *
                                               synthetic.YCBV_DIAMETERS[int(l)], 12, 24)
              for l in set(labels.tolist())}
    S = int(gd["in_S"])
    r = Renderer(image_size=(S, S), soft_blending=False, render_mask=False, seperate_lights=seps,
                 default_lights=deflt, meshes=meshes).to("cuda")
    out = r(*(torch.from_numpy(gd[k]).cuda() for k in ("in_R", "in_t", "in_K", "in_labels")))
    got = out["light_location"].cpu().numpy()
    rec = gd[f"d{int(deflt)}s{int(seps)}_light_location"]
    if rec.size == 0:  # PointLights() default location (pytorch3d's (0, 1, 0))
        rec = np.tile([0.0, 1.0, 0.0], (len(labels), 1))
    np.testing.assert_allclose(got, rec, rtol=1e-5, atol=1e-3)
