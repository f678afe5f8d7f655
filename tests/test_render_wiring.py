"""The renderer's reference-side wiring, pinned to the reference itself (§8(f)-3).

``tests/golden/golden_render_wiring.npz`` comes from the reference's own ``Renderer.forward``
(models/utils/rendering.py:185-248) with recording stand-ins for pytorch3d (make_golden.py
``render``): the PerspectiveCameras it builds (``cameras_from_opencv_projection`` :17-60), the
znear / zfar it rounds to 100 mm (:193-199) and the PointLights location / colours (:209-230), for
the four (default_lights, seperate_lights) settings.  Checked here (CPU):
* ``scflow_amd.renderer.cameras_from_opencv_projection`` and ``depth_range`` equal the recorded
  keywords (exact up to fp32 rounding);
* pytorch3d's PerspectiveCameras projection (NDC, ``in_ndc``: X_view = X·R + T, x = f·X/Z + p)
  applied to the RECORDED camera puts every vertex where ``oracle.render_oracle.project_ndc`` —
  the convention scflow_render's projection implements — puts it (1e-5 NDC);
* the oracle's light placement and the renderer's light colours equal the recorded ones.
The kernel's own light locations (``light_location`` output) are checked against the same
fixture on the GPU (tests/test_gpu_render.py).  The rasteriser itself stays parity-unpinned
(pytorch3d is absent).
"""
import numpy as np
import pytest
import torch

from tests.helpers import golden

ro = pytest.importorskip("oracle.render_oracle")
CASES = ((True, True), (True, False), (False, True), (False, False))


def _verts(labels):
    from scflow_amd import synthetic
    return [torch.from_numpy(synthetic.ellipsoid_mesh(np.array(synthetic.ELLIPSOID_AXES) *
                                                      synthetic.YCBV_DIAMETERS[int(l)], 12, 24)[0])
            for l in labels]


def _fixture():
    gd = golden("render_wiring")
    R, t, K = (torch.from_numpy(gd[k]) for k in ("in_R", "in_t", "in_K"))
    return gd, R, t, K, gd["in_labels"], int(gd["in_S"])


def test_fixture_meshes_are_the_generators():
    from scflow_amd import synthetic
    gd = golden("render_wiring")
    sums = [float(np.asarray(synthetic.ellipsoid_mesh(np.array(synthetic.ELLIPSOID_AXES) * d, 12, 24)[0],
                             np.float64).sum()) for d in synthetic.YCBV_DIAMETERS]
    np.testing.assert_allclose(sums, gd["mesh_verts_sum"], rtol=1e-12)


@pytest.mark.parametrize("deflt,seps", CASES)
def test_cameras_and_depth_range_match_reference(deflt, seps):
    from scflow_amd.renderer import cameras_from_opencv_projection, depth_range
    gd, R, t, K, labels, S = _fixture()
    tag = f"d{int(deflt)}s{int(seps)}"
    cam = cameras_from_opencv_projection(R, t, K, torch.tensor([S, S])[None].expand(len(labels), 2))
    for k in ("R", "T", "focal_length", "principal_point", "image_size"):
        np.testing.assert_allclose(getattr(cam, k).numpy(), gd[f"{tag}_cam_{k}"], rtol=1e-6, atol=1e-6,
                                   err_msg=k)
    zn, zf = depth_range(R, t, _verts(labels))
    np.testing.assert_array_equal([zn.item(), zf.item()], gd[f"{tag}_znear_zfar"])


def test_recorded_camera_projects_like_the_kernel_convention():
    """pytorch3d PerspectiveCameras (NDC) on the reference's recorded camera == project_ndc."""
    gd, R, t, K, labels, S = _fixture()
    verts = _verts(labels)
    Rp, Tp = torch.from_numpy(gd["d1s1_cam_R"]).double(), torch.from_numpy(gd["d1s1_cam_T"]).double()
    f, p = torch.from_numpy(gd["d1s1_cam_focal_length"]).double(), \
        torch.from_numpy(gd["d1s1_cam_principal_point"]).double()
    for i, v in enumerate(verts):
        v = v.double()
        Xv = v @ Rp[i] + Tp[i]                     # pytorch3d world → view (row vectors)
        ndc = torch.stack([f[i, 0] * Xv[:, 0] / Xv[:, 2] + p[i, 0],
                           f[i, 1] * Xv[:, 1] / Xv[:, 2] + p[i, 1], Xv[:, 2]], 1)
        ours = ro.project_ndc(v, R[i].double(), t[i].double(), K[i].double(), S)
        np.testing.assert_allclose(ndc.numpy(), ours.numpy(), atol=1e-5, rtol=1e-7)


@pytest.mark.parametrize("deflt,seps", CASES)
def test_light_placement_and_colours_match_reference(deflt, seps):
    gd, R, t, K, labels, S = _fixture()
    tag = f"d{int(deflt)}s{int(seps)}"
    loc = ro.light_location(_verts(labels), R.double(), t.double(), light=(seps, deflt))
    rec = gd[f"{tag}_light_location"]
    if rec.size == 0:  # PointLights() defaults: pytorch3d's location (0, 1, 0) — unpinned
        np.testing.assert_array_equal(loc.numpy(), np.tile([0.0, 1.0, 0.0], (len(labels), 1)))
    else:
        np.testing.assert_allclose(loc.numpy(), rec, rtol=1e-6, atol=1e-3)
    if not deflt:  # the ITODD colours the reference passes (:220); defaults are pytorch3d's own
        for k, v in (("ambient_color", 0.8), ("diffuse_color", 0.5), ("specular_color", 1.0)):
            np.testing.assert_array_equal(gd[f"{tag}_light_{k}"], np.full((1, 3), v, np.float32))
    else:
        assert all(gd[f"{tag}_light_{k}"].size == 0 for k in ("ambient_color", "diffuse_color",
                                                              "specular_color"))
    # one pose sits at 380 mm: its separate light clamps to the camera origin
    if seps:
        assert np.abs(rec[1]).max() == 0.0
