"""CPU: the renderer's oracle (oracle/render_oracle.py, a restatement of pytorch3d's rasteriser
and hard Phong shader — parity with pytorch3d itself is UNPINNED, pytorch3d is absent) pinned
analytically: the z-buffer of a finely tessellated ellipsoid matches the closed-form
ray/ellipsoid depth at pytorch3d's pixel-sample positions; plus PLY / OBJ I/O and the
Renderer's configuration checks (no GPU needed)."""
import math

import numpy as np
import pytest
import torch

ro = pytest.importorskip("oracle.render_oracle")


def analytic_depth(R, t, K, S, semi):
    """Ray/ellipsoid depth at the sample position of pixel (r, c): u = (c + ½)(S−1)/S."""
    s = (np.arange(S) + 0.5) * (S - 1) / S
    v, u = np.meshgrid(s, s, indexing="ij")
    rays = np.stack([u, v, np.ones_like(u)], -1) @ np.linalg.inv(K).T
    D = np.diag(1.0 / np.asarray(semi) ** 2)
    dr = rays @ R
    tr = R.T @ t
    a = np.einsum("hwi,ij,hwj->hw", dr, D, dr)
    b = -2.0 * np.einsum("hwi,ij,j->hw", dr, D, tr)
    c = float(tr @ D @ tr - 1.0)
    disc = b * b - 4 * a * c
    hit = disc > 0
    z = np.where(hit, (-b - np.sqrt(np.where(hit, disc, 0.0))) / (2 * a), -1.0)
    return z, hit


def scene(S, seed):
    from scflow_amd import synthetic
    sc = synthetic.make_scene(1, S, seed=seed)
    return (sc["ref_rotation"][0].astype(np.float64), sc["ref_translation"][0].astype(np.float64),
            sc["internel_k"][0].astype(np.float64), int(sc["labels"][0]))


@pytest.mark.parametrize("seed", [0, 1])
def test_oracle_zbuffer_matches_analytic_ellipsoid(seed):
    from scflow_amd import synthetic
    S = 64
    R, t, K, lab = scene(S, seed)
    semi = np.array(synthetic.ELLIPSOID_AXES) * synthetic.YCBV_DIAMETERS[lab]
    v, f, c = synthetic.ellipsoid_mesh(semi, 96, 192)
    ndc = ro.project_ndc(torch.from_numpy(v).double(), torch.from_numpy(R), torch.from_numpy(t),
                         torch.from_numpy(K), S)
    p2f, zbuf, bary = ro.rasterize(ndc, torch.from_numpy(f), S, face_chunk=2048)
    z_ref, hit = analytic_depth(R, t, K, S, semi)
    got = zbuf.numpy()
    inner = hit & (got > 0)
    # coverage agrees except along the silhouette (faceting); depth within the chord error
    assert (hit != (got > 0)).mean() < 0.02
    rel = np.abs(got[inner] - z_ref[inner]) / z_ref[inner]
    assert np.median(rel) < 1e-4 and rel.max() < 2e-3
    b = bary.numpy()[inner]
    np.testing.assert_allclose(b.sum(-1), 1.0, atol=1e-9)
    assert (b > 0).all()


def test_oracle_render_background_and_alpha():
    from scflow_amd import synthetic
    S = 32
    R, t, K, lab = scene(S, 3)
    v, f, c = synthetic.ellipsoid_mesh(np.array(synthetic.ELLIPSOID_AXES) * 150.0, 12, 24)
    imgs, zbuf, p2f, bary = ro.render({0: (torch.from_numpy(v).double(), torch.from_numpy(f),
                                           torch.from_numpy(c).double())},
                                      torch.from_numpy(R)[None], torch.from_numpy(t)[None],
                                      torch.from_numpy(K)[None], [0], S)
    empty = p2f[0] < 0
    assert empty.any() and (~empty).any()
    np.testing.assert_allclose(imgs[0][empty].numpy(), [[0.5, 0.5, 0.5, 0.0]] * int(empty.sum()))
    assert (imgs[0][~empty][:, 3] == 1).all()
    assert (imgs[0][~empty][:, :3] >= 0).all()
    assert (zbuf[0][empty] == -1).all()


@pytest.mark.parametrize("binary", [True, False])
def test_ply_round_trip(tmp_path, binary):
    from scflow_amd import synthetic
    from scflow_amd.renderer import load_ply, save_ply
    v, f, c = synthetic.ellipsoid_mesh((30.0, 20.0, 10.0), 6, 8)
    p = str(tmp_path / "obj_000001.ply")
    save_ply(p, v, f, c, binary=binary)
    v2, f2, c2 = load_ply(p)
    np.testing.assert_allclose(v2, v, rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(f2, f)
    np.testing.assert_allclose(c2, np.round(c * 255) / 255, atol=1e-6)


def test_renderer_loads_mesh_dir_and_rejects_unsupported(tmp_path):
    from scflow_amd import synthetic
    from scflow_amd.renderer import Renderer, save_ply
    for k in (1, 2):
        v, f, c = synthetic.ellipsoid_mesh((30.0 * k, 20.0, 10.0), 6, 8)
        save_ply(str(tmp_path / f"obj_{k:06d}.ply"), v, f, c)
    r = Renderer(str(tmp_path), image_size=(64, 64), soft_blending=False, render_mask=False)
    assert sorted(r.meshes) == [0, 1]
    assert r.meshes[1][0].shape[1] == 3 and r.meshes[1][3].shape == r.meshes[1][0].shape
    with pytest.raises(NotImplementedError):
        Renderer(str(tmp_path), soft_blending=True)
    with pytest.raises(NotImplementedError):
        Renderer(str(tmp_path), soft_blending=False, render_mask=True)
    from scflow_amd._lib import ScflowError
    with pytest.raises(ScflowError):  # no CPU path
        r(torch.eye(3)[None], torch.tensor([[0, 0, 500.0]]), torch.eye(3)[None], torch.tensor([0]))


def test_verts_normals_match_oracle():
    from scflow_amd import synthetic
    from scflow_amd.renderer import verts_normals
    v, f, _ = synthetic.ellipsoid_mesh((30.0, 20.0, 10.0), 10, 20)
    a = verts_normals(torch.from_numpy(v).double(), torch.from_numpy(f))
    b = ro.verts_normals(torch.from_numpy(v).double(), torch.from_numpy(f))
    torch.testing.assert_close(a, b)
    # outward: normals point away from the centre
    assert ((a * torch.from_numpy(v).double()).sum(1) > 0).all()
