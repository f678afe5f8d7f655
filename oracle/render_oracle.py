"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

CPU restatement (PyTorch on CPU, float32/float64) of the reference's mesh renderer
(``/root/reference/models/utils/rendering.py``: ``cameras_from_opencv_projection`` :17-60,
``Renderer.forward`` :196-248) as configured for SCFlow (``configs/refine_models/
scflow_ycbv_real.py:261-274``: HardPhongShader, faces_per_pixel=1, blur_radius=0,
seperate_lights=True with default light colours, background 0.5).  The reference delegates the
work to pytorch3d (``MeshRasterizer``, ``HardPhongShader``, ``PointLights``, ``TexturesVertex``),
which is NOT installed here; this file restates pytorch3d's published
algorithm (pytorch3d 0.7: ``csrc/rasterize_meshes/rasterize_meshes_cpu.cpp``, ``renderer/
mesh/shading.py::phong_shading``, ``renderer/lighting.py``, ``renderer/blending.py::
hard_rgb_blend``, ``structures/meshes.py::verts_normals``).

PARITY UNPINNED against pytorch3d itself (no pytorch3d, no reference renders to compare
with).  The geometry is pinned analytically instead: the z-buffer of a finely tessellated
ellipsoid agrees with the closed-form ray/ellipsoid depth at pytorch3d's pixel-sample
positions (tests/test_render_host.py).

Conventions restated:
* Camera: OpenCV R, t, K → pytorch3d NDC camera (:17-60).  A view-space point
  (X, Y, Z) = R·v + t projects to NDC  x = −(u − c0)/s,  y = −(v − c0)/s  with
  (u, v) = (fx·X/Z + cx, fy·Y/Z + cy),  c0 = (S − 1)/2,  s = (min(H, W) − 1)/2 (square S);
  z stays the view depth Z.
* Pixel (row r, col c) samples NDC (1 − (2c + 1)/W, 1 − (2r + 1)/H) (pytorch3d flips both
  axes: ``xi = W − 1 − c``, ``PixToNdc(i, S) = −1 + (2i + 1)/S``).
* Barycentrics from edge functions in NDC with area + 1e-8 (faces with |area| ≤ 1e-8
  skipped); perspective correction (w_i·z_j·z_k renormalised, denominator clamped at 1e-8);
  pz = Σ b_i z_i; the point counts iff all three corrected barycentrics are > 0 and pz ≥ 0;
  the smallest pz wins (faces_per_pixel=1; ties → the lower packed face index).
* Shading (hard Phong): normals / positions / vertex colours interpolated with the corrected
  barycentrics, lights.ambient·mat.ambient + diffuse + specular (shininess 64), colour =
  (ambient + diffuse)·texel + specular; background (0.5, 0.5, 0.5) alpha 0, foreground alpha 1.
* Light (seperate_lights, default colours ambient 0.5 / diffuse 0.3 / specular 0.2): location
  R_i·(0, 0, max(min_z_i − 400, 0)) with min_z_i the smallest view depth of image i's vertices
  (:209-213, :226-230); camera centre −Rᵀt.
"""
from __future__ import annotations

from typing import Dict, Sequence, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
K_EPS = 1e-8


def verts_normals(verts: Tensor, faces: Tensor) -> Tensor:
    """pytorch3d Meshes.verts_normals: area-weighted face normals accumulated per corner,
    then normalised (eps 1e-6)."""
    v0, v1, v2 = verts[faces[:, 0]], verts[faces[:, 1]], verts[faces[:, 2]]
    n = torch.zeros_like(verts)
    n.index_add_(0, faces[:, 1], torch.cross(v2 - v1, v0 - v1, dim=1))
    n.index_add_(0, faces[:, 2], torch.cross(v0 - v2, v1 - v2, dim=1))
    n.index_add_(0, faces[:, 0], torch.cross(v1 - v0, v2 - v0, dim=1))
    return F.normalize(n, eps=1e-6, dim=1)


def project_ndc(verts: Tensor, R: Tensor, t: Tensor, K: Tensor, S: int) -> Tensor:
    """[V, 3] object-frame vertices → [V, 3] (x_ndc, y_ndc, z_view)."""
    cam = verts @ R.T + t[None]
    z = cam[:, 2]
    u = K[0, 0] * cam[:, 0] / z + K[0, 2]
    v = K[1, 1] * cam[:, 1] / z + K[1, 2]
    c0 = (S - 1) / 2.0
    return torch.stack([-(u - c0) / c0, -(v - c0) / c0, z], 1)


def rasterize(ndc: Tensor, faces: Tensor, S: int, face_chunk: int = 256
              ) -> Tuple[Tensor, Tensor, Tensor]:
    """One image: returns pix_to_face [S, S] (−1 empty), zbuf [S, S] (−1 empty),
    bary [S, S, 3] (perspective-corrected; −1 empty)."""
    dt = ndc.dtype
    ar = torch.arange(S, dtype=dt)
    yf = (1 - (2 * ar + 1) / S)[:, None].expand(S, S)   # row r
    xf = (1 - (2 * ar + 1) / S)[None, :].expand(S, S)   # col c
    best_z = torch.full((S, S), float("inf"), dtype=dt)
    best_f = torch.full((S, S), -1, dtype=torch.long)
    for f0 in range(0, faces.shape[0], face_chunk):
        fc = faces[f0:f0 + face_chunk]
        v0, v1, v2 = ndc[fc[:, 0]], ndc[fc[:, 1]], ndc[fc[:, 2]]     # [F, 3]
        px, py = xf[None], yf[None]

        def edge(ax, ay, bx, by):  # EdgeFunctionForward(p, a, b)
            return (px - ax[:, None, None]) * (by - ay)[:, None, None] - \
                   (py - ay[:, None, None]) * (bx - ax)[:, None, None]
        # EdgeFunctionForward(v2, v0, v1) + kEpsilon; |area| ≤ eps faces are skipped
        area0 = (v2[:, 0] - v0[:, 0]) * (v1[:, 1] - v0[:, 1]) - (v2[:, 1] - v0[:, 1]) * (v1[:, 0] - v0[:, 0])
        area = area0 + K_EPS
        w0 = edge(v1[:, 0], v1[:, 1], v2[:, 0], v2[:, 1]) / area[:, None, None]
        w1 = edge(v2[:, 0], v2[:, 1], v0[:, 0], v0[:, 1]) / area[:, None, None]
        w2 = edge(v0[:, 0], v0[:, 1], v1[:, 0], v1[:, 1]) / area[:, None, None]
        z0, z1, z2 = (v[:, 2][:, None, None] for v in (v0, v1, v2))
        t0, t1, t2 = w0 * z1 * z2, z0 * w1 * z2, z0 * z1 * w2
        den = torch.clamp(t0 + t1 + t2, min=K_EPS)
        b0, b1, b2 = t0 / den, t1 / den, t2 / den
        pz = b0 * z0 + b1 * z1 + b2 * z2
        ok = (b0 > 0) & (b1 > 0) & (b2 > 0) & (pz >= 0) & (area0.abs() > K_EPS)[:, None, None]
        pz = torch.where(ok, pz, torch.full_like(pz, float("inf")))
        zmin, arg = pz.min(0)  # lowest index among equal z within the chunk
        take = zmin < best_z
        best_z = torch.where(take, zmin, best_z)
        best_f = torch.where(take, arg + f0, best_f)
    hit = best_f >= 0
    f = best_f.clamp(min=0)
    v0, v1, v2 = ndc[faces[f, 0]], ndc[faces[f, 1]], ndc[faces[f, 2]]   # [S, S, 3]

    def e(ax, ay, bx, by):
        return (xf - ax) * (by - ay) - (yf - ay) * (bx - ax)
    area = (v2[..., 0] - v0[..., 0]) * (v1[..., 1] - v0[..., 1]) - \
           (v2[..., 1] - v0[..., 1]) * (v1[..., 0] - v0[..., 0]) + K_EPS
    w0 = e(v1[..., 0], v1[..., 1], v2[..., 0], v2[..., 1]) / area
    w1 = e(v2[..., 0], v2[..., 1], v0[..., 0], v0[..., 1]) / area
    w2 = e(v0[..., 0], v0[..., 1], v1[..., 0], v1[..., 1]) / area
    t0, t1, t2 = w0 * v1[..., 2] * v2[..., 2], v0[..., 2] * w1 * v2[..., 2], v0[..., 2] * v1[..., 2] * w2
    den = torch.clamp(t0 + t1 + t2, min=K_EPS)
    bary = torch.stack([t0 / den, t1 / den, t2 / den], -1)
    z = (bary * torch.stack([v0[..., 2], v1[..., 2], v2[..., 2]], -1)).sum(-1)
    zbuf = torch.where(hit, z, torch.full_like(z, -1.0))
    bary = torch.where(hit[..., None], bary, torch.full_like(bary, -1.0))
    return torch.where(hit, best_f, torch.full_like(best_f, -1)), zbuf, bary


def phong(verts: Tensor, faces: Tensor, normals: Tensor, colors: Tensor, p2f: Tensor, bary: Tensor,
          light: Tensor, cam_center: Tensor, background=(0.5, 0.5, 0.5), shininess: float = 64.0,
          ambient=0.5, diffuse=0.3, specular=0.2) -> Tensor:
    """HardPhongShader + hard_rgb_blend for one image → [S, S, 4] RGBA."""
    hit = p2f >= 0
    f = p2f.clamp(min=0)

    def interp(attr):
        a = attr[faces[f]]                      # [S, S, 3 corners, C]
        return (bary[..., :, None] * a).sum(-2)
    pts, nrm, tex = interp(verts), interp(normals), interp(colors)
    n = F.normalize(nrm, eps=1e-6, dim=-1)
    d = F.normalize(light[None, None] - pts, eps=1e-6, dim=-1)
    cos = (n * d).sum(-1)
    dif = diffuse * torch.relu(cos)
    view = F.normalize(cam_center[None, None] - pts, eps=1e-6, dim=-1)
    refl = -d + 2 * (cos[..., None] * n)
    spec_a = torch.relu((view * refl).sum(-1)) * (cos > 0).to(pts)
    spec = specular * spec_a ** shininess
    rgb = (ambient + dif)[..., None] * tex + spec[..., None]
    bg = torch.tensor(background, dtype=rgb.dtype)
    rgb = torch.where(hit[..., None], rgb, bg.expand_as(rgb))
    return torch.cat([rgb, hit[..., None].to(rgb)], -1)


def light_location(verts: Sequence[Tensor], R: Tensor, t: Tensor, light=(True, True)) -> Tensor:
    """[N, 3] PointLights location of Renderer.forward (:209-230) for ``light`` = (seperate_lights,
    default_lights): R_i·(0, 0, max(min_z_i − 400, 0)) (seperate); pytorch3d's default (0, 1, 0)
    (default colours, one light); R_i·(0, 0, znear/4), znear = ⌊batch min z / 100⌋·100 (ITODD)."""
    seps, deflt = light
    zmin = torch.stack([(v.to(R.dtype) @ R[i].T + t[i][None])[:, 2].min() for i, v in enumerate(verts)])
    zero = torch.zeros_like(zmin)
    if seps:
        lz = torch.clamp(zmin - 400, min=0)
    elif deflt:
        return torch.tensor([0.0, 1.0, 0.0], dtype=R.dtype).expand(len(verts), 3).clone()
    else:
        lz = (torch.floor(zmin.min() / 100) * 100 / 4).expand_as(zmin)
    return (R @ torch.stack([zero, zero, lz], -1)[..., None])[..., 0]


def render(meshes: Dict[int, Tuple[Tensor, Tensor, Tensor]], R: Tensor, t: Tensor, K: Tensor,
           labels: Sequence[int], S: int, light=(True, True)):
    """Renderer.forward for a batch: meshes[label] = (verts [V,3], faces [F,3], colors [V,3]).
    ``light`` = (seperate_lights, default_lights) (:209-230).  Returns images [N, S, S, 4],
    zbuf [N, S, S], pix_to_face [N, S, S] (packed over the batch, −1 empty), bary [N, S, S, 3]."""
    seps, deflt = light
    imgs, zbufs, p2fs, barys = [], [], [], []
    offset = 0
    lights = light_location([meshes[int(lab)][0] for lab in labels], R, t, light)
    for i, lab in enumerate(labels):
        verts, faces, colors = meshes[int(lab)]
        dt = verts.dtype
        Ri, ti, Ki = R[i].to(dt), t[i].to(dt), K[i].to(dt)
        ndc = project_ndc(verts, Ri, ti, Ki, S)
        p2f, zbuf, bary = rasterize(ndc, faces, S)
        light_loc = lights[i].to(dt)
        cols = dict(ambient=0.5, diffuse=0.3, specular=0.2) if deflt else \
            dict(ambient=0.8, diffuse=0.5, specular=1.0)
        cam_center = -Ri.T @ ti
        img = phong(verts, faces, verts_normals(verts, faces), colors, p2f, bary, light_loc,
                    cam_center, **cols)
        imgs.append(img)
        zbufs.append(zbuf)
        p2fs.append(torch.where(p2f >= 0, p2f + offset, p2f))
        barys.append(bary)
        offset += faces.shape[0]
    return torch.stack(imgs), torch.stack(zbufs), torch.stack(p2fs), torch.stack(barys)
