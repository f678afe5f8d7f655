"""Mesh renderer: the reference's ``Renderer`` (models/utils/rendering.py:
77-248) with pytorch3d's rasteriser + hard Phong shader replaced by ``scflow_render`` (HIP,
scflow_amd/csrc/render.hip).

Same constructor keywords and ``forward(rotations, translations, internel_k, labels)`` →
``dict(images=[N, H, W, 4], fragments=Fragments(pix_to_face, zbuf, bary_coords, dists))`` with
pytorch3d's shapes (``[N, H, W, 1]``, ``[N, H, W, 1, 3]``) and values (zbuf = view depth, −1
where empty; pix_to_face indexes the batch's packed faces).  Meshes are read from
``mesh_dir`` (``*.ply`` / ``*.obj``; label from the file name ``obj_XXXXXX`` or
``label_obj_id_map``) or passed in as ``meshes={label: (verts, faces, colors)}``.

Supported configuration = what SCFlow uses (scflow_ycbv_real.py:261-274): Phong shading, hard
blending, faces_per_pixel 1, blur_radius 0, square images, all four light placements
(default/separate lights).  Soft blending and the silhouette (mask) renderer raise
NotImplementedError.  ``dists`` is not computed (None): nothing on the SCFlow path reads it.
"""
from __future__ import annotations

import glob
import os
import struct
from typing import Dict, NamedTuple, Optional, Sequence, Tuple

import numpy as np
import torch
from torch import nn

from . import _lib
from ._lib import ScflowError, check

Tensor = torch.Tensor


class Fragments(NamedTuple):
    pix_to_face: Tensor   # [N, H, W, 1] long, −1 empty
    zbuf: Tensor          # [N, H, W, 1], −1 empty
    bary_coords: Tensor   # [N, H, W, 1, 3], −1 empty
    dists: Optional[Tensor]


# ----------------------------------------------------------------------------------- mesh I/O
_PLY_TYPES = {"char": "b", "int8": "b", "uchar": "B", "uint8": "B", "short": "h", "int16": "h",
              "ushort": "H", "uint16": "H", "int": "i", "int32": "i", "uint": "I", "uint32": "I",
              "float": "f", "float32": "f", "double": "d", "float64": "d"}


def load_ply(path: str) -> Tuple[np.ndarray, np.ndarray, Optional[np.ndarray]]:
    """ASCII / binary PLY → (verts [V,3] float32, faces [F,3] int64, colors [V,3] float32 in
    [0, 1] or None).  Polygons are fanned into triangles."""
    with open(path, "rb") as f:
        if f.readline().strip() != b"ply":
            raise ValueError(f"{path}: not a PLY file")
        fmt, elements = None, []
        while True:
            line = f.readline()
            if not line:
                raise ValueError(f"{path}: truncated header")
            tok = line.decode("ascii", "replace").split()
            if not tok:
                continue
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "element":
                elements.append((tok[1], int(tok[2]), []))
            elif tok[0] == "property":
                if tok[1] == "list":
                    elements[-1][2].append((tok[4], ("list", tok[2], tok[3])))
                else:
                    elements[-1][2].append((tok[2], tok[1]))
            elif tok[0] == "end_header":
                break
        data = {}
        if fmt == "ascii":
            rest = f.read().decode("ascii").split()
            pos = 0
            for name, count, props in elements:
                rows = []
                for _ in range(count):
                    row = {}
                    for pname, ptype in props:
                        if isinstance(ptype, tuple):
                            n = int(rest[pos])
                            row[pname] = [float(x) for x in rest[pos + 1:pos + 1 + n]]
                            pos += 1 + n
                        else:
                            row[pname] = float(rest[pos])
                            pos += 1
                    rows.append(row)
                data[name] = rows
        elif fmt in ("binary_little_endian", "binary_big_endian"):
            end = "<" if fmt == "binary_little_endian" else ">"
            buf = f.read()
            pos = 0
            for name, count, props in elements:
                if all(not isinstance(t, tuple) for _, t in props):  # fixed-size rows: vectorised
                    dtype = np.dtype([(pn, end + _PLY_TYPES[pt]) for pn, pt in props])
                    arr = np.frombuffer(buf, dtype=dtype, count=count, offset=pos)
                    pos += dtype.itemsize * count
                    data[name] = arr
                    continue
                rows = []
                for _ in range(count):
                    row = {}
                    for pname, ptype in props:
                        if isinstance(ptype, tuple):
                            cf, vf = _PLY_TYPES[ptype[1]], _PLY_TYPES[ptype[2]]
                            (n,) = struct.unpack_from(end + cf, buf, pos)
                            pos += struct.calcsize(cf)
                            row[pname] = list(struct.unpack_from(end + vf * n, buf, pos))
                            pos += struct.calcsize(vf) * n
                        else:
                            (row[pname],) = struct.unpack_from(end + _PLY_TYPES[ptype], buf, pos)
                            pos += struct.calcsize(_PLY_TYPES[ptype])
                    rows.append(row)
                data[name] = rows
        else:
            raise ValueError(f"{path}: unsupported PLY format {fmt}")
    vert = data["vertex"]

    def col(name):
        if isinstance(vert, np.ndarray):
            return np.asarray(vert[name], np.float64)
        return np.asarray([r[name] for r in vert], np.float64)
    verts = np.stack([col("x"), col("y"), col("z")], 1).astype(np.float32)
    vprops = [p for p, _ in next(e for e in elements if e[0] == "vertex")[2]]
    colors = None
    if all(c in vprops for c in ("red", "green", "blue")):
        ctype = dict(next(e for e in elements if e[0] == "vertex")[2])["red"]
        scale = 255.0 if ctype in ("uchar", "uint8") else 1.0
        colors = (np.stack([col("red"), col("green"), col("blue")], 1) / scale).astype(np.float32)
    faces = []
    frows = data.get("face", [])
    key = None
    for name, ptype in next((e for e in elements if e[0] == "face"), ("face", 0, []))[2]:
        if isinstance(ptype, tuple) and name in ("vertex_indices", "vertex_index"):
            key = name
    for row in frows:
        idx = [int(i) for i in row[key]]
        for k in range(1, len(idx) - 1):
            faces.append((idx[0], idx[k], idx[k + 1]))
    return verts, np.asarray(faces, np.int64).reshape(-1, 3), colors


def save_ply(path: str, verts: np.ndarray, faces: np.ndarray, colors: Optional[np.ndarray] = None,
             binary: bool = True) -> None:
    """Write a triangle mesh (vertex colours as uchar) — test fixtures and synthetic models."""
    verts = np.asarray(verts, np.float32)
    faces = np.asarray(faces, np.int32)
    head = ["ply", f"format {'binary_little_endian' if binary else 'ascii'} 1.0",
            f"element vertex {len(verts)}", "property float x", "property float y", "property float z"]
    if colors is not None:
        head += ["property uchar red", "property uchar green", "property uchar blue"]
        c8 = np.clip(np.round(np.asarray(colors) * 255.0), 0, 255).astype(np.uint8)
    head += [f"element face {len(faces)}", "property list uchar int vertex_indices", "end_header"]
    with open(path, "wb") as f:
        f.write(("\n".join(head) + "\n").encode("ascii"))
        if binary:
            vd = [("x", "<f4"), ("y", "<f4"), ("z", "<f4")]
            if colors is not None:
                vd += [("r", "u1"), ("g", "u1"), ("b", "u1")]
            va = np.empty(len(verts), dtype=vd)
            va["x"], va["y"], va["z"] = verts[:, 0], verts[:, 1], verts[:, 2]
            if colors is not None:
                va["r"], va["g"], va["b"] = c8[:, 0], c8[:, 1], c8[:, 2]
            f.write(va.tobytes())
            fa = np.empty(len(faces), dtype=[("n", "u1"), ("i", "<i4", (3,))])
            fa["n"] = 3
            fa["i"] = faces
            f.write(fa.tobytes())
        else:
            for i, v in enumerate(verts):
                extra = "" if colors is None else " " + " ".join(str(int(x)) for x in c8[i])
                f.write(f"{v[0]:.9g} {v[1]:.9g} {v[2]:.9g}{extra}\n".encode("ascii"))
            for fc in faces:
                f.write(f"3 {fc[0]} {fc[1]} {fc[2]}\n".encode("ascii"))


def load_obj(path: str) -> Tuple[np.ndarray, np.ndarray, Optional[np.ndarray]]:
    """Minimal OBJ reader (v, optional per-vertex rgb after xyz, f with fan triangulation)."""
    verts, cols, faces = [], [], []
    with open(path) as f:
        for line in f:
            tok = line.split()
            if not tok:
                continue
            if tok[0] == "v":
                verts.append([float(x) for x in tok[1:4]])
                if len(tok) >= 7:
                    cols.append([float(x) for x in tok[4:7]])
            elif tok[0] == "f":
                idx = [int(x.split("/")[0]) - 1 for x in tok[1:]]
                for k in range(1, len(idx) - 1):
                    faces.append((idx[0], idx[k], idx[k + 1]))
    colors = np.asarray(cols, np.float32) if len(cols) == len(verts) and cols else None
    return np.asarray(verts, np.float32), np.asarray(faces, np.int64).reshape(-1, 3), colors


def verts_normals(verts: Tensor, faces: Tensor) -> Tensor:
    """pytorch3d ``Meshes.verts_normals_packed``: per-corner area-weighted face normals summed
    per vertex, normalised (eps 1e-6).  Once per mesh at load time."""
    v0, v1, v2 = verts[faces[:, 0]], verts[faces[:, 1]], verts[faces[:, 2]]
    n = torch.zeros_like(verts)
    n.index_add_(0, faces[:, 1], torch.cross(v2 - v1, v0 - v1, dim=1))
    n.index_add_(0, faces[:, 2], torch.cross(v0 - v2, v1 - v2, dim=1))
    n.index_add_(0, faces[:, 0], torch.cross(v1 - v0, v2 - v0, dim=1))
    return torch.nn.functional.normalize(n, eps=1e-6, dim=1)


# ----------------------------------------------------------------------------------- cameras
class PerspectiveCameraParams(NamedTuple):
    """The keyword arguments the reference hands pytorch3d's ``PerspectiveCameras``."""
    R: Tensor                # [N, 3, 3] (row-vector convention: X_view = X_world·R + T)
    T: Tensor                # [N, 3]
    focal_length: Tensor     # [N, 2] NDC units
    principal_point: Tensor  # [N, 2] NDC units
    image_size: Tensor       # [N, 2] (H, W)


def cameras_from_opencv_projection(R: Tensor, tvec: Tensor, camera_matrix: Tensor,
                                   image_size: Tensor) -> PerspectiveCameraParams:
    """rendering.py:17-60: OpenCV (R, t, K) → pytorch3d's NDC camera — transposed R with its
    first two columns negated, t with x, y negated, focal / principal point scaled by
    (min(H, W) − 1)/2 around the image centre.  scflow_render projects with (R, t, K) directly;
    both conventions put a vertex at the same NDC point (tests/test_render_wiring.py)."""
    focal = torch.stack([camera_matrix[:, 0, 0], camera_matrix[:, 1, 1]], dim=-1)
    pp = camera_matrix[:, :2, 2]
    wh = image_size.to(R).flip(dims=(1,))
    scale = ((wh.min(dim=1, keepdim=True)[0] - 1) / 2.0).expand(-1, 2)
    c0 = (wh - 1) / 2.0
    Rp = R.clone().permute(0, 2, 1)
    Tp = tvec.clone()
    Rp[:, :, :2] = Rp[:, :, :2] * -1
    Tp[:, :2] = Tp[:, :2] * -1
    return PerspectiveCameraParams(Rp, Tp, focal / scale, -(pp - c0) / scale, image_size)


def depth_range(rotations: Tensor, translations: Tensor, verts: Sequence[Tensor]) -> Tuple[Tensor, Tensor]:
    """(znear, zfar) of Renderer.forward (:193-199): the batch's vertex view depths, rounded down
    / up to 100 mm — as device tensors (the reference calls .item(); no host sync here)."""
    z = torch.cat([(R[2:3] @ v.T.to(R) + t[2]).reshape(-1)
                   for R, t, v in zip(rotations, translations, verts)])
    return torch.floor(z.min() / 100) * 100, (torch.floor(z.max() / 100) + 1) * 100


# ----------------------------------------------------------------------------------- renderer
class Renderer(nn.Module):
    """models/utils/rendering.py:77-248 on the HIP rasteriser."""

    def __init__(self, mesh_dir: Optional[str] = None, image_size=(256, 256), shader_type: str = "Phong",
                 soft_blending: bool = True, render_mask: bool = True, render_image: bool = True,
                 faces_per_pixel: int = 1, blur_radius: float = 0., sigma: float = 1e-4,
                 gamma: float = 1e-4, bin_size=None, default_lights: bool = True,
                 seperate_lights: bool = False, background_color=(0.5, 0.5, 0.5),
                 obj_label_in_file: bool = True, label_obj_id_map=None, mesh_ext: str = "ply",
                 meshes: Optional[Dict[int, Tuple]] = None) -> None:
        super().__init__()
        if shader_type != "Phong":
            raise NotImplementedError(f"shader {shader_type}: the HIP renderer implements Phong "
                                      "(the configured shader, scflow_ycbv_real.py:263)")
        if soft_blending or render_mask:
            raise NotImplementedError("soft blending / silhouette masks: the configured renderer is "
                                      "hard Phong with render_mask=False (scflow_ycbv_real.py:264-265)")
        if faces_per_pixel != 1 or blur_radius != 0:
            raise NotImplementedError("faces_per_pixel=1 and blur_radius=0 only")
        h, w = (image_size, image_size) if isinstance(image_size, int) else tuple(image_size)
        if h != w:
            raise NotImplementedError("square images only (SCFlow crops square patches)")
        self.image_size = (h, w)
        self.render_image = render_image
        self.render_mask = render_mask
        self.default_lights = default_lights
        self.seperate_lights = seperate_lights
        self.background_color = tuple(float(x) for x in background_color)
        self.obj_label_in_file = obj_label_in_file
        self.label_obj_id_map = label_obj_id_map
        self.mesh_ext = mesh_ext
        self.meshes: Dict[int, Tuple[Tensor, Tensor, Tensor, Tensor]] = {}
        if meshes is not None:
            for lab, m in meshes.items():
                self.add_mesh(int(lab), *m)
        if mesh_dir is not None:
            self.load_meshes(mesh_dir)
        self._device = torch.device("cpu")

    # mesh registry
    def add_mesh(self, label: int, verts, faces, colors=None) -> None:
        v = torch.as_tensor(np.asarray(verts), dtype=torch.float32)
        f = torch.as_tensor(np.asarray(faces), dtype=torch.long)
        c = (torch.full_like(v, 1.0) if colors is None
             else torch.as_tensor(np.asarray(colors), dtype=torch.float32))
        self.meshes[label] = (v, f, c, verts_normals(v.double(), f).float())

    def load_meshes(self, mesh_dir: str) -> None:
        """Renderer.load_meshes (:138-153): label = trailing integer of the file name − 1, or
        ``label_obj_id_map[name]``."""
        if not self.obj_label_in_file and self.label_obj_id_map is None:
            raise ValueError("label_obj_id_map is required when obj_label_in_file=False")
        paths = sorted(glob.glob(os.path.join(mesh_dir, "*." + self.mesh_ext))) if os.path.isdir(mesh_dir) \
            else [mesh_dir]
        for p in paths:
            stem = os.path.basename(p).split(".")[0]
            label = (int(stem.split("_")[-1]) - 1) if self.obj_label_in_file else self.label_obj_id_map[stem]
            v, f, c = load_ply(p) if p.endswith(".ply") else load_obj(p)
            self.add_mesh(label, v, f, c)

    def to(self, device):  # the reference's Renderer.to moves the meshes (:132-136)
        device = torch.device(device)
        self._device = device
        self.meshes = {k: tuple(x.to(device) for x in m) for k, m in self.meshes.items()}
        return self

    def forward(self, rotations: Tensor, translations: Tensor, internel_k: Tensor, labels: Tensor):
        if not (rotations.shape[0] == translations.shape[0] == internel_k.shape[0] == labels.shape[0]):
            raise ValueError("batch sizes differ")
        dev = rotations.device
        if dev.type != "cuda":
            raise ScflowError("the HIP renderer needs ROCm device tensors")
        n = rotations.shape[0]
        S = self.image_size[0]
        labs = labels.tolist()  # mesh selection is host-side, as in the reference (:198)
        ms = []
        for lab in labs:
            if lab not in self.meshes:
                raise KeyError(f"no mesh for label {lab}")
            m = self.meshes[lab]
            if m[0].device != dev:
                m = tuple(x.to(dev) for x in m)
                self.meshes[lab] = m
            ms.append(m)
        nv = [m[0].shape[0] for m in ms]
        nf = [m[1].shape[0] for m in ms]
        voff = np.concatenate([[0], np.cumsum(nv)[:-1]]).tolist()
        verts = torch.cat([m[0] for m in ms]).contiguous()
        colors = torch.cat([m[2] for m in ms]).contiguous()
        normals = torch.cat([m[3] for m in ms]).contiguous()
        faces = torch.cat([m[1] + o for m, o in zip(ms, voff)]).to(torch.int32).contiguous()
        ids = torch.arange(n, device=dev, dtype=torch.int32)
        vert_img = torch.repeat_interleave(ids, torch.tensor(nv, device=dev)).contiguous()
        face_img = torch.repeat_interleave(ids, torch.tensor(nf, device=dev)).contiguous()
        R = rotations.float().contiguous()
        t = translations.float().contiguous()
        K = internel_k.float().contiguous()
        lib = _lib.load()
        ws = torch.empty(int(lib.scflow_render_workspace(n, S, verts.shape[0])), dtype=torch.uint8,
                         device=dev)
        # light placement and colours (:209-230; pytorch3d PointLights defaults)
        if self.default_lights:
            amb, dif, spe = (0.5,) * 3, (0.3,) * 3, (0.2,) * 3
            mode = _lib.SCFLOW_LIGHT_PER_IMAGE if self.seperate_lights else _lib.SCFLOW_LIGHT_FIXED
        else:
            amb, dif, spe = (0.8,) * 3, (0.5,) * 3, (1.0,) * 3
            mode = _lib.SCFLOW_LIGHT_PER_IMAGE if self.seperate_lights else _lib.SCFLOW_LIGHT_BATCH_ZNEAR
        params = torch.tensor([*amb, *dif, *spe, *self.background_color, 0.0, 1.0, 0.0],
                              dtype=torch.float32, device=dev)
        images = torch.empty(n, S, S, 4, device=dev) if self.render_image else None
        zbuf = torch.empty(n, S, S, 1, device=dev)
        p2f = torch.empty(n, S, S, 1, device=dev, dtype=torch.int32)
        bary = torch.empty(n, S, S, 1, 3, device=dev)
        light = torch.empty(n, 3, device=dev)
        a = _lib.RenderArgs()
        a.verts, a.normals, a.colors, a.faces = (verts.data_ptr(), normals.data_ptr(), colors.data_ptr(),
                                                 faces.data_ptr())
        a.vert_img, a.face_img = vert_img.data_ptr(), face_img.data_ptr()
        a.R, a.t, a.K = R.data_ptr(), t.data_ptr(), K.data_ptr()
        a.n_img, a.size, a.total_verts, a.total_faces = n, S, verts.shape[0], faces.shape[0]
        a.light_mode = mode
        base = params.data_ptr()
        a.ambient, a.diffuse, a.specular, a.background = base, base + 12, base + 24, base + 36
        a.light_location = base + 48  # pytorch3d PointLights default location (0, 1, 0)
        a.shininess = 64.0
        a.images = 0 if images is None else images.data_ptr()
        a.zbuf, a.pix_to_face, a.bary = zbuf.data_ptr(), p2f.data_ptr(), bary.data_ptr()
        a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel()
        a.light_out = light.data_ptr()
        import ctypes
        check(lib.scflow_render(ctypes.byref(a), torch.cuda.current_stream(dev).cuda_stream),
              "scflow_render")
        frags = Fragments(pix_to_face=p2f.long(), zbuf=zbuf, bary_coords=bary, dists=None)
        # extension: the light location each image was shaded with (the reference builds it into
        # its PointLights, :209-230)
        out = {"fragments": frags, "light_location": light}
        if images is not None:
            out["images"] = images
        return out
