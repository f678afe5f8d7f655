"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

numpy restatement, loop for loop, of the reference's ADD metric core: ``project_3d_point``
(datasets/pose.py:18-75), ``ADD.eval_pose_error`` (metrics/add.py:354-400) and the threshold
branch of ``ADD.parse_error_to_metric`` (:309-330).  The reference itself cannot run here
(mmengine, trimesh, terminaltables absent) and ships no fixtures: parity unpinned beyond this
restatement of its arithmetic.
"""
import numpy as np


def project_3d_point(pt3d, K, rotation, translation):
    cam = np.matmul(rotation, pt3d.transpose()) + translation          # (N, 3, n)
    pts_2d = np.matmul(K, cam).transpose((0, 2, 1))
    pts_2d[..., 0] = pts_2d[..., 0] / (pts_2d[..., -1] + 1e-8)
    pts_2d[..., 1] = pts_2d[..., 1] / (pts_2d[..., -1] + 1e-8)
    return pts_2d[..., :-1], cam.transpose((0, 2, 1))


def eval_pose_error(verts_list, gt_t, gt_r, pred_t, pred_r, labels, k, symmetry_types, mesh_diameters):
    num_pred = len(gt_t)
    e3n, e2, e3 = np.zeros(num_pred), np.zeros(num_pred), np.zeros(num_pred)
    for i in np.unique(labels):
        idx = labels == i
        verts = verts_list[i]
        gt_2d, gt_3d = project_3d_point(verts, k[idx], gt_r[idx], gt_t[idx][..., None])
        pr_2d, pr_3d = project_3d_point(verts, k[idx], pred_r[idx], pred_t[idx][..., None])
        if symmetry_types.get(f"cls_{i + 1}", False):
            lst = []
            for g, p in zip(gt_3d, pr_3d):
                mi = np.argmin(np.linalg.norm(np.expand_dims(g, -2) - np.expand_dims(p, -3), axis=-1), axis=-1)
                lst.append(p[mi])
            pr_3d = np.stack(lst, 0)
        err = np.linalg.norm(gt_3d - pr_3d, axis=-1).mean(axis=-1)
        e3n[idx] = err / mesh_diameters[i]
        e2[idx] = np.linalg.norm(gt_2d - pr_2d, axis=-1).mean(axis=-1)
        e3[idx] = err
    return e3n, e2, e3


def precision(error, labels, thresholds, classnames):
    avg = [[] for _ in thresholds]
    out = {}
    for c in range(len(classnames)):
        e = error[labels == c]
        if e.shape[0] == 0:
            out[classnames[c]] = [-1.0] * len(thresholds)
            continue
        vals = []
        for i, thr in enumerate(thresholds):
            v = (e < thr).sum() / e.shape[0]
            vals.append(v)
            avg[i].append(v)
        out[classnames[c]] = vals
    return out, [sum(p) / len(p) for p in avg]
