"""BOP-format ADD evaluation (scflow_amd/bop_eval.py) on a synthetic BOP tree: annotation loading,
prediction↔GT matching (single / duplicate / missing predictions), ADD(-S) class-wise precision
and the flat metric dict, against a numpy restatement of the reference's metrics/add.py logic
written independently here; plus the scene_gt.json dump round trip.  (The reference's own ADD
metric pins the same functions in tests/test_metric_golden.py.)"""
import json
import os

import numpy as np
import pytest

from scflow_amd import bop_eval


def _rot(rng):
    q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
    return (q * np.sign(np.linalg.det(q))).astype(np.float32)


def _ref_errors(points, gR, gT, pR, pT, labels, K, sym, diam):
    """add.py:354-400 restated in numpy (float64)."""
    add = np.zeros(len(labels))
    rep = np.zeros(len(labels))
    for i in range(len(labels)):
        l = labels[i]
        P = points[l].astype(np.float64)
        g3 = P @ gR[i].T.astype(np.float64) + gT[i]
        p3 = P @ pR[i].T.astype(np.float64) + pT[i]
        g2 = g3 @ K[i].T.astype(np.float64)
        p2 = p3 @ K[i].T.astype(np.float64)
        g2 = g2[:, :2] / (g2[:, 2:] + 1e-8)
        p2 = p2[:, :2] / (p2[:, 2:] + 1e-8)
        if l in sym:
            d = np.linalg.norm(g3[:, None] - p3[None], axis=-1)
            p3 = p3[d.argmin(-1)]
        add[i] = np.linalg.norm(g3 - p3, axis=-1).mean() / diam[l]
        rep[i] = np.linalg.norm(g2 - p2, axis=-1).mean()
    return add, rep


@pytest.fixture
def bop_tree(tmp_path):
    rng = np.random.default_rng(3)
    C = 4
    points = [rng.standard_normal((200, 3)).astype(np.float32) * 40 for _ in range(C)]
    diam = [120.0, 90.0, 150.0, 60.0]
    sym = [2]
    K = [[600.0, 0, 320], [0, 600.0, 240], [0, 0, 1]]
    results, gt = [], {}
    for seq in (48, 51):
        scene_gt, scene_cam = {}, {}
        for img in range(3):
            objs, preds_l, preds_r, preds_t = [], [], [], []
            for oid in rng.choice(np.arange(1, C + 1), size=2, replace=False):
                R, t = _rot(rng), np.array([rng.normal() * 50, rng.normal() * 50, 700 + 100 * rng.random()],
                                           np.float32)
                objs.append(dict(obj_id=int(oid), cam_R_m2c=R.reshape(-1).tolist(), cam_t_m2c=t.tolist()))
                mode = rng.integers(0, 4)
                if mode == 3:   # missed object
                    continue
                n = 2 if mode == 2 else 1  # duplicates: a far one and a close one
                for k in range(n):
                    noise = 0.5 if k == n - 1 else 40.0
                    preds_l.append(int(oid) - 1)
                    preds_r.append(R if mode == 0 else _rot(rng) if k == 0 and n == 2 else R)
                    preds_t.append(t + rng.normal(size=3).astype(np.float32) * noise)
            scene_gt[str(img)] = objs
            scene_cam[str(img)] = dict(cam_K=np.asarray(K).reshape(-1).tolist())
            results.append(dict(img_metas=dict(img_path=f"{tmp_path}/data/{seq:06d}/rgb/{img:06d}.png"),
                                pred=dict(labels=np.asarray(preds_l, np.int64),
                                          rotations=np.asarray(preds_r, np.float32).reshape(-1, 3, 3),
                                          translations=np.asarray(preds_t, np.float32).reshape(-1, 3))))
        d = tmp_path / "data" / f"{seq:06d}"
        d.mkdir(parents=True)
        (d / "scene_gt.json").write_text(json.dumps(scene_gt))
        (d / "scene_camera.json").write_text(json.dumps(scene_cam))
        gt[f"{seq:06d}"] = dict(pose=scene_gt, camera=scene_cam)
    return tmp_path, results, gt, points, diam, sym, [f"cls_{i + 1}" for i in range(C)]


def test_load_match_evaluate(bop_tree):
    root, results, gt, points, diam, sym, names = bop_tree
    ann = bop_eval.load_bop_annotations(str(root / "data"), ["000048", "000051"])
    assert ann["000048"]["pose"] == gt["000048"]["pose"]
    flat = bop_eval.evaluate(results, ann, points, names, sym, diam, round_digits=None)
    # the reference's flow restated: matching (min normalised ADD among duplicates), fill values
    # for missing predictions, ADD(-S) precision per class at 5/10/20/50 % of the diameter
    add_all, labels = [], []
    for res in results:
        seq = res["img_metas"]["img_path"].split("/")[-3]
        img = str(int(res["img_metas"]["img_path"].split("/")[-1][:-4]))
        K = np.asarray(gt[seq]["camera"][img]["cam_K"], np.float64).reshape(3, 3)
        pl = res["pred"]["labels"] + 1
        for obj in gt[seq]["pose"][img]:
            oid = obj["obj_id"]
            gR = np.asarray(obj["cam_R_m2c"]).reshape(3, 3)
            gT = np.asarray(obj["cam_t_m2c"])
            labels.append(oid - 1)
            idx = np.nonzero(pl == oid)[0]
            if len(idx) == 0:
                add_all.append(1.0)
                continue
            cand = [_ref_errors(points, [gR], [gT], [res["pred"]["rotations"][j]],
                                [res["pred"]["translations"][j]], [oid - 1], [K], sym, diam)[0][0]
                    for j in idx]
            add_all.append(min(cand))
    add_all, labels = np.asarray(add_all), np.asarray(labels)
    for thr, tag in ((0.05, "05"), (0.10, "10"), (0.20, "20"), (0.50, "50")):
        vals = []
        for c, name in enumerate(names):
            sel = add_all[labels == c]
            v = -1.0 if sel.size == 0 else float((sel < thr).mean())
            assert flat[f"{name}/add_{tag}"] == pytest.approx(v, abs=1e-6), (name, tag)
            if sel.size:
                vals.append(v)
        assert flat[f"average/add_{tag}"] == pytest.approx(sum(vals) / len(vals), abs=1e-6)


def test_parse_error_to_metric_headers_and_absent_class():
    err = {"add": np.array([0.01, 0.3, 0.07]), "rep": np.array([1.0, 9.0, 3.0])}
    labels = np.array([0, 0, 2])
    md, headers = bop_eval.parse_error_to_metric(err, labels, {"auc": [], "add": [0.05, 0.1], "rep": [5]},
                                                 ["a", "b", "c"])
    assert headers == ["class", "add_05", "add_10", "rep_05"]
    assert md["b"] == [-1.0, -1.0, -1.0]
    assert md["a"] == [0.5, 0.5, 0.5]
    assert md["c"] == [0.0, 1.0, 1.0]
    assert md["average"] == pytest.approx([0.25, 0.75, 0.75])


def test_format_results_round_trip(bop_tree, tmp_path):
    root, results, gt, *_ = bop_tree
    paths = bop_eval.format_results(results, str(root / "data"), str(tmp_path / "out"))
    assert len(paths) == 2
    back = json.loads(open(os.path.join(tmp_path, "out", "000048", "scene_gt.json")).read())
    r0 = results[0]["pred"]
    assert [o["obj_id"] for o in back["0"]] == (r0["labels"] + 1).tolist()
    np.testing.assert_allclose(np.asarray(back["0"][0]["cam_t_m2c"]), r0["translations"][0], rtol=1e-6)
