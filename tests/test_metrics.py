"""CPU: the ADD / ADD-S / reprojection metric core (scflow_amd/metrics.py) against the numpy
restatement of the reference's ``eval_pose_error`` and class-wise precision
(oracle/metrics_oracle.py), on synthetic poses with the symmetric YCB-V classes included."""
import numpy as np
import pytest
import torch

mo = pytest.importorskip("oracle.metrics_oracle")


def test_pose_errors_and_precision_match_reference_arithmetic():
    from scflow_amd import metrics, synthetic
    rng = np.random.default_rng(0)
    n, C = 40, 21
    sc = synthetic.make_scene(n, 256, seed=3)
    labels = rng.choice([0, 4, 12, 15, 18, 20], n)
    tgt = synthetic.make_train_targets({**sc, "labels": labels}, 256, seed=3)
    pts = [rng.standard_normal((300, 3)) * 40 for _ in range(C)]
    diam = np.asarray(synthetic.YCBV_DIAMETERS)
    sym_labels = (12, 15, 18)
    ref = mo.eval_pose_error(pts, tgt["gt_translation"].astype(np.float64),
                             tgt["gt_rotation"].astype(np.float64),
                             sc["ref_translation"].astype(np.float64),
                             sc["ref_rotation"].astype(np.float64), labels,
                             sc["internel_k"].astype(np.float64),
                             {f"cls_{c + 1}": True for c in sym_labels}, diam)
    T = lambda a: torch.from_numpy(np.asarray(a, np.float64))  # noqa: E731
    got = metrics.pose_errors([T(p) for p in pts], T(tgt["gt_rotation"]), T(tgt["gt_translation"]),
                              T(sc["ref_rotation"]), T(sc["ref_translation"]), torch.from_numpy(labels),
                              T(sc["internel_k"]), sym_labels, diam)
    np.testing.assert_allclose(got["add"].numpy(), ref[0], rtol=1e-10)
    np.testing.assert_allclose(got["rep"].numpy(), ref[1], rtol=1e-10)
    np.testing.assert_allclose(got["add_mm"].numpy(), ref[2], rtol=1e-10)
    names = [f"cls_{c + 1}" for c in range(C)]
    thr = [0.05, 0.10, 0.20, 0.50]
    pc, avg = metrics.classwise_precision(got["add"], torch.from_numpy(labels), thr, names)
    rpc, ravg = mo.precision(ref[0], labels, thr, names)
    for k in names:
        np.testing.assert_allclose(pc[k], rpc[k])
    np.testing.assert_allclose(avg, ravg)
    # ADD-S ≤ ADD for the symmetric classes
    add_plain = metrics.pose_errors([T(p) for p in pts], T(tgt["gt_rotation"]), T(tgt["gt_translation"]),
                                    T(sc["ref_rotation"]), T(sc["ref_translation"]),
                                    torch.from_numpy(labels), T(sc["internel_k"]), (), diam)["add"]
    s = np.isin(labels, sym_labels)
    assert (got["add"].numpy()[s] <= add_plain.numpy()[s] + 1e-12).all()
