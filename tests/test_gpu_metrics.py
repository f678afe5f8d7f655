"""GPU: the metric core runs on device tensors and equals its CPU evaluation."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_pose_errors_on_device():
    from scflow_amd import metrics, synthetic
    rng = np.random.default_rng(1)
    n = 64
    sc = synthetic.make_scene(n, 256, seed=4)
    labels = torch.from_numpy(rng.choice([1, 12, 18], n))
    tgt = synthetic.make_train_targets({**sc, "labels": labels.numpy()}, 256, seed=4)
    pts = [torch.from_numpy(rng.standard_normal((1000, 3)) * 40).float() for _ in range(21)]
    args = [torch.from_numpy(x) for x in (tgt["gt_rotation"], tgt["gt_translation"],
                                          sc["ref_rotation"], sc["ref_translation"])]
    K = torch.from_numpy(sc["internel_k"])
    cpu = metrics.pose_errors(pts, *args, labels, K, (12, 18), synthetic.YCBV_DIAMETERS)
    gpu = metrics.pose_errors([p.cuda() for p in pts], *(a.cuda() for a in args), labels.cuda(), K.cuda(),
                              (12, 18), synthetic.YCBV_DIAMETERS)
    for k in cpu:
        np.testing.assert_allclose(gpu[k].cpu().numpy(), cpu[k].numpy(), rtol=1e-4, atol=1e-4)
