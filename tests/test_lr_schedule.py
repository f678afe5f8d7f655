"""The training step's OneCycleLR (configs/refine_models/scflow_ycbv_real.py:299-306) against
torch.optim.lr_scheduler.OneCycleLR with the same arguments (momentum cycling off: mmengine's
OneCycleLR schedules ``lr`` only).  CPU only."""
import math

import pytest
import torch

from scflow_amd.train.schedule import OneCycleLR, reference_schedule


def _torch_lrs(steps, **kw):
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.AdamW([p], lr=kw["max_lr"])
    sch = torch.optim.lr_scheduler.OneCycleLR(opt, cycle_momentum=False, **kw)
    out = {}
    for k in range(max(steps) + 1):
        if k in steps:
            out[k] = opt.param_groups[0]["lr"]
        opt.step()
        sch.step()
    return out


def test_reference_schedule_matches_torch_first_6000_and_end():
    ours = reference_schedule(4e-4)
    check = set(range(0, 6001)) | set(range(100000, 100100))
    ref = _torch_lrs(check, max_lr=4e-4, total_steps=100100, pct_start=0.05,
                     anneal_strategy="linear")
    for k in sorted(check):
        assert math.isclose(ours.lr_at(k), ref[k], rel_tol=1e-12, abs_tol=1e-18), (k, ours.lr_at(k), ref[k])
    assert math.isclose(ours.lr_at(0), 4e-4 / 25)
    assert math.isclose(ours.lr_at(5004), 4e-4)  # pct_start·total − 1: the peak
    assert math.isclose(ours.lr_at(100099), 4e-4 / 25 / 1e4)


@pytest.mark.parametrize("kw", [dict(total_steps=37, pct_start=0.3, anneal_strategy="cos"),
                                dict(total_steps=50, pct_start=0.25, anneal_strategy="linear",
                                     three_phase=True, div_factor=10.0, final_div_factor=100.0)])
def test_small_schedules_match_torch(kw):
    ours = OneCycleLR(1e-3, **kw)
    ref = _torch_lrs(set(range(kw["total_steps"])), max_lr=1e-3, **kw)
    for k, v in ref.items():
        assert math.isclose(ours.lr_at(k), v, rel_tol=1e-12, abs_tol=1e-18), (k, ours.lr_at(k), v)


def test_out_of_range_and_bad_args():
    s = OneCycleLR(1e-3, 10, anneal_strategy="linear")
    with pytest.raises(ValueError):
        s.lr_at(-1)
    for k in (10, 11, 10 ** 6):  # past the end: clamped at the minimum, never negative
        assert s.lr_at(k) == s.lr_at(9) and math.isclose(s.lr_at(k), s.min_lr, rel_tol=1e-9)
    with pytest.raises(ValueError):
        OneCycleLR(1e-3, 10, anneal_strategy="step")
    with pytest.raises(ValueError):
        OneCycleLR(1e-3, 0)
