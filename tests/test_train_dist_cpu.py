"""CPU, world_size 2 over gloo: the training step's data-parallel gradient exchange
(scflow_amd/train/step.py GradBuckets — flat buckets, all-reduce issued from post-accumulate
hooks during backward, then clip + AdamW) gives every rank the single-process full-batch
gradients and, after a few optimizer steps, the same weights as one process on the whole batch."""
import os
import socket

import pytest

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3, padding=1), torch.nn.ReLU(),
                               torch.nn.Conv2d(16, 16, 3, padding=1), torch.nn.ReLU(),
                               torch.nn.Flatten(), torch.nn.Linear(16 * 8 * 8, 10))


def _data():
    g = torch.Generator().manual_seed(1)
    return torch.randn(8, 3, 8, 8, generator=g), torch.randn(8, 10, generator=g)


def _run(rank, world, steps, max_norm, overlap=True):
    from scflow_amd.train.step import GradBuckets
    m = _model().double()
    x, y = _data()
    x, y = x.double(), y.double()
    if world > 1:
        n = x.shape[0] // world
        x, y = x[rank * n:(rank + 1) * n], y[rank * n:(rank + 1) * n]
    gb = GradBuckets(list(m.parameters()), bucket_bytes=8 << 10, overlap=overlap)  # several buckets
    opt = torch.optim.AdamW(gb.params, lr=1e-2, weight_decay=1e-4, foreach=True)
    hooked = []
    for _ in range(steps):
        gb.zero()
        loss = ((m(x) - y) ** 2).mean()
        loss.backward()
        hooked.append(sum(w is not None for w in gb._work))
        gb.finish()
        first_grads = [p.grad.clone() for p in m.parameters()] if not hooked[1:] else first_grads
        gb.clip_(max_norm)
        opt.step()
    return [p.detach().clone() for p in m.parameters()], first_grads, hooked, len(gb.buckets)


def _worker(rank, world, port, q, overlap):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        w, g, hooked, nb = _run(rank, world, 3, 0.5, overlap)
        q.put((rank, ([a.numpy() for a in w], [a.numpy() for a in g], hooked, nb)))  # by value
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [True, False])
def test_bucketed_allreduce_matches_single_process(overlap):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, overlap)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref_w, ref_g, _, nb = _run(0, 1, 3, 0.5)
    assert nb >= 3
    for rank in (0, 1):
        w, g, hooked, _ = res[rank]
        # overlap: every bucket's all-reduce was issued during backward; else all after it
        assert hooked == ([nb] * 3 if overlap else [0] * 3)
        for a, b in zip(g, ref_g):
            torch.testing.assert_close(torch.from_numpy(a), b, rtol=1e-12, atol=1e-14)
        for a, b in zip(w, ref_w):
            torch.testing.assert_close(torch.from_numpy(a), b, rtol=1e-10, atol=1e-12)


def test_clip_matches_torch():
    from scflow_amd.train.step import GradBuckets
    m = _model().double()
    x, y = _data()
    gb = GradBuckets(list(m.parameters()), bucket_bytes=4 << 10)
    gb.zero()
    ((m(x.double()) - y.double()) ** 2).sum().backward()
    ref = [p.grad.clone() for p in m.parameters()]
    total = gb.clip_(1.0)
    m2 = _model().double()
    for p, g in zip(m2.parameters(), ref):
        p.grad = g.clone()
    t2 = torch.nn.utils.clip_grad_norm_(m2.parameters(), 1.0)
    torch.testing.assert_close(total, t2)
    for p, q in zip(m.parameters(), m2.parameters()):
        torch.testing.assert_close(p.grad, q.grad)
