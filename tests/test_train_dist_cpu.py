"""CPU, world_size 2 over gloo: the training step's data-parallel gradient exchange
(scflow_amd/train/step.py GradBuckets — flat buckets, all-reduce issued from post-accumulate
hooks during backward, then clip + AdamW) gives every rank the single-process full-batch
gradients and, after a few optimizer steps, the same weights as one process on the whole batch."""
import os
import socket

import numpy as np
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


# --------------------------------------------------------------------------- the real refiner
_ITERS = 1
_LABELS = [12, 4]  # a multi-class batch: the shards' label[0] differ


def _refiner_worker(rank, world, port, q):
    """One replica: GradBuckets over the REAL refiner's de-duplicated parameter list (what
    TrainStep builds), filled with the oracle's fp64 single-process gradients of this rank's shard
    (context-encoder BatchNorm in train mode on the shard, the shard's own label[0]), then the
    bucketed all-reduce + average."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(4)
        from scflow_amd.dist import shard_train_batch
        from scflow_amd.train.step import GradBuckets, trainable_parameters
        from tests.test_train_host import build_train_refiner, oracle_loss_and_grads, train_batch
        r = build_train_refiner(_ITERS, dtype=torch.float64)
        params = trainable_parameters(r)
        name_of = {id(p): n for n, p in r.named_parameters()}
        names = [name_of[id(p)] for p in params]
        gb = GradBuckets(params)  # the default 8 MB buckets, as TrainStep
        batch, points, diam = train_batch(len(_LABELS), 256, seed=9, labels=_LABELS)
        shard = shard_train_batch(batch, rank, world)
        assert "head_label" not in shard
        _, _, _, grads = oracle_loss_and_grads(shard, points, diam, _ITERS, names)
        gb.zero()
        for p, n in zip(params, names):
            if grads[n] is not None:
                p.grad.copy_(grads[n])
        local = [p.grad.clone().numpy() for p in params]
        gb.finish()
        q.put((rank, (names, local, [p.grad.clone().numpy() for p in params], len(gb.buckets))))
    finally:
        dist.destroy_process_group()


def test_grad_buckets_real_refiner_per_replica_bn():
    """configs[3]'s data-parallel exchange on the real model (scflow_refiner.py:182-256,
    train.py:42-45, scflow_ycbv_real.py:198,285-296): every rank ends with the MEAN of the
    per-shard single-process gradients — per-replica BatchNorm statistics and per-replica
    label[0], the reference's DDP semantics — for all 149 parameters (the shared feature
    encoder once), and that differs from the full-batch single-process gradient."""
    from tests.test_train_host import build_train_refiner, oracle_loss_and_grads, train_batch
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_refiner_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    names, local0, red0, nb = res[0]
    _, local1, red1, _ = res[1]
    assert len(names) == 149 and len(set(names)) == 149 and nb >= 4
    enc = [n.split(".", 1)[1] for n in names if n.startswith(("real_encoder.", "render_encoder."))]
    assert enc and len(enc) == len(set(enc))  # the shared feature encoder once
    for a, b, l0, l1 in zip(red0, red1, local0, local1):
        np.testing.assert_array_equal(a, b)  # every rank holds the same averaged gradient
        np.testing.assert_array_equal(a, (l0 + l1) * 0.5)  # sum of two, then × ½: exact
    # the full batch in ONE process (batch-wide BN statistics, label[0] of the whole batch) is a
    # different gradient: the exchange must not be compared against it
    torch.set_num_threads(8)
    batch, points, diam = train_batch(len(_LABELS), 256, seed=9, labels=_LABELS)
    r = build_train_refiner(_ITERS, dtype=torch.float64)
    _, _, _, full = oracle_loss_and_grads(batch, points, diam, _ITERS, names)
    bn = [i for i, n in enumerate(names) if n.startswith("context.") and ".bn" in n]
    assert bn
    diff = max(float(np.abs(red0[i] - full[names[i]].numpy()).max() /
                     (np.abs(full[names[i]].numpy()).max() + 1e-30)) for i in bn)
    assert diff > 1e-3, diff
    del r
