"""CPU, world_size 2 over gloo: batch sharding + end-of-run gather reproduce the single-process
result on a MULTI-CLASS batch (each shard carries the global label[0] for the pose head) (the per-rank compute is the CPU oracle standing in for the GPU decoder, which
has no CPU path)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from scflow_amd.dist import gather_results, gather_shards, shard_batch, shard_range


def test_shard_range_covers_batch():
    for b in (1, 2, 3, 7, 16, 128):
        for w in (1, 2, 3, 8):
            rs = [shard_range(b, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == b
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            sz = [e - s for s, e in rs]
            assert max(sz) - min(sz) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(2)
        from oracle import scflow_oracle as orc
        from tests.helpers import decoder_inputs, oracle_state_dict
        inp = decoder_inputs(3, 256, seed=4)           # B=3: uneven 2 / 1 split
        inp["label"] = torch.tensor([5, 11, 2])          # mixed classes: rank 1's label[0] != 5
        mine = shard_batch(inp, rank, world)
        assert mine["head_label"].tolist() == [5]        # the global batch's label[0]
        sd = oracle_state_dict()
        out = orc.decoder_forward(sd, **mine, iters=2)
        flow, pred, R, t = gather_results(out)
        x = gather_shards(torch.arange(rank * 10, rank * 10 + mine["depth"].shape[0]).float())
        if rank == 0:
            q.put(tuple(a.numpy() for a in (flow, pred, R, t, x)))  # by value: the sender exits
    finally:
        dist.destroy_process_group()


def test_sharded_decode_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    flow, pred, R, t, x = (torch.from_numpy(a) for a in q.get(timeout=240))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert x.tolist() == [0.0, 1.0, 10.0]
    from oracle import scflow_oracle as orc
    from tests.helpers import decoder_inputs, oracle_state_dict
    inp = decoder_inputs(3, 256, seed=4)
    inp["label"] = torch.tensor([5, 11, 2])
    ref = orc.decoder_forward(oracle_state_dict(), **inp, iters=2)
    # CPU conv summation order depends on batch size / threads: equal to fp32 rounding, not bitwise
    assert float(orc.cal_epe_mean(ref[0][-1], flow).max()) < 1e-4
    assert float(orc.cal_epe_mean(ref[1][-1], pred).max()) < 1e-4
    torch.testing.assert_close(R, ref[2][-1], rtol=0, atol=1e-5)
    torch.testing.assert_close(t, ref[3][-1], rtol=1e-6, atol=1e-3)
