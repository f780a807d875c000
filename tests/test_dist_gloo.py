"""The multi-rank paths of selfplay.py on CPU with gloo, world size 2:
sharding covers every global game once, the target all-gather pools ragged
per-rank sets in rank order bit for bit, and the model broadcast makes every
rank hold rank 0's parameters."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from citadels_self_play_amd import models, selfplay
        seeds = selfplay.shard(10, base_seed=100)
        g = torch.Generator().manual_seed(rank)
        n = [3, 0, 5][rank]
        feat = torch.randint(0, 9, (n, 418), generator=g).float()
        value = torch.rand((n, 6), generator=g, dtype=torch.float64)
        pf, pv = selfplay.all_gather_targets(feat, value)
        torch.manual_seed(1000 + rank)
        m = models.ValueOnlyNN(418, 64)
        selfplay.broadcast_model(m)
        q.put((rank, seeds.tolist(), pf.numpy(), pv.numpy(),
               {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}))
    finally:
        dist.destroy_process_group()


def _run(ws):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in range(ws)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return sorted(out, key=lambda x: x[0])


def test_gloo_gather_shard_broadcast():
    for ws in (2, 3):
        out = _run(ws)
        seeds = sum((o[1] for o in out), [])
        assert seeds == list(range(100, 110))
        want_f, want_v = [], []
        for r in range(ws):
            g = torch.Generator().manual_seed(r)
            n = [3, 0, 5][r]
            want_f.append(torch.randint(0, 9, (n, 418), generator=g).float().numpy())
            want_v.append(torch.rand((n, 6), generator=g, dtype=torch.float64).numpy())
        wf, wv = np.concatenate(want_f), np.concatenate(want_v)
        for o in out:
            assert np.array_equal(o[2], wf) and np.array_equal(o[3], wv)
            for k in o[4]:
                assert np.array_equal(o[4][k], out[0][4][k]), k
        torch.manual_seed(1000)
        from citadels_self_play_amd import models
        m0 = models.ValueOnlyNN(418, 64)
        for k, v in m0.state_dict().items():
            assert np.array_equal(out[-1][4][k], v.numpy()), k


def _driven_worker(rank, ws, port, q):
    """Rank 0 reaches the all-gather first and drives a stand-in for its
    queue's slices while rank 1 (late by 1.5 s) has not joined; the pooled
    rows must be the blocking gather's."""
    import time
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from citadels_self_play_amd import selfplay
        g = torch.Generator().manual_seed(rank)
        n = [4, 2][rank]
        feat = torch.randint(0, 9, (n, 418), generator=g).float()
        value = torch.rand((n, 6), generator=g, dtype=torch.float64)
        if rank == 1:
            time.sleep(1.5)
        calls = [0]

        def drive():
            calls[0] += 1
            time.sleep(0.01)
            return calls[0] < 10_000
        pf, pv = selfplay.all_gather_targets(feat, value, drive=drive)
        bf, bv = selfplay.all_gather_targets(feat, value)
        q.put((rank, calls[0], bool(torch.equal(pf, bf) and torch.equal(pv, bv)), pf.shape[0]))
    finally:
        dist.destroy_process_group()


def test_gloo_gather_drives_while_waiting():
    """train_from_scratch.collect's async all-gathers: the rank that waits for
    a slower rank keeps calling drive() (its next round's queue slices)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_driven_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=120) for _ in range(2)])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert out[0][1] >= 20, out        # rank 0 drove slices for most of rank 1's 1.5 s delay
    assert all(o[2] and o[3] == 6 for o in out), out
