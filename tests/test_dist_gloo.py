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
