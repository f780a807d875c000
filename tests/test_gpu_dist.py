"""Multi-GPU readiness on one MI355X:

* shard invariance at the engine level: simulate_game trees of the two
  shards of a world of 2, run as two batches, equal (targets and stats,
  bitwise) the same seeds run as one batch, concatenated in rank order -- the
  "identical at any P" property;
* the RCCL ("nccl") branch of selfplay: a world-size-1 process group with
  device_id, the target all-gather and the model broadcast executed on the
  device."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def test_gpu_shard_invariance_simulate_games():
    from citadels_self_play_amd import selfplay
    from citadels_self_play_amd.engine import pool_bytes
    n, iters = 24, 2000
    whole_b, whole_stats, whole_t = selfplay.simulate_games(selfplay.shard(n, 4242, 0, 1), iters)
    parts = [selfplay.simulate_games(selfplay.shard(n, 4242, r, 2), iters) for r in range(2)]
    stats = torch.cat([p[1].cpu() for p in parts])
    assert torch.equal(stats, whole_stats.cpu())
    t = selfplay.concat_targets([p[2] for p in parts], [p[1].shape[0] for p in parts])
    for k in ("meta", "feat", "value", "dist", "opt_feat", "counts"):
        assert torch.equal(t[k].cpu(), whole_t[k].cpu()), k
    # and memory-bounded (3 trees at a time) within one rank: chunks, and the tree queue
    for queue in (False, True):
        cb, cstats, ct = selfplay.simulate_games(selfplay.shard(n, 4242, 0, 1), iters, queue=queue,
                                                 max_pool_bytes=pool_bytes(3, whole_b.node_cap, whole_b.edge_cap))
        assert torch.equal(cstats.cpu(), whole_stats.cpu())
        for k in ("meta", "feat", "value", "dist", "opt_feat", "counts"):
            assert torch.equal(ct[k].cpu(), whole_t[k].cpu()), k


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gpu_rccl_world1_collectives():
    from citadels_self_play_amd import models, selfplay
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _port(), rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        g = torch.Generator().manual_seed(0)
        feat = torch.randint(0, 9, (5, 418), generator=g).float().to(dev)
        value = torch.rand((5, 6), generator=g, dtype=torch.float64).to(dev)
        pf, pv = selfplay.all_gather_targets(feat, value)
        assert pf.device.type == "cuda"
        assert torch.equal(pf, feat) and torch.equal(pv, value)
        m = models.ValueOnlyNN(418, 64).to(dev)
        before = {k: v.clone() for k, v in m.state_dict().items()}
        selfplay.broadcast_model(m)
        for k, v in m.state_dict().items():
            assert torch.equal(v, before[k]), k
        objs = selfplay.all_gather_objects([1, 2, 3])
        assert objs == [1, 2, 3]
    finally:
        dist.destroy_process_group()
