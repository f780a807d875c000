"""train_from_scratch's data path across ranks, end to end on CPU with gloo
(reference: train_from_scratch.py:39-42 -- Pool.starmap of simulate_game over
the games, results pooled): each rank takes its shard of the global games
(selfplay.shard), searches them with the host build of the engine and search
headers (cith_random_position -> cith_cfr_decide -> cith_cfr_targets: the
same C++ the GPU kernels compile, the checker build of tests/hostcheck.py),
drops the trees that ended in an error (selfplay._roots_for_targets' rule)
and pools the (encode_game, node_value) targets with
selfplay.all_gather_targets.  The pooled targets of world 2 and world 3 equal
world 1's bit for bit, in global game order."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_GAMES, BASE, ITERS = 6, 31_000_500, 300


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_targets(seeds):
    """simulate_game on the host build for `seeds`: (feat [n,418] f32, value [n,6] f64, stats)."""
    from hostcheck import HostBatch, HostCfr, cfr_targets, random_position
    if len(seeds) == 0:
        return torch.zeros((0, 418)), torch.zeros((0, 6), dtype=torch.float64), np.zeros((0, 5), np.int32)
    hb = HostBatch([int(s) for s in seeds], True)
    random_position(hb, 100)
    cf = HostCfr(hb, node_cap=4096, edge_cap=16 * 4096, pred=False)
    chosen, stats = cf.decide(ITERS)
    roots = stats[:, 0].copy()
    roots[stats[:, 4] != 0] = -1                           # an error tree yields no targets
    t = cfr_targets(cf, roots, mode=2)                     # searched without a model: the pruned walk
    return torch.from_numpy(t["feat"]), torch.from_numpy(t["value"]), stats


def _worker(rank, ws, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from citadels_self_play_amd import selfplay
        seeds = selfplay.shard(N_GAMES, base_seed=BASE)
        feat, value, stats = _rank_targets(seeds)
        pf, pv = selfplay.all_gather_targets(feat, value)
        q.put((rank, seeds.tolist(), int(feat.shape[0]), pf.numpy(), pv.numpy(), stats.tolist()))
    finally:
        dist.destroy_process_group()


def _run(ws):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in ps:
        p.start()
    out = [q.get(timeout=600) for _ in range(ws)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return sorted(out, key=lambda x: x[0])


def test_gloo_simulate_game_pipeline_matches_world1():
    one = _run(1)[0]
    assert one[1] == list(range(BASE, BASE + N_GAMES)) and one[2] > 0
    for ws in (2, 3):
        out = _run(ws)
        assert sum((o[1] for o in out), []) == one[1]                     # every game once, in order
        assert sum(o[2] for o in out) == one[2]
        assert sum((o[5] for o in out), []) == one[5]                     # the same searches, game by game
        for o in out:                                                     # every rank holds the same pool
            assert np.array_equal(o[3].view(np.uint32), one[3].view(np.uint32))
            assert np.array_equal(o[4].view(np.uint64), one[4].view(np.uint64))
