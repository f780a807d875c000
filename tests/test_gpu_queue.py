"""The tree queue on MI355X (selfplay.simulate_queue over cit_cfr_train_slice
+ cit_cfr_arena_release): 24 simulate_game trees through 5 lanes in slices of
~20 µs .. 5 ms equal simulate_games' one launch bit for bit -- stats, targets
in seed order, final games and both streams -- also when small node caps make
trees overflow or the shared arena runs out and trees go through the
cfr_decide retry.  The cross-round queue (selfplay.TreeQueue: rounds of
positions back to back, later rounds' trees taking the slots an earlier
round's tail frees, rounds added while the queue runs) gives each round
exactly simulate_games' result for its seeds."""
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ("meta", "feat", "value", "dist", "opt_feat", "counts", "terminal", "overflow", "chosen")


def _same(a, b):
    ba, sa, ta = a
    bb, sb, tb = b
    assert torch.equal(sa.cpu(), sb.cpu())
    for k in KEYS:
        assert torch.equal(ta[k].cpu(), tb[k].cpu()), k
    for f in ("games", "mt", "mt_idx", "np_mt", "np_idx"):
        assert torch.equal(getattr(ba, f).cpu(), getattr(bb, f).cpu()), f


@pytest.mark.parametrize("slice_seconds", [2e-7, 5e-3])
def test_gpu_queue_matches_batch(slice_seconds):
    from citadels_self_play_amd import selfplay
    seeds = selfplay.shard(24, 5150, 0, 1)
    whole = selfplay.simulate_games(seeds, 2000)
    q = selfplay.simulate_queue(seeds, 2000, slots=5, slice_seconds=slice_seconds)
    _same(q, whole)
    assert int((q[1][:, 4] != 0).sum()) == int((whole[1][:, 4] != 0).sum())


def test_gpu_queue_overflow_retry():
    from citadels_self_play_amd import selfplay
    seeds = selfplay.shard(12, 6160, 0, 1)
    whole = selfplay.simulate_games(seeds, 2000, node_cap=2048, edge_cap=8192)
    q = selfplay.simulate_queue(seeds, 2000, slots=4, node_cap=2048, edge_cap=8192, slice_seconds=1e-3)
    assert int(((whole[1][:, 1]) > 2048).sum()) > 0      # some trees outgrew the first caps
    _same(q, whole)


def test_gpu_queue_arena_exhausted():
    # an arena far below the trees' needs: trees that find it exhausted stop
    # with the overflow bit and are searched again (cfr_decide), same results
    from citadels_self_play_amd import selfplay
    seeds = selfplay.shard(10, 7170, 0, 1)
    whole = selfplay.simulate_games(seeds, 2000)
    q = selfplay.simulate_queue(seeds, 2000, slots=6, arena_frac=(0.05, 0.05), slice_seconds=1e-3)
    _same(q, whole)


@pytest.mark.parametrize("overcommit,frac", [(3.0, (1.0, 1.0)), (2.5, (0.3, 0.5))])
def test_gpu_queue_overcommit_pauses(overcommit, frac):
    # more slots than the arena holds at the trees' final sizes: the slice
    # planner pauses the least advanced trees (and, with the tiny arena, trees
    # still overflow and go through the retry); results are unchanged
    from citadels_self_play_amd import selfplay
    seeds = selfplay.shard(20, 8180, 0, 1)
    whole = selfplay.simulate_games(seeds, 2000)
    msgs = []
    q = selfplay.simulate_queue(seeds, 2000, slots=4, arena_frac=frac, overcommit=overcommit, slice_seconds=2e-3,
                                log=msgs.append)
    _same(q, whole)
    assert any("tree-slices paused" in m for m in msgs)


@pytest.mark.parametrize("overcommit,frac", [(None, "auto"), (2.5, (0.3, 0.5))])
def test_gpu_tree_queue_rounds_match_batches(overcommit, frac):
    from citadels_self_play_amd import selfplay
    rounds = [selfplay.shard(10, 9190 + 100 * r, 0, 1) for r in range(3)]
    whole = [selfplay.simulate_games(sd, 2000) for sd in rounds]
    q = selfplay.TreeQueue(2000, 10, slots=4, slice_seconds=2e-3, overcommit=overcommit, arena_frac=frac)
    q.add(rounds[0])
    q.add(rounds[1])
    added = []

    def more(qq):                 # round 2 added from the slice callback once round 1's trees run
        if len(qq.rounds) == 2 and qq.rounds[1].n_done >= 1:
            added.append(qq.add(rounds[2]))
    got = []
    for r in range(3):
        q.run(r, on_slice=more)
        if len(q.rounds) == 2:    # (round 1 may have finished inside run(0))
            q.add(rounds[2])
        got.append(q.result(r))
        walked, n = q.targets_so_far(r)
        assert walked == 10 and n == int(got[-1][2]["counts"][:, 0].sum())
    q.close()
    assert len(q.rounds) == 3 and added in ([], [2])
    for a, b in zip(got, whole):
        _same(a, b)
