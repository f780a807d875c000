"""selfplay._SlicePlanner on the host: which trees of an overcommitted tree
queue search in the next slice (most advanced first, while the arena's free
blocks cover their growth; the oldest always runs)."""
import numpy as np
import torch

from citadels_self_play_amd import layout as L
from citadels_self_play_amd import selfplay


class _FakeBatch:
    def __init__(self, B, node_cap, edge_cap, arena):
        self.B = B
        per = L.cfr_pool_bytes(node_cap, edge_cap)
        self.pool = torch.full((B * per + 64,), 0xFF, dtype=torch.uint8)   # tables all -1
        self.arena = arena
        self.per = per // 4

    def hold(self, lane, n_blocks, e_blocks, nbt):
        t = self.pool[:self.B * self.per * 4].view(torch.int32).view(self.B, self.per)
        t[lane] = -1
        t[lane, :n_blocks] = torch.arange(n_blocks, dtype=torch.int32)
        t[lane, nbt:nbt + e_blocks] = torch.arange(e_blocks, dtype=torch.int32)


def _state(its):
    st = np.zeros((len(its), 16), np.int32)
    st[:, 5] = its
    return st


def test_planner_orders_by_progress_and_pauses_when_full():
    node_cap, edge_cap = 40 * L.CFR_NB, 40 * L.CFR_EB
    nbt = L.cfr_nblocks(node_cap)
    fb = _FakeBatch(4, node_cap, edge_cap, arena=(20, 20))
    p = selfplay._SlicePlanner(fb, node_cap, edge_cap, margin=1.0)
    live = np.ones(4, bool)
    # first slice: nothing held, prior growth = max(2, 40 // 16) = 2 blocks (+1) each: all four fit (12 <= 20)
    assert not p.plan(_state([0, 0, 0, 0]), live, np.zeros(4, bool)).any()
    # all grew: lanes 0..3 hold 6, 5, 2, 1 node blocks (grew by that much in the slice)
    for lane, n in enumerate((6, 5, 2, 1)):
        fb.hold(lane, n, 1, nbt)
    # free = 20 - 14 = 6 node blocks; need = growth + 1: lane 0 (most iterations) 7 -> always runs,
    # then nothing is left for the others
    pause = p.plan(_state([900, 500, 100, 50]), live, np.ones(4, bool))
    assert pause.tolist() == [False, True, True, True]
    # with lane 0 finished and released, lanes 1 (6) and 3 (2) fit in 20 - 8 = 12 (6 + 3 = 9), lane 2 (3) too
    fb.hold(0, 0, 0, nbt)
    live[0] = False
    pause = p.plan(_state([0, 500, 100, 50]), live, np.array([True, False, False, False]))
    assert pause.tolist() == [False, False, False, False]
    p.reset(np.array([0]))
    assert p.growth[0, 0] == -1 and p.last_held[0, 0] == 0
