"""A player's hand, just-drawn cards and museum share one card area
(csrc/cit_core.h, CIT_AREA_CAP): the list operations of cit_engine.h
(area_splice and the pl_* wrappers) against a Python-list model of the
reference's Deck methods (deck.py:49-67: get_a_card_like_it, draw_card,
add_card, `.cards = []`), on pseudo-random operation sequences that fill the
areas to capacity (csrc/cit_area_test.h) -- lengths past 64 (the wave paths'
second byte per lane) and the overflow check, which no golden game reaches.

CPU: the host build against the model.  GPU: the HIP kernel (the
lane-parallel CIT_WAVE paths) against the host build, row and log bytes."""
import ctypes as C

import numpy as np
import pytest

from citadels_self_play_amd import canon
from citadels_self_play_amd import layout as L
from hostcheck import lib as hostlib

M64 = (1 << 64) - 1
N_OPS = 3000
SEEDS = [0x9E3779B97F4A7C15 * (i + 1) & M64 for i in range(48)]


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _type(c):
    return 25 if c >= 40 else c


class Model:
    """Python lists for the 6 players' hand / jd / museum and the deck."""

    def __init__(self):
        self.lists = [[[], [], []] for _ in range(6)]
        self.deck = []
        self.err = False

    def used(self, p):
        return sum(len(x) for x in self.lists[p])

    def put(self, p, L_, c):
        if self.used(p) + 1 > L.AREA_CAP:
            self.err = True
            return
        self.lists[p][L_].append(c)

    def take_like(self, p, L_, c):
        lst = self.lists[p][L_]
        for i, x in enumerate(lst):
            if _type(x) == _type(c):
                return lst.pop(i)
        return c

    def op(self, s):
        s ^= s >> 12
        s ^= (s << 25) & M64
        s ^= s >> 27
        r = (s * 2685821657736338717) & M64
        op, p, L_, c, k = r % 6, (r >> 8) % 6, (r >> 16) % 3, (r >> 24) % 45, 1 + (r >> 32) % 5
        res = -1
        if op == 0:
            self.put(p, L_, c)
        elif op == 1:
            res = self.take_like(p, L_, c)
        elif op == 2:
            lst = self.lists[p][L_]
            res = lst.pop(0) if lst else 255
        elif op == 3:
            if ((r >> 40) & 7) == 0:
                self.lists[p][L_] = []
            else:
                self.put(p, L_, c)
        elif op == 4:
            while len(self.deck) < k + 2:
                self.deck.append((len(self.deck) * 7 + k) % 40)
            for _ in range(k):
                self.put(p, L_, self.deck.pop(0))
        else:
            q = (p + 1) % 6
            hp, hq = list(self.lists[p][0]), list(self.lists[q][0])
            for a, new in ((p, hq), (q, hp)):
                if self.used(a) - len(self.lists[a][0]) + len(new) > L.AREA_CAP:
                    self.err = True
                else:
                    self.lists[a][0] = list(new)
        log = op | (p << 4) | (L_ << 8) | (c << 12) | (k << 20) | ((res & 0xFF) << 24)
        return s, log


def host_run(seeds, n_ops):
    games = np.zeros((len(seeds), L.GAME_BYTES), np.uint8)
    log = np.zeros((len(seeds), n_ops), np.uint32)
    sd = np.asarray(seeds, np.uint64)
    hostlib().cith_area_test(_p(games), C.c_int(len(seeds)), _p(sd), C.c_int(n_ops), _p(log))
    return games, log


def test_host_area_ops_match_list_model():
    games, log = host_run(SEEDS, N_OPS)
    full = 0
    for l, seed in enumerate(SEEDS):
        m = Model()
        s = seed | 1
        for i in range(N_OPS):
            if m.err:
                assert log[l, i] == 0
                continue
            s, lg = m.op(s)
            assert int(log[l, i]) == lg, (l, i)
        g = L.game_from_bytes(games[l])
        d = canon.canon_game(g)
        assert bool(g.err) == m.err, l
        for p in range(6):
            P = d["players"][p]
            assert [P["hand"], P["jd"], P["museum"]] == m.lists[p], (l, p)
            full = max(full, m.used(p))
        assert canon.deck_list(g) == m.deck, l
    assert full > 64                      # the sequences reach the wave paths' second byte per lane


@pytest.mark.gpu
def test_gpu_area_ops_match_host():
    import torch
    import testkit
    lib = testkit.lib()
    B = len(SEEDS)
    ref_games, ref_log = host_run(SEEDS, N_OPS)
    games = torch.zeros((B, L.GAME_BYTES), dtype=torch.uint8, device="cuda")
    mt = torch.zeros((L.MT_N, B), dtype=torch.int32, device="cuda")
    idx = torch.zeros(B, dtype=torch.int32, device="cuda")
    seeds = torch.as_tensor(np.asarray(SEEDS, np.uint64).view(np.int64), device="cuda")
    log = torch.zeros((B, N_OPS), dtype=torch.int32, device="cuda")
    assert lib.citk_area_test(games.data_ptr(), mt.data_ptr(), idx.data_ptr(), B, seeds.data_ptr(), N_OPS,
                              log.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert np.array_equal(log.cpu().numpy().view(np.uint32), ref_log)
    assert np.array_equal(games.cpu().numpy(), ref_games)
