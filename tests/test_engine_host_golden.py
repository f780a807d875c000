"""The engine headers (compiled for the host by tests/hostcheck.py) against
the reference's golden trajectories, step by step: option lists, chosen
index (the lane's own CPython MT stream), post-state digests, full states."""
import numpy as np
import pytest

from citadels_self_play_amd import canon
from citadels_self_play_amd import layout as L
from hostcheck import HostBatch, lib


def test_layout_matches_native():
    import ctypes as C
    out = (C.c_int * 16)()
    n = lib().cith_layout(out, 16)
    assert list(out[:n]) == L.expected_layout()
    assert lib().cith_sizeof_game() <= L.GAME_BYTES == lib().cith_game_bytes()


def test_mt_streams(golden_rng):
    for rec in golden_rng["cpython"]:
        hb = HostBatch.__new__(HostBatch)
        hb.B = 1
        hb.mt = np.zeros((L.MT_N, 1), np.uint32)
        hb.idx = np.zeros(1, np.uint32)
        seeds = np.array([rec["seed"]], np.uint64)
        import ctypes as C
        from hostcheck import _p
        lib().cith_mt_seed(_p(hb.mt), _p(hb.idx), C.c_int(1), _p(seeds), C.c_int(0))
        assert hb.mt[:, 0].tolist() == rec["state0"][:624]
        out = np.zeros(len(rec["getrandbits32"]), np.uint32)
        lib().cith_mt_draw(_p(hb.mt), _p(hb.idx), C.c_int(1), C.c_int(0), C.c_int(len(out)), _p(out))
        assert out.tolist() == rec["getrandbits32"]
        lib().cith_mt_seed(_p(hb.mt), _p(hb.idx), C.c_int(1), _p(seeds), C.c_int(0))
        d = np.zeros(len(rec["random"]), np.float64)
        lib().cith_mt_random(_p(hb.mt), _p(hb.idx), C.c_int(1), C.c_int(0), C.c_int(len(d)), _p(d))
        assert d.tolist() == rec["random"]
        lib().cith_mt_seed(_p(hb.mt), _p(hb.idx), C.c_int(1), _p(seeds), C.c_int(0))
        for n, vals in rec["randbelow"]:
            assert [hb.randbelow(0, n) for _ in vals] == vals
    for rec in golden_rng["numpy"]:
        import ctypes as C
        from hostcheck import _p
        mt = np.zeros((L.MT_N, 1), np.uint32)
        idx = np.zeros(1, np.uint32)
        seeds = np.array([rec["seed"]], np.uint64)
        lib().cith_mt_seed(_p(mt), _p(idx), C.c_int(1), _p(seeds), C.c_int(1))
        assert mt[:, 0].tolist() == rec["key0"]
        d = np.zeros(len(rec["random_sample"]), np.float64)
        lib().cith_mt_random(_p(mt), _p(idx), C.c_int(1), C.c_int(0), C.c_int(len(d)), _p(d))
        assert d.tolist() == rec["random_sample"]


def _walk(rec):
    hb = HostBatch([rec["seed"]], rec["preset"])
    g = hb.game(0)
    assert canon.canon_game(g) == rec["states"]["0"]
    for i, (st, pid, n, oh, idx, ph) in enumerate(rec["steps"]):
        g = hb.game(0)
        assert (g.gs_state, g.gs_pid) == (st, pid), i
        opts, cnt = hb.get_options()
        g = hb.game(0)            # get_options may mutate (scholar)
        assert g.err == 0, (i, g.err)
        descs = [L.opt_from_bytes(opts[0, j]) for j in range(cnt[0])]
        if str(i) in rec["options"]:
            assert [canon.canon_option(o, g) for o in descs] == rec["options"][str(i)], i
        assert cnt[0] == n, (i, cnt[0], n)
        assert canon.hash_options(descs, g) == oh, i
        k = hb.randbelow(0, int(cnt[0]))
        assert k == idx, i
        hb.carry_out(opts[:, k])
        g = hb.game(0)
        assert g.err == 0, (i, g.err)
        d = canon.canon_game(g)
        if str(i + 1) in rec["states"]:
            assert d == rec["states"][str(i + 1)], i
        assert canon.hash_obj(d) == ph, i
    assert canon.canon_game(hb.game(0)) == rec["states"]["final"]


def test_engine_preset_stepwise(golden_preset):
    for rec in golden_preset:
        _walk(rec)


def test_engine_preset_rollout(golden_preset):
    hb = HostBatch([r["seed"] for r in golden_preset], True)
    steps, w = hb.rollout()
    for l, rec in enumerate(golden_preset):
        assert steps[l] == rec["n_steps"]
        assert w[l] == rec["winner"]
        assert canon.canon_game(hb.game(l)) == rec["states"]["final"]


def test_engine_random_role_stepwise(golden_random):
    for rec in golden_random:
        _walk(rec)
