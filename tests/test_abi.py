"""CPU-side checks of the C ABI: the shared library loads here (no GPU
needed to load it), exports every symbol include/citadels.h declares, and its
struct layout matches the Python mirror.  No compute calls."""
import ctypes as C
import os

import pytest

from citadels_self_play_amd import _lib
from citadels_self_play_amd import layout as L


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build_hip()
    return _lib.load()


def test_exports_every_declared_symbol(lib):
    names = _lib.declared_symbols()
    assert len(names) >= 9
    for n in names:
        assert hasattr(lib, n), n
        assert n in _lib._SIGS, n


def test_layout_matches(lib):
    out = (C.c_int * 16)()
    n = lib.cit_layout(out, 16)
    assert list(out[:n]) == L.expected_layout()
    assert lib.cit_game_bytes() == L.GAME_BYTES
    assert lib.cit_seer_scratch_words() == L.SEER_MAX
    assert lib.cit_abi_version() == 9


def test_cfr_pool_layout(lib):
    # per-tree block tables + one 64-bit arena (csrc/cit_cfr.h; layout.cfr_*)
    sizes = (C.c_int32 * 3)()
    assert lib.cit_cfr_block_sizes(sizes) == 0
    assert list(sizes) == [L.CFR_NB, L.CFR_EB, L.CFR_TBL_MAX]
    out = (C.c_int * 8)()
    h = __import__("tests.hostcheck", fromlist=["lib"]).lib()
    assert h.cith_cfr_sizes(out) == 5
    assert list(out[:5]) == [L.CFR_NODE_BYTES, L.CFR_EDGE_BYTES, lib.cit_cfr_opt_cap(), L.CFR_NB, L.CFR_EB]
    nc, ec = 700_512, 4 * 700_512 + 4096                      # pool_caps(200000)
    # per tree: tables, then its base row and a scratch row
    assert lib.cit_cfr_pool_bytes(nc, ec) == L.cfr_pool_bytes(nc, ec) == (4 * (172 + 172) + 15) // 16 * 16 + 2 * 1552
    assert lib.cit_cfr_pool_bytes(3, 5) % 16 == 0             # the next tree's tables 16-byte aligned
    assert lib.cit_cfr_arena_bytes(172 * 300, 172 * 300) == L.cfr_arena_bytes(172 * 300, 172 * 300) > 2 ** 38
    h.cith_cfr_arena_bytes_rows.restype = C.c_int64
    for rc in (0, 4, 128, 388):                               # diff rows: edge-slot runs, no row slots
        assert lib.cit_cfr_arena_bytes_rows(172, 17, rc) == L.cfr_arena_bytes(172, 17, rc) == \
            h.cith_cfr_arena_bytes_rows(172, 17, rc)
    assert L.cfr_node_block_bytes(128, False) == 4096 * 72 < L.cfr_node_block_bytes(0) == \
        4096 * (72 + 48 + 1552)                               # 72-B records (+ pred_node_value in pred pools)
    assert [L.cfr_row_slots(k) for k in (0, 10, 11, 70, 388)] == [2, 2, 3, 7, 34]   # 14 header words + k, 12 a slot
    h.cith_cfr_arena_bytes_fmt.restype = C.c_int64
    for rc in (0, 128):
        for pred in (0, 1):
            assert lib.cit_cfr_arena_bytes_fmt(172, 17, rc, pred) == L.cfr_arena_bytes(172, 17, rc, bool(pred)) == \
                h.cith_cfr_arena_bytes_fmt(172, 17, rc, pred)
    assert lib.cit_cfr_arena_bytes_fmt(1, 1, 130, 0) == -1
    for bad in (-4, 3, 130, 392):
        assert lib.cit_cfr_arena_bytes_rows(1, 1, bad) == -1
        assert lib.cit_cfr_arena_reset_rows(None, 4, 16, 16, 1, 1, bad, None) == -1
    assert lib.cit_cfr_pool_bytes(0, 10) == -1
    assert lib.cit_cfr_pool_bytes(L.CFR_TBL_MAX * L.CFR_NB + 1, 10) == -1   # table longer than a tree may hold
    assert lib.cit_cfr_arena_bytes(-1, 0) == -1
    assert lib.cit_cfr_arena_reset(None, 4, 16, 16, 1, 1, None) == -1


def test_arena_blocks():
    from citadels_self_play_amd.engine import arena_blocks, pool_bytes
    assert arena_blocks(10, 700_512, 2_806_144) == (1720, 1720)
    assert arena_blocks(10, 700_512, 2_806_144, (0.5, 0.8)) == (860, 1376)
    assert arena_blocks(1, 100, 500, 0.1) == (1, 1)           # never below one tree's worst case
    assert pool_bytes(2, 100, 500) == 2 * (16 + 2 * 1552) + L.cfr_arena_bytes(2, 2, 0, False)
    assert pool_bytes(2, 100, 500, pred=True) == 2 * (16 + 2 * 1552) + L.cfr_arena_bytes(2, 2)
    assert pool_bytes(2, 700_512, 2_806_144) == 2 * L.cfr_pool_bytes(700_512, 2_806_144) + \
        L.cfr_arena_bytes(344, 344, 388, False)                # large trees: diff rows, no pred
    from citadels_self_play_amd.engine import pool_caps
    assert pool_caps(200000) == (910_512, 14 * 910_512 + 4096)   # row runs in the edge cap
    assert pool_caps(200) == (1422, 4 * 1422 + 4096)            # small trees: raw rows
    nc, ec = pool_caps(200000)
    assert L.cfr_nblocks(nc) <= 1024 and L.cfr_eblocks(ec) <= 1024  # the tables fit a tree's LDS copy


def test_bad_args_rejected(lib):
    # argument validation happens before any launch: no GPU is touched
    assert lib.cit_rollout_random(None, None, None, None, 0, -1, 0, None, None, None) == -1
    assert lib.cit_init(None, None, None, 4, None, 1, None) == -1
    assert lib.cit_count_options(None, None, None, None, 4, None, None) == -1
    assert lib.cit_determinize(None, None, None, 4, None, 1, None) == -1
    assert lib.cit_skip_false_choice(None, None, None, None, 4, None, None) == -1
    assert lib.cit_cfr_action_choice(None, 4, 16, 16, None, None, None, None, None, None) == -1


def test_api_error_mapping():
    import pytest
    from citadels_self_play_amd import api
    with pytest.raises(IndexError):
        api.raise_for(0x2)
    with pytest.raises(ValueError):
        api.raise_for(0x8)
    with pytest.raises(KeyError):
        api.raise_for(0x4)
    api.raise_for(0)
