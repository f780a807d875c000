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
    assert lib.cit_abi_version() == 2


def test_cfr_pool_bytes_64bit(lib):
    # cfr_train(200000) pools exceed 2 GiB per tree (round 1 returned -1 there)
    nc, ec = 500_256, 5 * 500_256
    assert lib.cit_cfr_pool_bytes(nc, ec) == (nc * 168 + ec * 48 + 15) // 16 * 16 + nc * L.GAME_BYTES
    assert lib.cit_cfr_pool_bytes(3, 5) % 16 == 0   # rows (and the next tree's pool) 16-byte aligned
    assert lib.cit_cfr_pool_bytes(4_000_000, 20_000_000) > 2 ** 31
    assert lib.cit_cfr_pool_bytes(0, 10) == -1


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
