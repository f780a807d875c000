"""Capacity overflows in the host build of the search (csrc/cit_cfr.h): a node-
pool overflow carries a CIT_ERR_POOL_* bit (the tree is searched again with
more room and gives the reference's tree), an engine list capacity does not
(no retry can fix it; the tree is dropped and counted)."""
import numpy as np

from citadels_self_play_amd.engine import ERR_OVERFLOW, ERR_POOL, ERR_POOL_CAP, ERR_POOL_ROW, pool_caps
from hostcheck import HostBatch, HostCfr, random_position


def test_engine_list_capacity_is_not_a_pool_overflow():
    # simulate_game seed 31000322 at cfr_train(200000): a determinized player's
    # museum grows past its 16 slots (CIT_MUSEUM_CAP) deep in the search
    hb = HostBatch([31_000_322], True)
    random_position(hb, 100)
    nc, ec = pool_caps(200_000)
    _, stats = HostCfr(hb, node_cap=nc, edge_cap=ec).decide(200_000)
    assert int(stats[0][4]) == ERR_OVERFLOW


def test_pool_overflow_bits():
    for kw, bit in (({"node_cap": 64, "edge_cap": 5 * 64}, ERR_POOL_CAP), ({"row_cap": 8}, ERR_POOL_ROW)):
        hb = HostBatch([30_000_000], True)
        random_position(hb, 100)
        args = {"node_cap": 8192, "edge_cap": 8 * 8192}
        args.update(kw)
        _, stats = HostCfr(hb, **args).decide(2000)
        err = int(stats[0][4])
        assert err & ERR_OVERFLOW and err & bit and not (err & ERR_POOL & ~bit), hex(err)
