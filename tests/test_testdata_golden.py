"""generate_test_data.setup_game (create_game -> create_a_close_to_finished_game
-> encode_game -> run_mccfr -> encode_options_from_node / create_target_strategy)
in the oracle and in the host build of the engine, against the reference's
outputs (tests/golden/testdata500.json.gz, 500 MCCFR iterations)."""
import numpy as np
import pytest

import cfr_oracle as CO
import citadels_oracle as O
from citadels_self_play_amd import canon
from conftest import load_golden
from hostcheck import HostBatch, HostCfr, close_position, cfr_root_target
from test_cfr_host_golden import hash_obj
from test_targets_oracle_golden import check_targets


@pytest.mark.slow
def test_oracle_setup_game_matches_reference():
    for r in load_golden("testdata500.json.gz"):
        pos, res, tr = CO.setup_game(r["seed"], r["iters"])
        assert O.canon(pos) == r["position"], r["seed"]
        if isinstance(r["result"], str):
            assert res == r["result"], r["seed"]
            continue
        check_targets([res], [r["result"]], r["seed"])
        assert tr.count == r["nodes"] and tr.carry_outs == r["carry_outs"], r["seed"]
        g = tr.root.game
        assert hash_obj(list(g.rng.getstate()[1])) == r["rng_after"][0], r["seed"]


def test_host_setup_game_matches_reference():
    recs = load_golden("testdata500.json.gz")
    hb = HostBatch([r["seed"] for r in recs], True)
    close_position(hb)
    for l, r in enumerate(recs):
        assert canon.canon_game(hb.game(l)) == r["position"], r["seed"]
    from hostcheck import encode_games
    x = encode_games(hb)
    cf = HostCfr(hb, node_cap=4096, edge_cap=8 * 4096)
    chosen, stats = cf.decide(recs[0]["iters"])
    tgt = cfr_root_target(cf, stats[:, 0])
    for l, r in enumerate(recs):
        root, n_nodes, n_edges, carry, err = stats[l]
        if r["result"] == "ValueError":
            assert err != 0, r["seed"]
            continue
        assert err == 0, r["seed"]
        assert n_nodes == r["nodes"] and carry == r["carry_outs"], r["seed"]
        feat, opts, nv, dist = tgt[l]
        check_targets([(x[l], opts, nv, dist)], [r["result"]], r["seed"])
        assert hash_obj(hb.mt[:, l].tolist() + [int(hb.idx[l])]) == r["rng_after"][0], r["seed"]
        assert hash_obj(cf.npmt[:, l].tolist()) == r["rng_after"][1] and int(cf.npidx[l]) == r["rng_after"][2]
