"""Training-data path of train_from_scratch ("config 5": create_a_random_game(100)
-> cfr_train(2000, training=True) + live choice -> get_all_targets) in the host
build of the engine headers, against the reference's outputs
(tests/golden/targets2000.json.gz): positions, trees, decisions, RNG end
states and every target tuple (regret targets rtol 1e-12, np.exp)."""
import numpy as np
import pytest

from citadels_self_play_amd import canon
from citadels_self_play_amd import layout as L
from conftest import load_golden
from hostcheck import HostBatch, HostCfr, cfr_targets, random_position, split_targets
from test_cfr_host_golden import hash_obj
from test_targets_oracle_golden import check_targets


@pytest.mark.parametrize("mode,row_cap", [(0, 0), (2, 0), (2, 128)])   # 2: the pruned walk (no model);
def test_host_targets_match_reference(mode, row_cap):                    # 128: diff rows
    recs = load_golden("targets2000.json.gz")
    hb = HostBatch([r["seed"] for r in recs], True)
    random_position(hb, 100)
    for l, r in enumerate(recs):
        assert canon.canon_game(hb.game(l)) == r["position"], r["seed"]
    cf = HostCfr(hb, node_cap=8192, edge_cap=16 * 8192, row_cap=row_cap, pred=row_cap == 0)   # 72-B records too
    chosen, stats = cf.decide(2000)
    t = cfr_targets(cf, stats[:, 0], mode=mode)
    per = split_targets(t)
    for l, r in enumerate(recs):
        root, n_nodes, n_edges, carry, err = stats[l]
        assert err == 0, r["seed"]
        assert n_nodes == r["nodes"] and carry == r["carry_outs"], r["seed"]
        g = hb.game(l)
        assert canon.canon_option(L.opt_from_bytes(chosen[l]), g) == r["chosen"], r["seed"]
        assert hash_obj(hb.mt[:, l].tolist() + [int(hb.idx[l])]) == r["rng_after"][0], r["seed"]
        assert hash_obj(cf.npmt[:, l].tolist()) == r["rng_after"][1] and int(cf.npidx[l]) == r["rng_after"][2]
        check_targets(per[l], r["targets"], r["seed"])
