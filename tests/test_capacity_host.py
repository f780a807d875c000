"""Capacities in the host build of the search (csrc/cit_cfr.h, cit_core.h).

* The reference's unbounded per-player lists: simulate_game seed 31000322 at
  cfr_train(200000) grows a determinized player's museum to 17 cards deep in
  the search.  Round 3's fixed 16-card museum stopped that tree; with the
  shared 88-slot card area (hand | just_drawn | museum) it completes and
  equals the reference's own run (tests/golden/targets200000_cap.json.gz,
  tools/gen_golden_targets.py 200000 --seeds 31000322 --out
  targets200000_cap.json.gz): node and carry_out counts, the decision, both
  streams' end states and every target.
* A node-pool overflow carries a CIT_ERR_POOL_* bit (the tree is searched
  again with more room and gives the reference's tree)."""
import pytest

from citadels_self_play_amd import canon
from citadels_self_play_amd import layout as L
from citadels_self_play_amd.engine import ERR_OVERFLOW, ERR_POOL, ERR_POOL_CAP, ERR_POOL_ROW, pool_caps
from conftest import load_golden
from hostcheck import HostBatch, HostCfr, cfr_targets, random_position, split_targets
from test_cfr_host_golden import hash_obj
from test_targets_oracle_golden import check_targets


@pytest.mark.timeout(600)
def test_museum_past_16_matches_reference():
    recs = load_golden("targets200000_cap.json.gz")
    hb = HostBatch([r["seed"] for r in recs], True)
    random_position(hb, 100)
    for l, r in enumerate(recs):
        assert canon.canon_game(hb.game(l)) == r["position"], r["seed"]
    nc, ec = pool_caps(200_000)
    cf = HostCfr(hb, node_cap=nc, edge_cap=ec, row_cap=128, pred=False)     # the queue's pool format
    chosen, stats = cf.decide(200_000)
    per = split_targets(cfr_targets(cf, stats[:, 0], mode=2))
    for l, r in enumerate(recs):
        root, n_nodes, n_edges, carry, err = stats[l]
        assert r["error"] is None and err == 0, (r["seed"], hex(int(err)))
        assert n_nodes == r["nodes"] and carry == r["carry_outs"], (r["seed"], n_nodes, carry)
        g = hb.game(l)
        assert canon.canon_option(L.opt_from_bytes(chosen[l]), g) == r["chosen"], r["seed"]
        assert hash_obj(hb.mt[:, l].tolist() + [int(hb.idx[l])]) == r["rng_after"][0], r["seed"]
        assert hash_obj(cf.npmt[:, l].tolist()) == r["rng_after"][1] and int(cf.npidx[l]) == r["rng_after"][2]
        check_targets(per[l], r["targets"], r["seed"])


def test_pool_overflow_bits():
    for kw, bit in (({"node_cap": 64, "edge_cap": 5 * 64}, ERR_POOL_CAP), ({"row_cap": 8}, ERR_POOL_ROW)):
        hb = HostBatch([30_000_000], True)
        random_position(hb, 100)
        args = {"node_cap": 8192, "edge_cap": 8 * 8192}
        args.update(kw)
        _, stats = HostCfr(hb, **args).decide(2000)
        err = int(stats[0][4])
        assert err & ERR_OVERFLOW and err & bit and not (err & ERR_POOL & ~bit), hex(err)
