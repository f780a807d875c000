"""Pin the CFR oracle (oracle/cfr_oracle.py) to the reference's MCCFR
outputs (tests/golden/cfr_*.json.gz): position, node count, carry_out count,
chosen option, root arrays, RNG end states, and whole trees in DFS order.
The oracle uses numpy's own fp64 ops, so everything is compared exactly."""
import hashlib
import json

import numpy as np
import pytest

import cfr_oracle as CO
import citadels_oracle as O
from conftest import load_golden


def hash_obj(d):
    return hashlib.sha1(json.dumps(d, sort_keys=True, separators=(",", ":")).encode()).hexdigest()[:16]


def node_rec(n):
    return {
        "depth": n.depth, "player": n.player, "role_pick": int(bool(n.role_pick)),
        "terminal": int(bool(n.game.terminal)), "n_children": len(n.children),
        "node_value": np.asarray(n.nv, np.float64).tolist(), "wp": np.asarray(n.wp, np.float64).tolist(),
        "R": np.asarray(n.R, np.float64).tolist(), "S": np.asarray(n.S, np.float64).tolist(),
        "CS": np.asarray(n.CS, np.float64).tolist(),
        "game": hash_obj(O.canon(n.game)), "opts": [o.canon() for o, _ in n.children],
    }


def check(rec):
    pos = CO.config3_position(rec["seed"])
    if rec.get("skip"):
        assert pos is None
        return
    g, npr = pos
    assert O.canon(g) == rec["position"]
    chosen, tr = CO.run_mccfr(g, npr, rec["iters"])
    assert O.canon(tr.root.game) == rec["root_game"]
    assert tr.count == rec["nodes"]
    assert tr.carry_outs == rec["carry_outs"]
    assert chosen.canon() == rec["chosen"]
    assert node_rec(tr.root) == rec["root"]
    assert hash_obj(list(g.rng.getstate()[1])) == rec["rng_after"][0]
    st = npr.get_state()
    assert hash_obj(st[1].tolist()) == rec["rng_after"][1] and int(st[2]) == rec["rng_after"][2]
    if "tree" in rec:
        nodes = CO.dfs(tr.root, [])
        assert len(nodes) == len(rec["tree"])
        for i, (n, want) in enumerate(zip(nodes, rec["tree"])):
            assert node_rec(n) == want, i


def test_cfr_oracle_train200():
    for rec in load_golden("cfr_train200.json.gz"):
        check(rec)


@pytest.mark.slow
def test_cfr_oracle_train2000():
    for rec in load_golden("cfr_train2000.json.gz"):
        check(rec)
