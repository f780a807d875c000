"""MCCFR engine (csrc/cit_cfr.h, host build) against the reference's MCCFR
goldens: config-3 positions, node/carry_out counts, chosen option, root
arrays, RNG end states, and whole trees in DFS order.

Tolerance: node values, winning probabilities and regrets are exact (they
only involve correctly-rounded + - /); strategies go through exp(), where
libm differs from numpy's SIMD exp by <= 1 ulp, so S and CS are compared
with rtol = 1e-12."""
import hashlib
import json

import numpy as np
import pytest

from citadels_self_play_amd import canon
from citadels_self_play_amd import layout as L
from conftest import load_golden
from hostcheck import HostBatch, HostCfr, node_arrays

RTOL = 1e-12


def hash_obj(d):
    return hashlib.sha1(json.dumps(d, sort_keys=True, separators=(",", ":")).encode()).hexdigest()[:16]


def arrays(nodes, edges, i):
    R, S, CS = node_arrays(nodes, edges, i)
    return R.tolist(), S.tolist(), CS.tolist()


def dfs(nodes, edges, i, out):
    out.append(i)
    n = nodes[i]
    for a in range(int(n["n_children"])):
        dfs(nodes, edges, int(edges[n["first_edge"] + a]["child"]), out)
    return out


def compare_node(nodes, edges, rows, i, want, where):
    n = nodes[i]
    g = L.game_from_bytes(rows[i])
    assert int(n["depth"]) == want["depth"], where
    assert int(n["player"]) == want["player"], where
    assert int(n["flags"] & 1) == want["role_pick"], where
    assert int((n["flags"] >> 1) & 1) == want["terminal"], where
    assert int(n["n_children"]) == want["n_children"], where
    assert canon.hash_obj(canon.canon_game(g)) == want["game"], where
    assert n["nv"].tolist() == want["node_value"], where
    assert n["wp"].tolist() == want["wp"], where
    R, S, CS = arrays(nodes, edges, i)
    assert R == want["R"], where
    np.testing.assert_allclose(np.asarray(S, float), np.asarray(want["S"], float), rtol=RTOL, atol=0, err_msg=where)
    np.testing.assert_allclose(np.asarray(CS, float), np.asarray(want["CS"], float), rtol=RTOL, atol=0, err_msg=where)
    nch = int(n["n_children"])
    opts = [canon.canon_option(L.opt_from_bytes(edges[n["first_edge"] + a]["opt"]), g) for a in range(nch)]
    assert opts == want["opts"], where


def run_cases(recs, row_cap=0):
    recs = [r for r in recs if not r.get("skip")]
    hb = HostBatch([r["seed"] for r in recs], True)
    cf = HostCfr(hb, node_cap=8192, edge_cap=(16 if row_cap else 5) * 8192, row_cap=row_cap)   # rows in edge space
    cf.advance(0, 300)
    for l, r in enumerate(recs):
        assert canon.canon_game(hb.game(l)) == r["position"], r["seed"]
    iters = recs[0]["iters"]
    assert all(r["iters"] == iters for r in recs)
    chosen, stats = cf.decide(iters)
    for l, r in enumerate(recs):
        root, n_nodes, n_edges, carry, err = stats[l]
        assert err == 0, (r["seed"], err)
        g = hb.game(l)
        assert canon.canon_game(g) == r["root_game"], r["seed"]
        assert n_nodes == r["nodes"], r["seed"]
        assert carry == r["carry_outs"], r["seed"]
        assert canon.canon_option(L.opt_from_bytes(chosen[l]), g) == r["chosen"], r["seed"]
        nodes, edges, rows = cf.tree(l)
        compare_node(nodes, edges, rows, root, r["root"], (r["seed"], "root"))
        words = hb.mt[:, l].tolist() + [int(hb.idx[l])]
        assert hash_obj(words) == r["rng_after"][0], r["seed"]
        assert hash_obj(cf.npmt[:, l].tolist()) == r["rng_after"][1] and int(cf.npidx[l]) == r["rng_after"][2]
        if "tree" in r:
            order = dfs(nodes, edges, root, [])
            assert len(order) == len(r["tree"])
            for k, (i, want) in enumerate(zip(order, r["tree"])):
                compare_node(nodes, edges, rows, i, want, (r["seed"], k))


# row_cap 128: node rows stored as diffs against the tree's base row, runs of
# edge slots (the layout of large trees' pools, cit_cfr.h): same trees, rows
# and streams
@pytest.mark.parametrize("row_cap", [0, 128])
def test_cfr_host_train200(row_cap):
    run_cases(load_golden("cfr_train200.json.gz"), row_cap)


@pytest.mark.parametrize("row_cap", [0, 128])
def test_cfr_host_train2000(row_cap):
    run_cases(load_golden("cfr_train2000.json.gz"), row_cap)
