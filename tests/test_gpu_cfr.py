"""MCCFR on a real MI355X through the C ABI (cit_advance_random +
cit_cfr_decide): the reference's MCCFR goldens (positions, node and
carry_out counts, decisions, root arrays, RNG end states, whole trees), fresh
seeds against the CFR oracle, and batch-size properties at config-3 scale.
Same tolerance as the host test: exact except strategies (exp, rtol 1e-12)."""
import hashlib
import json

import numpy as np
import pytest
import torch

from citadels_self_play_amd import canon
from citadels_self_play_amd import layout as L
from conftest import load_golden
from test_cfr_host_golden import arrays, compare_node, dfs, hash_obj

pytestmark = pytest.mark.gpu


def _batch(seeds):
    from citadels_self_play_amd.engine import GameBatch
    return GameBatch(seeds, preset=True)


def _run_golden(name):
    recs = [r for r in load_golden(name) if not r.get("skip")]
    b = _batch([r["seed"] for r in recs])
    b.advance_random(0, 300)
    rows = b.rows()
    for l, r in enumerate(recs):
        assert canon.canon_game(L.game_from_bytes(rows[l])) == r["position"], r["seed"]
    b.seed_numpy()
    # 6144 nodes: the 2000-iteration seed 109 tree (6,604 nodes) overflows and is
    # searched again with a 4x pool -- the retry path is part of the check
    chosen, stats = b.cfr_decide(recs[0]["iters"], node_cap=6144, edge_cap=5 * 6144)
    torch.cuda.synchronize()
    chosen, stats, rows = chosen.cpu().numpy(), stats.cpu().numpy(), b.rows()
    mt = b.mt.cpu().numpy().view(np.uint32)
    idx = b.mt_idx.cpu().numpy()
    npmt = b.np_mt.cpu().numpy().view(np.uint32)
    npidx = b.np_idx.cpu().numpy()
    for l, r in enumerate(recs):
        root, n_nodes, n_edges, carry, err = stats[l]
        assert err == 0, (r["seed"], err)
        g = L.game_from_bytes(rows[l])
        assert canon.canon_game(g) == r["root_game"], r["seed"]
        assert n_nodes == r["nodes"], r["seed"]
        assert carry == r["carry_outs"], r["seed"]
        assert canon.canon_option(L.opt_from_bytes(chosen[l]), g) == r["chosen"], r["seed"]
        nodes, edges, trows = b.tree(l)
        compare_node(nodes, edges, trows, root, r["root"], (r["seed"], "root"))
        assert hash_obj(mt[:, l].tolist() + [int(idx[l])]) == r["rng_after"][0], r["seed"]
        assert hash_obj(npmt[:, l].tolist()) == r["rng_after"][1] and int(npidx[l]) == r["rng_after"][2]
        if "tree" in r:
            order = dfs(nodes, edges, root, [])
            assert len(order) == len(r["tree"])
            for k, (i, want) in enumerate(zip(order, r["tree"])):
                compare_node(nodes, edges, trows, i, want, (r["seed"], k))


def test_gpu_cfr_golden_200():
    _run_golden("cfr_train200.json.gz")


def test_gpu_cfr_golden_2000():
    _run_golden("cfr_train2000.json.gz")


def test_gpu_cfr_vs_oracle_fresh_seeds():
    import cfr_oracle as CO
    import citadels_oracle as O
    seeds = list(range(5000, 5016))
    b = _batch(seeds)
    b.advance_random(0, 300)
    b.seed_numpy()
    chosen, stats = b.cfr_decide(200)
    chosen, stats, rows = chosen.cpu().numpy(), stats.cpu().numpy(), b.rows()
    for l, s in enumerate(seeds):
        pos = CO.config3_position(s)
        if pos is None:
            assert L.game_from_bytes(rows[l]).terminal
            continue
        g, npr = pos
        want, tr = CO.run_mccfr(g, npr, 200)
        assert stats[l][4] == 0
        gg = L.game_from_bytes(rows[l])
        assert canon.canon_game(gg) == O.canon(tr.root.game), s
        assert stats[l][1] == tr.count and stats[l][3] == tr.carry_outs, s
        assert canon.canon_option(L.opt_from_bytes(chosen[l]), gg) == want.canon(), s


def test_gpu_cfr_batch_properties():
    """Config-3 scale (1024 decisions): no errors, deterministic, and a lane's
    result does not depend on the batch it runs in."""
    B = 1024
    seeds = np.arange(9_000_000, 9_000_000 + B)
    out = []
    for rep in range(2):
        b = _batch(seeds)
        b.advance_random(0, 300)
        b.seed_numpy()
        chosen, stats = b.cfr_decide(200)
        out.append((chosen.cpu().numpy(), stats.cpu().numpy(), b.rows()))
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    assert np.array_equal(out[0][2], out[1][2])
    terminal = np.array([L.game_from_bytes(r).terminal for r in out[0][2]])
    assert (out[0][1][~terminal, 4] == 0).all()
    small = _batch(seeds[::97])
    small.advance_random(0, 300)
    small.seed_numpy()
    c2, s2 = small.cfr_decide(200)
    assert np.array_equal(c2.cpu().numpy(), out[0][0][::97])
    assert np.array_equal(s2.cpu().numpy()[:, 1:], out[0][1][::97, 1:])


def test_gpu_cfr_strategy_lds_equals_hbm_path():
    """update_strategy's LDS copies (nodes of <= 96 children) and its HBM
    path (larger nodes; forced for every node by CIT_CFR_STRATEGY_HBM) build
    bitwise the same trees: every node and edge record, decisions, streams."""
    from citadels_self_play_amd.engine import CFR_STRATEGY_HBM
    seeds = np.arange(9_100_000, 9_100_000 + 64)
    res = []
    for flags in (0, CFR_STRATEGY_HBM):
        b = _batch(seeds)
        b.advance_random(0, 300)
        b.seed_numpy()
        chosen, stats = b.cfr_decide(2000, node_cap=8192, edge_cap=5 * 8192, flags=flags)
        trees = [b.tree(l)[:2] for l in range(len(seeds))]
        res.append((chosen.cpu().numpy(), stats.cpu().numpy(), b.rows(), b.mt.cpu().numpy(),
                    b.np_mt.cpu().numpy(), b.np_idx.cpu().numpy(), trees))
    a, h = res
    for x, y in zip(a[:6], h[:6]):
        assert np.array_equal(x, y)
    for l, ((na, ea), (nh, eh)) in enumerate(zip(a[6], h[6])):
        n = int(a[1][l][1])
        for f in na.dtype.names:
            if f != "pad":
                assert np.ascontiguousarray(na[f][:n]).tobytes() == np.ascontiguousarray(nh[f][:n]).tobytes(), (l, f)
        for i in range(n):                       # the written edge records of every node (reserved slots aside)
            assert repr(arrays(na, ea, i)) == repr(arrays(nh, eh, i)), (l, i)
            fe, nch = int(na[i]["first_edge"]), int(na[i]["n_children"])
            if nch:
                assert ea[fe:fe + nch]["opt"].tobytes() == eh[fe:fe + nch]["opt"].tobytes(), (l, i)
                assert ea[fe:fe + nch]["child"].tobytes() == eh[fe:fe + nch]["child"].tobytes(), (l, i)


@pytest.mark.parametrize("shape", [(4, 256, 2), (12, 1024, 3)], ids=["4x256_2streams", "timed_12x1024_3streams"])
def test_gpu_cfr_streams_overlap(shape):
    """Config-3 batches searched on HIP streams at once (bench.py's
    continuous loop) equal the same batches searched one after another:
    decisions, stats, root games and both streams, bit for bit -- at a small
    shape and at the timed one (12 batches of 1,024 positions on the bench's
    3 streams, engine.side_streams)."""
    from citadels_self_play_amd.engine import GameBatch, side_streams
    K, B, S = shape

    def make():
        bs = []
        for k in range(K):
            b = GameBatch(np.arange(9_000_000 + 10_000 * k, 9_000_000 + 10_000 * k + B), preset=True)
            b.advance_random(0, 300)
            b.seed_numpy()
            b._pool(4096, 5 * 4096)
            bs.append(b)
        torch.cuda.synchronize()
        return bs

    def grab(bs, res):
        torch.cuda.synchronize()
        return [(c.cpu().numpy(), s.cpu().numpy(), b.rows(), b.mt.cpu().numpy(), b.np_mt.cpu().numpy())
                for b, (c, s) in zip(bs, res)]

    alone = make()
    ref = grab(alone, [b._cfr_decide(200, 4096, 5 * 4096) for b in alone])
    over = make()
    sts = side_streams(torch.device("cuda"), S)
    res = []
    for k, b in enumerate(over):
        with torch.cuda.stream(sts[k % S]):
            res.append(b._cfr_decide(200, 4096, 5 * 4096))
    got = grab(over, res)
    for a, g in zip(ref, got):
        assert (a[1][:, 4] == 0).mean() > 0.9
        for x, y in zip(a, g):
            assert np.array_equal(x, y)
