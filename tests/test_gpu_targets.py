"""Training-data generation on a real MI355X through the C ABI
(cit_random_position -> cit_cfr_decide(2000) -> cit_cfr_target_count /
cit_cfr_targets) against the reference's own outputs
(tests/golden/targets2000.json.gz), and batch-size invariance at scale."""
import numpy as np
import pytest
import torch

from citadels_self_play_amd import canon
from citadels_self_play_amd import layout as L
from conftest import load_golden
from test_cfr_host_golden import hash_obj
from test_targets_oracle_golden import check_targets

pytestmark = pytest.mark.gpu


def _split(t):
    t = {k: v.cpu().numpy() for k, v in t.items()}
    per = [[] for _ in range(len(t["counts"]))]
    for k, (lane, node, pid, nch, c0) in enumerate(t["meta"]):
        per[lane].append((t["feat"][k], t["opt_feat"][c0:c0 + nch], t["value"][k], t["dist"][c0:c0 + nch]))
    return per


@pytest.mark.parametrize("name,iters", [("targets2000.json.gz", 2000), ("targets20000.json.gz", 20000)])
def test_gpu_targets_golden(name, iters):
    """simulate_game trees of the reference (cfr_train(2000), 16 seeds; and the
    config-5 quick setting cfr_train(20000), 4 seeds): positions, node and
    carry_out counts, decisions, both streams' end states, every target."""
    from citadels_self_play_amd.engine import GameBatch, pool_caps
    recs = [r for r in load_golden(name) if not r.get("error")]
    b = GameBatch([r["seed"] for r in recs], preset=True)
    b.random_position(100)
    rows = b.rows()
    for l, r in enumerate(recs):
        assert canon.canon_game(L.game_from_bytes(rows[l])) == r["position"], r["seed"]
    b.seed_numpy()
    nc, ec = pool_caps(iters)
    chosen, stats = b.cfr_decide(iters, node_cap=nc, edge_cap=ec)
    per = _split(b.cfr_targets(stats[:, 0]))
    chosen, stats, rows = chosen.cpu().numpy(), stats.cpu().numpy(), b.rows()
    mt = b.mt.cpu().numpy().view(np.uint32)
    idx = b.mt_idx.cpu().numpy()
    npmt = b.np_mt.cpu().numpy().view(np.uint32)
    npidx = b.np_idx.cpu().numpy()
    for l, r in enumerate(recs):
        root, n_nodes, n_edges, carry, err = stats[l]
        assert err == 0, r["seed"]
        assert n_nodes == r["nodes"] and carry == r["carry_outs"], r["seed"]
        g = L.game_from_bytes(rows[l])
        assert canon.canon_option(L.opt_from_bytes(chosen[l]), g) == r["chosen"], r["seed"]
        assert hash_obj(mt[:, l].tolist() + [int(idx[l])]) == r["rng_after"][0], r["seed"]
        assert hash_obj(npmt[:, l].tolist()) == r["rng_after"][1] and int(npidx[l]) == r["rng_after"][2]
        check_targets(per[l], r["targets"], r["seed"])


def test_gpu_targets_batch_invariance():
    """512 trees of cfr_train(500): every lane's targets are the same whether it
    runs in the full batch or in a strided sub-batch."""
    from citadels_self_play_amd.engine import GameBatch
    seeds = np.arange(7_000_000, 7_000_512)
    out = []
    for sel in (slice(None), slice(None, None, 37)):
        b = GameBatch(seeds[sel], preset=True)
        steps = b.random_position(100).cpu().numpy()
        assert (steps >= 0).all()
        b.seed_numpy()
        chosen, stats = b.cfr_decide(500, node_cap=4096)
        t = b.cfr_targets(stats[:, 0])
        torch.cuda.synchronize()
        out.append((stats.cpu().numpy(), _split(t)))
    (s_all, t_all), (s_sub, t_sub) = out
    assert np.array_equal(s_all[::37, 1:], s_sub[:, 1:])
    assert sum(len(x) for x in t_all) > 100
    for a, bb in zip(t_all[::37], t_sub):
        assert len(a) == len(bb)
        for x, y in zip(a, bb):
            for u, v in zip(x, y):
                assert np.array_equal(u, v)


def test_gpu_setup_game_golden():
    """generate_test_data.setup_game (500 iterations) on the device vs the reference."""
    from citadels_self_play_amd import _lib
    from citadels_self_play_amd.engine import GameBatch
    recs = load_golden("testdata500.json.gz")
    b = GameBatch([r["seed"] for r in recs], preset=True)
    index = b.close_position().cpu().numpy()
    assert (index >= 0).all()
    rows = b.rows()
    for l, r in enumerate(recs):
        assert canon.canon_game(L.game_from_bytes(rows[l])) == r["position"], r["seed"]
    feat = torch.zeros((b.B, 418), dtype=torch.float32, device=b.device)
    _lib.check(b.lib.cit_encode_games(b.games.data_ptr(), b.B, -1, feat.data_ptr(), None), "encode")
    b.seed_numpy()
    chosen, stats = b.cfr_decide(recs[0]["iters"], node_cap=4096)
    t = {k: v.cpu().numpy() for k, v in b.cfr_targets(stats[:, 0], mode=1).items()}
    feat, stats = feat.cpu().numpy(), stats.cpu().numpy()
    by_lane = {int(m[0]): (k, m) for k, m in enumerate(t["meta"])}
    for l, r in enumerate(recs):
        if r["result"] == "ValueError":
            assert stats[l][4] != 0 and l not in by_lane, r["seed"]
            continue
        assert stats[l][4] == 0 and stats[l][1] == r["nodes"] and stats[l][3] == r["carry_outs"], r["seed"]
        k, (lane, node, pid, nch, c0) = by_lane[l]
        check_targets([(feat[l], t["opt_feat"][c0:c0 + nch], t["value"][k], t["dist"][c0:c0 + nch])],
                      [r["result"]], r["seed"])


def test_gpu_pool_overflow_retry():
    """A tree that outgrows its node pool is searched again with a larger pool:
    decisions, stats, streams and targets equal those of a run whose pool was
    large enough from the start (reference behaviour has no pool at all)."""
    from citadels_self_play_amd.engine import GameBatch
    seeds = np.arange(7_100_000, 7_100_064)
    out = []
    for cap, retries in ((96, 3), (8192, 0)):
        b = GameBatch(seeds, preset=True)
        b.random_position(100)
        b.seed_numpy()
        chosen, stats = b.cfr_decide(500, node_cap=cap, max_retries=retries)
        t = b.cfr_targets(stats[:, 0])
        torch.cuda.synchronize()
        out.append((chosen.cpu().numpy(), stats.cpu().numpy(), _split(t), b.rows(), b.mt.cpu().numpy(),
                    b.mt_idx.cpu().numpy(), b.np_mt.cpu().numpy(), b.np_idx.cpu().numpy()))
    small, big = out
    assert (big[1][:, 4] == 0).all() and (small[1][:, 4] == 0).all()
    assert (big[1][:, 1] > 96).sum() > 8            # most lanes did overflow the small pool
    for x, y in zip(small[:2] + small[3:], big[:2] + big[3:]):
        assert np.array_equal(x, y)
    for a, bb in zip(small[2], big[2]):
        assert len(a) == len(bb)
        for x, y in zip(a, bb):
            for u, v in zip(x, y):
                assert np.array_equal(u, v)


@pytest.mark.parametrize("row_cap", [128, 8])
def test_gpu_diff_rows_match_raw_rows(row_cap):
    """Node rows stored as diffs against the tree's base row (the default for
    large trees, engine.row_cap_for) give the trees, decisions, streams and
    targets of raw rows; with a cap too small for any row (8 dwords) every
    tree overflows and is searched again with raw rows, same results."""
    from citadels_self_play_amd.engine import GameBatch
    seeds = np.arange(7_200_000, 7_200_048)
    out = []
    for rc in (0, row_cap):
        b = GameBatch(seeds, preset=True)
        b.random_position(100)
        b.seed_numpy()
        b.row_cap = rc
        chosen, stats = b.cfr_decide(2000, node_cap=8192, edge_cap=16 * 8192)   # diff rows take edge slots
        t = b.cfr_targets(stats[:, 0])
        torch.cuda.synchronize()
        trees = [b.tree(l) for l in (0, 7, 31)]
        out.append((chosen.cpu().numpy(), stats.cpu().numpy(), _split(t), b.rows(), b.mt.cpu().numpy(),
                    b.np_mt.cpu().numpy(), trees, getattr(b, "_retry", None) is not None))
    raw, diff = out
    assert diff[7] == (row_cap == 8)                  # the tiny cap overflowed every tree into the retry
    # stats but n_edges (diff rows are runs of edge slots: more slots, other edge indices)
    assert np.array_equal(raw[1][:, [0, 1, 3, 4]], diff[1][:, [0, 1, 3, 4]])
    for x, y in zip(raw[:1] + raw[3:6], diff[:1] + diff[3:6]):
        assert np.array_equal(x, y)
    for a, bb in zip(raw[2], diff[2]):
        assert len(a) == len(bb)
        for x, y in zip(a, bb):
            for u, v in zip(x, y):
                assert np.array_equal(u, v)
    def written(nodes, n):
        # each node's written edge slots in node order (reserved ones never filled hold garbage)
        f, c, rp = nodes["first_edge"][:n], nodes["n_children"][:n], (nodes["flags"][:n] & 1) != 0
        idx = np.concatenate([np.arange(a, a + (40 if r else k)) for a, k, r in zip(f, c, rp) if k > 0])
        unused = [np.arange(a + k, a + 10) for a, k, r in zip(f, c, rp) if r and k > 0]   # (childless: no run)
        return idx[~np.isin(idx, np.concatenate(unused))] if unused else idx

    for l, (n0, e0, r0), (n1, e1, r1) in zip((0, 7, 31), raw[6], diff[6]):
        n = int(raw[1][l, 1])
        for k in n0.dtype.names:                            # first_edge / pad (the row run) are pool addresses
            if k not in ("first_edge", "pad"):
                assert np.array_equal(n0[:n][k], n1[:n][k]), k
        assert np.array_equal(r0[:n], r1[:n])               # every node's game row, decoded
        ed0, ed1 = written(n0, n), written(n1, n)
        for k in ("opt", "child", "R", "S", "CS"):           # (an edge's 4 pad bytes are never written)
            assert np.array_equal(e0[ed0][k], e1[ed1][k]), k


@pytest.mark.parametrize("queue", [False, True])
def test_gpu_capacity_trees_match_reference(queue):
    """The two cfr_train(200000) trees whose card areas outgrew round 3's
    fixed lists (seed 31000322: a museum past 16; 31007440), through the
    config-5 product path -- simulate_games (one batch), and the tree queue
    with one slot (each tree searched in 0.5-s slices, targets extracted after
    its last) -- against the reference's own outputs: node and carry_out
    counts, decision, both streams' end states, every target
    (tests/golden/targets200000_cap.json.gz)."""
    from citadels_self_play_amd import selfplay
    recs = load_golden("targets200000_cap.json.gz")
    seeds = np.array([r["seed"] for r in recs], np.int64)
    if queue:
        b, stats, t = selfplay.simulate_queue(seeds, 200_000, slots=1, slice_seconds=0.5)
    else:
        b, stats, t = selfplay.simulate_games(seeds, 200_000)
    torch.cuda.synchronize()
    per = _split({k: t[k] for k in ("counts", "meta", "feat", "opt_feat", "value", "dist")})
    stats, rows, chosen = stats.cpu().numpy(), b.rows(), t["chosen"].cpu().numpy()
    mt, idx = b.mt.cpu().numpy().view(np.uint32), b.mt_idx.cpu().numpy()
    npmt, npidx = b.np_mt.cpu().numpy().view(np.uint32), b.np_idx.cpu().numpy()
    for l, r in enumerate(recs):
        root, n_nodes, n_edges, carry, err = stats[l]
        assert err == 0, (r["seed"], hex(int(err)))
        assert n_nodes == r["nodes"] and carry == r["carry_outs"], (r["seed"], n_nodes, carry)
        g = L.game_from_bytes(rows[l])
        assert canon.canon_option(L.opt_from_bytes(chosen[l]), g) == r["chosen"], r["seed"]
        assert hash_obj(mt[:, l].tolist() + [int(idx[l])]) == r["rng_after"][0], r["seed"]
        assert hash_obj(npmt[:, l].tolist()) == r["rng_after"][1] and int(npidx[l]) == r["rng_after"][2]
        check_targets(per[l], r["targets"], r["seed"])
