"""The tree queue's pieces on the host build (csrc/cit_cfr.h cfr_train_slice,
cit_host.cpp): cfr_train run as resumable slices, and lanes whose finished
trees release their arena blocks and take the next position while the other
trees keep running, reproduce the cfr_train(2000) goldens exactly (node and
carry_out counts, chosen option, root game and arrays, both RNG end states,
whole trees) -- the same checks as test_cfr_host_golden."""
import numpy as np

from citadels_self_play_amd import canon
from citadels_self_play_amd import layout as L
from conftest import load_golden
from hostcheck import HostBatch, HostCfr
from test_cfr_host_golden import compare_node, dfs, hash_obj

CP_DONE = 3


def check_tree(cf, hb, l, stats, chosen, r):
    root, n_nodes, n_edges, carry, err = stats[l]
    assert err == 0, (r["seed"], err)
    g = hb.game(l)
    assert canon.canon_game(g) == r["root_game"], r["seed"]
    assert n_nodes == r["nodes"] and carry == r["carry_outs"], r["seed"]
    assert canon.canon_option(L.opt_from_bytes(chosen[l]), g) == r["chosen"], r["seed"]
    nodes, edges, rows = cf.tree(l)
    compare_node(nodes, edges, rows, root, r["root"], (r["seed"], "root"))
    assert hash_obj(hb.mt[:, l].tolist() + [int(hb.idx[l])]) == r["rng_after"][0], r["seed"]
    assert hash_obj(cf.npmt[:, l].tolist()) == r["rng_after"][1] and int(cf.npidx[l]) == r["rng_after"][2]
    if "tree" in r:
        order = dfs(nodes, edges, root, [])
        assert len(order) == len(r["tree"])
        for k, (i, want) in enumerate(zip(order, r["tree"])):
            compare_node(nodes, edges, rows, i, want, (r["seed"], k))


def recs2000(n):
    return [r for r in load_golden("cfr_train2000.json.gz") if not r.get("skip")][:n]


def test_slices_match_one_call():
    recs = recs2000(4)
    hb = HostBatch([r["seed"] for r in recs], True)
    cf = HostCfr(hb, node_cap=8192, edge_cap=5 * 8192)
    cf.advance(0, 300)
    cf.reset()
    st = np.zeros((hb.B, 16), np.int32)
    chosen = np.zeros((hb.B, 16), np.uint8)
    stats = np.zeros((hb.B, 5), np.int32)
    calls = 0
    while cf.train_slice(2000, st, 113, chosen, stats):
        calls += 1
    assert calls >= 2000 // 113 - 1
    assert (st[:, 6] == CP_DONE).all()
    for l, r in enumerate(recs):
        check_tree(cf, hb, l, stats, chosen, r)


def test_queue_release_and_refill():
    # 5 positions through 2 lanes: a finished lane is checked, releases its
    # blocks (reused, stale, by the next tree) and takes the next position
    recs = recs2000(5)
    src = HostBatch([r["seed"] for r in recs], True)
    HostCfr(src).advance(0, 300)
    hb = HostBatch([recs[0]["seed"], recs[1]["seed"]], True)
    cf = HostCfr(hb, node_cap=8192, edge_cap=5 * 8192)
    # two trees' worst case, less than the queue needs: released blocks are reused
    cf.pool = np.zeros(2 * L.cfr_pool_bytes(8192, 5 * 8192) + L.cfr_arena_bytes(4, 6), np.uint8)
    from hostcheck import lib, _p
    import ctypes as C
    lib().cith_cfr_arena_reset(_p(cf.pool), C.c_int(2), C.c_int(8192), C.c_int(5 * 8192), C.c_int(4), C.c_int(6))
    st = np.zeros((2, 16), np.int32)
    chosen = np.zeros((2, 16), np.uint8)
    stats = np.zeros((2, 5), np.int32)
    seed_np = HostCfr(src)                      # numpy streams of the queue's seeds

    def load(slot, q):
        hb.games[slot] = src.games[q]
        hb.mt[:, slot] = src.mt[:, q]
        hb.idx[slot] = src.idx[q]
        hb.seer[slot] = src.seer[q]
        cf.npmt[:, slot] = seed_np.npmt[:, q]
        cf.npidx[slot] = seed_np.npidx[q]
        st[slot] = 0

    slot_of = [0, 1]
    load(0, 0)
    load(1, 1)
    nxt, done = 2, 0
    while done < len(recs):
        cf.train_slice(2000, st, 97 + 31 * done, chosen, stats)
        for slot in range(2):
            q = slot_of[slot]
            if q is None or st[slot, 6] != CP_DONE:
                continue
            check_tree(cf, hb, slot, stats, chosen, recs[q])
            done += 1
            cf.release([slot])
            if nxt < len(recs):
                load(slot, nxt)
                slot_of[slot] = nxt
                nxt += 1
            else:
                slot_of[slot] = None
    hdr = cf.pool[2 * L.cfr_pool_bytes(8192, 5 * 8192):][:32].view("<u4")
    assert hdr[4] > 0 and hdr[5] >= hdr[4]          # trees took released node blocks from the ring
