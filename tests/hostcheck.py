"""Loader for the TEST-ONLY host build of the engine headers
(csrc/cit_host.cpp -> build/libcitadels_hostcheck.so).  Used by the CPU test
suite to validate engine logic against the golden fixtures without a GPU."""
import ctypes as C
import os
import subprocess

import numpy as np

from citadels_self_play_amd import layout as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "citadels_self_play_amd", "csrc")
LIB = os.path.join(ROOT, "build", "libcitadels_hostcheck.so")

_lib = None


def build(force=False):
    srcs = [os.path.join(SRC, f) for f in ("cit_host.cpp", "cit_engine.h", "cit_core.h", "cit_cfr.h", "cit_area_test.h")]
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(s) for s in srcs):
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.check_call(["g++", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-strict-aliasing", "-shared", "-fPIC",
                           "-pthread", srcs[0], "-o", LIB])
    return LIB


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class HostBatch:
    """B games + their CPython MT streams in host memory, row layout identical to the device."""

    def __init__(self, seeds, preset=True):
        self.B = len(seeds)
        self.games = np.zeros((self.B, L.GAME_BYTES), np.uint8)
        self.mt = np.zeros((L.MT_N, self.B), np.uint32)
        self.idx = np.zeros(self.B, np.uint32)
        self.seeds = np.asarray(seeds, np.uint64)
        self.seer = np.zeros((self.B, L.SEER_MAX), np.uint64)
        lib().cith_init(_p(self.games), _p(self.mt), _p(self.idx), C.c_int(self.B), _p(self.seeds),
                        C.c_int(int(preset)))

    def game(self, l):
        return L.game_from_bytes(self.games[l])

    def get_options(self, max_opts=4096):
        out = np.zeros((self.B, max_opts, 16), np.uint8)
        n = np.zeros(self.B, np.int32)
        lib().cith_get_options(_p(self.games), _p(self.mt), _p(self.idx), _p(self.seer), C.c_int(self.B), _p(out),
                               C.c_int(max_opts), _p(n))
        return out, n

    def carry_out(self, chosen):
        w = np.zeros(self.B, np.int32)
        chosen = np.ascontiguousarray(chosen, np.uint8)
        lib().cith_carry_out(_p(self.games), _p(self.mt), _p(self.idx), C.c_int(self.B), _p(chosen), _p(w))
        return w

    def randbelow(self, lane, bound):
        out = np.zeros(1, np.uint32)
        lib().cith_mt_randbelow(_p(self.mt), _p(self.idx), C.c_int(self.B), C.c_int(lane), C.c_uint32(bound),
                                C.c_int(1), _p(out))
        return int(out[0])

    def rollout(self, max_steps=-1):
        steps = np.zeros(self.B, np.int32)
        w = np.zeros(self.B, np.int32)
        lib().cith_rollout(_p(self.games), _p(self.mt), _p(self.idx), _p(self.seer), C.c_int(self.B), C.c_int(max_steps),
                           _p(steps), _p(w))
        return steps, w


NODE_DT = np.dtype([("parent", "<i4"), ("first_edge", "<i4"), ("n_children", "<i2"), ("edge_cap", "<i2"),
                    ("depth", "<i2"), ("player", "i1"), ("gs_state", "i1"), ("flags", "u1"), ("winner", "i1"),
                    ("sib", "<i2"), ("pad", "u1", 4), ("nv", "<f8", 6), ("wp", "<f8", 6), ("pred", "<f8", 6)])
EDGE_DT = np.dtype([("opt", "u1", 16), ("child", "<i4"), ("pad", "<i4"), ("R", "<f8"), ("S", "<f8"), ("CS", "<f8")])
WIDE_DT = np.dtype([("R", "<f8", 6), ("S", "<f8", 6), ("CS", "<f8", 6)])
assert NODE_DT.itemsize == 168 and EDGE_DT.itemsize == 48 and WIDE_DT.itemsize == 3 * 48


def cfr_pool_bytes(node_cap, edge_cap, B=1, row_cap=0, pred=True):
    """A host pool of B trees with the worst-case arena (layout.cfr_* / cit_cfr.h)."""
    return B * L.cfr_pool_bytes(node_cap, edge_cap) + \
        L.cfr_arena_bytes(B * L.cfr_nblocks(node_cap), B * L.cfr_eblocks(edge_cap), row_cap, pred)


def node_arrays(nodes, edges, n):
    """(R, S, CS) of node n as the reference holds them: [nch] for a normal
    node, [6, 10] for a role-pick node (its wide records follow its 10 edges)."""
    N = nodes[n]
    nch, f = int(N["n_children"]), int(N["first_edge"])
    if nch == 0:
        return np.zeros(0), np.zeros(0), np.zeros(0)
    if N["flags"] & 1:
        W = edges[f + 10:f + 40].view(WIDE_DT)[:nch]
        return W["R"].T.copy(), W["S"].T.copy(), W["CS"].T.copy()
    E = edges[f:f + nch]
    return E["R"].copy(), E["S"].copy(), E["CS"].copy()


class HostCfr:
    """Host-build MCCFR decisions over a HostBatch (config-3 harness)."""

    def __init__(self, hb, node_cap=2048, edge_cap=4096, row_cap=0, pred=True):
        self.hb = hb
        B = hb.B
        self.node_cap, self.edge_cap, self.row_cap, self.pred = node_cap, edge_cap, row_cap, pred
        self.npmt = np.zeros((L.MT_N, B), np.uint32)
        self.npidx = np.zeros(B, np.uint32)
        lib().cith_mt_seed(_p(self.npmt), _p(self.npidx), C.c_int(B), _p(hb.seeds), C.c_int(1))
        self.pool = np.zeros(cfr_pool_bytes(node_cap, edge_cap, B, row_cap, pred), np.uint8)
        self.optbuf = np.zeros((B, 512, 16), np.uint8)

    def advance(self, lo, hi):
        steps = np.zeros(self.hb.B, np.int32)
        hb = self.hb
        lib().cith_advance_random(_p(hb.games), _p(hb.mt), _p(hb.idx), _p(hb.seer), C.c_int(hb.B), C.c_int(lo),
                                  C.c_int(hi), _p(steps))
        return steps

    def reset(self):
        """Empty block tables and arena (before each search; cfr_pred resumptions keep them)."""
        B = self.hb.B
        lib().cith_cfr_arena_reset_fmt(_p(self.pool), C.c_int(B), C.c_int(self.node_cap), C.c_int(self.edge_cap),
                                       C.c_int(B * L.cfr_nblocks(self.node_cap)),
                                       C.c_int(B * L.cfr_eblocks(self.edge_cap)), C.c_int(self.row_cap),
                                       C.c_int(int(self.pred)))

    def decide(self, iters, flags=0):
        hb = self.hb
        self.reset()
        chosen = np.zeros((hb.B, 16), np.uint8)
        stats = np.zeros((hb.B, 5), np.int32)
        lib().cith_cfr_decide(_p(hb.games), _p(hb.mt), _p(hb.idx), _p(self.npmt), _p(self.npidx), _p(hb.seer),
                              C.c_int(hb.B), C.c_int(iters), C.c_int(flags), _p(self.pool), C.c_int(self.node_cap),
                              C.c_int(self.edge_cap), _p(self.optbuf), _p(chosen), _p(stats))
        return chosen, stats

    def train_slice(self, iters, state, slice_iters, chosen, stats, flags=0):
        """One cit_cfr_train_slice call (budget: slice_iters iterations per tree);
        returns the number of trees still running."""
        hb = self.hb
        return lib().cith_cfr_train_slice(_p(hb.games), _p(hb.mt), _p(hb.idx), _p(self.npmt), _p(self.npidx),
                                          _p(hb.seer), C.c_int(hb.B), C.c_int(iters), C.c_int(flags), _p(self.pool),
                                          C.c_int(self.node_cap), C.c_int(self.edge_cap), _p(self.optbuf), _p(state),
                                          C.c_int(slice_iters), _p(chosen), _p(stats))

    def release(self, lanes):
        lanes = np.ascontiguousarray(lanes, np.int32)
        lib().cith_cfr_arena_release(_p(self.pool), C.c_int(self.hb.B), C.c_int(self.node_cap), C.c_int(self.edge_cap),
                                     _p(lanes), C.c_int(len(lanes)))

    def tree(self, l):
        nodes, edges, rows = L.cfr_tree_bytes(lambda o, n: self.pool[o:o + n], self.hb.B, l, self.node_cap,
                                              self.edge_cap)
        return nodes.view(NODE_DT), edges.view(EDGE_DT), rows


def encode_games(hb, pid=-1):
    out = np.zeros((hb.B, 418), np.float32)
    lib().cith_encode_games(_p(hb.games), C.c_int(hb.B), C.c_int(pid), _p(out))
    return out


def encode_options(game_row, opts):
    opts = np.ascontiguousarray(opts, np.uint8)
    out = np.zeros((len(opts), 131), np.float32)
    row = np.ascontiguousarray(game_row, np.uint8)
    lib().cith_encode_options(_p(row), _p(opts), C.c_int(len(opts)), _p(out))
    return out


def cfr_pred(cf, iters, max_depth, mlp):
    """Drive the resumable host-build cfr_pred: between resumptions, evaluate
    the suspended lanes' feature rows with `mlp` (feat [k,418] -> probs [k,6])."""
    hb = cf.hb
    B = hb.B
    st = np.zeros((B, 16), np.int32)            # CfrState (64 B)
    probs = np.zeros((B, 6), np.float32)
    feat = np.zeros((B, 418), np.float32)
    chosen = np.zeros((B, 16), np.uint8)
    rounds = 0
    cf.reset()
    while True:
        w = lib().cith_cfr_pred_step(_p(hb.games), _p(hb.mt), _p(hb.idx), _p(cf.npmt), _p(cf.npidx), _p(hb.seer),
                                     C.c_int(B), C.c_int(iters), C.c_int(max_depth), _p(cf.pool),
                                     C.c_int(cf.node_cap), C.c_int(cf.edge_cap), _p(cf.optbuf), _p(st), _p(probs),
                                     _p(feat), _p(chosen))
        if w == 0:
            break
        waiting = st[:, 6] == 2
        probs[waiting] = mlp(feat[waiting])
        rounds += 1
    stats = np.stack([st[:, 8], st[:, 0], st[:, 1], st[:, 3], st[:, 2]], axis=1)
    return chosen, stats, rounds


def random_position(hb, max_move=100):
    """random.seed(seed); create_a_random_game(max_move) on every lane."""
    lib().cith_mt_seed(_p(hb.mt), _p(hb.idx), C.c_int(hb.B), _p(hb.seeds), C.c_int(0))
    ring = np.zeros(max_move * L.GAME_BYTES // 4, np.uint32)
    steps = np.zeros(hb.B, np.int32)
    lib().cith_random_position(_p(hb.games), _p(hb.mt), _p(hb.idx), _p(hb.seer), C.c_int(hb.B), C.c_int(max_move),
                               _p(ring), _p(steps))
    return steps


def close_position(hb):
    """create_a_close_to_finished_game on every lane's created game."""
    store = np.zeros(130 * L.GAME_BYTES // 4, np.uint32)
    index = np.zeros(hb.B, np.int32)
    lib().cith_close_position(_p(hb.games), _p(hb.mt), _p(hb.idx), _p(hb.seer), C.c_int(hb.B), _p(store), _p(index))
    return index


def cfr_root_target(cf, roots):
    """create_target_strategy + encode_options_from_node at each lane's root ->
    per lane (None, options, node_value, target) or None."""
    t = cfr_targets(cf, roots, mode=1)
    out = [None] * cf.hb.B
    for k, (lane, node, pid, nch, c0) in enumerate(t["meta"]):
        out[lane] = (None, t["opt_feat"][c0:c0 + nch], t["value"][k], t["dist"][c0:c0 + nch])
    return out


def cfr_targets(cf, roots, mode=0):
    """get_all_targets over every lane's finished tree -> dict of arrays (see cfr_emit_targets)."""
    hb = cf.hb
    roots = np.ascontiguousarray(roots, np.int32)
    counts = np.zeros((hb.B, 2), np.int32)
    lib().cith_cfr_target_count(_p(cf.pool), C.c_int(hb.B), C.c_int(cf.node_cap), C.c_int(cf.edge_cap), _p(roots),
                                C.c_int(mode), _p(counts))
    offs = np.zeros_like(counts)
    offs[1:] = np.cumsum(counts, axis=0)[:-1]
    nt, nc = int(counts[:, 0].sum()), int(counts[:, 1].sum())
    out = {"meta": np.zeros((nt, 5), np.int32), "feat": np.zeros((nt, 418), np.float32),
           "value": np.zeros((nt, 6), np.float64), "dist": np.zeros(nc, np.float64),
           "opt_feat": np.zeros((nc, 131), np.float32), "counts": counts}
    lib().cith_cfr_targets(_p(cf.pool), C.c_int(hb.B), C.c_int(cf.node_cap), C.c_int(cf.edge_cap), _p(roots),
                           C.c_int(mode), _p(hb.mt), _p(hb.idx), _p(offs), _p(out["meta"]), _p(out["feat"]), _p(out["value"]),
                           _p(out["dist"]), _p(out["opt_feat"]))
    return out


def split_targets(t):
    """Per-lane lists of (feat, options [nch,131], node_value, regret target) tuples."""
    per = [[] for _ in range(len(t["counts"]))]
    for k, (lane, node, pid, nch, c0) in enumerate(t["meta"]):
        per[lane].append((t["feat"][k], t["opt_feat"][c0:c0 + nch], t["value"][k], t["dist"][c0:c0 + nch]))
    return per


def compare_game(seed, fma, pred_iters, train_iters, node_cap=2048):
    """compare_to_random's loop for one game on the host build of the engine:
    cith_advance_policy between decisions, cith_cfr_pred_step (seat 0, `fma`
    leaf evaluator) and cith_cfr_decide (seat 1).  Returns (hb, random steps,
    decisions [(seat, option descriptor, game before carry_out)])."""
    hb = HostBatch([seed], True)
    cf = HostCfr(hb, node_cap=node_cap, edge_cap=8 * node_cap)
    status = np.zeros(1, np.int32)
    steps = np.zeros(1, np.int32)
    decisions = []
    while True:
        lib().cith_advance_policy(_p(hb.games), _p(hb.mt), _p(hb.idx), _p(hb.seer), C.c_int(1), C.c_int(3),
                                  C.c_int(-1), _p(status), _p(steps))
        seat = int(status[0])
        if seat < 0:
            return hb, int(steps[0]), decisions
        if seat == 0:
            chosen, stats, _ = cfr_pred(cf, pred_iters, 10, fma)
        else:
            chosen, stats = cf.decide(train_iters)
        assert stats[0][4] == 0, stats
        decisions.append((seat, chosen[0].copy(), hb.game(0)))
        hb.carry_out(chosen)
