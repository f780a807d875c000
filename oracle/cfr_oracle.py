"""CPU ORACLE (test infrastructure only) — MCCFR search restated.

Restates algorithms/deep_mccfr.py (no-model and model paths) and
Game.sample_private_information (game/game.py:183-339) over the oracle's own
game model (citadels_oracle.OGame).  Randomness: one CPython stream per tree
(the games of a tree share it, as every reference game shares the module
`random`), one numpy RandomState per tree (the reference's global
np.random).  fp64 arithmetic is numpy's own (np.exp, np.sum, choice).

Pinned by tests/test_cfr_oracle_golden.py against tests/golden/cfr_*.json.gz
(made from the reference by tools/gen_golden_cfr.py).
"""
import copy

import numpy as np

import citadels_oracle as O
from citadels_oracle import BEWITCHED, OGS, rank, rprop

LN13 = np.log(1.3)


# ---------------------------------------------------------------- cloning
def clone(g):
    """deepcopy(game) keeping the shared streams shared (the reference's games
    all draw from the module-level `random`)."""
    rng, nprng = g.rng, getattr(g, "nprng", None)
    g.rng = None
    g.nprng = None
    try:
        c = copy.deepcopy(g)
    finally:
        g.rng, g.nprng = rng, nprng
    c.rng, c.nprng = rng, nprng
    return c


def _gs_eq(self, o):
    """GameState.__eq__ (helper_classes.py:29-32): state and player only."""
    return isinstance(o, OGS) and self.state == o.state and self.pid == o.pid


OGS.__eq__ = _gs_eq
OGS.__hash__ = object.__hash__


# ------------------------------------------- determinization (game.py:183-339)
def unknown_cards(g, pc):
    """get_unknown_cards (game.py:183-213)."""
    unk = list(g.used_cards)
    for p in g.players:
        for c in p.build:
            O.take_like(unk, c)
    for p in g.players:
        for c in p.museum:
            O.take_like(unk, c)
    for c in pc.hand:
        O.take_like(unk, c)
    for h in pc.kh:
        if h.used:
            for c in h.cards:
                O.take_like(unk, c)
    return unk


def _strip(kr, role, g):
    """remove_role_from_role_knowledge (game.py:298-301) on a copied knowledge list."""
    for k in kr:
        if not k[1]:
            m = 0
            for rid in range(-1, 8):
                if (k[0] >> (rid + 1)) & 1 and g.role_mask_name(rid) != role:
                    m |= 1 << (rid + 1)
            k[0] = m


def sample_private_information(g, pc, role_sample=True):
    """game.py:215-242, 245-339."""
    for h in pc.kh:
        r = g.rng.random()
        h.used = (h.conf - 1) * 0.2 > r
    unk = unknown_cards(g, pc)
    # sample_deck (:245-262)
    n = len(g.deck)
    lk = next((h for h in pc.kh if h.pid == -1 and h.used), None)
    lk_cards = list(lk.cards) if lk is not None else None
    g.deck = []
    if lk_cards is not None:
        for _ in range(min(len(lk_cards), n)):
            O.put(g.deck, lk_cards.pop(0))
            n -= 1
    g.rng.shuffle(unk)
    for _ in range(n):
        O.put(g.deck, O.draw(unk))
    # sample_warrants_and_blackmails (:321-336)
    bm = [r for r in range(8) if g.rp[r][4] is not None]
    if bm:
        g.rng.shuffle(bm)
        for r in bm:
            g.rp[r][4] = "Real" if r == bm[0] else "Fake"
    wr = [r for r in range(8) if g.rp[r][1] is not None]
    if wr:
        g.rng.shuffle(wr)
        for r in wr:
            g.rp[r][1] = "Real" if r == wr[0] else "Fake"
    kr = [[k[0], k[1]] for k in pc.kr]
    if role_sample:
        # remove_role_and_smaller_id_roles_from_role_knowledge_if_unconfirmed (:304-310)
        role = g.players[g.gs.pid].role
        _strip(kr, role, g)
        if role is not None:
            for rid in range(8):
                if rid < rank(role):
                    _strip(kr, g.roles[rid], g)
    for p in g.players:
        # sample_cards_for_opponent (:264-280)
        if p is not pc:
            hk = next((h for h in pc.kh if h.pid == p.id and h.used), None)
            hk_cards = list(hk.cards) if hk is not None else None
            n = len(p.hand)
            p.hand = []
            if hk_cards is not None:
                for _ in range(min(len(hk_cards), n)):
                    O.put(p.hand, hk_cards.pop(0))
                    n -= 1
            for _ in range(n):
                O.put(p.hand, O.draw(unk))
        # sample_roles_for_opponent (:283-295)
        if role_sample and p is not pc and p.id != g.gs.pid and g.gs.state != 0:
            mask = kr[p.id][0]
            vals = [g.role_mask_name(rid) for rid in range(-1, 8) if (mask >> (rid + 1)) & 1]
            k = g.rng._randbelow(len(vals))
            if vals:
                p.role = vals[k]
                _strip(kr, p.role, g)
            else:   # the IndexError band-aid
                p.role = next(g.roles[rid] for rid in range(8) if rid not in g.used_roles)
    if role_sample and g.gs.state != 0:
        g.refresh_used_roles()


# ------------------------------------------------------------- search tree
class Node:
    """CFRNode (deep_mccfr.py:8-35)."""

    def __init__(self, tree, game, parent=None, depth=0):
        self.tree = tree
        self.game = game
        self.depth = depth
        tree.count += 1
        self.skip_forced()
        self.parent = parent
        self.children = []
        self.player = game.gs.pid
        self.R = np.array([])
        self.S = np.array([])
        self.CS = np.array([])
        self.nv = np.zeros(6)
        self.wp = np.zeros(6)
        self.role_pick = game.gs.state == 0
        self.pred = None

    def skip_forced(self):
        """skip_false_choice (:37-49): plays single-option steps on this node's game."""
        g = self.game
        i = 0
        opts = g.get_options()
        done = False
        while len(opts) == 1 and not done:
            i += 1
            done = self.tree.carry(g, opts[0]) is not None
            opts = g.get_options()
            if i > 100:
                done = True

    # -- strategies ---------------------------------------------------------
    def update_strategy(self):
        """:292-319"""
        t = np.exp(-self.R * LN13)
        if not self.role_pick:
            tot = np.sum(t)
            self.S = t / tot if tot > 0 else np.ones_like(t) / len(t)
        else:
            tot = np.sum(t, axis=0)
            if np.any(tot <= 1e-8):
                self.S = np.where(tot > 1e-8, t / tot, 1.0 / t.shape[0])
            else:
                self.S = t / tot
        self.CS = self.CS + self.S
        self.CS = self.CS / self.CS.sum()

    def choose(self, live=False):
        """action_choice (:67-91) and weighted_average_strategy (:51-65)."""
        npr = self.tree.np
        if not self.role_pick:
            p = self.CS / self.CS.sum()
            k = npr.choice(range(len(self.children)), p=p)
            return self.children[k][1], self.children[k][0]
        if live:
            return None, self.role_preference(self.S[self.game.gs.pid])
        order = self.game.turn
        w = np.zeros(self.CS.shape[1])
        for i, pidx in enumerate(order):
            w += self.CS[pidx] * (len(order) - i)
        avg = w / sum(order)
        p = np.ones(len(self.children)) / len(self.children) if avg.sum() == 0 else avg / avg.sum()
        k = npr.choice(range(len(self.children)), p=p)
        return self.children[k][1], self.children[k][0]

    def role_preference(self, strat):
        """Game.get_option_from_role_preference (game.py:312-317)."""
        opts = self.game.get_options()
        ids = [rank(O.R[o.a["choice"]]) for o in opts]
        sub = strat[ids]
        sub /= sub.sum()
        return self.tree.np.choice(opts, p=sub)

    # -- expansion ----------------------------------------------------------
    def expand(self):
        """:93-100"""
        if self.game.gs.state == 0 and not self.children:
            self.role_pick = True
            self.expand_role_pick()
        elif self.player == self.tree.orig and not self.children:
            self.expand_own()
        elif self.player != self.tree.orig and len(self.children) < 10:
            self.expand_opponent()

    def _needs_sample(self, g):
        return self.parent is None or g.gs.pid != self.parent.game.gs.pid

    def _role_sample(self):
        return self.parent.game.gs.state != 0 if self.parent is not None else False

    def expand_role_pick(self):
        """:102-131 (child keyed by the LAST pick of the playout)."""
        tr = self.tree
        for _ in range(10):
            h = clone(self.game)
            last = None
            while h.gs.state != 1:
                opts = h.get_options()
                k = tr.np.choice(range(len(opts)), p=np.ones(len(opts)) / len(opts))
                last = opts[k]
                tr.carry(h, opts[k])
            self.children.append((last, Node(tr, h, self, self.depth + 1)))
        n = len(self.children)
        if tr.model is not None:
            for i in range(6):
                h = clone(self.game)
                h.gs.pid = i
                wp = tr.infer(h)
            if not tr.training:
                self.pred = tr.weight * wp
        self.R = np.zeros((n, 6)).T
        self.S = np.zeros((n, 6)).T
        self.CS = np.zeros((n, 6)).T

    def expand_own(self):
        """:133-151"""
        tr = self.tree
        opts = self.game.get_options()
        for o in opts:
            h = clone(self.game)
            if self._needs_sample(h):
                sample_private_information(h, h.players[tr.orig], self._role_sample())
            tr.carry(h, o)
            self.children.append((o, Node(tr, h, self, self.depth + 1)))
        if tr.model is not None:
            wp = tr.infer(self.game)
            if not tr.training:
                self.pred = tr.weight * wp
        self.R = np.zeros(len(self.children))
        self.S = np.zeros(len(self.children))
        self.CS = np.zeros(len(self.children))

    def expand_opponent(self):
        """:153-179"""
        tr = self.tree
        h = clone(self.game)
        if self._needs_sample(h):
            sample_private_information(h, h.players[tr.orig], self._role_sample())
        opts = h.get_options()
        if tr.model is not None:
            tr.infer(h)
        k = tr.np.choice(range(len(opts)), p=np.ones(len(opts)) / len(opts))
        tr.carry(h, opts[k])
        if not any(opts[k] == c for c, _ in self.children):
            self.children.append((opts[k], Node(tr, h, self, self.depth + 1)))
            self.R = np.append(self.R, 0)
            self.S = np.append(self.S, 0)
            if tr.model is not None:
                wp = tr.infer(self.game)
                if not tr.training:
                    self.pred = tr.weight * wp
            self.CS = np.append(self.CS, 0)

    # -- backup ---------------------------------------------------------------
    def backpropagate(self, reward):
        """:276-290 (iterative: same order of updates as the recursion)."""
        n = self
        tr = self.tree
        while n is not None:
            if tr.training or (n.nv.sum() == 0 or tr.model is None):
                n.nv += reward
            n.wp = n.nv / n.nv.sum()
            if n.children:
                n.update_regrets()
            n = n.parent

    def update_regrets(self):
        """:231-256"""
        if not self.role_pick:
            p = self.player
            act = [c.wp[p] for _, c in self.children]
            mx = max(act)
            for a in range(len(self.children)):
                self.R[a] += mx - act[a]
        else:
            A = np.array([c.wp for _, c in self.children]).T
            self.R += np.max(A, axis=0) - A


class Tree:
    def __init__(self, game, orig, model=None, training=False, weight=5, np_rng=None):
        self.orig = orig
        self.model = model
        self.training = training
        self.weight = weight
        self.np = np_rng
        self.count = 0
        self.carry_outs = 0
        self.root = Node(self, game)

    def carry(self, g, o):
        self.carry_outs += 1
        return g.carry_out(o)

    def infer(self, g):
        """model_inference (deep_mccfr.py:364-374): float32 winning probabilities."""
        return np.asarray(self.model(g), np.float32)

    def cfr_train(self, iters):
        """:187-205"""
        root = self.root
        if root.game.terminal:
            return
        root.expand()
        n = root
        for _ in range(iters):
            n.update_strategy()
            n, _ = n.choose()
            if n.game.terminal:
                n.backpropagate(reward(n.game))
                n.update_strategy()
                n = root
            else:
                n.expand()
        root.update_strategy()

    def cfr_pred(self, iters, max_depth):
        """:207-229"""
        root = self.root
        if root.game.terminal:
            return
        root.expand()
        n = root
        for _ in range(iters):
            n.update_strategy()
            n, _ = n.choose()
            if n.depth > max_depth and not n.game.terminal:
                n.expand()
                n.backpropagate(n.pred)
                n.update_strategy()
                n = root
            elif n.game.terminal:
                n.backpropagate(reward(n.game))
                n.update_strategy()
                n = root
            else:
                n.expand()
        root.update_strategy()


def reward(g):
    r = np.zeros(6)
    if g.winner >= 0:
        r[g.winner] = 1
    return r


def run_mccfr(game, np_rng, iters, model=None, training=False):
    """run_utils.run_mccfr (run_utils.py:74-87): returns (chosen option, tree)."""
    game.nprng = np_rng
    tr = Tree(game, game.gs.pid, model=model, training=training, np_rng=np_rng)
    if model is not None and not training:
        tr.cfr_pred(iters, 10)
    else:
        tr.cfr_train(iters)
    _, chosen = tr.root.choose(live=True)
    return chosen, tr


def config3_position(seed):
    """The config-3 harness of tools/gen_golden_cfr.py: returns (game, np_rng) or None."""
    g = O.new_game(seed, True)
    npr = np.random.RandomState(seed)
    k = g.rng.randint(0, 300)
    for _ in range(k):
        opts = g.get_options()
        if g.carry_out(opts[g.rng._randbelow(len(opts))]) is not None:
            break
    if g.terminal:
        return None
    return g, npr


def dfs(node, out):
    out.append(node)
    for _, c in node.children:
        dfs(c, out)
    return out


# ------------------------------------------------------- training targets
def random_position(seed, max_move=100):
    """create_a_random_game(max_move) (run_utils.py:55-73) after random.seed(seed),
    np.random.seed(seed): k = randint(1, max_move); a preset game played to the
    end by random.choice, keeping a deep copy after every step; returns
    (games[-k], np_rng).  The stream continues from the end of the playout."""
    import random as _random
    rng = _random.Random(seed)
    k = rng.randint(1, max_move)
    g = O.new_game(None, True, rng)
    snaps = [clone(g)]
    while True:
        opts = g.get_options()
        w = g.carry_out(opts[rng._randbelow(len(opts))])
        snaps.append(clone(g))
        if w is not None:
            break
    return snaps[-k], np.random.RandomState(seed)


BUILD_THRESHOLD = 15    # build_train_targets' default; get_all_targets never passes its own (:268)


def build_train_targets(node, rng):
    """deep_mccfr.py:321-345 -> (encode_game f32[418], options f32[nch,131],
    node_value f64[6], regret target f64[nch] or f64[10])."""
    import mlp_oracle as M
    if not node.children or node.nv.sum() < BUILD_THRESHOLD:
        return []
    opts = np.stack([M.encode_option(o) for o, _ in node.children])
    if node.role_pick:
        i = rng.randint(0, 5)
        x = M.encode_game(node.game, i)
        dist = np.array(node.R[i], dtype=np.float64)
    else:
        x = M.encode_game(node.game)
        dist = np.array(node.R, dtype=np.float64)
    if dist.sum() == 0:
        dist = np.ones_like(dist)
    return [(x, opts, node.nv.copy(), dist)]


def get_all_targets(node, rng, out=None):
    """get_all_targets (deep_mccfr.py:258-274): pre-order over the tree."""
    out = [] if out is None else out
    out += build_train_targets(node, rng)
    for _, c in node.children:
        get_all_targets(c, rng, out)
    return out


def simulate_game(seed, iters, max_move=100):
    """simulate_game (train_from_scratch.py:23-36, pretrain: no model, training=True)
    on a seeded position; returns (position, chosen, tree, targets) or raises like
    the reference on a terminal position (action_choice on a childless root)."""
    g, npr = random_position(seed, max_move)
    pos = clone(g)
    chosen, tr = run_mccfr(g, npr, iters, training=True)
    return pos, chosen, tr, get_all_targets(tr.root, g.rng)


# --------------------------------------------------- generate_test_data
def close_position(g, max_back=30):
    """create_a_close_to_finished_game(game) (run_utils.py:29-53): plays `g` to
    the end (deep copy before the first and after every step), then examines
    games[-k] for k = randint(1, max_back), k-1, ... (Python indexing, so k <= 0
    wraps to the front) until one has >= 2 options, at most 100 times."""
    rng = g.rng
    k = rng.randint(1, max_back)
    games = [clone(g)]
    while True:
        opts = g.get_options()
        w = g.carry_out(opts[rng._randbelow(len(opts))])
        games.append(clone(g))
        if w is not None:
            break
    opts, limit, pos = [], 0, None
    while len(opts) < 2 and limit < 100:
        pos = games[-k]
        opts = pos.get_options()
        k -= 1
        limit += 1
    return pos


def setup_game(seed, iters):
    """generate_test_data.setup_game (generate_test_data.py:9-31) after
    random.seed(seed), np.random.seed(seed), with run_mccfr(max_iterations=iters).
    Returns (position, result) where result is "ValueError", "empty" or
    (encode_game, options [nch,131], node_value, target) (create_target_strategy,
    run_utils.py:98-109), and the tree (or None)."""
    import mlp_oracle as M
    g = O.new_game(seed, True)
    npr = np.random.RandomState(seed)
    pos = close_position(g)
    snap = clone(pos)
    x = M.encode_game(pos)
    try:
        _, tr = run_mccfr(pos, npr, iters)
    except ValueError:
        return snap, "ValueError", None
    root = tr.root
    opts = np.stack([M.encode_option(o) for o, _ in root.children]) if root.children else None
    if len(root.R) == 0:
        return snap, "empty", tr
    R = np.array(root.R, dtype=np.float64)
    if R.shape == (6, 10):
        R = R[pos.rng.randint(0, 5)]
    if R.sum() == 0:
        R = np.ones_like(R)
    return snap, (x, opts, root.nv.copy(), R), tr


# ---------------------------------------------------- compare_to_random
def compare_game(seed, model, pred_iters=200, train_iters=2000):
    """compare_to_random.play_games' loop (compare_to_random.py:16-35) for one
    game after random.seed(seed), np.random.seed(seed): seat 0 run_mccfr with
    the model (cfr_pred(pred_iters, 10)), seat 1 run_mccfr(train_iters), both
    only with > 1 option; other seats random.choice.  `model` maps a game to
    float32 winning probabilities.  Returns (game, steps, decisions)."""
    g = O.new_game(seed, True)
    npr = np.random.RandomState(seed)
    g.nprng = npr
    steps, decisions = 0, []
    while True:
        pid = g.gs.pid
        if pid == 0 and len(g.get_options()) > 1:
            chosen, _ = run_mccfr(g, npr, pred_iters, model=model)
            decisions.append([0, steps, chosen.canon()])
            w = g.carry_out(chosen)
        elif pid == 1 and len(g.get_options()) > 1:
            chosen, _ = run_mccfr(g, npr, train_iters)
            decisions.append([1, steps, chosen.canon()])
            w = g.carry_out(chosen)
        else:
            opts = g.get_options()
            w = g.carry_out(opts[g.rng._randbelow(len(opts))])
        steps += 1
        if w is not None:
            return g, steps, decisions
