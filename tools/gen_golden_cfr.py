"""Golden fixtures for the MCCFR search (algorithms/deep_mccfr.py) from the
reference itself (build container only; writes tests/golden/cfr_*.json.gz).

Harness ("config 3" position + decision), per seed s:
    random.seed(s); np.random.seed(s)
    game = create_game()                                  # run_utils.py:20-27
    for _ in range(random.randint(0, 300)):               # advance by random play
        if random.choice(game.get_options_from_state()).carry_out(game): break
    chosen, root = run_mccfr(game, max_iterations=N)      # run_utils.py:74-87 (no model)

Recorded: the position, the root game after the search (the root's
skip_false_choice mutates it), node count, carry_out calls made by the
search, the chosen option, root arrays, and for some seeds the whole tree in
DFS order.  `seaborn` (plotting only, absent here) is stubbed.
"""
import gzip
import json
import os
import random
import sys
import time
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "tests", "golden")
sys.path.insert(0, HERE)
sys.path.insert(0, REF)
sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))

import refcanon as rc  # noqa: E402


def arr(x):
    return np.asarray(x, dtype=np.float64).tolist()


def node_rec(n):
    extra = {}
    if hasattr(n, "pred_node_value"):
        extra["pred"] = arr(n.pred_node_value)
    return {**extra,
        "depth": n.depth, "player": n.current_player_id, "role_pick": int(bool(n.role_pick_node)),
        "terminal": int(bool(n.game.terminal)), "n_children": len(n.children),
        "node_value": arr(n.node_value), "wp": arr(n.winning_probabilities),
        "R": arr(n.cumulative_regrets), "S": arr(n.strategy), "CS": arr(n.cumulative_strategy),
        "game": rc.hash_obj(rc.canon_game(n.game)),
        "opts": [rc.canon_option(o) for o, _ in n.children],
    }


def dfs(n, out):
    out.append(node_rec(n))
    for _, c in n.children:
        dfs(c, out)


def count_nodes(n):
    return 1 + sum(count_nodes(c) for _, c in n.children)


def seeded_model():
    """ValueOnlyNN(418, 512): torch.manual_seed(0) init + the seeded BatchNorm
    statistics of tools/gen_golden_mlp.py ("bn" variant), eval mode."""
    import torch
    from algorithms.models import ValueOnlyNN
    torch.manual_seed(0)
    m = ValueOnlyNN(418, hidden_size=512)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for bn in (m.bn1, m.bn2):
            n = bn.num_features
            bn.running_mean.copy_(torch.randn(n, generator=g) * 0.5)
            bn.running_var.copy_(torch.rand(n, generator=g) * 2 + 0.1)
            bn.weight.copy_(torch.rand(n, generator=g) + 0.5)
            bn.bias.copy_(torch.randn(n, generator=g) * 0.1)
    return m.eval()


def case(seed, iters, tree, model=None):
    import game.option as gopt
    from run_utils import create_game, run_mccfr
    random.seed(seed)
    np.random.seed(seed)
    g = create_game()
    k = random.randint(0, 300)
    for _ in range(k):
        if random.choice(g.get_options_from_state()).carry_out(g):
            break
    rec = {"seed": seed, "iters": iters, "advance": k}
    if g.terminal:
        rec["skip"] = True
        return rec
    rec["position"] = rc.canon_game(g)
    counter = [0]
    orig = gopt.option.carry_out

    def counting(self, game):
        counter[0] += 1
        return orig(self, game)

    gopt.option.carry_out = counting
    t = time.time()
    try:
        if model is None:
            chosen, root = run_mccfr(g, max_iterations=iters)
        else:   # run_mccfr's model branch (run_utils.py:78-81) on the CPU
            from algorithms.deep_mccfr import CFRNode
            root = CFRNode(g, original_player_id=g.gamestate.player_id, model=model, training=False, device="cpu")
            root.cfr_pred(max_iterations=iters, max_depth=10)
            _, chosen = root.action_choice(live=True)
        rec["error"] = None
    except Exception as e:
        rec["error"] = type(e).__name__
        gopt.option.carry_out = orig
        return rec
    finally:
        gopt.option.carry_out = orig
    rec["seconds"] = time.time() - t
    rec["carry_outs"] = counter[0]
    rec["root_game"] = rc.canon_game(root.game)
    rec["nodes"] = count_nodes(root)
    rec["chosen"] = rc.canon_option(chosen)
    rec["root"] = node_rec(root)
    rec["rng_after"] = [rc.hash_obj(list(random.getstate()[1])), rc.hash_obj(np.random.get_state()[1].tolist()),
                        int(np.random.get_state()[2])]
    if tree:
        nodes = []
        dfs(root, nodes)
        rec["tree"] = nodes
    return rec


def main_pred():
    model = seeded_model()
    recs = []
    t = time.time()
    for s in range(16):
        recs.append(case(s, 200, tree=s < 4, model=model))
        print("pred", s, recs[-1].get("nodes"), recs[-1].get("carry_outs"), "%.1fs" % (time.time() - t), flush=True)
    with gzip.open(os.path.join(OUT, "cfr_pred200.json.gz"), "wt") as f:
        json.dump(recs, f, separators=(",", ":"))


def main_2000():
    """cfr_train2000.json.gz: 16 seeds, root records, no trees."""
    recs = []
    t = time.time()
    for s in range(100, 116):
        recs.append(case(s, 2000, tree=False))
        print(s, recs[-1].get("nodes"), recs[-1].get("carry_outs"), "%.1fs" % (time.time() - t), flush=True)
    with gzip.open(os.path.join(OUT, "cfr_train2000.json.gz"), "wt") as f:
        json.dump(recs, f, separators=(",", ":"))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "pred":
    main_pred()
elif __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "2000":
    main_2000()
elif __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    recs = []
    t = time.time()
    for s in range(24):
        recs.append(case(s, 200, tree=s < 6))
        print(s, recs[-1].get("nodes"), recs[-1].get("carry_outs"), "%.1fs" % (time.time() - t), flush=True)
    with gzip.open(os.path.join(OUT, "cfr_train200.json.gz"), "wt") as f:
        json.dump(recs, f, separators=(",", ":"))
    recs = []
    for s in (100, 101):
        recs.append(case(s, 2000, tree=False))
        print(s, recs[-1].get("nodes"), recs[-1].get("carry_outs"), "%.1fs" % (time.time() - t), flush=True)
    with gzip.open(os.path.join(OUT, "cfr_train2000.json.gz"), "wt") as f:
        json.dump(recs, f, separators=(",", ":"))
