"""Golden fixtures for generate_test_data.setup_game (generate_test_data.py:9-31)
from the reference itself (build container only; writes
tests/golden/testdata500.json.gz).

Harness, per seed s:
    random.seed(s); np.random.seed(s)
    setup_game(s) with run_mccfr(..., max_iterations=500) instead of 20000
      game = create_game(); g = create_a_close_to_finished_game(game)   # run_utils.py:29-53
      x = g.encode_game(); _, root = run_mccfr(g, max_iterations=500)
      options = encode_options_from_node(root); target = create_target_strategy(root)

Recorded: the position (after the get_options calls that picked it), the
tuple (encode row, options sha256 + shape, node_value, target) or the
ValueError that setup_game swallows, node / carry_out counts, RNG end states.
"""
import gzip
import hashlib
import json
import os
import random
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "tests", "golden")
sys.path.insert(0, HERE)
sys.path.insert(0, REF)
sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))

import refcanon as rc  # noqa: E402
from gen_golden_cfr import count_nodes  # noqa: E402

ITERS = 500


def case(seed):
    import game.option as gopt
    from run_utils import (create_a_close_to_finished_game, create_game, create_target_strategy,
                           encode_options_from_node, run_mccfr)
    random.seed(seed)
    np.random.seed(seed)
    rec = {"seed": seed, "iters": ITERS}
    game = create_game()
    g = create_a_close_to_finished_game(game)
    rec["position"] = rc.canon_game(g)
    x = g.encode_game()
    counter = [0]
    orig = gopt.option.carry_out

    def counting(self, gm):
        counter[0] += 1
        return orig(self, gm)

    gopt.option.carry_out = counting
    try:
        _, root = run_mccfr(game=g, max_iterations=ITERS)
        opts = encode_options_from_node(root)
        if len(root.cumulative_regrets) == 0:
            rec["result"] = "empty"
        else:
            t = create_target_strategy(root)
            o = opts.detach().numpy().astype(np.float32)
            rec["result"] = {"encode": [int(v) for v in x.tolist()], "opts_shape": list(o.shape),
                             "opts_sha": hashlib.sha256(o.tobytes()).hexdigest()[:32],
                             "nv": np.asarray(root.node_value, np.float64).tolist(),
                             "dist": np.asarray(t.numpy(), np.float64).tolist()}
            rec["nodes"] = count_nodes(root)
    except ValueError as e:
        rec["result"] = "ValueError"
        rec["msg"] = str(e)[:80]
    finally:
        gopt.option.carry_out = orig
    rec["carry_outs"] = counter[0]
    rec["rng_after"] = [rc.hash_obj(list(random.getstate()[1])), rc.hash_obj(np.random.get_state()[1].tolist()),
                        int(np.random.get_state()[2])]
    return rec


def main():
    os.makedirs(OUT, exist_ok=True)
    recs = []
    for s in range(40):
        recs.append(case(s))
        r = recs[-1]["result"]
        print(s, r if isinstance(r, str) else len(r["dist"]), recs[-1].get("nodes"), flush=True)
    with gzip.open(os.path.join(OUT, "testdata500.json.gz"), "wt") as f:
        json.dump(recs, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
