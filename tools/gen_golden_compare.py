"""Golden fixtures for compare_to_random.play_games (compare_to_random.py:8-37)
from the reference itself (build container only; writes
tests/golden/compare.json.gz).

The loop is play_games' own, per game seeded with random.seed(s),
np.random.seed(s), with smaller searches so it runs in minutes: seat 0 uses
the model path of run_mccfr (cfr_pred(PRED_ITERS, max_depth=10) + live choice
on the CPU, run_utils.py:78-81) with the seeded ValueOnlyNN of
gen_golden_cfr.seeded_model(); seat 1 uses run_mccfr(game, max_iterations=
TRAIN_ITERS); other seats random.choice.  Recorded: winner, step count,
searched-decision count, final game hash, RNG end states, and the decisions.
"""
import gzip
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
from gen_golden_cfr import seeded_model  # noqa: E402

PRED_ITERS, TRAIN_ITERS = 30, 60


def play(seed, model):
    from algorithms.deep_mccfr import CFRNode
    from run_utils import create_game, run_mccfr
    random.seed(seed)
    np.random.seed(seed)
    game = create_game()
    winner = False
    steps, decisions = 0, []
    while not winner:
        if game.gamestate.player_id == 0 and len(game.get_options_from_state()) > 1:
            root = CFRNode(game, original_player_id=game.gamestate.player_id, model=model, training=False,
                           device="cpu")
            root.cfr_pred(max_iterations=PRED_ITERS, max_depth=10)
            _, chosen = root.action_choice(live=True)
            decisions.append([0, steps, rc.canon_option(chosen)])
            winner = chosen.carry_out(game)
        elif game.gamestate.player_id == 1 and len(game.get_options_from_state()) > 1:
            chosen, _ = run_mccfr(game, max_iterations=TRAIN_ITERS)
            decisions.append([1, steps, rc.canon_option(chosen)])
            winner = chosen.carry_out(game)
        else:
            options = game.get_options_from_state()
            winner = random.choice(options).carry_out(game)
        steps += 1
    return {"seed": seed, "winner": winner.id, "steps": steps, "decisions": decisions,
            "final": rc.hash_obj(rc.canon_game(game)),
            "rng_after": [rc.hash_obj(list(random.getstate()[1])), rc.hash_obj(np.random.get_state()[1].tolist()),
                          int(np.random.get_state()[2])]}


def main():
    model = seeded_model()
    recs = []
    for s in range(3):
        recs.append(play(s, model))
        print(s, recs[-1]["winner"], recs[-1]["steps"], len(recs[-1]["decisions"]), flush=True)
    with gzip.open(os.path.join(OUT, "compare.json.gz"), "wt") as f:
        json.dump({"pred_iters": PRED_ITERS, "train_iters": TRAIN_ITERS, "games": recs}, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
