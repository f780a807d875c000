"""Golden encode_game rows (game/game.py:91-128) and encode_option rows
(game/option.py:52-115) from the reference (build container only).

For preset and random-role games seeded 0..11, every 5th state of the
random-policy trajectory: the canonical state hash, Game.encode_game() (418
values, integers stored as ints) and encode_option() for the state's whole
option list (131 values each).  Also encode_game with gamestate.player_id
overridden to every player (deep_mccfr.py:120-123 does that on a role pick)."""
import gzip
import json
import os
import random
import sys

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "tests", "golden")
sys.path.insert(0, HERE)
sys.path.insert(0, REF)

import refcanon as rc  # noqa: E402


def ints(t):
    a = t.detach().cpu().numpy().astype(np.float64).ravel()
    assert (a == np.round(a)).all()
    return [int(x) for x in a]


def main():
    from game.game import Game
    recs = []
    for preset in (True, False):
        for seed in range(12):
            random.seed(seed)
            g = Game(preset=preset)
            g.setup_round()
            step = 0
            w = False
            while not w:
                opts = g.get_options_from_state()
                if step % 5 == 0:
                    rec = {"preset": preset, "seed": seed, "step": step, "state": rc.hash_obj(rc.canon_game(g)),
                           "encode": ints(g.encode_game()),
                           "options": [[rc.canon_option(o), ints(o.encode_option())] for o in opts[:40]]}
                    pid = g.gamestate.player_id
                    over = []
                    for i in range(6):
                        g.gamestate.player_id = i
                        over.append(ints(g.encode_game()))
                    g.gamestate.player_id = pid
                    rec["encode_pid"] = over
                    recs.append(rec)
                w = random.choice(opts).carry_out(g)
                step += 1
    with gzip.open(os.path.join(OUT, "encode.json.gz"), "wt") as f:
        json.dump(recs, f, separators=(",", ":"))
    print(len(recs), "records")


if __name__ == "__main__":
    main()
