"""Generate the golden fixtures under tests/golden/ from the reference itself.

Runs ONLY in the build container (it imports /root/reference, which does not
exist on the GPU box).  The fixtures it writes are plain data (JSON, gzip):
inputs (seeds) and the reference's outputs (canonical states, option-list
digests, RNG streams).  No reference source is copied.

    python tools/gen_golden.py            # regenerate everything
"""
import gzip
import json
import os
import random
import sys
import time

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "tests", "golden")
sys.path.insert(0, HERE)
sys.path.insert(0, REF)

import refcanon as rc  # noqa: E402


def dump(name, obj):
    path = os.path.join(OUT, name)
    with gzip.open(path, "wt") as f:
        json.dump(obj, f, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes")


def rng_fixtures():
    """CPython `random` (MT19937 + init_by_array + _randbelow) and numpy legacy
    RandomState (init_genrand + random_sample + choice(p)) streams."""
    out = {"cpython": [], "numpy": []}
    for s in [0, 1, 7, 12345, 2**32 + 5, 2**40 + 7]:
        r = random.Random(s)
        st = r.getstate()[1]
        words = [r.getrandbits(32) for _ in range(1500)]
        r2 = random.Random(s)
        dbl = [r2.random() for _ in range(100)]
        r3 = random.Random(s)
        below = []
        for n in [1, 2, 3, 5, 7, 8, 9, 31, 56, 100, 1000, 2594]:
            below.append([n, [r3.randrange(n) for _ in range(20)]])
        r4 = random.Random(s)
        shuf = []
        for n in [0, 1, 2, 8, 76]:
            x = list(range(n))
            r4.shuffle(x)
            shuf.append(x)
        r5 = random.Random(s)
        samp = r5.sample(list(range(24)), 14)
        out["cpython"].append({"seed": s, "state0": list(st), "getrandbits32": words, "random": dbl,
                               "randbelow": below, "shuffle": shuf, "sample24_14": samp})
    for s in [0, 1, 7, 12345, 2**32 - 1]:
        rs = np.random.RandomState(s)
        key = rs.get_state()[1].tolist()
        dbl = rs.random_sample(100).tolist()
        rs2 = np.random.RandomState(s)
        ch = []
        for n in [1, 2, 3, 6, 10, 44]:
            p = rs2.random_sample(n)
            p = p / p.sum()
            ch.append([n, p.tolist(), [int(rs2.choice(range(n), p=p)) for _ in range(10)]])
        out["numpy"].append({"seed": s, "key0": key, "random_sample": dbl, "choice": ch})
    dump("rng_streams.json.gz", out)


def trajectory(seed, preset, full_opts=False, full_every=50):
    from game.game import Game
    random.seed(seed)
    np.random.seed(seed)
    g = Game(preset=preset)
    g.setup_round()
    rec = {"seed": seed, "preset": preset, "steps": [], "states": {}, "options": {}, "error": None}
    rec["states"]["0"] = rc.canon_game(g)
    winner = False
    step = 0
    try:
        while not winner:
            opts = g.get_options_from_state()
            oh = rc.hash_options(opts)
            if full_opts or step % full_every == 0:
                rec["options"][str(step)] = [rc.canon_option(o) for o in opts]
            pre_state, pre_pid = g.gamestate.state, g.gamestate.player_id
            # random.choice on the global stream, exactly as compare_to_random.py:37-39
            idx = random.randrange(len(opts)) if opts else None
            if idx is None:
                random.choice(opts)  # raises IndexError like the reference
            c = opts[idx]
            winner = c.carry_out(g)
            step += 1
            d = rc.canon_game(g)
            rec["steps"].append([pre_state, pre_pid, len(opts), oh, idx, rc.hash_obj(d)])
            if step % full_every == 0:
                rec["states"][str(step)] = d
    except Exception as e:  # reference crash: record it, the engine must flag the same step
        rec["error"] = [type(e).__name__, step]
    rec["states"]["final"] = rc.canon_game(g)
    rec["winner"] = winner.id if winner else -1
    rec["n_steps"] = step
    return rec


def trajectories(preset, seeds, full_opt_seeds, name):
    t = time.time()
    recs = [trajectory(s, preset, full_opts=(s in full_opt_seeds)) for s in seeds]
    print(name, "games", len(recs), "steps", sum(r["n_steps"] for r in recs),
          "errors", sum(1 for r in recs if r["error"]), "%.1fs" % (time.time() - t))
    dump(name, recs)


def fingerprint(preset, n):
    """Seat win-rate / steps-per-game fingerprint over n seeds."""
    from game.game import Game
    wins = [0] * 6
    steps = 0
    pts = 0
    errs = 0
    for s in range(n):
        random.seed(s)
        g = Game(preset=preset)
        g.setup_round()
        w = False
        try:
            while not w:
                w = random.choice(g.get_options_from_state()).carry_out(g)
                steps += 1
            wins[w.id] += 1
            pts += max(g.points)
        except Exception:
            errs += 1
    return {"preset": preset, "games": n, "wins": wins, "steps": steps, "winner_points": pts, "errors": errs}


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    rng_fixtures()
    trajectories(True, list(range(64)), {0, 1, 2, 3}, "traj_preset.json.gz")
    trajectories(False, list(range(32)), {0, 1}, "traj_random.json.gz")
    dump("fingerprint.json.gz", [fingerprint(True, 400), fingerprint(False, 200)])
