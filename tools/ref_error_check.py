"""Does the reference itself raise on a config-5 tree the engine reports as an
error lane?  Runs simulate_game's search for one seed with the reference
(build container only; `seaborn` stubbed), counting carry_out calls, and
prints the exception (type, message) and the carry_out count at which it was
raised, to compare with the engine's stats row (carry_outs, err) for the
same seed (tools/diag_cfr_errors.py / tests/hostcheck.py):
    python tools/ref_error_check.py SEED ITERS"""
import json
import os
import random
import sys
import time
import types

import numpy as np

REF = "/root/reference"
sys.path.insert(0, REF)
sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))
sys.setrecursionlimit(100000)


def main():
    seed, iters = int(sys.argv[1]), int(sys.argv[2])
    import game.option as gopt
    from run_utils import create_a_random_game, run_mccfr
    random.seed(seed)
    np.random.seed(seed)
    g = create_a_random_game(100)
    counter = [0]
    orig = gopt.option.carry_out

    def counting(self, game):
        counter[0] += 1
        return orig(self, game)

    gopt.option.carry_out = counting
    t0 = time.time()
    err = None
    try:
        run_mccfr(g, model=None, max_iterations=iters, training=True)
    except Exception as e:
        err = [type(e).__name__, str(e)[:200]]
    print(json.dumps({"seed": seed, "iters": iters, "carry_outs": counter[0], "error": err,
                      "seconds": time.time() - t0}), flush=True)


if __name__ == "__main__":
    main()
