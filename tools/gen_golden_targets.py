"""Golden fixtures for the training-data path of train_from_scratch
("config 5") from the reference itself (build container only; writes
tests/golden/targets2000.json.gz).

Harness, per seed s (simulate_game, train_from_scratch.py:23-36, pretrain):
    random.seed(s); np.random.seed(s)
    game = create_a_random_game(100)                        # run_utils.py:55-73
    _, root = run_mccfr(game, None, max_iterations=M, training=True)   # run_utils.py:75-87
    targets = root.get_all_targets(usefulness_treshold=200) # deep_mccfr.py:258-274,321-345

Recorded per seed: the position, node / carry_out counts, the chosen option,
RNG end states, and every target tuple: encode_game row (small ints), the
options' encode_option rows (sha256 of the float32 bytes + shape),
node_value and the regret target (float64 lists).  `seaborn` is stubbed.
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


def case(seed, iters):
    import game.option as gopt
    from run_utils import create_a_random_game, run_mccfr
    random.seed(seed)
    np.random.seed(seed)
    g = create_a_random_game(100)
    rec = {"seed": seed, "iters": iters, "position": rc.canon_game(g)}
    counter = [0]
    orig = gopt.option.carry_out

    def counting(self, game):
        counter[0] += 1
        return orig(self, game)

    gopt.option.carry_out = counting
    try:
        chosen, root = run_mccfr(g, model=None, max_iterations=iters, training=True)
    except Exception as e:           # a terminal position, or the reference's ValueErrors
        rec["error"] = type(e).__name__
        rec["message"] = str(e)
        rec["carry_outs"] = counter[0]
        return rec
    finally:
        gopt.option.carry_out = orig
    rec["error"] = None
    rec["carry_outs"] = counter[0]
    rec["nodes"] = count_nodes(root)
    rec["chosen"] = rc.canon_option(chosen)
    targets = root.get_all_targets(usefulness_treshold=200)
    rec["rng_after"] = [rc.hash_obj(list(random.getstate()[1])), rc.hash_obj(np.random.get_state()[1].tolist()),
                        int(np.random.get_state()[2])]
    tl = []
    for x, opts, nv, dist in targets:
        o = opts.detach().numpy().astype(np.float32)
        tl.append({"encode": [int(v) for v in x.tolist()],
                   "opts_shape": list(o.shape), "opts_sha": hashlib.sha256(o.tobytes()).hexdigest()[:32],
                   "nv": np.asarray(nv.numpy(), np.float64).tolist(),
                   "dist": np.asarray(dist.numpy(), np.float64).tolist()})
    rec["targets"] = tl
    return rec


def main():
    """python tools/gen_golden_targets.py [ITERS N_SEEDS]: targets2000.json.gz (16
    seeds) by default; targets20000.json.gz = cfr_train(20000), 4 seeds.

    python tools/gen_golden_targets.py ITERS --seeds S1,S2,... [--out NAME]: the
    listed seeds only, one record per line to NAME.part (so seeds can run in
    separate processes), then --merge NAME joins the parts in seed order.
    targets200000.json.gz (the reference's own train_from_scratch setting,
    train_from_scratch.py:39,45,58): seeds 30000000, 30000001 (error-free),
    30000012 (ValueError after 1 carry_out) and 30000017 (ValueError deep in
    the search)."""
    os.makedirs(OUT, exist_ok=True)
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    if "--merge" in sys.argv:
        name = sys.argv[sys.argv.index("--merge") + 1]
        recs = []
        for fn in sorted(os.listdir(OUT)):
            if fn.startswith(name + ".") and fn.endswith(".part"):
                with open(os.path.join(OUT, fn)) as f:
                    recs += [json.loads(line) for line in f if line.strip()]
        recs.sort(key=lambda r: r["seed"])
        with gzip.open(os.path.join(OUT, name), "wt") as f:
            json.dump(recs, f, separators=(",", ":"))
        return
    if "--seeds" in sys.argv:
        seeds = [int(x) for x in sys.argv[sys.argv.index("--seeds") + 1].split(",")]
        name = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else "targets%d.json.gz" % iters
        for s in seeds:
            rec = case(s, iters)
            print(s, rec.get("error"), rec.get("nodes"), len(rec.get("targets", [])), flush=True)
            with open(os.path.join(OUT, "%s.%d.part" % (name, s)), "w") as f:
                f.write(json.dumps(rec, separators=(",", ":")) + "\n")
        return
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    recs = []
    for s in range(n):
        recs.append(case(s, iters))
        print(s, recs[-1].get("error"), recs[-1].get("nodes"), len(recs[-1].get("targets", [])), flush=True)
    with gzip.open(os.path.join(OUT, "targets%d.json.gz" % iters), "wt") as f:
        json.dump(recs, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
