"""Error-bit histogram of config-5 trees (simulate_games) and config-3
decisions on the GPU; prints the seeds of lanes that end with an error so the
CPU oracle can be asked whether the reference raises on them too."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from citadels_self_play_amd import selfplay  # noqa: E402


def report(tag, seeds, b, stats):
    err_row = b.errors().cpu().numpy()
    st = stats.cpu().numpy()
    term = b.terminal().cpu().numpy()
    bad = np.nonzero((st[:, 4] != 0) & ~term)[0]
    print(json.dumps({"tag": tag, "lanes": int(len(seeds)), "err_lanes": int(len(bad)),
                      "cases": [{"seed": int(seeds[i]), "tree_err": int(st[i, 4]), "row_err": int(err_row[i]),
                                 "nodes": int(st[i, 1]), "edges": int(st[i, 2])} for i in bad[:64]]}), flush=True)


def main():
    torch.cuda.set_device(0)
    if len(sys.argv) > 2:                 # diag_cfr_errors.py ITERS TREES
        iters, n = int(sys.argv[1]), int(sys.argv[2])
        seeds = selfplay.shard(n, base_seed=30_000_000)
        b, stats, _ = selfplay.simulate_games(seeds, iters)
        torch.cuda.synchronize()
        report("config5_%d" % iters, seeds, b, stats)
        return
    seeds = selfplay.shard(1024, base_seed=30_000_000)
    b, stats, _ = selfplay.simulate_games(seeds, 2000)
    torch.cuda.synchronize()
    report("config5_2000", seeds, b, stats)
    seeds = selfplay.shard(256, base_seed=30_000_000)
    b, stats, _ = selfplay.simulate_games(seeds, 20000)
    torch.cuda.synchronize()
    report("config5_20000", seeds, b, stats)


if __name__ == "__main__":
    main()
