"""How many dwords of a node's game row differ from its tree's base (root)
row, on cfr_train trees of the host build (the evidence for the diff-row
slot size, engine.CFR_ROW_CAP).  python tools/row_diff_stats.py [iters] [seeds...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import hostcheck as H  # noqa: E402
from citadels_self_play_amd.engine import pool_caps  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    seeds = [int(x) for x in sys.argv[2:]] or [30000000, 30000001, 30000003, 30000005]
    allmax = 0
    for seed in seeds:
        hb = H.HostBatch([seed], True)
        H.random_position(hb, 100)
        nc, ec = pool_caps(iters)
        cf = H.HostCfr(hb, node_cap=nc, edge_cap=ec)
        chosen, stats = cf.decide(iters)
        nodes, edges, rows = cf.tree(0)
        n, root = int(stats[0][1]), int(stats[0][0])
        r = rows[:n].reshape(n, -1).view(np.uint32)
        d = (r != r[root]).sum(1)
        nz = (r != 0).sum(1)
        allmax = max(allmax, int(d.max()))
        print("seed %d cfr_train(%d): %d nodes; dwords differing from the root row: mean %.1f p99 %.0f max %d "
              "(of %d; nonzero dwords mean %.1f)" % (seed, iters, n, d.mean(), np.percentile(d, 99), d.max(),
                                                     r.shape[1], nz.mean()), flush=True)
    print("max over all nodes: %d (diff slot cap %d)" % (allmax, 128))


if __name__ == "__main__":
    main()
