"""Config 3 measurement: B preset positions (random.randint(0,300) random
steps in), one no-model MCCFR decision (cfr_train(iters) + live choice) per
position, all on one GPU.  Reports decisions/s and the carry_out transitions
made inside the search per second (BASELINE.md config 3 unit).
--pred: config 4 (cfr_pred(iters, depth 10) with a seeded ValueOnlyNN(418,512)
leaf evaluator; B default 4096 per GPU)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from citadels_self_play_amd.engine import GameBatch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--node-cap", type=int, default=1024)
    ap.add_argument("--pred", action="store_true")
    ap.add_argument("--fused", type=int, default=-1, help="config 4: 1 in-kernel leaves, 0 leaf rounds, -1 default")
    a = ap.parse_args()
    net = None
    if a.pred:
        from citadels_self_play_amd import models
        torch.manual_seed(0)
        net = models.ValueNet(models.ValueOnlyNN(418, 512), "cuda")
    for rep in range(a.reps):
        s0 = 20_000_000 + rep * a.batch
        b = GameBatch(np.arange(s0, s0 + a.batch), preset=True)
        b.advance_random(0, 300)
        b.seed_numpy()
        term0 = b.terminal().cpu().numpy()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        rounds = 0
        if net is None:
            chosen, stats = b.cfr_decide(a.iters, node_cap=a.node_cap)
        else:
            chosen, stats, rounds = b.cfr_pred(a.iters, net, max_depth=10, node_cap=a.node_cap,
                                               fused="auto" if a.fused < 0 else bool(a.fused))
        e1.record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ms = e0.elapsed_time(e1)
        st = stats.cpu().numpy()
        ok = st[:, 4] == 0
        print(json.dumps({"config": "config4" if net else "config3", "fused": a.fused, "rounds": rounds, "B": a.batch, "iters": a.iters, "kernel_ms": ms, "wall_s": wall,
                          "decisions_per_s": a.batch / (ms * 1e-3),
                          "carry_out_per_s": float(st[:, 3].sum()) / (ms * 1e-3),
                          "nodes_mean": float(st[:, 1].mean()), "nodes_max": int(st[:, 1].max()),
                          "edges_max": int(st[:, 2].max()), "terminal_positions": int(term0.sum()),
                          "errors_nonterminal": int((~ok & ~term0).sum()),
                          "err_bits": int(np.bitwise_or.reduce(st[~term0, 4])) if (~term0).any() else 0,
                          "carry_outs": int(st[:, 3].sum())}), flush=True)


if __name__ == "__main__":
    main()
