"""Config 5 (simulate_game trees at cfr_train(ITERS) through the tree queue)
with the queue's per-slice trace (selfplay CIT_QUEUE_TRACE): how many trees
search in each slice, how many are paused for arena room, and how the run
ends (the tail of long trees).  GPU box:

    python tools/cfg5_trace.py [TREES] [ITERS] [OUT_PREFIX]
      -> OUT_PREFIX.jsonl (one line per slice) + a summary line on stdout
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    trees = int(sys.argv[1]) if len(sys.argv) > 1 else 1920
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "gpurun_out", "cfg5_trace")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    os.environ["CIT_QUEUE_TRACE"] = out + ".jsonl"
    import numpy as np
    import torch
    from citadels_self_play_amd import selfplay
    seeds = np.arange(30_000_000, 30_000_000 + trees)
    t0 = time.perf_counter()
    b, stats, t = selfplay.simulate_games(seeds, iters, log=lambda m: print(m, file=sys.stderr, flush=True))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = stats.cpu().numpy()
    _, cls = selfplay.error_classes(stats, t["terminal"])
    rows = [json.loads(x) for x in open(out + ".jsonl")]
    busy = [r["searching"] for r in rows]
    print(json.dumps({"trees": trees, "iters": iters, "seconds": el, "trees_per_s": trees / el,
                      "carry_outs": int(st[:, 3].sum()), "carry_out_per_s": float(st[:, 3].sum()) / el,
                      "slices": len(rows), "searching_mean": float(np.mean(busy)) if busy else 0,
                      "searching_max": max(busy) if busy else 0,
                      "t_half_done": next((r["t"] for r in rows if r["done"] >= trees // 2), None),
                      "t_90_done": next((r["t"] for r in rows if r["done"] >= 0.9 * trees), None),
                      "t_last": rows[-1]["t"] if rows else None, "error_classes": cls}), flush=True)


if __name__ == "__main__":
    main()
