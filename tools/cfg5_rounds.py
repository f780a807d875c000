"""Config 5 through the cross-round tree queue (selfplay.TreeQueue), with
the wall time split into its phases: position setup (the rounds' adds and the
pool), slices, each round's completion, result() (retries + target
assembly) and the final target walk.  One JSON line; CIT_QUEUE_PROF=1 adds the
queue's own per-phase sums (synchronising after each phase).

    python tools/cfg5_rounds.py [--trees 1920] [--rounds 2] [--iters 200000]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from citadels_self_play_amd import selfplay  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trees", type=int, default=1920)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--iters", type=int, default=200000)
    ap.add_argument("--seed", type=int, default=30_000_000 + 90 * 1_000_000)
    ap.add_argument("--slots", type=int, default=0, help="queue slots (0: sized from one round)")
    ap.add_argument("--overcommit", type=float, default=0.0, help="0: selfplay.QUEUE_OVERCOMMIT")
    a = ap.parse_args()
    msgs = []
    log = (lambda m: (msgs.append((round(time.perf_counter() - t0, 3), m)), print(m, file=sys.stderr, flush=True)))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    q = selfplay.TreeQueue(a.iters, a.trees, log=log, slots=a.slots or None, overcommit=a.overcommit or None)
    t_init = time.perf_counter() - t0
    for r in range(a.rounds):
        q.add(selfplay.shard(a.trees, base_seed=a.seed + r * 1_000_000))
    torch.cuda.synchronize()
    t_add = time.perf_counter() - t0
    ph = []
    n_t = 0
    for r in range(a.rounds):
        ta = time.perf_counter()
        q.run(r)
        tb = time.perf_counter()
        _, stats, t = q.result(r)
        torch.cuda.synchronize()
        tc = time.perf_counter()
        n_t += int(t["feat"].shape[0])
        ph.append({"round": r, "run_s": tb - ta, "result_s": tc - tb, "done_at": q.rounds[r].t_done - t0,
                   "carry_outs": int(stats[:, 3].double().sum()), "errors": int((stats[:, 4] != 0).sum())})
    S, oc, slices = q.S, q.overcommit, q.n_slices
    qprof = dict(q.qprof) if q.qprof else None
    q.close()
    el = time.perf_counter() - t0
    print(json.dumps({"trees": a.trees, "rounds": a.rounds, "iters": a.iters, "seconds": el,
                      "trees_per_s": a.trees * a.rounds / el, "init_s": t_init, "setup_s": t_add, "rounds_detail": ph,
                      "slots": S, "overcommit": oc, "slices": slices, "targets": n_t, "qprof": qprof,
                      "log_tail": msgs[-6:]}), flush=True)


if __name__ == "__main__":
    main()
