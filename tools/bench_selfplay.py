"""Measurement of BASELINE.json configs 3-5 (the MCCFR workloads), one process
per GPU (run under torchrun for N > 1; 1 GPU otherwise):

  --config 3  B positions per GPU, one cfr_train(200) decision each (no NN)
  --config 4  B positions per GPU, one cfr_pred(200, depth 10) decision each
              with ValueOnlyNN(418,512) (torch.manual_seed(0) weights,
              broadcast from rank 0), leaf rows batched into the MFMA kernel
  --config 5  B simulate_game trees per GPU: create_a_random_game(100) ->
              cfr_train(M) -> get_all_targets, targets pooled over ranks with
              the RCCL all-gather

Timed region: barrier + synchronize on both sides, max over ranks; inputs
(positions) are built before it except for config 5, whose position
generation is part of simulate_game.  One untimed-for-the-summary warm-up
rep, then --reps timed reps; prints one JSON line (rank 0) with the MEDIAN
rep (decisions/s or trees/s, carry_out transitions/s inside the searches)
and every rep.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from citadels_self_play_amd import selfplay  # noqa: E402
from citadels_self_play_amd.engine import GameBatch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3, choices=(3, 4, 5))
    ap.add_argument("--batch", type=int, default=None, help="per GPU")
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--node-cap", type=int, default=None)
    ap.add_argument("--edge-cap", type=int, default=None, help="default engine.pool_caps(iters)")
    ap.add_argument("--queue", type=int, default=None,
                    help="config 5: this many trees per GPU through a tree queue of --batch lanes (selfplay.simulate_queue)")
    ap.add_argument("--slice", type=float, default=0.5, help="queue slice seconds")
    ap.add_argument("--overcommit", type=float, default=None,
                    help="queue slots per slot that fits at ARENA_FRAC (default selfplay.QUEUE_OVERCOMMIT)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seed", type=int, default=30_000_000)
    a = ap.parse_args()
    rank, world, dev = selfplay.init_distributed()
    # config 5: 1024 trees per GPU at 20000 iterations (one wave per SIMD); 320 lanes
    # at the reference's 200000 (block arenas hold ~0.5 of the worst case, ~0.7 GB
    # per tree), fed 960 trees through the tree queue
    iters = a.iters or {3: 200, 4: 200, 5: 20000}[a.config]
    if a.queue is None:      # config 5 at the reference's 200k: 3 trees per lane through the tree queue
        a.queue = 960 if (a.config == 5 and iters > 20000 and not a.batch) else 0
    B = a.batch or {3: 1024, 4: 4096 // max(1, world) if world > 1 else 4096,
                    5: 1024 if iters <= 20000 else 320}[a.config]
    net = None
    if a.config == 4:
        from citadels_self_play_amd import models
        torch.manual_seed(0)
        m = selfplay.broadcast_model(models.ValueOnlyNN(418, 512).to(dev).eval())
        net = models.ValueNet(m, dev)
    out = []
    for rep in range(a.warmup + a.reps):
        n_per = a.queue if (a.config == 5 and a.queue) else B
        seeds = selfplay.shard(n_per * world, base_seed=a.seed + rep * n_per * world)
        b = None
        if a.config in (3, 4):
            b = GameBatch(seeds, preset=True, device=dev)
            b.advance_random(0, 300)
            b.seed_numpy()
            term = b.terminal()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        rounds, n_targets = 0, 0
        if a.config == 3:
            chosen, stats = b.cfr_decide(iters, node_cap=a.node_cap or 1024)
        elif a.config == 4:
            chosen, stats, rounds = b.cfr_pred(iters, net, max_depth=10, node_cap=a.node_cap or 2048)
        else:
            logf = (lambda m: print(m, file=sys.stderr, flush=True))
            if a.queue:
                b, stats, t = selfplay.simulate_queue(seeds, iters, slots=B, node_cap=a.node_cap, edge_cap=a.edge_cap,
                                                      slice_seconds=a.slice, log=logf, overcommit=a.overcommit)
            else:
                b, stats, t = selfplay.simulate_games(seeds, iters, node_cap=a.node_cap, edge_cap=a.edge_cap, log=logf)
            f, v = selfplay.all_gather_targets(t["feat"], t["value"])
            n_targets = int(f.shape[0])
            # k = 1 picks the final (terminal) game: ValueError in the reference
            term = t["terminal"]
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        eb = stats[:, 4].to(dev)[~term.to(dev)]
        err_bits = {hex(1 << k): int(((eb >> k) & 1).sum()) for k in range(12) if int(((eb >> k) & 1).sum())}
        st = stats.to(dev).to(torch.float64)
        tot = torch.tensor([el, float(st.shape[0]), float(st[:, 3].sum()), float(((st[:, 4] != 0) & ~term).sum()),
                            float(term.sum()), float(st[:, 1].sum()), float(st[:, 1].max()), float(st[:, 2].max())],
                           dtype=torch.float64,
                           device=dev)
        if world > 1:
            tmax = tot.clone()
            dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
            dist.all_reduce(tot)
            tot[0], tot[6], tot[7] = tmax[0], tmax[6], tmax[7]
        el, units, carry, errs, terms, nodes, nodes_max, edges_max = [float(x) for x in tot]
        if rank == 0:
            print("rep %d: %.2fs" % (rep, el), file=sys.stderr, flush=True)
        out.append({"config": a.config, "n_gpus": world, "per_gpu": int(units) // world, "lanes": B,
                    "overcommit": a.overcommit if a.overcommit is not None else
                    (selfplay.QUEUE_OVERCOMMIT if (a.config == 5 and a.queue) else None),
                    "queue": bool(a.config == 5 and a.queue), "iters": iters, "seconds": el,
                    "warmup": rep < a.warmup,
                    ("trees_per_s" if a.config == 5 else "decisions_per_s"): units / el,
                    "carry_out_per_s": carry / el, "nodes_mean": nodes / units, "nodes_max": int(nodes_max), "edges_max": int(edges_max), "rounds": rounds,
                    "pooled_targets": n_targets, "error_lanes_nonterminal": int(errs),
                    "terminal_positions": int(terms), "error_bits_rank0": err_bits})
    if rank == 0:
        timed = sorted([r for r in out if not r["warmup"]], key=lambda r: r["carry_out_per_s"])
        median = timed[len(timed) // 2] if timed else None
        print(json.dumps({"median": median, "reps": out}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
