"""compare_to_random (compare_to_random.py:8-42) on the device engine, one
process per GPU:

    torchrun --nproc-per-node 8 -m citadels_self_play_amd.compare_to_random --games 800 --model best_model.pt

Every game plays the reference's loop: seat 0 decides with run_mccfr(game,
model, 200) (cfr_pred, depth 10, value-net leaves), seat 1 with
run_mccfr(game) (cfr_train 2000), both only when they have more than one
option; the other seats play random.choice.  All games of a rank advance
together: cit_advance_policy runs the random steps of every lane up to its
next searched decision; the lanes waiting on seat 0 and on seat 1 are then
searched as two sub-batches and their choices carried out.  Winner counts
are summed over ranks (RCCL all-reduce of 6 counters).
"""
import argparse

import numpy as np
import torch
import torch.distributed as dist

from . import selfplay
from .engine import GameBatch


def play_games(seeds, net, pred_iters=200, train_iters=2000, device=None, node_cap=None, log=None):
    """Returns (winners [B] int, steps [B], searched decisions [B], batch)."""
    b = GameBatch(seeds, preset=True, device=device)
    b.seed_numpy()
    decisions = torch.zeros(b.B, dtype=torch.int32, device=b.device)
    rounds = 0
    while True:
        status = b.advance_policy(0b11)
        s = status.cpu()
        if bool((s < 0).all()):
            break
        for seat in (0, 1):
            lanes = torch.nonzero(s == seat).flatten()
            if lanes.numel() == 0:
                continue
            sub = b.subset(lanes)
            if seat == 0:
                chosen, stats, _ = sub.cfr_pred(pred_iters, net, max_depth=10,
                                                node_cap=node_cap or max(2048, 8 * pred_iters))
            else:
                chosen, stats = sub.cfr_decide(train_iters, node_cap=node_cap or max(1024, 4 * train_iters))
            sub.carry_out(chosen)
            b.scatter(sub, lanes)
            decisions[lanes.to(b.device)] += 1
        rounds += 1
        if log and rounds % 10 == 0:
            log("round %d: %d games still running" % (rounds, int((s >= 0).sum())))
    winners = torch.tensor([b.row(l).winner for l in range(b.B)], dtype=torch.int32)
    return winners, b.steps.cpu(), decisions.cpu(), b


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=100, help="total over all ranks (5 x 20 in the reference)")
    ap.add_argument("--model", default=None, help="state_dict of ValueOnlyNN(418,512) (this framework's or yours)")
    ap.add_argument("--pred-iters", type=int, default=200)
    ap.add_argument("--train-iters", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args(argv)
    rank, world, dev = selfplay.init_distributed()
    from .models import ValueNet, ValueOnlyNN
    m = ValueOnlyNN(418, 512)
    if args.model:
        m.load_state_dict(torch.load(args.model, map_location="cpu", weights_only=True))
    m = selfplay.broadcast_model(m.to(dev).eval())
    net = ValueNet(m, dev)
    seeds = selfplay.shard(args.games, base_seed=args.seed)

    def log(msg):
        if rank == 0:
            print(msg, flush=True)

    winners, steps, decisions, _ = play_games(seeds, net, args.pred_iters, args.train_iters, device=dev, log=log)
    counts = torch.tensor(np.bincount(winners[winners >= 0].numpy(), minlength=6)[:6], dtype=torch.int64,
                          device=dev)
    if world > 1:
        dist.all_reduce(counts)
    log("winners per seat: %s" % counts.cpu().tolist())
    return counts.cpu().tolist()


if __name__ == "__main__":
    main()
