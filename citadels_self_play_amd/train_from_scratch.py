"""train_from_scratch (train_from_scratch.py:23-111) on the device engine, one
process per GPU:

    torchrun --nproc-per-node 8 -m citadels_self_play_amd.train_from_scratch --iters 200000

Each data round, every rank runs `--games-per-gpu` simulate_game trees
(create_a_random_game(100) -> cfr_train(iters, training=True) ->
get_all_targets) through one selfplay.TreeQueue per phase (a tree queue over
as many slots as its block arena -- ~0.8 of HBM -- holds, the least advanced
trees paused for a slice when it runs short; when a round's finished trees
project that another round will be needed, that round's trees enter the
slots the current round's tail frees); the (encode_game,
node_value) pairs are pooled across ranks with an RCCL all-gather until
`--min-targets` are collected (get_mccfr_targets, :45-63).  Rank 0 trains the
value net (train.train_node_value_only) and the weights are broadcast.  The
full target tuples are written per rank in the reference's pickle layout
(list of (x, options, node_value, target) tensors).  The model passed to the
search in the training phases does not change the search (training=True uses
no predictions, deep_mccfr.py:119-126,279), so every phase runs the same
device search.

Error semantics (--on-error).  A reference tree whose search raises (a
ValueError from np.random.choice over an empty or NaN strategy row, or
run_mccfr on an already-terminal position) propagates out of Pool.starmap and
ends the run: get_mccfr_targets catches only RanOutOfMemory
(train_from_scratch.py:56-63).  `--on-error raise` reproduces that (a
TreeError, a ValueError, on every rank).  The default `drop` keeps going
without those trees and logs per round how many were dropped and why
(selfplay.error_classes: reference value errors, terminal positions, and
the engine-only classes -- a player past the 88-slot card area, a node pool
past its retries -- which raise EngineCapacityError under `raise`); none of
them contributes targets.
"""
import argparse
import os
import pickle
import time

import torch

from . import selfplay
from .models import ValueOnlyNN


class TreeError(ValueError):
    """--on-error raise: a simulate_game tree ended in one of the reference's
    exceptions (train_from_scratch.py:56-63 catches only RanOutOfMemory, so
    the reference's data generation stops there)."""


class EngineCapacityError(RuntimeError):
    """--on-error raise: a tree hit a limit of this engine that the reference
    does not have (selfplay.error_classes "capacity" / "pool" / "unsupported"), so its targets
    cannot be reproduced; not a reference exception."""


def lane_errors(stats, t, seeds):
    """Per-round error accounting: (counts by selfplay.ERROR_CLASSES, first
    failing seed of the reference's classes, first seed of the engine's)."""
    from .selfplay import error_classes
    cls, counts = error_classes(stats, t["terminal"])
    ref = ((cls == 0) | (cls == 1)).nonzero().flatten()
    eng = (cls >= 2).nonzero().flatten()
    first_ref = int(seeds[int(ref[0])]) if ref.numel() else None
    first_eng = int(seeds[int(eng[0])]) if eng.numel() else None
    return counts, first_ref, first_eng


def round_seeds(args, world, phase, rnd):
    """This rank's seeds of data round `rnd` of `phase` (a disjoint block per round and rank)."""
    base = args.seed + (phase * 1000 + rnd) * args.games_per_gpu * world
    return selfplay.shard(args.games_per_gpu * world, base_seed=base)


# _Lookahead estimates a round's targets from its first walked trees once this
# fraction of the round is walked (round 5 waited for half, leaving the slots of
# the earliest finished trees idle until then)
LOOKAHEAD_WALKED = float(os.environ.get("CIT_LOOKAHEAD_WALKED", str(1.0 / 8)))
# rounds the queue may hold beyond the one collect waits for: with one, a round that
# fills every slot (960 trees per GPU: 1,920 slots) leaves the slots its tail frees
# idle until collect moves on, so the rounds finished in pairs
LOOKAHEAD_DEPTH = int(os.environ.get("CIT_LOOKAHEAD_DEPTH", "2"))


class _Lookahead:
    """collect's cross-round queue (selfplay.TreeQueue): while round r's
    longest trees finish, round r + 1's trees already search in the slots the
    finished ones freed -- once the targets of round r's finished trees
    project that the pooled targets will still fall short of min_targets
    (the estimate only decides whether to start the next round early: the
    rounds actually used are decided by the pooled count, as in the
    reference, and a round started but not needed is dropped).  Each round's
    trees and targets are those of simulate_games on its seeds, bit for bit.
    `max_rounds` (the bench's fixed-round runs) never starts a round past it."""

    def __init__(self, args, world, phase, min_targets, log, max_rounds=None):
        self.args, self.world, self.phase, self.min_targets = args, world, phase, min_targets
        self.max_rounds = max_rounds
        # slots for two rounds (as many as the arena holds, TreeQueue caps them): the next round's trees
        # take the slots beside the current round's, not only those its finished trees free
        self.q = selfplay.TreeQueue(args.iters, args.games_per_gpu, slots=2 * args.games_per_gpu, max_move=100,
                                    node_cap=args.node_cap, log=log)
        self.pooled = 0
        self.speculated = 0
        self.rnd = 0
        self.rate = None          # pooled targets per tree of the rounds done (collect sets it)

    def maybe_next(self, q):
        """Add round last + 1 (last: the newest round in the queue, up to
        LOOKAHEAD_DEPTH past the one collect waits for) once 1/8 of round
        `last` is walked, if the rounds in flight project short of min_targets."""
        rnd, last = self.rnd, len(q.rounds) - 1
        if last - rnd >= LOOKAHEAD_DEPTH or (self.max_rounds is not None and last + 1 >= self.max_rounds):
            return
        walked, n = q.targets_so_far(last)
        Q = q.rounds[last].Q
        if walked < max(1, int(Q * LOOKAHEAD_WALKED)):
            if last > rnd or self.rate is None:
                return
            rate = self.rate                 # the finished rounds' yield until this round's own estimate
        elif last == rnd:
            rate = n / walked
        else:                                # the finished rounds' yield, else the current round's so far
            w0, n0 = q.targets_so_far(rnd)
            rate = self.rate if self.rate is not None else n0 / max(1, w0)
        projected = self.pooled + rate * Q * self.world * (last - rnd + 1)
        if projected < 1.25 * self.min_targets:
            q.add(round_seeds(self.args, self.world, self.phase, last + 1))
            self.speculated += 1

    def round(self, rnd):
        self.rnd = rnd
        while len(self.q.rounds) <= rnd:
            self.q.add(round_seeds(self.args, self.world, self.phase, len(self.q.rounds)))
        self.q.run(rnd, on_slice=self.maybe_next)
        return self.q.result(rnd)

    def drive(self):
        """One slice of whatever the queue holds beyond the finished round
        (collect calls it while a collective waits for slower ranks); False
        when there is nothing to search."""
        if self.q.idle():
            return False
        return self.q.step(on_slice=self.maybe_next)

    def close(self):
        self.q.close()


def collect(rank, world, args, phase, min_targets, log, max_rounds=None):
    """get_mccfr_targets (train_from_scratch.py:45-64): data rounds of
    `games_per_gpu` simulate_game trees per rank until the pooled targets
    reach min_targets (or `max_rounds` rounds).  The per-round collectives
    (the --on-error check, the target all-gathers) are async: while a slower
    rank has not finished its round, this rank's host keeps driving the next
    round's queue slices instead of blocking."""
    feats, values, tuples = [], [], []
    dropped = {k: 0 for k in selfplay.ERROR_CLASSES}
    pooled = 0
    rnd = 0
    look = _Lookahead(args, world, phase, min_targets, log, max_rounds) if getattr(args, "lookahead", True) else None
    drive = look.drive if look is not None else None
    collect.round_done = []
    collect.queue = None
    try:
        while pooled < min_targets and (max_rounds is None or rnd < max_rounds):
            seeds = round_seeds(args, world, phase, rnd)
            t0 = time.time()
            if look is None:
                b, stats, t = selfplay.simulate_games(seeds, args.iters, max_move=100, node_cap=args.node_cap,
                                                      log=log)
            else:
                look.pooled = pooled
                b, stats, t = look.round(rnd)
            counts, first_ref, first_eng = lane_errors(stats, t, seeds)
            if args.on_error == "raise":
                bad = torch.tensor([0 if first_ref is None else 1, 0 if first_eng is None else 1],
                                   device=stats.device)
                if world > 1:                                  # every rank stops together
                    selfplay.wait_driving(torch.distributed.all_reduce(bad, async_op=True), drive)
                if int(bad[0].item()):
                    raise TreeError("simulate_game raised in the search (first failing seed on this rank: %s; "
                                    "%d value errors, %d terminal positions)"
                                    % (first_ref, counts["value_error"], counts["terminal"]))
                if int(bad[1].item()):
                    raise EngineCapacityError("a tree exceeded an engine capacity the reference does not have "
                                              "(first seed on this rank: %s; %d capacity, %d pool, %d unsupported)"
                                              % (first_eng, counts["capacity"], counts["pool"],
                                                 counts["unsupported"]))
            f, v = selfplay.all_gather_targets(t["feat"], t["value"], drive=drive)
            feats.append(f.cpu())
            values.append(v.cpu())
            if args.save_tuples:
                tuples += selfplay.targets_to_tuples(t)
            pooled += f.shape[0]
            if look is not None:
                look.rate = pooled / float((rnd + 1) * len(seeds) * world)
            for k in dropped:
                dropped[k] += counts[k]
            collect.round_done.append(time.perf_counter())
            log("phase %d round %d: %d trees/rank, %d pooled targets (%d/%d), dropped trees on rank %d: %d value "
                "errors (the reference's ValueError), %d already-terminal positions, %d engine capacity, %d node "
                "pool, %d unsupported branch / engine fault, %.1fs"
                % (phase, rnd, len(seeds), f.shape[0], pooled, min_targets, rank, counts["value_error"],
                   counts["terminal"], counts["capacity"], counts["pool"], counts["unsupported"], time.time() - t0))
            rnd += 1
    finally:
        if look is not None:
            q = look.q
            collect.queue = {"slots": q.S, "overcommit": q.overcommit, "slices": q.n_slices,
                             "paused_tree_slices": 0 if q.planner is None else q.planner.paused_slices,
                             "speculated_rounds": look.speculated}
            look.close()
    collect.dropped = dropped
    collect.rounds = rnd
    return torch.cat(feats), torch.cat(values), tuples


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200000)
    # the tree queue runs as many 200k-iteration trees at once as the 288 GB HBM3E
    # holds (all 1,920 of the bench's config 5 at ~0.5 KB per node)
    # and queues the rest (selfplay.TreeQueue)
    ap.add_argument("--games-per-gpu", type=int, default=960)
    ap.add_argument("--node-cap", type=int, default=None)
    ap.add_argument("--pretrain-targets", type=int, default=20000)
    ap.add_argument("--train-targets", type=int, default=5000)
    ap.add_argument("--phases", type=int, default=5)
    ap.add_argument("--epochs", type=int, default=1000)
    ap.add_argument("--batch-size", type=int, default=2048)
    ap.add_argument("--val", default="validation_targets.pkl", help="generate_test_data output")
    ap.add_argument("--out", default=".")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--save-tuples", action="store_true")
    ap.add_argument("--no-lookahead", dest="lookahead", action="store_false",
                    help="one simulate_games call per data round instead of one tree queue across rounds (the next "
                         "round's trees taking the slots the current round's tail frees; same targets)")
    ap.add_argument("--on-error", choices=("drop", "raise"), default="drop",
                    help="a tree whose search raises one of the reference's exceptions (ValueError: an empty or NaN "
                         "choice; a terminal position): drop it and count it (default), or stop the run as the "
                         "reference does (train_from_scratch.py:56-63 catches only RanOutOfMemory)")
    args = ap.parse_args(argv)
    rank, world, dev = selfplay.init_distributed()

    def log(msg):
        if rank == 0:
            print(msg, flush=True)

    if os.path.exists(args.val):
        with open(args.val, "rb") as f:          # this framework's own generate_test_data output
            val = pickle.load(f)
    else:
        log("no %s: building a validation set with generate_test_data.setup_games" % args.val)
        seeds = selfplay.shard(max(64, args.games_per_gpu) * world, base_seed=10 ** 9 + args.seed)
        b, feat, stats, t = selfplay.setup_games(seeds, min(args.iters, 20000))
        val = selfplay.all_gather_objects(selfplay.targets_to_tuples(t, feat))
    plan = [("pretrain", args.pretrain_targets, 0.3703517140136571)] + \
        [("train%d" % u, args.train_targets, 0.02) for u in range(args.phases)]
    model = ValueOnlyNN(418, 512)
    log("error policy: --on-error %s" % args.on_error)
    for phase, (name, need, lr) in enumerate(plan):
        folder = os.path.join(args.out, name)
        feat, value, tuples = collect(rank, world, args, phase, need, log)
        if args.save_tuples:
            os.makedirs(folder, exist_ok=True)
            with open(os.path.join(folder, "targets_rank%d.pkl" % rank), "wb") as f:
                pickle.dump(tuples, f)
        if rank == 0:
            best, model, _ = selfplay_train(feat, value, val, args, lr, folder, dev)
            log("%s: %d targets, best eval loss %.5f" % (name, feat.shape[0], best))
        model = selfplay.broadcast_model(model.to(dev))
    return model


def selfplay_train(feat, value, val, args, lr, folder, dev):
    from .train import train_node_value_only
    return train_node_value_only((feat, value), val, epochs=args.epochs, lr=lr, hidden_size=512,
                                 gamma=0.8851980333411889, batch_size=args.batch_size, device=dev,
                                 parent_folder=folder)


if __name__ == "__main__":
    main()
