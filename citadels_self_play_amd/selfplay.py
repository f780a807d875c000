"""Batched self-play drivers over the device engine (one process per GPU).

The reference fans games out over `multiprocessing.Pool` workers, each
running one game through the Python object API (train_from_scratch.py:39-42,
compare_to_random.py:40-42, generate_test_data.py:28-31).  Here one rank owns
a contiguous block of the global games (seeded by global index, so results
do not depend on the world size) and runs them as one batch on its GPU:

* `decide`        - configs 3/4: positions `random.randint(lo, hi)` random steps
                    into create_game(), one run_mccfr decision each (cfr_train
                    without a model, cfr_pred with the value net).
* `simulate_games`- config 5 / simulate_game (train_from_scratch.py:23-36):
                    create_a_random_game(100) -> cfr_train(M) (+ live choice) ->
                    get_all_targets.
* `setup_games`   - generate_test_data.setup_game (generate_test_data.py:9-26).
* `all_gather_targets` - the only data-path collective: pools the (encode_game,
                    node_value) pairs of all ranks (replaces Pool.starmap's
                    result pooling); two RCCL all_gathers (counts, packed rows).
* `broadcast_model`    - rank 0's value-net parameters to every rank, once.

All device work goes through libcitadels_hip.so (engine.GameBatch); nothing
here falls back to the CPU.
"""
import json
import os
import time

import numpy as np
import torch
import torch.distributed as dist

from .engine import GameBatch, pool_caps

TARGET_ROW_BYTES = 418 * 4 + 6 * 8      # encode_game f32[418] | node_value f64[6]


def init_distributed():
    """One process per GPU under torchrun (RANK / LOCAL_RANK / WORLD_SIZE); RCCL
    ("nccl") process group when WORLD_SIZE > 1.  Returns (rank, world, device).
    CIT_DIST_BACKEND=gloo (with ranks folded onto the visible GPUs) exists only
    to rehearse N ranks on a one-GPU box; the product path is RCCL."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_dev = torch.cuda.device_count()
    backend = os.environ.get("CIT_DIST_BACKEND", "nccl")
    if ws > 1 and backend == "nccl" and ws > n_dev:
        raise RuntimeError("WORLD_SIZE=%d ranks but %d visible GPUs: RCCL runs one rank per GPU "
                           "(CIT_DIST_BACKEND=gloo only rehearses folded ranks)" % (ws, n_dev))
    dev = torch.device("cuda", local % max(1, n_dev))
    torch.cuda.set_device(dev)
    if ws > 1 and not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    r, w = world()
    return r, w, dev


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard(n_total, base_seed=0, rank=None, world_size=None):
    """Global game indices [rank*n/P, (rank+1)*n/P) -> their seeds."""
    r, w = world()
    rank = r if rank is None else rank
    world_size = w if world_size is None else world_size
    lo = n_total * rank // world_size
    hi = n_total * (rank + 1) // world_size
    return np.arange(base_seed + lo, base_seed + hi, dtype=np.int64)


def broadcast_model(model, src=0):
    """dist.broadcast of every parameter / buffer of `model` (in place)."""
    if not (dist.is_available() and dist.is_initialized()):
        return model
    for t in list(model.parameters()) + list(model.buffers()):
        dist.broadcast(t.data, src)
    return model


def decide(seeds, iters, net=None, lo=0, hi=300, node_cap=None, device=None, fused="auto"):
    """Configs 3/4 (tools/gen_golden_cfr.py harness): per seed s, random.seed(s),
    np.random.seed(s), create_game(), randint(lo, hi) random steps, then
    run_mccfr(game, net, iters) (fused: GameBatch.cfr_pred's leaf-evaluation
    mode).  Returns (batch, chosen, stats[, rounds])."""
    b = GameBatch(seeds, preset=True, device=device)
    b.advance_random(lo, hi)
    b.seed_numpy()
    if net is None:
        chosen, stats = b.cfr_decide(iters, node_cap=node_cap or 1024)
        return b, chosen, stats, 0
    chosen, stats, rounds = b.cfr_pred(iters, net, max_depth=10, node_cap=node_cap or 2048, fused=fused)
    return b, chosen, stats, rounds


# Arena share of the trees' worst case (node blocks, edge blocks) for batches of
# >= ARENA_MIN_TREES trees of >= ARENA_MIN_BLOCKS node blocks each: cfr_train(200000)
# trees average ~1.35 nodes / iteration against round 4's caps of 3.5,
# and ~9 edge slots per node (children ~2, row ~7) against its 4 +
# ROW_EDGE_SLOTS: about 0.38 and 0.25 of those caps, so node and edge blocks run
# out together; pool_caps is now 1.3x those caps, the fractions 1/1.3 of round 4's.
ARENA_FRAC = (0.385, 0.254)      # round 4's (0.5, 0.33) of the 1.3x smaller caps (engine.pool_caps)
ARENA_MIN_TREES, ARENA_MIN_BLOCKS = 32, 16
# Tree-queue slots per slot that fits at ARENA_FRAC (simulate_queue's overcommit).
# With diff row slots a slot is smaller, so fewer paused trees pay: 1920 trees
# at cfr_train(200000), two A/B sessions (profiles/r03/overcommit/): 1.0 60.8,
# 1.25 61.4, 1.5 65.4 / 77.4, 2.0 61.0 (round 2's best), 2.5 63.2, 3.0 60.9
# trees/s.
QUEUE_OVERCOMMIT = float(os.environ.get("CIT_QUEUE_OVERCOMMIT", "1.5"))
# share of the device memory not held by live tensors that node pools may take by default
POOL_FRAC = float(os.environ.get("CIT_POOL_FRAC", "0.8"))
# wall-clock seconds per queue slice (cit_cfr_train_slice's budget)
QUEUE_SLICE_S = float(os.environ.get("CIT_QUEUE_SLICE_S", "0.5"))


def arena_frac_for(B, node_cap):
    from . import layout as L
    return ARENA_FRAC if B >= ARENA_MIN_TREES and L.cfr_nblocks(node_cap) >= ARENA_MIN_BLOCKS else None


def simulate_games(seeds, iters, max_move=100, node_cap=None, device=None, edge_cap=None, max_pool_bytes=None,
                   log=None, arena_frac="auto", queue=True):
    """simulate_game (train_from_scratch.py:23-36, pretrain / training=True: the
    search ignores the model) for every seed: random.seed(s), np.random.seed(s),
    create_a_random_game(max_move), run_mccfr(iters, training=True),
    get_all_targets.  Returns (batch, stats, targets dict of device tensors).

    Node pools are sized from `iters` (engine.pool_caps: a cfr_train(200000)
    tree may grow to ~1.3 GB).  Trees take node blocks from one shared arena
    as they grow, so a batch of many large trees holds `arena_frac` of their
    summed worst case (default ARENA_FRAC: ~1.3x the measured mean; a tree
    that finds the arena exhausted is searched again, bit-identically, in a
    batch of its own).  When the seeds' pools do not fit in `max_pool_bytes`
    (default: 80 % of the device memory not held by live tensors) they go
    through a tree queue over as many lanes as fit (simulate_queue; with
    queue=False: consecutive equal chunks, the returned batch then being the
    last chunk's); results are concatenated in seed order either way.
    targets["terminal"] [B] marks the positions that were already over (the
    reference's run_mccfr raises ValueError on them); targets["overflow"] [B]
    the trees that still overflowed after their retries; targets["chosen"]
    [B,16] every tree's live decision.  A tree whose search ended in an error
    (the reference's ValueError, or a surviving overflow) yields no targets."""
    from .engine import pool_bytes
    if node_cap is None:
        node_cap, ec = pool_caps(iters)
        edge_cap = edge_cap or ec
    edge_cap = edge_cap or 5 * node_cap
    dev = torch.device(device or "cuda")
    if max_pool_bytes is None:
        from .engine import device_avail_bytes   # (cached blocks of earlier pools count as free)
        max_pool_bytes = int(POOL_FRAC * device_avail_bytes(dev))
    seeds = np.asarray(seeds, np.int64)
    frac = (lambda B: arena_frac_for(B, node_cap)) if arena_frac == "auto" else (lambda B: arena_frac)
    chunk = len(seeds)
    while chunk > 1 and pool_bytes(chunk, node_cap, edge_cap, frac(chunk)) > max_pool_bytes:
        per = pool_bytes(chunk, node_cap, edge_cap, frac(chunk)) / chunk
        chunk = max(1, min(chunk - 1, int(max_pool_bytes // per)))
    if chunk < len(seeds) and queue:
        # more trees than fit at once: a tree queue over `chunk` lanes (same results)
        return simulate_queue(seeds, iters, slots=chunk, max_move=max_move, node_cap=node_cap, edge_cap=edge_cap,
                              device=dev, max_pool_bytes=max_pool_bytes, arena_frac=arena_frac, log=log)
    n_chunks = -(-len(seeds) // chunk)
    chunk = -(-len(seeds) // n_chunks)           # equal chunks: no short last launch
    parts = []
    b = None
    for i in range(0, len(seeds), chunk):
        if b is not None:
            b.pool = None                      # free the previous chunk's trees
        b = GameBatch(seeds[i:i + chunk], preset=True, device=dev)
        b.arena_frac = frac(b.B)
        b.random_position(max_move)
        b.seed_numpy()
        term = b.terminal()
        chosen, stats = b.cfr_decide(iters, node_cap=node_cap, edge_cap=edge_cap)
        t = b.cfr_targets(_roots_for_targets(stats), mode=0)
        t["terminal"] = term
        t["overflow"] = _overflowed(stats)
        t["chosen"] = chosen
        parts.append((stats, t))
        if log is not None:
            used, cap = b.arena_used()
            log("simulate_games: trees %d-%d of %d done (arena node blocks %d / %d, edge blocks %d / %d)"
                % (i, i + b.B - 1, len(seeds), used[0], cap[0], used[1], cap[1]))
    if len(parts) == 1:
        return b, parts[0][0], parts[0][1]
    return b, torch.cat([p[0] for p in parts]), concat_targets([p[1] for p in parts], [p[0].shape[0] for p in parts])


CP_DONE = 3                             # CfrState.phase of a finished tree (csrc/cit_cfr.h)


class _SlicePlanner:
    """Which trees of an overcommitted tree queue search in the next slice.

    With more slots than the arena holds at the trees' final sizes, the queue
    relies on trees being at different stages of growth (a tree holds, on
    average over its life, about half its final blocks).  Before each slice
    the planner reads every tree's held blocks (its block tables) and its
    iteration count, and lets trees run, most advanced first, while the
    arena's free blocks cover their expected growth over one slice (the
    growth each showed in its last slice, else the largest growth seen) with
    `margin`; the rest sit the slice out (paused: CfrState.phase reads
    CP_DONE for one launch, so the kernel returns at once).  Trees enter
    paused and start when the arena has room: the queue staggers itself, and
    the most advanced trees, which release the most blocks when they finish,
    always go first.  The oldest tree always runs; if the arena still runs
    out it overflows and is searched again after the queue (simulate_queue's
    retry), so pausing never changes a result, only where the search waits."""

    def __init__(self, sb, node_cap, edge_cap, margin=1.5):
        from . import layout as L
        self.nbt, self.ebt = L.cfr_nblocks(node_cap), L.cfr_eblocks(edge_cap)
        per = L.cfr_pool_bytes(node_cap, edge_cap) // 4
        self.tables = sb.pool[:sb.B * per * 4].view(torch.int32).view(sb.B, per)[:, :self.nbt + self.ebt]
        self.cap = np.array(sb.arena, np.int64)
        self.margin = margin
        self.last_held = np.zeros((sb.B, 2), np.int64)
        self.growth = np.full((sb.B, 2), -1, np.int64)      # blocks per slice (-1: not seen running)
        self.prior = np.array([max(2, self.nbt // 16), max(2, self.ebt // 16)], np.int64)
        self.paused_slices = 0

    def held(self):
        t = (self.tables >= 0)
        return torch.stack([t[:, :self.nbt].sum(1), t[:, self.nbt:].sum(1)], 1).cpu().numpy().astype(np.int64)

    def plan(self, state_np, live, ran):
        """live: slots holding an unfinished tree; ran: slots that searched in the
        last slice.  Returns the bool mask of live slots to pause."""
        held = self.held()
        grew = held - self.last_held
        seen = ran & (grew.sum(1) > 0)
        self.growth[seen] = grew[seen]
        if seen.any():
            self.prior = np.maximum(self.prior, grew[seen].max(0))
        self.last_held = held
        free = self.cap - held.sum(0)
        order = np.flatnonzero(live)
        order = order[np.argsort(-state_np[order, 5], kind="stable")]       # most iterations first
        pause = np.zeros(live.shape[0], bool)
        for k, i in enumerate(order):
            g = self.growth[i] if self.growth[i, 0] >= 0 else self.prior
            need = np.ceil(g * self.margin).astype(np.int64) + 1
            if k == 0 or (need <= free).all():
                free -= need
            else:
                pause[i] = True
        self.paused_slices += int(pause.sum())
        return pause

    def reset(self, slots):
        """`slots` (numpy indices) took new trees."""
        self.growth[slots] = -1
        self.last_held[slots] = 0


def simulate_queue(seeds, iters, slots=None, max_move=100, node_cap=None, edge_cap=None, device=None,
                   slice_seconds=None, max_pool_bytes=None, arena_frac="auto", log=None, overcommit=None,
                   max_requeue=0):
    """simulate_games through a tree queue: `slots` trees search at once (one
    per workgroup, sharing one block arena); the search runs in slices of
    ~slice_seconds (cit_cfr_train_slice), and after each slice the finished
    trees' targets are extracted, their blocks released and their lanes given
    the next positions, so a long tree no longer holds the whole batch.

    overcommit > 1 (default QUEUE_OVERCOMMIT for large trees): the arena
    takes all of max_pool_bytes and the queue runs `overcommit` times the
    slots that fit at ARENA_FRAC, relying on trees being at different stages
    of growth; _SlicePlanner pauses the least advanced trees for a slice when
    the arena's free blocks do not cover everyone's growth.

    Results (stats, targets in seed order, final games and streams) are those
    of simulate_games bit for bit; trees that overflow are searched again
    through GameBatch.cfr_decide (its retry).  Returns (batch of all seeds,
    stats, targets).  One round of a TreeQueue (which can also run rounds
    back to back, the next round's trees taking the slots the current
    round's tail leaves)."""
    q = TreeQueue(iters, len(seeds), slots=slots, max_move=max_move, node_cap=node_cap, edge_cap=edge_cap,
                  device=device, slice_seconds=slice_seconds, max_pool_bytes=max_pool_bytes, arena_frac=arena_frac,
                  log=log, overcommit=overcommit, max_requeue=max_requeue, multi_round=False)
    r = q.add(seeds)
    q.run(r)
    out = q.result(r)
    q.close()
    return out


class _Round:
    """One round of positions in a TreeQueue: its source batch (positions,
    then the finished games and streams), per-tree outputs and target parts."""

    def __init__(self, seeds, base, max_move, dev):
        self.src = GameBatch(np.asarray(seeds, np.int64), preset=True, device=dev)
        self.src.random_position(max_move)
        self.src.seed_numpy()
        self.term = self.src.terminal()
        self.Q = self.src.B
        self.base = base
        self.snap = self.src._snapshot()
        self.out_stats = torch.zeros((self.Q, 5), dtype=torch.int32, device=dev)
        self.out_chosen = torch.zeros((self.Q, 16), dtype=torch.uint8, device=dev)
        self.parts, self.early = [], []
        self.n_done = 0          # trees finished (targets walked or pending)
        self.counted = self.n_walked = self.n_targets = 0   # TreeQueue.targets_so_far's running totals
        self.t_done = None       # perf_counter when run() saw the round complete


class TreeQueue:
    """simulate_game trees (create_a_random_game(max_move) -> cfr_train(iters)
    -> get_all_targets) through one tree queue over rounds of positions
    (train_from_scratch.collect's rounds, the reference's get_mccfr_targets
    loop, train_from_scratch.py:45-64).  `add(seeds)` appends a round; its
    trees enter the queue's slots in order after the earlier rounds' trees,
    so while one round's longest trees finish, the next round's trees already
    search in the slots (and arena blocks) the finished ones freed.
    `run(r)` searches until round r is complete, `result(r)` returns it as
    simulate_queue does (bit-identical to searching the round alone: a
    tree's search depends only on its own position and streams).  A round
    that turns out not to be needed is simply never run to its end (close()).

    `per_round` (the trees in one round) sizes the slots: as simulate_queue
    sizes them for a batch of that many positions."""

    def __init__(self, iters, per_round, slots=None, max_move=100, node_cap=None, edge_cap=None, device=None,
                 slice_seconds=None, max_pool_bytes=None, arena_frac="auto", log=None, overcommit=None,
                 max_requeue=0, multi_round=True):
        from .engine import pool_bytes, side_streams, row_cap_for
        from . import layout as L
        if node_cap is None:
            node_cap, ec = pool_caps(iters)
            edge_cap = edge_cap or ec
        edge_cap = edge_cap or 5 * node_cap
        self.iters, self.node_cap, self.edge_cap, self.max_move, self.log = iters, node_cap, edge_cap, max_move, log
        self.max_requeue, self.multi_round = max_requeue, multi_round
        dev = self.dev = torch.device(device or "cuda")
        self.t_setup = time.perf_counter()
        if max_pool_bytes is None:
            from .engine import device_avail_bytes
            max_pool_bytes = int(POOL_FRAC * device_avail_bytes(dev))
        frac = (lambda B: arena_frac_for(B, node_cap)) if arena_frac == "auto" else (lambda B: arena_frac)
        Q = max(1, int(per_round))
        if slots and multi_round:
            Q = max(Q, int(slots))      # a round-to-round queue may hold more trees than one round
        S = min(Q, slots or Q)
        while S > 1 and pool_bytes(S, node_cap, edge_cap, frac(S)) > max_pool_bytes:
            S = max(1, min(S - 1, int(max_pool_bytes // (pool_bytes(S, node_cap, edge_cap, frac(S)) / S))))
        if overcommit is None:
            overcommit = QUEUE_OVERCOMMIT if (arena_frac == "auto" and frac(S) is not None) else 1.0
        arena_f = frac(S)
        if overcommit > 1 and arena_f is not None and S < Q:
            # the same bytes as S trees at ARENA_FRAC, shared by more slots
            fn, fe = arena_f if isinstance(arena_f, tuple) else (arena_f, arena_f)
            nbt, ebt = L.cfr_nblocks(node_cap), L.cfr_eblocks(edge_cap)
            nb0, eb0 = fn * S * nbt, fe * S * ebt
            S2 = min(Q, int(S * overcommit))
            scale = (max_pool_bytes - S2 * L.cfr_pool_bytes(node_cap, edge_cap)) / float(
                L.cfr_arena_bytes(int(nb0), int(eb0), row_cap_for(node_cap), False))
            S, arena_f = S2, (min(1.0, nb0 * scale / (S2 * nbt)), min(1.0, eb0 * scale / (S2 * ebt)))
        else:
            overcommit = 1.0
        self.S, self.overcommit = S, overcommit
        self.sb = None
        self.arena_f = arena_f
        self.rounds = []
        self.total = 0                        # positions added over all rounds (global queue ids)
        self.nxt = 0                          # next global id to admit
        self.state = torch.zeros((S, 16), dtype=torch.int32, device=dev)
        self.state[:, 6] = CP_DONE            # an idle slot searches nothing (a slot taking a tree is zeroed)
        self.chosen = torch.zeros((S, 16), dtype=torch.uint8, device=dev)
        self.stats = torch.zeros((S, 5), dtype=torch.int32, device=dev)
        self.running = torch.zeros(1, dtype=torch.int32, device=dev)
        self.slot_q = torch.full((S,), -1, dtype=torch.long, device=dev)    # global id per slot (-1 idle, -2 walk pending)
        self.pending = None                   # (slots, global ids) finished last slice: targets walked during this one
        self.requeue, self.retries = [], {}
        self.n_slices = self.n_requeued = 0
        self.ticks = max(1, int((QUEUE_SLICE_S if slice_seconds is None else slice_seconds) * 1e8))
        self.ran = np.zeros(S, bool)
        self.side, self.rstream = side_streams(dev, 2)
        self.planner = None
        # CIT_QUEUE_PROF=1: wall time per phase (synchronising after each; diagnosis only)
        self.qprof = {"plan": 0.0, "slice+targets": 0.0, "finish": 0.0} if os.environ.get("CIT_QUEUE_PROF") else None
        # CIT_QUEUE_TRACE=path: one JSON line per slice (time, live / paused / searching trees, trees done,
        # arena blocks held) -- where the queue's time goes (diagnosis only)
        self.qtrace = open(os.environ["CIT_QUEUE_TRACE"], "w") if os.environ.get("CIT_QUEUE_TRACE") else None
        self.t_q0 = time.perf_counter()

    # ---------------------------------------------------------------- rounds
    def add(self, seeds):
        """Append a round of positions (random.seed(s), np.random.seed(s),
        create_a_random_game(max_move) per seed); returns its index."""
        t_pos = time.perf_counter()
        r = _Round(seeds, self.total, self.max_move, self.dev)
        if self.log is not None:
            torch.cuda.synchronize()
            t_pos = time.perf_counter() - t_pos
        self.total += r.Q
        self.rounds.append(r)
        if self.sb is None:
            # the slots' batch and pool, shaped from the first round's lanes
            sb = r.src.subset(torch.arange(min(self.S, r.Q), device=self.dev))
            if sb.B < self.S:
                sb = GameBatch.from_tensors(*[t for t in _pad_lanes(sb, self.S)])
            sb.arena_frac = self.arena_f
            sb._pool(self.node_cap, self.edge_cap)
            self.sb = sb
            # the planner keeps a queue of large trees inside its arena: overcommitted slots, and the
            # trees of later rounds entering beside a round's tail
            self.planner = _SlicePlanner(sb, self.node_cap, self.edge_cap) if (
                self.overcommit > 1 or (self.arena_f is not None and self.multi_round)) else None
            if self.log is not None:
                torch.cuda.synchronize()
                self.log("simulate_queue: %d positions and a %d-slot pool set up in %.1f s (positions %.2f s)"
                         % (r.Q, self.S, time.perf_counter() - self.t_setup, t_pos))
        self._admit()
        return len(self.rounds) - 1

    def _round_of(self, g):
        for r in self.rounds:
            if r.base <= g < r.base + r.Q:
                return r
        raise KeyError(g)

    def _split(self, ids, slots=None):
        """Global ids (device long) -> [(round, local ids, matching slots)]."""
        out = []
        for r in self.rounds:
            m = (ids >= r.base) & (ids < r.base + r.Q)
            if bool(m.any()):
                out.append((r, ids[m] - r.base, None if slots is None else slots[m]))
        return out

    def _admit(self):
        """Idle slots take the next positions (after the initial fill: slots
        freed by finished trees take them in _finish)."""
        idle = (self.slot_q == -1).nonzero().flatten()
        if idle.numel():
            self._fill(idle)

    def _fill(self, fs):
        ids = self.requeue[:int(fs.numel())]
        del self.requeue[:len(ids)]
        take = min(int(fs.numel()) - len(ids), self.total - self.nxt)
        ids += list(range(self.nxt, self.nxt + take))
        self.nxt += take
        k = len(ids)
        if k:
            new_q = torch.tensor(ids, dtype=torch.long, device=self.dev)
            for r, loc, sl in self._split(new_q, fs[:k]):
                self.sb.scatter(r.src.subset(loc), sl)
            self.state[fs[:k]] = 0
            if self.planner is not None:
                self.planner.reset(fs[:k].cpu().numpy())
            self.slot_q[fs[:k]] = new_q
        self.slot_q[fs[k:]] = -1
        self.state[fs[k:], 6] = CP_DONE

    def targets_so_far(self, r):
        """(trees of round r whose targets were walked, targets they yielded):
        host counts for deciding whether another round will be needed."""
        R = self.rounds[r]
        while R.counted < len(R.parts):
            t, slots, ids = R.parts[R.counted]
            R.n_targets += int(t["counts"][slots.long(), 0].sum())
            R.n_walked += int(slots.numel())
            R.counted += 1
        return R.n_walked, R.n_targets

    def done(self, r):
        R = self.rounds[r]
        return R.n_done == R.Q and not self._pending_in(R)

    def _pending_in(self, R):
        if self.pending is None:
            return False
        q = self.pending[1]
        return bool(((q >= R.base) & (q < R.base + R.Q)).any())

    # ----------------------------------------------------------------- slices
    def _tick(self, key, t0):
        if self.qprof is None:
            return t0
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        self.qprof[key] += t1 - t0
        return t1

    def run(self, r=None, on_slice=None):
        """Slices until round r (default: every round added) is complete;
        on_slice(queue) after each slice (may add rounds)."""
        while True:
            self._stamp()
            if r is not None and self.done(r):
                break
            if not self.step(on_slice):
                break
        self._stamp()

    def idle(self):
        """True when no tree is searching, waiting for its target walk or queued."""
        return (self.pending is None and bool((self.slot_q < 0).all()) and not self.requeue
                and self.nxt >= self.total)

    def step(self, on_slice=None):
        """One slice of every searching tree (the finished trees of the last
        slice walked beside it, freed slots refilled).  Returns False once the
        queue has nothing left to search."""
        from .engine import ERR_OVERFLOW, ERR_POOL, ERR_POOL_ARENA
        sb, state, dev, S = self.sb, self.state, self.dev, self.S
        if sb is None:
            return False
        tq = time.perf_counter()
        self.running.zero_()
        paused = None
        if self.planner is not None:
            st_np = state.cpu().numpy()
            live = (self.slot_q.cpu().numpy() >= 0) & (st_np[:, 6] != CP_DONE)
            pmask = self.planner.plan(st_np, live, self.ran)
            self.ran = live & ~pmask
            if pmask.any():
                paused = torch.from_numpy(np.flatnonzero(pmask)).to(dev)
                saved = state[paused, 6].clone()
                state[paused, 6] = CP_DONE           # sits this slice out (the kernel returns at once)
        tq = self._tick("plan", tq)
        sb.train_slice(self.iters, state, self.ticks, self.chosen, self.stats, self.running)
        self.n_slices += 1
        if self.pending is not None:
            # last slice's finished trees: their targets are walked on a second stream while this
            # slice runs (their slots sit this slice out, their blocks stay held until the walk ends)
            p_slots, p_qs = self.pending
            with torch.cuda.stream(self.side):      # (everything it reads was complete at the last sync)
                roots = torch.full((S,), -1, dtype=torch.int32, device=dev)
                for R, loc, sl in self._split(p_qs, p_slots):
                    roots[sl] = _roots_for_targets(R.out_stats[loc])
                t = sb._cfr_targets(roots, 0)
                for R, loc, sl in self._split(p_qs, p_slots):
                    R.parts.append((t, sl, loc))
        # the slice and the walk -- not the device: an overflowed tree searched again on the
        # retry stream (seconds for a 200k tree) must not hold the queue's next slice
        torch.cuda.current_stream(dev).synchronize()
        self.side.synchronize()
        tq = self._tick("slice+targets", tq)
        if paused is not None:
            state[paused, 6] = saved
            self.running += int(paused.numel())       # paused trees are unfinished
        free = []
        if self.pending is not None:
            p_slots, p_qs = self.pending
            for R, loc, sl in self._split(p_qs, p_slots):
                R.src.scatter(sb.subset(sl), loc)
            sb.release(p_slots)
            free.append(p_slots)
            self.pending = None
        done = ((state[:, 6] == CP_DONE) & (self.slot_q >= 0)).nonzero().flatten()
        if done.numel():
            qs = self.slot_q[done]
            st_done = self.stats[done]
            # max_requeue > 0: a tree stopped only by the shared arena running out starts again
            # from its position later in the queue (the same search, bit for bit; at most
            # max_requeue times, then the final retry)
            redo = torch.zeros(done.numel(), dtype=torch.bool, device=dev)
            (n_used, e_used), (n_cap, e_cap) = sb.arena_used() if self.max_requeue else ((0, 0), (1, 1))
            if n_used > n_cap or e_used > e_cap:
                st_np = st_done.cpu().numpy()
                for i, (q, row) in enumerate(zip(qs.cpu().tolist(), st_np)):
                    if row[4] == ERR_OVERFLOW | ERR_POOL_ARENA and self.retries.get(q, 0) < self.max_requeue:
                        self.retries[q] = self.retries.get(q, 0) + 1
                        redo[i] = True
                        self.requeue.append(q)
                        self.n_requeued += 1
            fin = ~redo
            ov = fin & ((st_done[:, 4] & ERR_POOL) != 0)        # pool overflows: searched again
            if bool(ov.any()):
                for R, loc, sl in self._split(qs[ov]):
                    R.early.append(_early_retry(R.snap, loc, st_done[ov][(qs[ov] >= R.base) &
                                                                         (qs[ov] < R.base + R.Q)],
                                                self.iters, self.node_cap, self.edge_cap, self.rstream))
                if self.log is not None:
                    self.log("simulate_queue: tree(s) %s overflowed after slice %d (nodes, edges: %s of caps %d, "
                             "%d); searched again beside the queue"
                             % (qs[ov].tolist(), self.n_slices, st_done[ov][:, 1:3].tolist(), self.node_cap,
                                self.edge_cap))
            if bool(fin.any()):
                qf, sf = qs[fin], st_done[fin]
                cf = self.chosen[done[fin]]
                for R in self.rounds:
                    m = (qf >= R.base) & (qf < R.base + R.Q)
                    if bool(m.any()):
                        R.out_stats[qf[m] - R.base] = sf[m]
                        R.out_chosen[qf[m] - R.base] = cf[m]
                        R.n_done += int(m.sum())
                self.pending = (done[fin], qf)
                self.slot_q[done[fin]] = -2                 # held: targets pending
            if bool(redo.any()):
                sb.release(done[redo])
                free.append(done[redo])
                self.slot_q[done[redo]] = -1
            if self.log is not None:
                self.log("simulate_queue: %s trees done after %d slices"
                         % (" + ".join("%d of %d" % (R.n_done, R.Q) for R in self.rounds), self.n_slices))
        if free:
            self._fill(torch.cat(free))
        if on_slice is not None:
            on_slice(self)
        tq = self._tick("finish", tq)
        if self.qtrace is not None:
            held = self.planner.held().sum(0).tolist() if self.planner is not None else None
            self.qtrace.write(json.dumps({
                "slice": self.n_slices, "t": round(time.perf_counter() - self.t_q0, 4),
                "slots_busy": int((self.slot_q >= 0).sum()), "searching": int(self.ran.sum()),
                "paused": 0 if paused is None else int(paused.numel()),
                "done": [R.n_done for R in self.rounds], "held_blocks": held,
                "arena_blocks": None if self.planner is None else self.planner.cap.tolist()}) + "\n")
        if (int(self.running.item()) == 0 and self.pending is None and bool((self.slot_q < 0).all())
                and not self.requeue):
            return False
        return True

    def _stamp(self):
        for R in self.rounds:
            if R.t_done is None and R.n_done == R.Q and not self._pending_in(R):
                R.t_done = time.perf_counter()

    def result(self, r):
        """(batch of round r's positions, stats, targets) once run(r) returned:
        the trees that overflowed are settled first (the early retries beside
        the queue, cfr_decide's retries for any still overflowing)."""
        from .engine import ERR_POOL
        R = self.rounds[r]
        dev = self.dev
        if self.log is not None and self.planner is not None:
            self.log("simulate_queue: %d slots (overcommit %.2f), %d tree-slices paused, %d trees restarted after "
                     "the arena ran out" % (self.S, self.overcommit, self.planner.paused_slices, self.n_requeued))
        if self.log is not None and self.qprof is not None:
            self.log("simulate_queue phases (s): %s over %d slices"
                     % ({k: round(v, 2) for k, v in self.qprof.items()}, self.n_slices))
        t_retry = time.perf_counter()
        keep_from = len(R.parts)
        torch.cuda.synchronize()
        over = []
        for oq, sub, c2, st2 in R.early:
            # still overflowing (the early search had 4x caps at most): cfr_decide's retries from the snapshot
            if bool(((st2[:, 4] & ERR_POOL) != 0).any()):
                g, mt, idx, seer, npm, npi, steps = R.snap
                sub = GameBatch.from_tensors(g[oq].contiguous(), mt[:, oq].contiguous(), idx[oq].contiguous(),
                                             seer[oq].contiguous(), npm[:, oq].contiguous(), npi[oq].contiguous())
                sub.row_cap = 0
                c2, st2 = sub.cfr_decide(self.iters, self.node_cap, self.edge_cap)
            R.out_stats[oq] = st2
            R.out_chosen[oq] = c2
            R.parts.append((sub.cfr_targets(_roots_for_targets(st2), 0), torch.arange(sub.B, device=dev), oq))
            R.src.scatter(sub, oq)
            over.append(oq)
        R.early = []
        over = torch.cat(over) if over else torch.zeros(0, dtype=torch.long, device=dev)
        if self.log is not None and over.numel():
            torch.cuda.synchronize()
            self.log("simulate_queue: %d trees overflowed and were searched again beside the queue (%.1f s after it)"
                     % (int(over.numel()), time.perf_counter() - t_retry))
        t = _assemble_targets(R.parts, R.Q, exclude=over, keep_from=keep_from)
        t["terminal"] = R.term
        t["overflow"] = _overflowed(R.out_stats)
        t["chosen"] = R.out_chosen
        return R.src, R.out_stats, t

    def close(self):
        """Release the pool (the planner's view of the block tables included)
        and the rounds' target parts (their results were assembled)."""
        if self.qtrace is not None:
            self.qtrace.close()
            self.qtrace = None
        if self.sb is not None:
            torch.cuda.synchronize()
            self.sb.pool = None
            self.sb = None
        self.planner = None
        for R in self.rounds:
            R.parts, R.early, R.snap = [], [], None


def _pad_lanes(b, S):
    """The state tensors of batch b padded to S lanes (repeating lane 0): the
    slot batch of a queue whose first round has fewer trees than slots."""
    idx = torch.cat([torch.arange(b.B, device=b.device), torch.zeros(S - b.B, dtype=torch.long, device=b.device)])
    return (b.games[idx].contiguous(), b.mt[:, idx].contiguous(), b.mt_idx[idx].contiguous(),
            b.seer[idx].contiguous(), b.np_mt[:, idx].contiguous(), b.np_idx[idx].contiguous())


def _early_retry(snap, oq, st, iters, node_cap, edge_cap, stream):
    """Trees of queue ids `oq` that overflowed (stats `st`) are searched again
    at once from their pre-search snapshot, in a batch of their own on
    `stream` (beside the queue's slices): raw rows, 4x caps when one reached
    its own caps.  Returns (oq, batch, chosen, stats); results are read after
    the queue (GameBatch._retry_overflow's rule, without blocking the queue)."""
    from .engine import ERR_POOL_CAP
    from . import layout as L
    g, mt, idx, seer, npm, npi, steps = snap
    cap_hit = bool(((st[:, 4] & ERR_POOL_CAP) != 0).any())
    grow = 4 if cap_hit else 1
    nc = min(grow * node_cap, L.CFR_TBL_MAX * L.CFR_NB)
    ec = min(grow * edge_cap, L.CFR_TBL_MAX * L.CFR_EB)
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        sub = GameBatch.from_tensors(g[oq].contiguous(), mt[:, oq].contiguous(), idx[oq].contiguous(),
                                     seer[oq].contiguous(), npm[:, oq].contiguous(), npi[oq].contiguous())
        sub.row_cap = 0
        c, s = sub._cfr_decide(iters, nc, ec)
    return oq, sub, c, s


def _overflowed(stats):
    """Lanes whose search still carries CIT_ERR_OVERFLOW after its retries."""
    from .engine import ERR_OVERFLOW
    return (stats[:, 4] & ERR_OVERFLOW) != 0


ERROR_CLASSES = ("value_error", "terminal", "capacity", "pool", "unsupported")
ERR_UNSUPPORTED = 0x40       # CIT_ERR_UNSUPPORTED (csrc/cit_core.h): an engine limit, not a reference exception


def error_classes(stats, terminal):
    """Per-lane class of a tree that yields no targets (-1: none) and the count
    of each class, in ERROR_CLASSES order:
      value_error  the search raised one of the reference's own exceptions
                   (CIT_ERR_* other than the overflow and unsupported bits: a
                   ValueError from np.random.choice over an empty or NaN row,
                   ...);
      terminal     the position was already over (run_mccfr raises on it);
      capacity     an engine list limit the reference does not have
                   (CIT_ERR_OVERFLOW without a pool bit: a player holding more
                   than 88 cards, or more than 32 hand-knowledge entries);
      pool         a node pool still overflowed after its retries;
      unsupported  CIT_ERR_UNSUPPORTED: a branch the engine stops on (the
                   magician / cardinal option tables of a hand over 32 cards)
                   or an engine / configuration fault (a failed tree setup,
                   cfr_pred on a pool reset without pred, no crown holder in
                   setup_round) -- counted apart from the list limits so a
                   fault is never filed as an expected capacity stop."""
    from .engine import ERR_OVERFLOW, ERR_POOL
    err = stats[:, 4].cpu()
    term = terminal.cpu().to(torch.bool)
    over = (err & ERR_OVERFLOW) != 0
    pool = over & ((err & ERR_POOL) != 0)
    unsup = (err & ERR_UNSUPPORTED) != 0
    cls = torch.full(err.shape, -1, dtype=torch.int64)
    cls[(err != 0) & ~over & ~unsup] = 0
    cls[term] = 1
    cls[over & ~pool & ~term] = 2
    cls[pool & ~term] = 3
    cls[unsup & ~over & ~term] = 4
    return cls, {k: int((cls == i).sum()) for i, k in enumerate(ERROR_CLASSES)}


def _roots_for_targets(stats):
    """Root ids for cfr_targets with every lane whose search ended in an error
    set to -1, so it yields no targets: a reference ValueError ends
    simulate_game before get_all_targets, and a pool overflow that survived
    its retries is a truncated search (the reference's search has no pool)."""
    roots = stats[:, 0].to(torch.int32).clone()
    roots[(stats[:, 4] != 0).to(roots.device)] = -1
    return roots


def _assemble_targets(parts, n, exclude=None, keep_from=None):
    """cfr_targets dicts of trees spread over slot lanes -> one dict in output
    lane order: part (t, slots, ids) holds output lanes `ids` in its lanes
    `slots`; targets of `exclude` lanes are taken only from parts keep_from..
    (default: the last part)."""
    keep_from = len(parts) - 1 if keep_from is None else keep_from
    d = parts[0][0]["meta"].device
    metas, firsts, feats, values, dists, opts = [], [], [], [], [], []
    counts = torch.zeros((n, 2), dtype=torch.int32, device=d)
    off = 0
    for i, (t, slots, ids) in enumerate(parts):
        m = torch.full((t["counts"].shape[0],), -1, dtype=torch.long, device=d)
        m[slots] = ids.long()
        if exclude is not None and exclude.numel() and i < keep_from:
            m[slots[torch.isin(ids, exclude)]] = -1
        meta = t["meta"].clone()
        lane = m[meta[:, 0].long()]
        keep = lane >= 0
        meta[:, 0] = lane.to(meta.dtype)
        metas.append(meta[keep])
        firsts.append(t["meta"][:, 4].long()[keep] + off)
        feats.append(t["feat"][keep])
        values.append(t["value"][keep])
        dists.append(t["dist"])
        opts.append(t["opt_feat"])
        off += t["dist"].shape[0]
        ok = m[slots] >= 0
        counts[ids[ok].long()] = t["counts"][slots[ok]]
    meta = torch.cat(metas)
    order = torch.sort(meta[:, 0].long() * (1 << 32) + torch.arange(meta.shape[0], device=d), stable=True).indices
    meta = meta[order]
    first = torch.cat(firsts)[order]
    nch = meta[:, 3].long()
    new_first = torch.cumsum(nch, 0) - nch
    rows = torch.repeat_interleave(first - new_first, nch) + torch.arange(int(nch.sum()), device=d)
    meta[:, 4] = new_first.to(meta.dtype)
    return {"meta": meta, "feat": torch.cat(feats)[order], "value": torch.cat(values)[order],
            "dist": torch.cat(dists)[rows], "opt_feat": torch.cat(opts)[rows], "counts": counts}


def concat_targets(ts, sizes):
    """cfr_targets dicts of consecutive lane chunks -> one dict (lane and option
    row indices shifted)."""
    lane0, row0 = 0, 0
    metas = []
    for t, n in zip(ts, sizes):
        m = t["meta"].clone()
        m[:, 0] += lane0
        m[:, 4] += row0
        metas.append(m)
        lane0 += n
        row0 += t["dist"].shape[0]
    out = {"meta": torch.cat(metas)}
    for k in ("feat", "value", "dist", "opt_feat", "counts", "terminal", "overflow", "chosen"):
        if all(k in t for t in ts):
            out[k] = torch.cat([t[k] for t in ts])
    return out


def setup_games(seeds, iters, node_cap=None, device=None):
    """generate_test_data.setup_game for every seed: random.seed(s), np.random.seed(s),
    create_game(), create_a_close_to_finished_game, encode_game, run_mccfr(iters),
    encode_options_from_node + create_target_strategy at the root.  Lanes whose
    search raised ValueError (terminal positions) yield no tuple, as setup_game
    returns [].  Returns (batch, feat [B,418], stats, root targets)."""
    from . import _lib
    b = GameBatch(seeds, preset=True, device=device)
    b.close_position()
    feat = torch.zeros((b.B, 418), dtype=torch.float32, device=b.device)
    _lib.check(b.lib.cit_encode_games(b.games.data_ptr(), b.B, -1, feat.data_ptr(),
                                      torch.cuda.current_stream(b.device).cuda_stream), "cit_encode_games")
    b.seed_numpy()
    nc, ec = pool_caps(iters)
    chosen, stats = b.cfr_decide(iters, node_cap=node_cap or nc, edge_cap=None if node_cap else ec)
    targets = b.cfr_targets(stats[:, 0], mode=1)
    return b, feat, stats, targets


def pack_targets(feat, value):
    """[n,418] f32 + [n,6] f64 -> [n, TARGET_ROW_BYTES] uint8 rows."""
    n = feat.shape[0]
    f = feat.contiguous().view(torch.uint8).reshape(n, 418 * 4)
    v = value.contiguous().view(torch.uint8).reshape(n, 6 * 8)
    return torch.cat([f, v], dim=1)


def unpack_targets(rows):
    n = rows.shape[0]
    f = rows[:, :418 * 4].contiguous().view(torch.float32).reshape(n, 418)
    v = rows[:, 418 * 4:].contiguous().view(torch.float64).reshape(n, 6)
    return f, v


def wait_driving(work, drive=None):
    """Wait for an async collective; while it is incomplete, call drive() (e.g.
    one slice of a tree queue) instead of blocking the host, until drive()
    returns False (nothing left to run) -- then block."""
    if work is None:
        return
    while drive is not None and not work.is_completed():
        if not drive():
            break
    work.wait()


def all_gather_targets(feat, value, group=None, drive=None):
    """Pool every rank's (encode_game, node_value) target pairs on every rank,
    in rank order: all_gather of the int64 counts, then of the rows padded to
    the largest count.  Works on any backend (RCCL on device tensors, gloo on
    CPU tensors).  Both collectives are issued async: with `drive`, the host
    keeps calling drive() (train_from_scratch: the next round's queue slices)
    while a slower rank has not yet joined, instead of blocking on the counts."""
    if not (dist.is_available() and dist.is_initialized()):
        return feat, value
    ws = dist.get_world_size(group)
    dev = feat.device
    n = torch.tensor([feat.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(ws)]
    wait_driving(dist.all_gather(counts, n, group=group, async_op=True), drive)
    counts = [int(c.item()) for c in counts]
    m = max(counts)
    rows = torch.zeros((m, TARGET_ROW_BYTES), dtype=torch.uint8, device=dev)
    if feat.shape[0]:
        rows[:feat.shape[0]] = pack_targets(feat, value)
    bufs = [torch.empty_like(rows) for _ in range(ws)]
    wait_driving(dist.all_gather(bufs, rows, group=group, async_op=True), drive)
    pooled = torch.cat([b[:c] for b, c in zip(bufs, counts)], dim=0)
    return unpack_targets(pooled)


def targets_to_tuples(t, feat=None):
    """The reference's target tuples (deep_mccfr.py:321-345 / generate_test_data.py:26)
    from a cfr_targets dict: (encode_game f32[418], options f32[1,nch,131],
    node_value f64[6], regret target f64[nch]) per target, CPU tensors, in
    target order.  `feat` [B,418] overrides the per-target encode rows by lane
    (generate_test_data encodes the position before the search)."""
    h = {k: v.cpu() for k, v in t.items()}
    fx = feat.cpu() if feat is not None else None
    out = []
    for k, (lane, node, pid, nch, c0) in enumerate(h["meta"].tolist()):
        x = fx[lane].clone() if fx is not None else h["feat"][k].clone()
        out.append((x, h["opt_feat"][c0:c0 + nch].clone().unsqueeze(0), h["value"][k].clone(),
                    h["dist"][c0:c0 + nch].clone()))
    return out


def all_gather_objects(obj, group=None):
    """Pool a picklable per-rank list on every rank (rank order)."""
    if not (dist.is_available() and dist.is_initialized()):
        return list(obj)
    bufs = [None] * dist.get_world_size(group)
    dist.all_gather_object(bufs, obj, group=group)
    return [x for b in bufs for x in b]
