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


def decide(seeds, iters, net=None, lo=0, hi=300, node_cap=None, device=None):
    """Configs 3/4 (tools/gen_golden_cfr.py harness): per seed s, random.seed(s),
    np.random.seed(s), create_game(), randint(lo, hi) random steps, then
    run_mccfr(game, net, iters).  Returns (batch, chosen, stats[, rounds])."""
    b = GameBatch(seeds, preset=True, device=device)
    b.advance_random(lo, hi)
    b.seed_numpy()
    if net is None:
        chosen, stats = b.cfr_decide(iters, node_cap=node_cap or 1024)
        return b, chosen, stats, 0
    chosen, stats, rounds = b.cfr_pred(iters, net, max_depth=10, node_cap=node_cap or 2048)
    return b, chosen, stats, rounds


# Arena share of the trees' worst case (node blocks, edge blocks) for batches of
# >= ARENA_MIN_TREES trees of >= ARENA_MIN_BLOCKS node blocks each: cfr_train(200000)
# trees average ~1.35 nodes / iteration against pool_caps' 3.5,
# and ~9 edge slots per node (children ~2, row ~7) against its 4 +
# ROW_EDGE_SLOTS: about 0.38 and 0.25 of the caps, so node and edge blocks run
# out together.
ARENA_FRAC = (0.5, 0.33)
ARENA_MIN_TREES, ARENA_MIN_BLOCKS = 32, 16
# Tree-queue slots per slot that fits at ARENA_FRAC (simulate_queue's overcommit).
# With diff row slots a slot is smaller, so fewer paused trees pay: 1920 trees
# at cfr_train(200000), two A/B sessions (profiles/r03/overcommit/): 1.0 60.8,
# 1.25 61.4, 1.5 65.4 / 77.4, 2.0 61.0 (round 2's best), 2.5 63.2, 3.0 60.9
# trees/s.
QUEUE_OVERCOMMIT = float(os.environ.get("CIT_QUEUE_OVERCOMMIT", "1.5"))


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
        torch.cuda.empty_cache()                # cached blocks of earlier pools count as free
        max_pool_bytes = int(0.8 * torch.cuda.mem_get_info(dev)[0])
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
                   slice_seconds=0.5, max_pool_bytes=None, arena_frac="auto", log=None, overcommit=None,
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
    stats, targets)."""
    from .engine import ERR_OVERFLOW, ERR_POOL, ERR_POOL_ARENA, ERR_POOL_CAP, pool_bytes
    from . import layout as L
    if node_cap is None:
        node_cap, ec = pool_caps(iters)
        edge_cap = edge_cap or ec
    edge_cap = edge_cap or 5 * node_cap
    dev = torch.device(device or "cuda")
    t_setup = time.perf_counter()
    src = GameBatch(np.asarray(seeds, np.int64), preset=True, device=dev)
    src.random_position(max_move)
    src.seed_numpy()
    term = src.terminal()
    Q = src.B
    snap = src._snapshot()
    if max_pool_bytes is None:
        torch.cuda.empty_cache()
        max_pool_bytes = int(0.8 * torch.cuda.mem_get_info(dev)[0])
    frac = (lambda B: arena_frac_for(B, node_cap)) if arena_frac == "auto" else (lambda B: arena_frac)
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
        from .engine import row_cap_for
        scale = (max_pool_bytes - S2 * L.cfr_pool_bytes(node_cap, edge_cap)) / float(
            L.cfr_arena_bytes(int(nb0), int(eb0), row_cap_for(node_cap), False))
        S, arena_f = S2, (min(1.0, nb0 * scale / (S2 * nbt)), min(1.0, eb0 * scale / (S2 * ebt)))
    else:
        overcommit = 1.0
    sb = src.subset(torch.arange(S, device=dev))
    sb.arena_frac = arena_f
    sb._pool(node_cap, edge_cap)
    planner = _SlicePlanner(sb, node_cap, edge_cap) if overcommit > 1 else None
    if log is not None:
        torch.cuda.synchronize()
        log("simulate_queue: %d positions and a %d-slot pool set up in %.1f s"
            % (Q, S, time.perf_counter() - t_setup))
    state = torch.zeros((S, 16), dtype=torch.int32, device=dev)
    chosen = torch.zeros((S, 16), dtype=torch.uint8, device=dev)
    stats = torch.zeros((S, 5), dtype=torch.int32, device=dev)
    running = torch.zeros(1, dtype=torch.int32, device=dev)
    out_stats = torch.zeros((Q, 5), dtype=torch.int32, device=dev)
    out_chosen = torch.zeros((Q, 16), dtype=torch.uint8, device=dev)
    slot_q = torch.arange(S, device=dev)         # queue index held by each slot (-1: idle)
    parts, nxt, n_slices, n_done = [], S, 0, 0
    ticks = max(1, int(slice_seconds * 1e8))
    ran = np.zeros(S, bool)
    from .engine import side_streams
    main = torch.cuda.current_stream(dev)
    side, rstream = side_streams(dev, 2)
    early = []            # overflowed trees searched again at once, beside the queue: (queue ids, batch, chosen, stats)
    requeue, retries = [], {}
    pending = None        # (slots, queue ids) finished last slice: targets extracted during this slice
    n_requeued = 0
    # CIT_QUEUE_PROF=1: wall time per phase (synchronising after each; diagnosis only)
    qprof = {"plan": 0.0, "slice+targets": 0.0, "finish": 0.0} if os.environ.get("CIT_QUEUE_PROF") else None
    # CIT_QUEUE_TRACE=path: one JSON line per slice (time, live / paused / searching trees, trees done,
    # arena blocks held) -- where the queue's time goes (diagnosis only)
    qtrace = open(os.environ["CIT_QUEUE_TRACE"], "w") if os.environ.get("CIT_QUEUE_TRACE") else None
    t_q0 = time.perf_counter()

    def tick(key, t0):
        if qprof is None:
            return t0
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        qprof[key] += t1 - t0
        return t1

    def next_ids(k):
        nonlocal nxt
        ids = requeue[:k]
        del requeue[:k]
        take = min(k - len(ids), Q - nxt)
        ids += list(range(nxt, nxt + take))
        nxt += take
        return ids
    tq = time.perf_counter()
    while True:
        running.zero_()
        paused = None
        if planner is not None:
            st_np = state.cpu().numpy()
            live = (slot_q.cpu().numpy() >= 0) & (st_np[:, 6] != CP_DONE)
            pmask = planner.plan(st_np, live, ran)
            ran = live & ~pmask
            if pmask.any():
                paused = torch.from_numpy(np.flatnonzero(pmask)).to(dev)
                saved = state[paused, 6].clone()
                state[paused, 6] = CP_DONE           # sits this slice out (the kernel returns at once)
        tq = tick("plan", tq)
        sb.train_slice(iters, state, ticks, chosen, stats, running)
        n_slices += 1
        if pending is not None:
            # last slice's finished trees: their targets are walked on a second stream while this
            # slice runs (their slots sit this slice out, their blocks stay held until the walk ends)
            p_slots, p_qs = pending
            with torch.cuda.stream(side):           # (everything it reads was complete at the last sync)
                roots = torch.full((S,), -1, dtype=torch.int32, device=dev)
                roots[p_slots] = _roots_for_targets(out_stats[p_qs])
                parts.append((sb._cfr_targets(roots, 0), p_slots, p_qs))
        torch.cuda.synchronize()
        tq = tick("slice+targets", tq)
        if paused is not None:
            state[paused, 6] = saved
            running += int(paused.numel())         # paused trees are unfinished
        free = []
        if pending is not None:
            p_slots, p_qs = pending
            src.scatter(sb.subset(p_slots), p_qs)
            sb.release(p_slots)
            free.append(p_slots)
            pending = None
        done = ((state[:, 6] == CP_DONE) & (slot_q >= 0)).nonzero().flatten()
        if done.numel():
            qs = slot_q[done]
            st_done = stats[done]
            # max_requeue > 0: a tree stopped only by the shared arena running out starts again
            # from its position later in the queue (the same search, bit for bit; at most
            # max_requeue times, then the final retry)
            redo = torch.zeros(done.numel(), dtype=torch.bool, device=dev)
            (n_used, e_used), (n_cap, e_cap) = sb.arena_used() if max_requeue else ((0, 0), (1, 1))
            if n_used > n_cap or e_used > e_cap:
                st_np = st_done.cpu().numpy()
                for i, (q, row) in enumerate(zip(qs.cpu().tolist(), st_np)):
                    if row[4] == ERR_OVERFLOW | ERR_POOL_ARENA and retries.get(q, 0) < max_requeue:
                        retries[q] = retries.get(q, 0) + 1
                        redo[i] = True
                        requeue.append(q)
                        n_requeued += 1
            fin = ~redo
            ov = fin & ((st_done[:, 4] & ERR_POOL) != 0)        # pool overflows: searched again
            if bool(ov.any()):
                early.append(_early_retry(snap, qs[ov], st_done[ov], iters, node_cap, edge_cap, rstream))
                if log is not None:
                    log("simulate_queue: tree(s) %s overflowed after slice %d (nodes, edges: %s of caps %d, %d); "
                        "searched again beside the queue" % (qs[ov].tolist(), n_slices, st_done[ov][:, 1:3].tolist(),
                                                             node_cap, edge_cap))
            if bool(fin.any()):
                out_stats[qs[fin]] = st_done[fin]
                out_chosen[qs[fin]] = chosen[done[fin]]
                pending = (done[fin], qs[fin])
                slot_q[done[fin]] = -2                 # held: targets pending
                n_done += int(fin.sum())
            if bool(redo.any()):
                sb.release(done[redo])
                free.append(done[redo])
                slot_q[done[redo]] = -1
            if log is not None:
                log("simulate_queue: %d of %d trees done after %d slices" % (n_done, Q, n_slices))
        if free:
            fs = torch.cat(free)
            ids = next_ids(int(fs.numel()))
            k = len(ids)
            if k:
                new_q = torch.tensor(ids, dtype=torch.long, device=dev)
                sb.scatter(src.subset(new_q), fs[:k])
                state[fs[:k]] = 0
                if planner is not None:
                    planner.reset(fs[:k].cpu().numpy())
                slot_q[fs[:k]] = new_q
            slot_q[fs[k:]] = -1
        tq = tick("finish", tq)
        if qtrace is not None:
            held = planner.held().sum(0).tolist() if planner is not None else None
            qtrace.write(json.dumps({"slice": n_slices, "t": round(time.perf_counter() - t_q0, 4),
                                     "slots_busy": int((slot_q >= 0).sum()), "searching": int(ran.sum()),
                                     "paused": 0 if paused is None else int(paused.numel()), "done": n_done,
                                     "held_blocks": held, "arena_blocks": None if planner is None
                                     else planner.cap.tolist()}) + "\n")
        if int(running.item()) == 0 and pending is None and bool((slot_q < 0).all()) and not requeue:
            break
    if log is not None and planner is not None:
        log("simulate_queue: %d slots (overcommit %.2f), %d tree-slices paused, %d trees restarted after the "
            "arena ran out" % (S, overcommit, planner.paused_slices, n_requeued))
    if qtrace is not None:
        qtrace.close()
    if log is not None and qprof is not None:
        log("simulate_queue phases (s): %s over %d slices" % ({k: round(v, 2) for k, v in qprof.items()}, n_slices))
    sb.pool = None
    t_retry = time.perf_counter()
    keep_from = len(parts)
    torch.cuda.synchronize()
    over = []
    for oq, sub, c2, st2 in early:
        # still overflowing (the early search had 4x caps at most): cfr_decide's retries from the snapshot
        if bool(((st2[:, 4] & ERR_POOL) != 0).any()):
            g, mt, idx, seer, npm, npi, steps = snap
            sub = GameBatch.from_tensors(g[oq].contiguous(), mt[:, oq].contiguous(), idx[oq].contiguous(),
                                         seer[oq].contiguous(), npm[:, oq].contiguous(), npi[oq].contiguous())
            sub.row_cap = 0
            c2, st2 = sub.cfr_decide(iters, node_cap, edge_cap)
        out_stats[oq] = st2
        out_chosen[oq] = c2
        parts.append((sub.cfr_targets(_roots_for_targets(st2), 0), torch.arange(sub.B, device=dev), oq))
        src.scatter(sub, oq)
        over.append(oq)
    over = torch.cat(over) if over else torch.zeros(0, dtype=torch.long, device=dev)
    if log is not None and over.numel():
        torch.cuda.synchronize()
        log("simulate_queue: %d trees overflowed and were searched again beside the queue (%.1f s after it)"
            % (int(over.numel()), time.perf_counter() - t_retry))
    t = _assemble_targets(parts, Q, exclude=over, keep_from=keep_from)
    t["terminal"] = term
    t["overflow"] = _overflowed(out_stats)
    t["chosen"] = out_chosen
    return src, out_stats, t


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


ERROR_CLASSES = ("value_error", "terminal", "capacity", "pool")


def error_classes(stats, terminal):
    """Per-lane class of a tree that yields no targets (-1: none) and the count
    of each class, in ERROR_CLASSES order:
      value_error  the search raised one of the reference's own exceptions
                   (CIT_ERR_* other than the overflow bit: a ValueError from
                   np.random.choice over an empty or NaN row, ...);
      terminal     the position was already over (run_mccfr raises on it);
      capacity     an engine list overflowed (CIT_ERR_OVERFLOW without a pool
                   bit): only a player holding more than 88 cards, or more
                   than 32 hand-knowledge entries, can -- the reference has no
                   such limit;
      pool         a node pool still overflowed after its retries."""
    from .engine import ERR_OVERFLOW, ERR_POOL
    err = stats[:, 4].cpu()
    term = terminal.cpu().to(torch.bool)
    over = (err & ERR_OVERFLOW) != 0
    pool = over & ((err & ERR_POOL) != 0)
    cls = torch.full(err.shape, -1, dtype=torch.int64)
    cls[(err != 0) & ~over] = 0
    cls[term] = 1
    cls[over & ~pool & ~term] = 2
    cls[pool & ~term] = 3
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


def all_gather_targets(feat, value, group=None):
    """Pool every rank's (encode_game, node_value) target pairs on every rank,
    in rank order: all_gather of the int64 counts, then of the rows padded to
    the largest count.  Works on any backend (RCCL on device tensors, gloo on
    CPU tensors)."""
    if not (dist.is_available() and dist.is_initialized()):
        return feat, value
    ws = dist.get_world_size(group)
    dev = feat.device
    n = torch.tensor([feat.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(ws)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts)
    rows = torch.zeros((m, TARGET_ROW_BYTES), dtype=torch.uint8, device=dev)
    if feat.shape[0]:
        rows[:feat.shape[0]] = pack_targets(feat, value)
    bufs = [torch.empty_like(rows) for _ in range(ws)]
    dist.all_gather(bufs, rows, group=group)
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
