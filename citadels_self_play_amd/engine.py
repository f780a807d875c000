"""Batched engine API: B independent games resident in HBM as packed rows,
driven by the HIP kernels of libcitadels_hip.so.

    b = GameBatch(seeds, preset=True)          # random.seed(s); create_game()
    opts, n = b.get_options()                  # Game.get_options_from_state()
    chosen, k = b.random_choice(opts, n)       # random.choice(options)
    winner = b.carry_out(chosen)               # option.carry_out(game)
    steps, winner = b.rollout()                # the fused step loop to terminal

PyTorch supplies device memory and the stream; the compute is the native
library.  Every call is asynchronous on torch's current stream.
"""
import math
import os
import warnings

import numpy as np
import torch

from . import _lib
from . import canon as _canon
from . import layout as L


NODE_DT = np.dtype([("parent", "<i4"), ("first_edge", "<i4"), ("n_children", "<i2"), ("edge_cap", "<i2"),
                    ("depth", "<i2"), ("player", "i1"), ("gs_state", "i1"), ("flags", "u1"), ("winner", "i1"),
                    ("sib", "<i2"), ("pad", "u1", 4), ("nv", "<f8", 6), ("wp", "<f8", 6), ("pred", "<f8", 6)])
ERR_OVERFLOW = 0x1         # CIT_ERR_OVERFLOW (csrc/cit_core.h)
# With ERR_OVERFLOW: which node-pool capacity ran out (CIT_ERR_POOL_*); only
# these are searched again (an overflow without them is an engine list
# capacity no retry fixes)
ERR_POOL_ARENA, ERR_POOL_CAP, ERR_POOL_ROW = 0x1000, 0x2000, 0x4000
ERR_POOL = ERR_POOL_ARENA | ERR_POOL_CAP | ERR_POOL_ROW
EDGE_DT = np.dtype([("opt", "u1", 16), ("child", "<i4"), ("pad", "<i4"), ("R", "<f8"), ("S", "<f8"), ("CS", "<f8")])
WIDE_DT = np.dtype([("R", "<f8", 6), ("S", "<f8", 6), ("CS", "<f8", 6)])   # role-pick columns (csrc/cit_cfr.h)
CFR_ROOT_SKIPPED = 1       # CIT_CFR_ROOT_SKIPPED (include/citadels.h)
CFR_STRATEGY_HBM = 2       # CIT_CFR_STRATEGY_HBM: update_strategy without the LDS copies (checking aid)


def node_arrays(nodes, edges, n):
    """(cumulative_regrets, strategy, cumulative_strategy) of node n in the
    reference's shapes: [nch] for a normal node, [6, 10] for a role-pick node
    (whose [6]-wide columns follow its 10 edges in the pool)."""
    N = nodes[n]
    nch, f = int(N["n_children"]), int(N["first_edge"])
    if nch == 0:
        return np.zeros(0), np.zeros(0), np.zeros(0)
    if N["flags"] & 1:
        W = edges[f + 10:f + 40].view(WIDE_DT)[:nch]
        return W["R"].T.copy(), W["S"].T.copy(), W["CS"].T.copy()
    E = edges[f:f + nch]
    return E["R"].copy(), E["S"].copy(), E["CS"].copy()


def pool_caps(iters):
    """Node / edge capacity for a cfr_train(iters) tree: measured 1.2-3.5 nodes
    per iteration (2000 iterations: up to 6,604 nodes; 200000: up to 646,897
    in 10,000 trees, and one past 700,512 in the next 3,840) and up to ~4
    edge slots per node (~2 measured since opponent nodes' runs grow as they
    fill), plus ROW_EDGE_SLOTS per node for the diff rows of large trees
    (row_cap_for: ~7 slots measured); caps are 1.3x the 3.5 nodes per
    iteration that bounded round 4's trees, because a tree that still
    outgrows its pool is searched again from the start with a 4x pool
    (GameBatch._retry_overflow) -- alone at the end of a data round that is
    ~13 s of one wavefront.  Caps bound a tree's tables (224 node / 778 edge
    blocks at 200k, under CFR_TBL_MAX); the arena holds what the trees use
    (selfplay.ARENA_FRAC is relative to these caps)."""
    node_cap = max(1024, int(4.55 * iters) + 512)
    rows = ROW_EDGE_SLOTS * node_cap if row_cap_for(node_cap) else 0
    return node_cap, 4 * node_cap + 4096 + rows


# Rows of large trees' node pools: diffs against the tree's base row, each a
# run of edge slots as long as its diff (cit_cfr.h; a cfr_train(200000) node
# differs in ~70 of 388 dwords: ~7 slots, 336 B, against round 3's fixed
# 576-B slot and a raw row's 1,552 B), with at most CFR_ROW_CAP differing
# dwords (388, the default: never past; a smaller cap is a testing aid whose
# overflowing trees are searched again with raw rows, _retry_overflow).
# Small trees (configs 3/4) keep raw rows.
CFR_ROW_CAP = int(os.environ.get("CIT_ROW_CAP", str(L.CFR_ROW_W)))      # (0: raw rows everywhere, for A/B runs)
ROW_EDGE_SLOTS = 10        # edge slots per node pool_caps reserves for its row run
# cfr_pred splits batches of at least this many trees into 2 stream groups
PRED_GROUP_MIN = int(os.environ.get("CIT_PRED_GROUP_MIN", "2048"))
PRED_GROUPS = int(os.environ.get("CIT_PRED_GROUPS", "3"))
# cfr_pred time slices (cit_cfr_pred_slice), 100 MHz GPU wall-clock ticks per
# search launch; 0 = a launch runs every tree to its next leaf (cit_cfr_pred_step)
# cfr_pred rounds enqueued per host poll: a search launch, the leaf evaluation,
# the next launch, ... without reading the waiting counters in between (each
# round counts into its own slot, read once per batch), so a group's stream
# never idles for the host's round turnaround; launches past the end find
# every tree done and return at once
PRED_AHEAD = int(os.environ.get("CIT_PRED_AHEAD", "4"))
# cfr_pred as one launch whose trees evaluate their leaves in their own kernel
# (cit_cfr_pred_fused, the single-row MLP of cit_mlp_wave.h) instead of rounds
# of search launches and batched MFMA leaf launches; the trees are bitwise
# the same either way (tests/test_gpu_mlp.py, tests/test_gpu_configs.py)
PRED_FUSED = os.environ.get("CIT_PRED_FUSED", "1") != "0"
PRED_SLICE_TICKS = int(os.environ.get("CIT_PRED_SLICE_TICKS", "0"))   # 1 / 2 / 3 / 4: 87.0k / 96.9k / 100.3k / 61.4k decisions/s (config 4, profiles/r03/pred_groups)
_side_streams = {}
# search-kernel launches made by this process, per kernel (bench.py's counter
# child attributes each leg's dispatches with them)
LAUNCHES = {}


def _launched(kernel):
    LAUNCHES[kernel] = LAUNCHES.get(kernel, 0) + 1


def side_streams(device, n):
    """The first n of one pool of HIP streams per device, shared by every
    caller (the bench's stream legs, cfr_pred's groups, the tree queue): a
    stream's first launches set up its hardware queue, and a process gets 4
    of them (GPU_MAX_HW_QUEUES on the box), so streams past that share a
    queue and serialise -- fresh streams per leg would leave later legs'
    streams on shared queues."""
    pool = _side_streams.setdefault(str(device), [])
    while len(pool) < n:
        pool.append(torch.cuda.Stream(device=device))
    return pool[:n]


ROW_CAP_MIN_BLOCKS = 16


def row_cap_for(node_cap):
    return CFR_ROW_CAP if L.cfr_nblocks(node_cap) >= ROW_CAP_MIN_BLOCKS else 0


def arena_blocks(B, node_cap, edge_cap, frac=None):
    """Arena blocks (node, edge) for B trees: `frac` (a number, or a (node, edge)
    pair) of their worst case, at least one tree's worst case (None: all of it)."""
    nbt, ebt = L.cfr_nblocks(node_cap), L.cfr_eblocks(edge_cap)
    fn, fe = (1.0, 1.0) if frac is None else (frac if isinstance(frac, tuple) else (frac, frac))
    return (min(B * nbt, max(nbt, math.ceil(fn * B * nbt))), min(B * ebt, max(ebt, math.ceil(fe * B * ebt))))


def pool_bytes(B, node_cap, edge_cap, frac=None, row_cap="auto", pred=False):
    """Device bytes of a B-tree node pool: per-tree regions + arena (cit_cfr.h;
    pred: room for pred_node_value, cfr_pred pools)."""
    nb, eb = arena_blocks(B, node_cap, edge_cap, frac)
    rc = row_cap_for(node_cap) if row_cap == "auto" else row_cap
    return B * L.cfr_pool_bytes(node_cap, edge_cap) + L.cfr_arena_bytes(nb, eb, rc, pred)


def device_avail_bytes(device):
    """Device bytes a new pool may take: free memory plus what torch's caching
    allocator holds but does not use (a released node pool stays cached, so
    the next search of the same size reuses it instead of a fresh hipMalloc of
    up to ~230 GB; torch frees cached blocks itself if a request does not fit)."""
    free = torch.cuda.mem_get_info(device)[0]
    return free + torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device)


def _ptr(t):
    return t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


class GameBatch:
    def __init__(self, seeds, preset=True, device=None, games_per_block=0, seer=None):
        if not torch.cuda.is_available():
            raise _lib.NativeError("GameBatch needs a GPU (the engine has no CPU fallback)")
        self.lib = _lib.load()
        self.device = torch.device(device or "cuda")
        seeds = torch.as_tensor(np.asarray(seeds, dtype=np.int64))
        self.B = int(seeds.numel())
        self.preset = bool(preset)
        self.games_per_block = games_per_block
        d = self.device
        self.seeds = seeds.to(d)
        self.games = torch.zeros((self.B, L.GAME_BYTES), dtype=torch.uint8, device=d)
        self.mt = torch.zeros((L.MT_N, self.B), dtype=torch.int32, device=d)
        self.mt_idx = torch.zeros(self.B, dtype=torch.int32, device=d)
        # Seer give-back scratch (only state 8 of random-role games writes it); may be shared
        # between batches that are never stepped concurrently.
        if seer is not None and tuple(seer.shape) == (self.B, L.SEER_MAX):
            self.seer = seer
        else:
            self.seer = torch.zeros((self.B, L.SEER_MAX), dtype=torch.int64, device=d)
        self.steps = torch.zeros(self.B, dtype=torch.int32, device=d)
        self.winner = torch.full((self.B,), -1, dtype=torch.int32, device=d)
        self.reset()

    @classmethod
    def from_tensors(cls, games, mt, mt_idx, seer, np_mt=None, np_idx=None):
        """A batch over existing device state (no init): games [B,1552] u8, mt [624,B],
        mt_idx [B], seer [B,SEER_MAX] and optionally numpy streams np_mt/np_idx."""
        self = cls.__new__(cls)
        self.lib = _lib.load()
        self.device = games.device
        self.B = int(games.shape[0])
        self.preset = True
        self.games_per_block = 0
        self.games, self.mt, self.mt_idx, self.seer = games, mt, mt_idx, seer
        if np_mt is not None:
            self.np_mt, self.np_idx = np_mt, np_idx
        self.steps = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        self.winner = torch.full((self.B,), -1, dtype=torch.int32, device=self.device)
        return self

    def reset(self):
        """Re-create every lane's game from its seed (cit_init)."""
        _lib.check(self.lib.cit_init(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), self.B, _ptr(self.seeds),
                                     int(self.preset), _stream()), "cit_init")
        self.steps.zero_()
        self.winner.fill_(-1)

    # --- per-step API ---------------------------------------------------------
    def get_options(self, max_opts=64):
        opts = torch.zeros((self.B, max_opts, 16), dtype=torch.uint8, device=self.device)
        n = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.cit_get_options(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), _ptr(self.seer),
                                            self.B, _ptr(opts), max_opts, _ptr(n), _stream()), "cit_get_options")
        return opts, n

    def random_choice(self, opts, n):
        max_opts = opts.shape[1]
        chosen = torch.zeros((self.B, 16), dtype=torch.uint8, device=self.device)
        k = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.cit_random_choice(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), self.B,
                                              _ptr(opts), max_opts, _ptr(n), _ptr(chosen), _ptr(k), _stream()),
                   "cit_random_choice")
        return chosen, k

    def carry_out(self, chosen):
        chosen = chosen.contiguous()
        w = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.cit_carry_out(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), self.B, _ptr(chosen),
                                          _ptr(w), _stream()), "cit_carry_out")
        return w

    # --- fused hot loop --------------------------------------------------------
    def rollout(self, max_steps=-1, games_per_block=None):
        g = self.games_per_block if games_per_block is None else games_per_block
        _lib.check(self.lib.cit_rollout_random(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), _ptr(self.seer),
                                               self.B, int(max_steps), int(g), _ptr(self.steps), _ptr(self.winner),
                                               _stream()), "cit_rollout_random")
        return self.steps, self.winner

    def rollout_queue(self, max_steps=-1, grid=None):
        """rollout() as a work queue (cit_rollout_queue): `grid` resident waves
        (default 8 per SIMD of the device) take the games one after another, so
        a long game no longer holds the launch; same results game by game."""
        if grid is None:
            grid = 8 * 4 * torch.cuda.get_device_properties(self.device).multi_processor_count
        nxt = torch.zeros(1, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.cit_rollout_queue(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), _ptr(self.seer),
                                              self.B, int(max_steps), int(grid), _ptr(self.steps), _ptr(self.winner),
                                              _ptr(nxt), _stream()), "cit_rollout_queue")
        return self.steps, self.winner

    # --- MCCFR (algorithms/deep_mccfr.py) ------------------------------------------
    def advance_random(self, lo, hi):
        """The config-3 position harness: random.randint(lo, hi) random-policy steps per lane."""
        steps = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.cit_advance_random(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), _ptr(self.seer),
                                               self.B, int(lo), int(hi), _ptr(steps), _stream()),
                   "cit_advance_random")
        return steps

    def seed_numpy(self, seeds=None):
        """np.random.seed(s) per lane (numpy's legacy global stream used by the search)."""
        d = self.device
        seeds = self.seeds if seeds is None else torch.as_tensor(np.asarray(seeds, np.int64)).to(d)
        self.np_mt = torch.zeros((L.MT_N, self.B), dtype=torch.int32, device=d)
        self.np_idx = torch.zeros(self.B, dtype=torch.int32, device=d)
        _lib.check(self.lib.cit_mt_seed(_ptr(self.np_mt), _ptr(self.np_idx), self.B, _ptr(seeds), 1, _stream()),
                   "cit_mt_seed")

    def _snapshot(self):
        return tuple(t.clone() for t in (self.games, self.mt, self.mt_idx, self.seer, self.np_mt, self.np_idx,
                                         self.steps))

    def _retry_overflow(self, snap, stats, chosen, run, max_retries, orig=None):
        """Lanes whose search overflowed its node / edge pool (stats err bit
        CIT_ERR_OVERFLOW with a CIT_ERR_POOL_* bit) are searched again from their pre-search state in a
        batch of their own, with 4x the tree capacity (the same capacity when
        it was the shared arena that ran out); results and streams are scattered back, and the
        sub-batch is kept so cfr_targets can read those lanes' trees."""
        self._retry = None
        over = ((stats[:, 4].to(self.device) & ERR_POOL) != 0).nonzero().flatten()
        if max_retries <= 0 or over.numel() == 0:
            return chosen, stats
        # 4x caps when a lane reached its own node / edge cap, else the same caps
        # (the retry batch's arena holds every sub-tree's worst case and raw
        # rows, so a lane stopped by the arena or a diff row cannot be again)
        cap_hit = bool(((stats[over.to(stats.device), 4] & ERR_POOL_CAP) != 0).any())
        grow = 4 if cap_hit else 1
        g, mt, idx, seer, npm, npi, steps = snap
        sub = GameBatch.from_tensors(g[over].contiguous(), mt[:, over].contiguous(), idx[over].contiguous(),
                                     seer[over].contiguous(), npm[:, over].contiguous(), npi[over].contiguous())
        sub.steps = steps[over].contiguous()
        sub.row_cap = 0                           # a row past the diff-slot cap overflows too: raw rows
        sub_orig = None if orig is None else \
            np.broadcast_to(np.asarray(orig, np.int32), (self.B,))[over.cpu().numpy()].copy()
        nc = min(grow * self.node_cap, L.CFR_TBL_MAX * L.CFR_NB)
        ec = min(grow * self.edge_cap, L.CFR_TBL_MAX * L.CFR_EB)
        c2, s2 = run(sub, nc, ec, max_retries - 1, sub_orig)
        self.scatter(sub, over)
        chosen = chosen.clone()
        stats = stats.clone()
        chosen[over.to(chosen.device)] = c2.to(chosen.device)
        stats[over.to(stats.device)] = s2.to(stats.device)
        self._retry = (over, sub)
        return chosen, stats

    def cfr_decide(self, iters, node_cap=1024, edge_cap=None, max_retries=3, flags=0, orig=None):
        """run_mccfr(game, max_iterations=iters) (no model) on every lane; returns
        (chosen [B,16] uint8 descriptors, stats [B,5] = root, nodes, edges, carry_outs, err).
        A tree that outgrows its pool is searched again with a 4x pool (up to
        `max_retries` times), so pool capacity never changes a result."""
        if not hasattr(self, "np_mt"):
            self.seed_numpy()
        snap = self._snapshot() if max_retries > 0 else None
        chosen, stats = self._cfr_decide(iters, node_cap, edge_cap, flags, orig)
        return self._retry_overflow(snap, stats, chosen,
                                    lambda sub, nc, ec, mr, o: sub.cfr_decide(iters, nc, ec, mr, flags, o),
                                    max_retries, orig)

    def _orig(self, orig):
        """CFRNode's original_player_id per lane as a device int32 tensor (None: the game's own)."""
        if orig is None:
            return None
        return torch.as_tensor(np.broadcast_to(np.asarray(orig, np.int32), (self.B,)).copy()).to(self.device)

    def _cfr_decide(self, iters, node_cap, edge_cap, flags=0, orig=None):
        self._pool(node_cap, edge_cap)
        self._model_tree = False
        node_cap, edge_cap = self.node_cap, self.edge_cap
        o = self._orig(orig)
        chosen = torch.zeros((self.B, 16), dtype=torch.uint8, device=self.device)
        stats = torch.zeros((self.B, 5), dtype=torch.int32, device=self.device)
        _launched("k_cfr_decide")
        _lib.check(self.lib.cit_cfr_decide(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), _ptr(self.np_mt),
                                           _ptr(self.np_idx), _ptr(self.seer), self.B, int(iters), int(flags),
                                           None if o is None else _ptr(o), _ptr(self.pool),
                                           node_cap, edge_cap, _ptr(self.optbuf), _ptr(chosen), _ptr(stats),
                                           _stream()), "cit_cfr_decide")
        return chosen, stats

    def advance_policy(self, search_mask=0b11, max_steps=-1):
        """compare_to_random's step loop up to each lane's next searched decision
        (cit_advance_policy).  Returns status [B] (seat to decide, -1 over, -2 error)."""
        status = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.cit_advance_policy(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), _ptr(self.seer),
                                               self.B, int(search_mask), int(max_steps), _ptr(status),
                                               _ptr(self.steps), _stream()), "cit_advance_policy")
        return status

    def subset(self, lanes):
        """A new batch holding copies of `lanes` (rows, both streams, seer scratch)."""
        lanes = torch.as_tensor(lanes, dtype=torch.long, device=self.device)
        sub = GameBatch.from_tensors(self.games[lanes].contiguous(), self.mt[:, lanes].contiguous(),
                                     self.mt_idx[lanes].contiguous(), self.seer[lanes].contiguous(),
                                     self.np_mt[:, lanes].contiguous() if hasattr(self, "np_mt") else None,
                                     self.np_idx[lanes].contiguous() if hasattr(self, "np_idx") else None)
        sub.steps = self.steps[lanes].contiguous()
        return sub

    def scatter(self, sub, lanes):
        """Write a subset batch back into `lanes`."""
        lanes = torch.as_tensor(lanes, dtype=torch.long, device=self.device)
        self.games[lanes] = sub.games
        self.mt[:, lanes] = sub.mt
        self.mt_idx[lanes] = sub.mt_idx
        self.seer[lanes] = sub.seer
        self.steps[lanes] = sub.steps
        if hasattr(sub, "np_mt"):
            self.np_mt[:, lanes] = sub.np_mt
            self.np_idx[lanes] = sub.np_idx

    def random_position(self, max_move=100, seeds=None):
        """random.seed(seed); create_a_random_game(max_move) (run_utils.py:55-73) on every
        lane.  Returns steps into the game of each position (-1 on a lane error)."""
        d = self.device
        seeds = self.seeds if seeds is None else torch.as_tensor(np.asarray(seeds, np.int64)).to(d)
        _lib.check(self.lib.cit_mt_seed(_ptr(self.mt), _ptr(self.mt_idx), self.B, _ptr(seeds), 0, _stream()),
                   "cit_mt_seed")
        ring = torch.empty(self.B * max_move * L.GAME_BYTES, dtype=torch.uint8, device=d)
        steps = torch.zeros(self.B, dtype=torch.int32, device=d)
        _lib.check(self.lib.cit_random_position(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), _ptr(self.seer),
                                                self.B, int(max_move), _ptr(ring), _ptr(steps), _stream()),
                   "cit_random_position")
        del ring
        return steps

    def close_position(self):
        """create_a_close_to_finished_game (run_utils.py:29-53) on every lane's created
        game.  Returns the snapshot index of each position (-1 on a lane error)."""
        d = self.device
        store = torch.empty(self.B * self.lib.cit_close_rows() * L.GAME_BYTES, dtype=torch.uint8, device=d)
        index = torch.zeros(self.B, dtype=torch.int32, device=d)
        _lib.check(self.lib.cit_close_position(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), _ptr(self.seer),
                                               self.B, _ptr(store), _ptr(index), _stream()), "cit_close_position")
        del store
        return index

    def cfr_targets(self, roots, mode=0):
        """get_all_targets over the trees of the last cfr_decide (roots = stats[:, 0]).
        Returns a dict: meta [n,5] (lane, node, player override, n_children, first
        option row), feat [n,418] f32, value [n,6] f64, dist [m] f64, opt_feat [m,131]
        f32, counts [B,2]."""
        d = self.device
        roots = roots.to(device=d, dtype=torch.int32).contiguous()
        groups = getattr(self, "_groups", None)
        if groups is not None:                 # a cfr_pred split into stream groups: each sub-batch holds its trees
            parts, subs = groups
            outs = []
            for lanes, sub in zip(parts, subs):
                outs.append(sub.cfr_targets(roots[lanes].clone(), mode))
                self.mt[:, lanes] = sub.mt
                self.mt_idx[lanes] = sub.mt_idx
            return _merge_parts(outs, parts, self.B)
        retry = getattr(self, "_retry", None)
        if retry is not None:
            over, sub = retry
            roots = roots.clone()
            sub_roots = roots[over].clone()
            roots[over] = -1
            main = self._cfr_targets(roots, mode)
            extra = sub.cfr_targets(sub_roots, mode)
            self.mt[:, over] = sub.mt
            self.mt_idx[over] = sub.mt_idx
            return _merge_targets(main, extra, over)
        return self._cfr_targets(roots, mode)

    def _cfr_targets(self, roots, mode):
        d = self.device
        if getattr(self, "_groups", None) is not None:
            raise RuntimeError("the last search ran in stream groups: its trees are in the sub-batches")
        if mode == 0 and getattr(self, "_model_tree", True) is False:
            mode = 2                                  # CFR_TGT_PRUNE: searched without a model

        counts = torch.zeros((self.B, 2), dtype=torch.int32, device=d)
        _lib.check(self.lib.cit_cfr_target_count(_ptr(self.pool), self.B, self.node_cap, self.edge_cap, _ptr(roots),
                                                 int(mode), _ptr(counts), _stream()), "cit_cfr_target_count")
        offs = torch.zeros_like(counts)
        offs[1:] = torch.cumsum(counts, dim=0)[:-1]
        tot = counts.sum(dim=0).cpu()
        nt, nc = int(tot[0]), int(tot[1])
        out = {"meta": torch.zeros((nt, 5), dtype=torch.int32, device=d),
               "feat": torch.zeros((nt, 418), dtype=torch.float32, device=d),
               "value": torch.zeros((nt, 6), dtype=torch.float64, device=d),
               "dist": torch.zeros(nc, dtype=torch.float64, device=d),
               "opt_feat": torch.zeros((nc, 131), dtype=torch.float32, device=d), "counts": counts}
        _lib.check(self.lib.cit_cfr_targets(_ptr(self.pool), self.B, self.node_cap, self.edge_cap, _ptr(roots),
                                            int(mode), _ptr(self.mt), _ptr(self.mt_idx), _ptr(offs), _ptr(out["meta"]),
                                            _ptr(out["feat"]), _ptr(out["value"]), _ptr(out["dist"]),
                                            _ptr(out["opt_feat"]), _stream()), "cit_cfr_targets")
        return out

    arena_frac = None       # arena blocks as a fraction of the trees' worst case (arena_blocks)
    row_cap = "auto"        # row slot format: 0 raw rows, K diff rows (row_cap_for by node_cap)

    def _pool(self, node_cap, edge_cap, pred=False):
        """Node pool for B trees of (node_cap, edge_cap): block tables + an arena
        of arena_blocks(..., self.arena_frac) blocks, reset (empty) for a new
        search.  An arena that would not fit in device memory is cut to what
        does; a tree that finds it exhausted overflows and is searched again
        (_retry_overflow)."""
        edge_cap = edge_cap or 5 * node_cap
        self._groups = None                     # a new search: trees live in this batch's pool
        per = self.lib.cit_cfr_pool_bytes(node_cap, edge_cap)
        if per <= 0 or node_cap >= 2 ** 31 or edge_cap >= 2 ** 31:
            raise ValueError("bad node pool capacity (%d nodes, %d edges)" % (node_cap, edge_cap))
        nb, eb = arena_blocks(self.B, node_cap, edge_cap, self.arena_frac)
        rc = row_cap_for(node_cap) if self.row_cap == "auto" else int(self.row_cap)
        need = per * self.B + self.lib.cit_cfr_arena_bytes_fmt(nb, eb, rc, int(pred))
        have = self.pool.numel() if getattr(self, "pool", None) is not None else 0
        if need > have and self.device.type == "cuda":
            avail = int(0.9 * (device_avail_bytes(self.device) + have))
            if need > avail:
                nbt, ebt = L.cfr_nblocks(node_cap), L.cfr_eblocks(edge_cap)
                scale = max(0.0, (avail - per * self.B) / float(need - per * self.B))
                nb0, eb0 = nb, eb
                nb, eb = max(nbt, int(nb * scale)), max(ebt, int(eb * scale))
                need = per * self.B + self.lib.cit_cfr_arena_bytes_fmt(nb, eb, rc, int(pred))
                warnings.warn("node arena cut to %.0f%% of the requested %d node / %d edge blocks (%d trees): "
                              "device memory is short, trees that find it exhausted are searched again "
                              "(slower, same results); use fewer trees per batch to avoid this"
                              % (100.0 * nb / max(1, nb0), nb0, eb0, self.B), RuntimeWarning, stacklevel=3)
        if have and have < need:
            self.pool = None                        # free the old pool before allocating the new one
            torch.cuda.empty_cache()
        if getattr(self, "pool", None) is None:
            self.pool = torch.empty(need, dtype=torch.uint8, device=self.device)
        if getattr(self, "optbuf", None) is None or self.optbuf.shape[0] != self.B:
            self.optbuf = torch.empty((self.B, self.lib.cit_cfr_opt_cap(), 16), dtype=torch.uint8, device=self.device)
        self.node_cap, self.edge_cap, self.arena, self.pool_row_cap = node_cap, edge_cap, (nb, eb), rc
        _lib.check(self.lib.cit_cfr_arena_reset_fmt(_ptr(self.pool), self.B, node_cap, edge_cap, nb, eb, rc,
                                                    int(pred), _stream()), "cit_cfr_arena_reset_fmt")

    def train_slice(self, iters, state, ticks, chosen, stats, running, flags=0):
        """One cit_cfr_train_slice launch over the pool bound by _pool (state [B,16]
        int32 CfrState, zero rows start a tree); `running` [1] int32 receives the
        count of trees left unfinished."""
        self._model_tree = False
        _launched("k_cfr_train_slice")
        _lib.check(self.lib.cit_cfr_train_slice(
            _ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), _ptr(self.np_mt), _ptr(self.np_idx), _ptr(self.seer),
            self.B, int(iters), int(flags), None, _ptr(self.pool), self.node_cap, self.edge_cap, _ptr(self.optbuf),
            _ptr(state), int(ticks), _ptr(chosen), _ptr(stats), _ptr(running), _stream()), "cit_cfr_train_slice")

    def release(self, lanes):
        """Trees of `lanes` (device int32) give their arena blocks back (cit_cfr_arena_release)."""
        lanes = lanes.to(device=self.device, dtype=torch.int32).contiguous()
        _lib.check(self.lib.cit_cfr_arena_release(_ptr(self.pool), self.B, self.node_cap, self.edge_cap, _ptr(lanes),
                                                  int(lanes.numel()), _stream()), "cit_cfr_arena_release")

    def arena_used(self):
        """(node blocks, edge blocks) handed out by the last search's arena and its
        capacity (node, edge); a count above capacity means it ran out."""
        if getattr(self, "_groups", None) is not None:
            raise RuntimeError("the last search ran in stream groups: see the sub-batches' arena_used()")
        off = self.B * self.lib.cit_cfr_pool_bytes(self.node_cap, self.edge_cap)
        h = self.pool[off:off + 16].cpu().numpy().view("<u4")
        return (int(h[0]), int(h[2])), (int(h[1]), int(h[3]))

    def cfr_pred(self, iters, net, max_depth=10, node_cap=1024, edge_cap=None, max_rounds=100000, max_retries=3,
                 flags=0, orig=None, groups="auto", slice_ticks="auto", fused="auto"):
        """run_mccfr(game, model, max_iterations=iters) with a model and training=False
        (cfr_pred(iters, max_depth) + live action choice) on every lane.  `net` is a
        models.ValueNet.  fused (auto: PRED_FUSED): one launch, each tree
        evaluating its leaves in its own kernel (rounds = 0); otherwise leaf rows
        of all suspended trees are evaluated in one MFMA launch per round.
        Both search bitwise the same trees.  Trees that outgrow their pool are
        searched again with a 4x pool (as cfr_decide).  Returns (chosen, stats
        [B,5], rounds).

        groups > 1 (auto: PRED_GROUPS = 3 from 2,048 trees): the trees are split into that many
        sub-batches whose rounds run on their own HIP streams, interleaved, so
        one group's search kernel fills the SIMDs while another waits for its
        leaf evaluation and the host's round turnaround (a round lasts as long
        as its slowest tree); every tree is searched exactly as in one batch.
        slice_ticks > 0 (auto: PRED_SLICE_TICKS): each search launch also
        stops a tree at an iteration boundary after that much GPU wall clock,
        so a round ends with the slice rather than its slowest tree; results
        are the same."""
        self._slice_ticks = PRED_SLICE_TICKS if slice_ticks == "auto" else int(slice_ticks)
        if not hasattr(self, "np_mt"):
            self.seed_numpy()
        snap = self._snapshot() if max_retries > 0 else None
        F = PRED_FUSED if fused == "auto" else bool(fused)
        G = (PRED_GROUPS if self.B >= PRED_GROUP_MIN else 1) if groups == "auto" else max(1, min(int(groups), self.B))
        if F:
            self._groups = None
            chosen, stats, rounds = self._cfr_pred_fused(iters, net, max_depth, node_cap, edge_cap, flags, orig)
        elif G > 1:
            chosen, stats, rounds = self._cfr_pred_groups(G, iters, net, max_depth, node_cap, edge_cap, max_rounds,
                                                          flags, orig)
        else:
            self._groups = None
            chosen, stats, rounds = self._cfr_pred(iters, net, max_depth, node_cap, edge_cap, max_rounds, flags, orig)
        box = [rounds]

        def run(sub, nc, ec, mr, o):
            c, st, r = sub.cfr_pred(iters, net, max_depth, nc, ec, max_rounds, mr, flags, o,
                                    slice_ticks=self._slice_ticks, fused=F)
            box[0] += r
            return c, st
        chosen, stats = self._retry_overflow(snap, stats, chosen, run, max_retries, orig)
        return chosen, stats, box[0]

    def _pred_begin(self, node_cap, edge_cap, orig):
        """Pool and per-tree buffers of a cfr_pred run (state, feat, probs, chosen, waiting)."""
        self._pool(node_cap, edge_cap, pred=True)
        self._model_tree = True
        d = self.device
        self._pred = {"o": self._orig(orig),
                      "state": torch.zeros((self.B, self.lib.cit_cfr_state_bytes() // 4), dtype=torch.int32, device=d),
                      "feat": torch.zeros((self.B, 418), dtype=torch.float32, device=d),
                      "probs": torch.zeros((self.B, 6), dtype=torch.float32, device=d),
                      "chosen": torch.zeros((self.B, 16), dtype=torch.uint8, device=d),
                      "waiting": torch.zeros((max(1, PRED_AHEAD), 2), dtype=torch.int32, device=d),
                      "ticks": getattr(self, "_slice_ticks", 0)}       # (waiting, running) per round of a batch

    def _cfr_pred_fused(self, iters, net, max_depth, node_cap, edge_cap, flags=0, orig=None):
        """cit_cfr_pred_fused: every tree to its decision in one launch."""
        self._pred_begin(node_cap, edge_cap, orig)
        P = self._pred
        o = P["o"]
        stats = torch.empty((self.B, 5), dtype=torch.int32, device=self.device)
        _launched("k_cfr_pred_fused")
        _lib.check(self.lib.cit_cfr_pred_fused(
            _ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), _ptr(self.np_mt), _ptr(self.np_idx),
            _ptr(self.seer), self.B, int(iters), int(flags), None if o is None else _ptr(o), int(max_depth),
            _ptr(self.pool), self.node_cap, self.edge_cap, _ptr(self.optbuf), net.wave.data_ptr(), _ptr(P["state"]),
            _ptr(P["chosen"]), _ptr(stats), _stream()), "cit_cfr_pred_fused")
        return P["chosen"], stats.cpu(), 0

    def _pred_step(self, iters, max_depth, flags, slot=0):
        """One cit_cfr_pred_step launch (every tree runs to its next leaf evaluation
        or its end); its waiting / running counts go to round slot `slot` (zeroed
        by the caller)."""
        P = self._pred
        o = P["o"]
        w = _ptr(P["waiting"]) + 8 * slot
        _launched("k_cfr_pred_step")
        _lib.check(self.lib.cit_cfr_pred_slice(
            _ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), _ptr(self.np_mt), _ptr(self.np_idx),
            _ptr(self.seer), self.B, int(iters), int(flags), None if o is None else _ptr(o), int(max_depth),
            _ptr(self.pool), self.node_cap, self.edge_cap, _ptr(self.optbuf), _ptr(P["state"]), _ptr(P["probs"]),
            _ptr(P["feat"]), _ptr(P["chosen"]), int(P["ticks"]), w, w + 4, _stream()), "cit_cfr_pred_slice")

    def _pred_leaves(self, net):
        P = self._pred
        if P.get("work") is None:
            P["work"] = net.workspace(self.B)
        _lib.check(self.lib.cit_mlp_forward_packed(_ptr(P["feat"]), self.B, net.packed.data_ptr(), _ptr(P["probs"]),
                                                   None, _ptr(P["work"]), P["work"].numel(), _stream()),
                   "cit_mlp_forward_packed")

    def _pred_end(self):
        P = self._pred
        st = P["state"].cpu()
        stats = torch.stack([st[:, 8], st[:, 0], st[:, 1], st[:, 3], st[:, 2]], dim=1)
        return P["chosen"], stats

    def _pred_batch(self, net, iters, max_depth, flags, lead, n):
        """Enqueue n rounds (PRED_AHEAD): search launch j counts into slot j, and
        a leaf evaluation runs between launches (and first when `lead`: the
        previous batch's last launch left trees waiting).  A leaf evaluation
        with no tree waiting rewrites the same probabilities, and a launch
        after every tree is done returns at once, so the trees are searched
        exactly as with a host check after every launch."""
        self._pred["waiting"].zero_()
        for j in range(n):
            if j or lead:
                self._pred_leaves(net)
            self._pred_step(iters, max_depth, flags, j)

    def _pred_poll(self, n):
        """(done, leaf rounds, lead) from the slots of the last batch of n rounds:
        the rounds whose launch left trees waiting, up to the first launch
        after which no tree waits or runs."""
        rounds = 0
        cnt = self._pred["waiting"][:n].tolist()
        for waiting, running in cnt:
            if waiting == 0 and running == 0:
                return True, rounds, False
            rounds += waiting > 0
        return False, rounds, cnt[-1][0] > 0

    def _cfr_pred(self, iters, net, max_depth, node_cap, edge_cap, max_rounds, flags=0, orig=None):
        self._pred_begin(node_cap, edge_cap, orig)
        A = self._pred["waiting"].shape[0]
        rounds, lead = 0, False
        while rounds < max_rounds:
            n = max(1, min(A, max_rounds - rounds))
            self._pred_batch(net, iters, max_depth, flags, lead, n)
            done, r, lead = self._pred_poll(n)
            rounds += r
            if done:
                break
        chosen, stats = self._pred_end()
        return chosen, stats, rounds

    def _cfr_pred_groups(self, G, iters, net, max_depth, node_cap, edge_cap, max_rounds, flags, orig):
        """cfr_pred over G sub-batches on G streams, rounds interleaved (see cfr_pred)."""
        cur = torch.cuda.current_stream(self.device)
        parts = [torch.arange(self.B, device=self.device)[g::G] for g in range(G)]
        o = None if orig is None else np.broadcast_to(np.asarray(orig, np.int32), (self.B,))
        subs, streams = [], []
        for g, lanes in enumerate(parts):
            sub = self.subset(lanes)
            sub._slice_ticks = getattr(self, "_slice_ticks", 0)
            st = side_streams(self.device, G)[g]
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                sub._pred_begin(node_cap, edge_cap, None if o is None else o[lanes.cpu().numpy()])
                n0 = max(1, min(sub._pred["waiting"].shape[0], max_rounds))
                sub._pred_batch(net, iters, max_depth, flags, False, n0)
            subs.append(sub)
            streams.append(st)
        rounds = [0] * G
        last = [n0] * G
        active = list(range(G))
        while active:
            for g in list(active):
                sub = subs[g]
                with torch.cuda.stream(streams[g]):
                    done, r, lead = sub._pred_poll(last[g])
                    rounds[g] += r
                    if done or rounds[g] >= max_rounds:
                        active.remove(g)
                        continue
                    last[g] = max(1, min(sub._pred["waiting"].shape[0], max_rounds - rounds[g]))
                    sub._pred_batch(net, iters, max_depth, flags, lead, last[g])
        chosen = torch.zeros((self.B, 16), dtype=torch.uint8, device=self.device)
        stats = torch.zeros((self.B, 5), dtype=torch.int32)
        for g, (sub, lanes) in enumerate(zip(subs, parts)):
            with torch.cuda.stream(streams[g]):
                c, s = sub._pred_end()
            cur.wait_stream(streams[g])
            chosen[lanes] = c
            stats[lanes.cpu()] = s
            self.scatter(sub, lanes)
        self._groups = (parts, subs)
        self._model_tree = True
        return chosen, stats, max(rounds)

    def lane_batch(self, lane):
        """(batch, lane in it) holding `lane`'s last search tree: the retry
        sub-batch (recursively) when the lane was searched again after an
        overflow, else this batch."""
        retry = getattr(self, "_retry", None)
        if retry is not None:
            over = retry[0].cpu().tolist()
            if lane in over:
                return retry[1].lane_batch(over.index(lane))
        groups = getattr(self, "_groups", None)
        if groups is not None:                 # a cfr_pred run split into stream groups
            parts, subs = groups
            for lanes, sub in zip(parts, subs):
                ll = lanes.cpu().tolist()
                if lane in ll:
                    return sub.lane_batch(ll.index(lane))
        return self, lane

    def tree(self, lane):
        """(nodes, edges, rows) numpy views of one lane's search tree (host copy);
        a lane searched again after a pool overflow is read from its retry batch."""
        b, lane = self.lane_batch(lane)
        nodes, edges, rows = L.cfr_tree_bytes(lambda o, n: b.pool[o:o + n].cpu().numpy(), b.B, lane,
                                              b.node_cap, b.edge_cap)
        return nodes.view(NODE_DT), edges.view(EDGE_DT), rows

    # --- single-game pieces of the search, exposed for the object API -------------
    def count_options(self):
        """len(get_options_from_state()) per lane (cit_count_options; may mutate like get_options)."""
        n = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.cit_count_options(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), _ptr(self.seer),
                                              self.B, _ptr(n), _stream()), "cit_count_options")
        return n

    def determinize(self, orig_player, role_sample=True):
        """Game.sample_private_information(players[orig], role_sample) per lane."""
        o = torch.as_tensor(np.broadcast_to(np.asarray(orig_player, np.int32), (self.B,)).copy()).to(self.device)
        _lib.check(self.lib.cit_determinize(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx), self.B, _ptr(o),
                                            int(bool(role_sample)), _stream()), "cit_determinize")

    def skip_false_choice(self):
        """CFRNode.skip_false_choice on every lane's game; returns carry_outs played."""
        c = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.cit_skip_false_choice(_ptr(self.games), _ptr(self.mt), _ptr(self.mt_idx),
                                                  _ptr(self.seer), self.B, _ptr(c), _stream()),
                   "cit_skip_false_choice")
        return c

    # --- inspection --------------------------------------------------------------
    def rows(self):
        return self.games.cpu().numpy()

    def row(self, lane):
        return L.game_from_bytes(self.games[lane].cpu().numpy())

    def canon(self, lane):
        return _canon.canon_game(self.row(lane))

    def errors(self):
        """Per-lane error words (CIT_ERR_* bits)."""
        off = L.CitGame.err.offset
        return self.games[:, off:off + 4].contiguous().view(torch.int32).view(-1)

    def terminal(self):
        return self.games[:, L.CitGame.terminal.offset].to(torch.bool)


def _merge_parts(outs, parts, B):
    """cfr_targets of sub-batches (sub lane i of part g = global lane parts[g][i])
    -> one dict in global lane order (see _merge_targets)."""
    d = outs[0]["meta"].device
    metas, firsts, feats, values, dists, opts = [], [], [], [], [], []
    counts = torch.zeros((B, 2), dtype=torch.int32, device=d)
    base = 0
    for out, lanes in zip(outs, parts):
        lanes = lanes.to(d)
        m = out["meta"].clone()
        m[:, 0] = lanes[m[:, 0].long()].to(m.dtype)
        metas.append(m)
        firsts.append(out["meta"][:, 4].long() + base)
        base += out["dist"].shape[0]
        feats.append(out["feat"])
        values.append(out["value"])
        dists.append(out["dist"])
        opts.append(out["opt_feat"])
        counts[lanes] = out["counts"]
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


def _merge_targets(main, extra, over):
    """cfr_targets of the main pool (retried lanes empty) + those of a retry
    sub-batch (sub lane i = global lane over[i]) -> one dict in lane order, CSR
    option rows re-laid out in target order."""
    d = main["meta"].device
    over = over.to(d)
    em = extra["meta"].clone()
    em[:, 0] = over[em[:, 0].long()].to(em.dtype)
    meta = torch.cat([main["meta"], em])
    order = torch.sort(meta[:, 0].long() * (1 << 32) + torch.arange(meta.shape[0], device=d), stable=True).indices
    meta = meta[order]
    nc_main = main["dist"].shape[0]
    first = torch.cat([main["meta"][:, 4].long(), extra["meta"][:, 4].long() + nc_main])[order]
    nch = meta[:, 3].long()
    new_first = torch.cumsum(nch, 0) - nch
    rows = torch.repeat_interleave(first - new_first, nch) + torch.arange(int(nch.sum()), device=d)
    dist = torch.cat([main["dist"], extra["dist"]])[rows]
    opt_feat = torch.cat([main["opt_feat"], extra["opt_feat"]])[rows]
    meta[:, 4] = new_first.to(meta.dtype)
    counts = main["counts"].clone()
    counts[over] = extra["counts"]
    return {"meta": meta, "feat": torch.cat([main["feat"], extra["feat"]])[order],
            "value": torch.cat([main["value"], extra["value"]])[order], "dist": dist, "opt_feat": opt_feat,
            "counts": counts}
