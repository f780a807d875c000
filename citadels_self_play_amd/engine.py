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
import numpy as np
import torch

from . import _lib
from . import canon as _canon
from . import layout as L


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
