"""CPU ORACLE (test infrastructure only): ctypes wrapper of oracle/mlp_fma.c
and encode_game restated over the oracle's game model (game/game.py:91-128)."""
import ctypes as C
import os
import subprocess

import numpy as np

import citadels_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "mlp_fma.c")
LIB = os.path.join(HERE, "_ref", "libmlp_fma.so")
_lib = None


def build():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-shared", "-fPIC", SRC, "-o", LIB, "-lm"])
    return LIB


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
    return _lib


class FmaMLP:
    """folded = models.fold(ValueOnlyNN) tensors (w1t, b1, ..., w4t, b4)."""

    def __init__(self, folded):
        self.w = [np.ascontiguousarray(t.numpy() if hasattr(t, "numpy") else t, np.float32) for t in folded]

    def __call__(self, feat, logits=False):
        x = np.ascontiguousarray(np.atleast_2d(feat), np.float32)
        M = x.shape[0]
        probs = np.zeros((M, 6), np.float32)
        lg = np.zeros((M, 6), np.float32)
        p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        lib().mlp_forward(p(x), C.c_int(M), *[p(w) for w in self.w], p(probs), p(lg))
        return (probs, lg) if logits else probs


def encode_game(g, pid=None):
    """game.py:91-128 over citadels_oracle.OGame; pid overrides gamestate.player_id."""
    cur = g.gs.pid if pid is None else pid
    v = np.zeros(418, np.float32)
    for r in range(8):
        v[r * 3 + g.roles[r] % 3] = 1
    for p in g.players:
        if p.role is None or p.role == O.BEWITCHED:
            continue
        if g.players[cur].kr[p.id][1]:
            v[24 + p.id * 8 + p.role // 3] = 1
    for i, p in enumerate(g.players):
        v[72 + i] = O.count_points(p)
        v[78 + i] = p.gold
        v[84 + i] = len(p.hand)
        for c in p.build:
            v[90 + i * 40 + O.ctype(c)] += 1
            v[330 + i * 5 + O.csuit(c)] += 1
    v[360 + cur] = 1
    v[366 + g.gs.state] = 1
    v[377] = 1 if g.ending else 0
    for r in range(8):
        rp = g.rp[r]
        v[378 + r * 5:378 + r * 5 + 5] = [bool(rp[0]), rp[1] is not None, bool(rp[2]), bool(rp[3]), rp[4] is not None]
    return v
