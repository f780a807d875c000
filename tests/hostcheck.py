"""Loader for the TEST-ONLY host build of the engine headers
(csrc/cit_host.cpp -> build/libcitadels_hostcheck.so).  Used by the CPU test
suite to validate engine logic against the golden fixtures without a GPU."""
import ctypes as C
import os
import subprocess

import numpy as np

from citadels_self_play_amd import layout as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "citadels_self_play_amd", "csrc")
LIB = os.path.join(ROOT, "build", "libcitadels_hostcheck.so")

_lib = None


def build(force=False):
    srcs = [os.path.join(SRC, f) for f in ("cit_host.cpp", "cit_engine.h", "cit_core.h")]
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(s) for s in srcs):
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", srcs[0], "-o", LIB])
    return LIB


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class HostBatch:
    """B games + their CPython MT streams in host memory, row layout identical to the device."""

    def __init__(self, seeds, preset=True):
        self.B = len(seeds)
        self.games = np.zeros((self.B, L.GAME_BYTES), np.uint8)
        self.mt = np.zeros((L.MT_N, self.B), np.uint32)
        self.idx = np.zeros(self.B, np.uint32)
        self.seeds = np.asarray(seeds, np.uint64)
        self.seer = np.zeros((self.B, L.SEER_MAX), np.uint64)
        lib().cith_init(_p(self.games), _p(self.mt), _p(self.idx), C.c_int(self.B), _p(self.seeds),
                        C.c_int(int(preset)))

    def game(self, l):
        return L.game_from_bytes(self.games[l])

    def get_options(self, max_opts=4096):
        out = np.zeros((self.B, max_opts, 16), np.uint8)
        n = np.zeros(self.B, np.int32)
        lib().cith_get_options(_p(self.games), _p(self.mt), _p(self.idx), _p(self.seer), C.c_int(self.B), _p(out),
                               C.c_int(max_opts), _p(n))
        return out, n

    def carry_out(self, chosen):
        w = np.zeros(self.B, np.int32)
        chosen = np.ascontiguousarray(chosen, np.uint8)
        lib().cith_carry_out(_p(self.games), _p(self.mt), _p(self.idx), C.c_int(self.B), _p(chosen), _p(w))
        return w

    def randbelow(self, lane, bound):
        out = np.zeros(1, np.uint32)
        lib().cith_mt_randbelow(_p(self.mt), _p(self.idx), C.c_int(self.B), C.c_int(lane), C.c_uint32(bound),
                                C.c_int(1), _p(out))
        return int(out[0])

    def rollout(self, max_steps=-1):
        steps = np.zeros(self.B, np.int32)
        w = np.zeros(self.B, np.int32)
        lib().cith_rollout(_p(self.games), _p(self.mt), _p(self.idx), _p(self.seer), C.c_int(self.B), C.c_int(max_steps),
                           _p(steps), _p(w))
        return steps, w
