"""Engine scopes of the config-2 rollout (k_rollout_u) on the GPU: the
CIT_PROF_SCOPE blocks 25..31 of csrc/cit_engine.h -- state 5's option
generation split into type mask / builds / role abilities / the rest, the
whole enumeration, and finish_round's round end vs next player -- as
shader-clock cycles per call and per rollout step.

    python tools/prof_rollout_scopes.py build      # here (CPU): build/rollscope/libcitscope.so
    python tools/prof_rollout_scopes.py [B]        # GPU box"""
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "rollscope")
LIB = os.path.join(OUT, "libcitscope.so")
sys.path.insert(0, ROOT)
SCOPES = {25: "state5_type_mask", 26: "state5_builds", 27: "state5_role", 28: "state5_rest",
          29: "enum_options_all", 30: "finish_round_end", 31: "finish_next_player"}


def build():
    import __graft_entry__ as G
    os.makedirs(OUT, exist_ok=True)
    o = os.path.join(OUT, "cit_hip.o")
    subprocess.check_call([G.HIPCC] + G.HIP_FLAGS + G.UNIT_FLAGS.get("cit_hip.hip", []) +
                          ["-DCIT_PROF", "-DCIT_PROF_MASK=0xfe000000ull", "-c", os.path.join(G.CSRC, "cit_hip.hip"),
                           "-o", o])
    objs = [o] + [os.path.join(ROOT, "build", "hip", u.replace(".hip", ".o")) for u in G.HIP_UNITS[1:]]
    subprocess.check_call([G.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", LIB])
    print(LIB)


def run(B):
    import numpy as np
    import torch
    import citadels_self_play_amd._lib as LL
    LL.LIB_PATH = LIB
    from citadels_self_play_amd.engine import GameBatch
    lib = LL.load()
    lib.cit_hip_prof_read.argtypes = [C.c_void_p]
    buf = (C.c_ulonglong * 64)()
    gb = GameBatch(np.arange(1_000_000_000, 1_000_000_000 + B), preset=True, device="cuda:0")
    torch.cuda.synchronize()
    lib.cit_hip_prof_read(buf)
    steps, _ = gb.rollout()
    torch.cuda.synchronize()
    lib.cit_hip_prof_read(buf)
    v = np.array(list(buf), dtype=np.float64)
    n = float(steps.sum().item())
    out = {"B": B, "steps": n, "scopes": {name: {"calls": v[32 + i], "cycles_per_call": v[i] / max(v[32 + i], 1),
                                                  "cycles_per_step": v[i] / n} for i, name in SCOPES.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 4096)
