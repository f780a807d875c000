"""Per-phase cycle accounting of the config-2 rollout step on the GPU.

Builds a profiling variant of the library (-DCIT_PROF_ROLLOUT) into
build/rollprof/libcitprof_roll.so beforehand (`python tools/prof_rollout.py build`, on
the CPU); on the GPU box run `python tools/prof_rollout.py [B]`.  Prints mean
shader-clock cycles per step for prepare / enumerate / randbelow / pick /
carry_out and enumerate+carry cycles per game state."""
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "build", "rollprof", "libcitprof_roll.so")
sys.path.insert(0, ROOT)


NAMES = ("role_pick gold_or_card which_card blackmail_response reveal_blackmail reveal_warrant build empty "
         "finish_round ghost_town smithy lab magic_school weapon_storage lighthouse museum graveyard take_gold_war "
         "assassination magistrate_warrant bewitching steal blackmail spy magic_hand_change discard_and_draw "
         "look_at_hand take_from_hand seer give_back_card take_crown_king give_crown take_crown_pat bishop cardinal "
         "abbot_gold_or_card abbot_beg merchant alchemist trader architect navigator scholar scholar_pick warlord "
         "marshal diplomat").split()


def build():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as G
    objs = []
    os.makedirs(os.path.join(ROOT, "build", "rollprof"), exist_ok=True)
    for u in ["cit_hip.hip"]:
        o = os.path.join(ROOT, "build", "rollprof", u.replace(".hip", ".o"))
        subprocess.check_call([G.HIPCC] + G.HIP_FLAGS + ["-DCIT_PROF_ROLLOUT", "-c", os.path.join(G.CSRC, u), "-o", o])
        objs.append(o)
    subprocess.check_call([G.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + [os.path.join(ROOT, "build", "hip", u.replace(".hip", ".o")) for u in G.HIP_UNITS[1:]] + ["-o", LIB])


def run(B):
    import numpy as np
    import torch
    import citadels_self_play_amd._lib as LL
    LL.LIB_PATH = LIB
    from citadels_self_play_amd.engine import GameBatch
    lib = LL.load()
    buf = (C.c_ulonglong * 160)()
    gb = GameBatch(np.arange(1_000_000_000, 1_000_000_000 + B), preset=True, device="cuda:0")
    torch.cuda.synchronize()
    lib.cit_roll_prof_read(buf)
    gb.rollout()
    torch.cuda.synchronize()
    lib.cit_roll_prof_read(buf)
    v = np.array(list(buf), dtype=np.float64)
    steps = v[5]
    names = ["prepare", "enumerate", "randbelow", "pick", "carry_out"]
    out = {"B": B, "steps": steps, "cycles_per_step": {n: v[i] / steps for i, n in enumerate(names)},
           "total_cycles_per_step": v[:5].sum() / steps,
           "twists": v[7], "cycles_per_twist": v[6] / max(v[7], 1), "twist_cycles_per_step": v[6] / steps,
           "per_state": {str(s): {"steps": v[32 + s], "share_of_steps": v[32 + s] / steps,
                                  "enum_carry_cycles_per_step": v[16 + s] / max(v[32 + s], 1)}
                         for s in range(11) if v[32 + s]},
           "carry_by_name": sorted([(NAMES[o], v[112 + o], v[64 + o] / max(v[112 + o], 1), v[64 + o] / steps)
                                    for o in range(47) if v[112 + o]], key=lambda t: -t[3])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 4096)
