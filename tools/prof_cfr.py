"""MCCFR phase-cycle breakdown (SURVEY §8(d) CFR row) on the GPU box.

Builds (here, on the CPU: `python tools/prof_cfr.py build`) a variant of
libcitadels_hip.so whose search translation unit is compiled with -DCIT_PROF
(per-function clock64 accounting by lane 0 of each tree, csrc/cit_cfr.h
CIT_PROF_SCOPE) into build/cfrprof/; on the box `python tools/prof_cfr.py run`
runs config 3 (1024 positions, cfr_train(200)) and config 5 trees
(cfr_train(2000)), and prints one JSON line per workload: calls, cycles per
call and share of the search's cycles per phase.  Nested scopes: cfr_node
contains skip-carry/prepare/list; expand_* contain copy_row, sample, carry,
cfr_node; shares are of the top-level sum (expand_*, update_strategy, choose,
backprop, live_choice)."""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build", "cfrprof")
LIB = os.path.join(OUT, "libcitprof.so")
NAMES = ["carry", "prepare", "count", "pick", "list", "sample", "copy_row", "cfr_node", "exp_role", "exp_own",
         "exp_opp", "upd_strategy", "choose", "upd_regrets", "backprop", "live_choice"]


def build():
    import __graft_entry__ as G
    os.makedirs(OUT, exist_ok=True)
    objs = []
    for u in G.HIP_UNITS:
        o = os.path.join(OUT, u.replace(".hip", ".o"))
        extra = ["-DCIT_PROF"] if u == "cit_cfr.hip" else []
        if u != "cit_cfr.hip":
            o = os.path.join(ROOT, "build", "hip", u.replace(".hip", ".o"))
        else:
            subprocess.check_call([G.HIPCC] + G.HIP_FLAGS + extra + ["-c", os.path.join(G.CSRC, u), "-o", o])
        objs.append(o)
    subprocess.check_call([G.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", LIB])
    print(LIB)


def run():
    import torch
    import citadels_self_play_amd._lib as LL
    LL.LIB_PATH = LIB
    from citadels_self_play_amd import _lib
    from citadels_self_play_amd.engine import GameBatch, pool_caps
    lib = _lib.load()
    lib.cit_prof_read.argtypes = [C.c_void_p]
    buf = (C.c_ulonglong * 32)()
    for tag, B, iters in (("config3", 1024, 200), ("config5_2000", 1024, 2000)):
        b = GameBatch(np.arange(20_000_000, 20_000_000 + B), preset=True)
        if iters == 200:
            b.advance_random(0, 300)
        else:
            b.random_position(100)
        b.seed_numpy()
        torch.cuda.synchronize()
        lib.cit_prof_read(buf)
        nc, ec = pool_caps(iters)
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        chosen, stats = b.cfr_decide(iters, node_cap=nc, edge_cap=ec)
        t1.record()
        torch.cuda.synchronize()
        lib.cit_prof_read(buf)
        v = np.array(list(buf), dtype=np.float64)
        cyc, cnt = v[:16], v[16:]
        st = stats.cpu().numpy()
        top = cyc[[8, 9, 10, 11, 12, 14, 15]].sum()      # the top-level scopes of the search loop
        phases = {n: {"calls": int(cnt[i]), "cycles_per_call": cyc[i] / max(cnt[i], 1),
                      "share_of_search": cyc[i] / top} for i, n in enumerate(NAMES)}
        print(json.dumps({"workload": tag, "trees": B, "iters": iters, "ms": t0.elapsed_time(t1),
                          "carry_outs": int(st[:, 3].sum()), "nodes": int(st[:, 1].sum()),
                          "cycles_per_tree": top / B, "phases": phases}), flush=True)


if __name__ == "__main__":
    build() if sys.argv[1:] == ["build"] else run()
