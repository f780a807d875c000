"""MCCFR phase-cycle breakdown (SURVEY §8(d) CFR row) on the GPU box.

`python tools/prof_cfr.py build` (here, on the CPU) compiles variants of
libcitadels_hip.so whose search translation unit has -DCIT_PROF (per-scope
clock64 accounting by lane 0 of each tree, csrc/cit_cfr.h CIT_PROF_SCOPE),
each timing only the scopes of one CIT_PROF_MASK, so that a variant's
accounting perturbs the search little (one s_memtime pair per timed scope):

  top    expand_role / expand_own / expand_opp / update_strategy / choose /
         backprop / live_choice  (once per search iteration)
  node   sample / copy_row / cfr_node
  engine carry / prepare / list (LDS) / pick / list (HBM)
  sample the determinization's parts (cit_engine.h cit_sample_private_wave)

`python tools/prof_cfr.py run` (GPU box) runs config 3 (1024 positions,
cfr_train(200)) and config-5-style trees (cfr_train(2000)) with the plain
library and with each variant, and prints one JSON line per (variant,
workload): kernel ms (plain and profiled: the perturbation), calls, cycles per
call, and each scope's share of the tree's cycles (scopes nest: cfr_node
contains carry/prepare/list; expand_* contain copy_row, sample, carry,
cfr_node)."""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build", "cfrprof")
NAMES = ["carry", "prepare", "list_lds", "pick", "list", "sample", "copy_row", "cfr_node", "exp_role", "exp_own",
         "exp_opp", "upd_strategy", "choose", "upd_regrets", "backprop", "live_choice",
         "smp_used", "smp_unknown", "smp_deck", "smp_warrants", "smp_opponents", "skip_false", "row_store",
         "row_load", "leaf_eval"] + ["s%d" % i for i in range(25, 32)]
VARIANTS = {"top": (8, 9, 10, 11, 12, 14, 15), "node": (5, 6, 7), "engine": (0, 1, 2, 3, 4),
            "sample": (5, 16, 17, 18, 19, 20), "rows": (7, 21, 22, 23), "pred": (8, 9, 10, 11, 12, 14, 24)}


# PROF_TAG / PROF_FLAGS: a tagged set of variants built with extra flags (A/B of a
# change inside one scope), e.g. PROF_TAG=base PROF_FLAGS="-DCIT_SHUFFLE_TRACE=0"
TAG = os.environ.get("PROF_TAG", "")
EXTRA = os.environ.get("PROF_FLAGS", "").split()


def lib_of(name):
    return os.path.join(OUT, "libcitprof_%s%s.so" % (name, "_" + TAG if TAG else ""))


def build(only=None):
    """Compile the variants in parallel (PROF_ONLY=name,name: a subset)."""
    import __graft_entry__ as G
    os.makedirs(OUT, exist_ok=True)
    others = [os.path.join(ROOT, "build", "hip", u.replace(".hip", ".o")) for u in G.HIP_UNITS if u != "cit_cfr.hip"]
    only = only or [n for n in os.environ.get("PROF_ONLY", "").split(",") if n]
    names = [n for n in VARIANTS if not only or n in only]
    procs = []
    for name in names:
        mask = sum(1 << i for i in VARIANTS[name])
        o = os.path.join(OUT, "cit_cfr_%s%s.o" % (name, "_" + TAG if TAG else ""))
        procs.append((name, o, subprocess.Popen([G.HIPCC] + G.HIP_FLAGS + EXTRA + [
            "-DCIT_PROF", "-DCIT_PROF_MASK=%dull" % mask, "-c", os.path.join(G.CSRC, "cit_cfr.hip"), "-o", o])))
    for name, o, p in procs:
        if p.wait():
            raise RuntimeError("hipcc failed for variant %s" % name)
        subprocess.check_call([G.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", o] + others + ["-o", lib_of(name)])
        print(lib_of(name))


_NET = []


def _workload(GameBatch, pool_caps, torch, B, iters, pred=False):
    b = GameBatch(np.arange(20_000_000, 20_000_000 + B), preset=True)
    if iters <= 200:
        b.advance_random(0, 300)
    else:
        b.random_position(100)
    b.seed_numpy()
    torch.cuda.synchronize()
    nc, ec = pool_caps(iters)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    if pred and not _NET:
        from citadels_self_play_amd import models
        torch.manual_seed(0)
        _NET.append(models.ValueNet(models.ValueOnlyNN(418, 512), "cuda"))
    t0.record()
    if pred:               # config 4: cfr_pred(iters, 10) with in-kernel leaves
        chosen, stats, _ = b.cfr_pred(iters, _NET[0], max_depth=10, node_cap=4096, fused=True)
    else:
        chosen, stats = b._cfr_decide(iters, nc, ec)
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1), stats.cpu().numpy()


def run(which=None, workloads=None):
    import torch
    import citadels_self_play_amd._lib as LL
    from citadels_self_play_amd.engine import GameBatch, pool_caps
    which = None if which in ("", "all") else which
    loads = [("plain", LL.LIB_PATH)] + [(n, lib_of(n)) for n in VARIANTS if which in (None, n) or
                                        (which and n in which.split("+"))]
    plain = {}
    for vname, path in loads:
        LL._lib = None
        LL.LIB_PATH = path
        lib = LL.load()
        if vname != "plain":
            lib.cit_prof_read.argtypes = [C.c_void_p]
            buf = (C.c_ulonglong * 64)()
        # workloads "ITERS:B" (cfr_train) or "pred:ITERS:B" (cfr_pred, config 4)
        wl = (("config3", 1024, 200, False), ("config5_2000", 1024, 2000, False)) if not workloads else \
            [("%s_b%s" % (w.rsplit(":", 1)[0].replace(":", ""), w.rsplit(":", 1)[1]), int(w.rsplit(":", 1)[1]),
              int(w.split(":")[-2]), w.startswith("pred:")) for w in workloads.split(",")]
        for tag, B, iters, pred in wl:
            if vname != "plain":
                lib.cit_prof_read(buf)
            ms, st = _workload(GameBatch, pool_caps, torch, B, iters, pred)
            if vname == "plain":
                plain[tag] = ms
                continue
            lib.cit_prof_read(buf)
            v = np.array(list(buf), dtype=np.float64)
            cyc, cnt = v[:32], v[32:]
            ids = VARIANTS[vname]
            phases = {NAMES[i]: {"calls": int(cnt[i]), "cycles_per_call": cyc[i] / max(cnt[i], 1),
                                 "cycles_per_tree": cyc[i] / B, "cycles_per_carry": cyc[i] / max(st[:, 3].sum(), 1)}
                      for i in ids}
            print(json.dumps({"variant": vname + ("_" + TAG if TAG else ""), "workload": tag, "trees": B, "iters": iters, "ms": ms,
                              "ms_plain": plain.get(tag), "carry_outs": int(st[:, 3].sum()),
                              "nodes": int(st[:, 1].sum()), "phases": phases}), flush=True)


if __name__ == "__main__":
    # run [variant] [iters:B ...]  (workloads comma- or space-separated)
    build() if sys.argv[1:] == ["build"] else run(*(sys.argv[2:3] + ([",".join(sys.argv[3:])] if sys.argv[3:] else [])))
