"""Per-tree duration distribution of k_cfr_decide (how much of a launch is the
tail of its slowest trees).

`python tools/cfr_tree_clock.py build` (here, CPU) compiles cit_cfr.hip with
-DCFR_TREE_CLOCK into build/treeclock/libcittc.so (other units from the main
build); `python tools/cfr_tree_clock.py run [LIB]` (GPU box) runs config 3
(1024 positions, cfr_train(200)) and 1024 config-5-style trees at
cfr_train(2000), and prints per workload: kernel ms, per-tree ms quantiles,
busy fraction = sum(tree time) / (trees x launch span), and the correlation of
tree time with its carry_outs / nodes."""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build", "treeclock")
LIB = os.path.join(OUT, "libcittc.so")


def build(extra=()):
    import __graft_entry__ as G
    os.makedirs(OUT, exist_ok=True)
    objs = []
    for u in G.HIP_UNITS:
        if u == "cit_cfr.hip":
            o = os.path.join(OUT, "cit_cfr.o")
            subprocess.check_call([G.HIPCC] + G.HIP_FLAGS + ["-DCFR_TREE_CLOCK"] + list(extra) +
                                  ["-c", os.path.join(G.CSRC, u), "-o", o])
        else:
            o = os.path.join(ROOT, "build", "hip", u.replace(".hip", ".o"))
        objs.append(o)
    subprocess.check_call([G.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", LIB])
    print(LIB)


def run(lib_path=LIB):
    import torch
    import citadels_self_play_amd._lib as LL
    LL.LIB_PATH = lib_path
    from citadels_self_play_amd import _lib, selfplay
    from citadels_self_play_amd.engine import GameBatch, pool_caps
    lib = _lib.load()
    lib.cit_tree_clock_read.argtypes = [C.c_void_p, C.c_int]
    loads = (("config3", 1024, 200, 0), ("config3", 1024, 200, 1), ("config3", 1024, 200, 2),
             ("config5_2000", 1024, 2000, 0), ("config4", 512, 200, 0), ("config4", 512, 200, 1),
             ("config4", 4096, 200, 0), ("config4", 4096, 200, 1))
    only = os.environ.get("TREE_CLOCK_ONLY")          # e.g. "config4": those workloads only
    net = None
    for tag, B, iters, rep in loads:
        if only and tag not in only.split(","):
            continue
        seeds = selfplay.shard(B, base_seed=30_000_000 + rep * B)
        b = GameBatch(seeds, preset=True)
        if iters == 200:
            b.advance_random(0, 300)
        else:
            b.random_position(100)
        b.seed_numpy()
        nc, ec = pool_caps(iters)
        if tag == "config4" and net is None:
            from citadels_self_play_amd import models
            torch.manual_seed(0)
            net = models.ValueNet(models.ValueOnlyNN(418, 512), "cuda")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if tag == "config4":           # cfr_pred with in-kernel leaves (k_cfr_pred_fused keeps the same clock)
            chosen, stats, _ = b.cfr_pred(iters, net, max_depth=10, node_cap=4096, fused=True)
        else:
            chosen, stats = b._cfr_decide(iters, nc, ec)
        e1.record()
        torch.cuda.synchronize()
        buf = (C.c_ulonglong * (2 * B))()
        _lib.check(lib.cit_tree_clock_read(buf, B), "cit_tree_clock_read")
        t = np.array(list(buf), dtype=np.float64).reshape(B, 2)
        dur = (t[:, 1] - t[:, 0]) / 100e3          # 100 MHz -> ms
        span = (t[:, 1].max() - t[:, 0].min()) / 100e3
        st = stats.cpu().numpy().astype(np.float64)
        q = np.percentile(dur, [0, 10, 50, 90, 99, 100])
        print(json.dumps({
            "workload": tag, "rep": rep, "trees": B, "iters": iters, "kernel_ms": e0.elapsed_time(e1),
            "span_ms": span, "tree_ms": dict(zip(["min", "p10", "p50", "p90", "p99", "max"], q.tolist())),
            "tree_ms_mean": float(dur.mean()), "busy_frac": float(dur.sum() / (B * span)),
            "start_spread_ms": float((t[:, 0].max() - t[:, 0].min()) / 100e3),
            "carry_outs_mean": float(st[:, 3].mean()), "carry_outs_max": float(st[:, 3].max()),
            "us_per_carry_median": float(np.median(dur * 1e3 / np.maximum(st[:, 3], 1))),
            "corr_carry": float(np.corrcoef(dur, st[:, 3])[0, 1]), "corr_nodes": float(np.corrcoef(dur, st[:, 1])[0, 1]),
            "slowest": [{"ms": float(dur[i]), "carry": int(st[i, 3]), "nodes": int(st[i, 1]), "err": int(st[i, 4])}
                        for i in np.argsort(-dur)[:5]],
            "errors": int((st[:, 4] != 0).sum())}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        run(*sys.argv[2:])
