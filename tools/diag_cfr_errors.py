"""Error-bit histogram of config-5 trees (simulate_games) and config-3
decisions on the GPU; prints the seeds of lanes that end with an error so the
CPU oracle can be asked whether the reference raises on them too.

`python tools/diag_cfr_errors.py build` (CPU) compiles a CFR_ERR_DIAG variant
(build/cfrdiag/libcfrdiag.so) whose tree error words also say which
np.random.choice check raised (0x200 empty option list, 0x400 NaN/negative
probability, 0x800 probabilities not summing to 1); `DIAG_LIB=... python
tools/diag_cfr_errors.py ITERS TREES` uses it."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from citadels_self_play_amd import selfplay  # noqa: E402


def report(tag, seeds, b, stats, t=None):
    err_row = b.errors().cpu().numpy() if b.B == stats.shape[0] else np.zeros(stats.shape[0], np.int64)
    st = stats.cpu().numpy()
    term = t["terminal"].cpu().numpy() if t is not None and "terminal" in t else b.terminal().cpu().numpy()
    bad = np.nonzero((st[:, 4] != 0) & ~term)[0]
    print(json.dumps({"tag": tag, "lanes": int(len(seeds)), "err_lanes": int(len(bad)),
                      "cases": [{"seed": int(seeds[i]), "tree_err": int(st[i, 4]), "row_err": int(err_row[i]),
                                 "nodes": int(st[i, 1]), "edges": int(st[i, 2])} for i in bad[:64]]}), flush=True)


def build():
    import subprocess
    import __graft_entry__ as G
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "build", "cfrdiag")
    os.makedirs(out, exist_ok=True)
    o = os.path.join(out, "cit_cfr.o")
    subprocess.check_call([G.HIPCC] + G.HIP_FLAGS + ["-DCFR_ERR_DIAG", "-c", os.path.join(G.CSRC, "cit_cfr.hip"),
                                                      "-o", o])
    others = [os.path.join(root, "build", "hip", u.replace(".hip", ".o")) for u in G.HIP_UNITS if u != "cit_cfr.hip"]
    lib = os.path.join(out, "libcfrdiag.so")
    subprocess.check_call([G.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", o] + others + ["-o", lib])
    print(lib)


def main():
    if sys.argv[1:] == ["build"]:
        return build()
    if os.environ.get("DIAG_LIB"):
        import citadels_self_play_amd._lib as LL
        LL.LIB_PATH = os.environ["DIAG_LIB"]
    torch.cuda.set_device(0)
    if len(sys.argv) > 2:                 # diag_cfr_errors.py ITERS TREES
        iters, n = int(sys.argv[1]), int(sys.argv[2])
        seeds = selfplay.shard(n, base_seed=30_000_000)
        b, stats, t = selfplay.simulate_games(seeds, iters)
        torch.cuda.synchronize()
        report("config5_%d" % iters, seeds, b, stats, t)
        return
    seeds = selfplay.shard(1024, base_seed=30_000_000)
    b, stats, _ = selfplay.simulate_games(seeds, 2000)
    torch.cuda.synchronize()
    report("config5_2000", seeds, b, stats)
    seeds = selfplay.shard(256, base_seed=30_000_000)
    b, stats, _ = selfplay.simulate_games(seeds, 20000)
    torch.cuda.synchronize()
    report("config5_20000", seeds, b, stats)


if __name__ == "__main__":
    main()
