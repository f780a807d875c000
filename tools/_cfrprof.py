import sys, ctypes as C, numpy as np, torch
sys.path.insert(0, ".")
import citadels_self_play_amd._lib as LL
LL.LIB_PATH = "build/libcitprof.so"
from citadels_self_play_amd import _lib
from citadels_self_play_amd.engine import GameBatch
lib = _lib.load()
names = ["carry", "prepare", "count", "pick", "list", "sample", "copy_row", "cfr_node", "exp_role", "exp_own",
         "exp_opp", "upd_strategy", "choose", "upd_regrets", "backprop", "live_choice"]
buf = (C.c_ulonglong * 32)()
lib.cit_prof_read(buf)
for B, iters in ((1024, 200), (1024, 2000)):
    b = GameBatch(np.arange(20_000_000, 20_000_000 + B), preset=True)
    if iters == 200:
        b.advance_random(0, 300)
    else:
        b.random_position(100)
    b.seed_numpy()
    torch.cuda.synchronize()
    lib.cit_prof_read(buf)
    chosen, stats = b.cfr_decide(iters, node_cap=max(1024, 4 * iters))
    torch.cuda.synchronize()
    lib.cit_prof_read(buf)
    v = np.array(list(buf), dtype=np.float64)
    cyc, cnt = v[:16], v[16:]
    st = stats.cpu().numpy()
    tot = cyc[[5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15]].sum()
    print("B", B, "iters", iters, "carry_outs", st[:, 3].sum(), "nodes", st[:, 1].sum())
    for i, n in enumerate(names):
        print("  %-13s calls %10d  cycles/call %9.0f  share %.3f" % (n, cnt[i], cyc[i] / max(cnt[i], 1), cyc[i] / tot))
