"""Target walk (get_all_targets: k_cfr_target_count + k_cfr_targets) timed
alone after one cfr_decide of N simulate_game trees at ITERS iterations
(CIT_LIB_PATH picks the build: CFR_WALK_TPW 1 or 64).  One JSON line: the
walk's seconds per call (HIP events, 3 calls on snapshots of the same
streams) and a hash of the first call's targets (the builds must agree)."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from citadels_self_play_amd import selfplay  # noqa: E402
from citadels_self_play_amd.engine import GameBatch, pool_caps  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 960
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
seeds = selfplay.shard(N, base_seed=30_000_000)
nc, ec = pool_caps(ITERS)
b = GameBatch(np.asarray(seeds, np.int64), preset=True, device="cuda")
b.random_position(100)
b.seed_numpy()
chosen, stats = b.cfr_decide(ITERS, node_cap=nc, edge_cap=ec)
roots = selfplay._roots_for_targets(stats)
mt0, idx0 = b.mt.clone(), b.mt_idx.clone()
times, digest = [], None
for k in range(3):
    b.mt.copy_(mt0)
    b.mt_idx.copy_(idx0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t = b.cfr_targets(roots, mode=0)
    e1.record()
    torch.cuda.synchronize()
    times.append(e0.elapsed_time(e1) / 1e3)
    h = hashlib.sha256()
    for key in ("meta", "feat", "value", "dist", "opt_feat", "counts"):
        h.update(t[key].cpu().numpy().tobytes())
    if digest is None:
        digest = h.hexdigest()
    assert h.hexdigest() == digest, "the walk is not repeatable"
print(json.dumps({"lib": os.environ.get("CIT_LIB_PATH", "default"), "trees": N, "iters": ITERS,
                  "targets": int(t["feat"].shape[0]), "walk_s": times, "digest": digest,
                  "carry_outs": int(stats[:, 3].sum())}), flush=True)
