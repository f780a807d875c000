"""Config 5 through train_from_scratch.collect at one admission setting
(CIT_LOOKAHEAD_WALKED / CIT_LOOKAHEAD_DEPTH, read at import): R rounds of N trees per GPU at
cfr_train(ITERS); one JSON line with the rounds' completion times."""
import json
import os
import sys
import time
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from citadels_self_play_amd import train_from_scratch as tfs  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1920
R = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ITERS = int(sys.argv[3]) if len(sys.argv) > 3 else 200000
args = SimpleNamespace(iters=ITERS, games_per_gpu=N, node_cap=None, seed=30_000_000 + 90_000_000, on_error="drop",
                       save_tuples=False, lookahead=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
T0 = time.perf_counter()
log = (lambda m: print("%8.2f %s" % (time.perf_counter() - T0, m), flush=True)) if os.environ.get("CIT_LOG") else (
    lambda m: None)
feat, value, _ = tfs.collect(0, 1, args, 0, 10 ** 15, log, max_rounds=R)
torch.cuda.synchronize()
el = time.perf_counter() - t0
print(json.dumps({"walked": tfs.LOOKAHEAD_WALKED, "depth": tfs.LOOKAHEAD_DEPTH, "trees": N, "rounds": R, "seconds": el,
                  "trees_per_s": N * R / el, "round_done_s": [t - t0 for t in tfs.collect.round_done],
                  "targets": int(feat.shape[0]), "queue": tfs.collect.queue}), flush=True)
