"""Config-2 rollouts of K pre-initialised batches (inputs resident in HBM, as
bench.py's timed region) launched one after another on one stream, and
alternately on 2 or 4 HIP streams so consecutive batches overlap (the next
batch's games take the SIMD slots the previous batch's finished games free).
Prints one JSON line: transitions/s per stream count and whether every
variant played the same transitions.

    python tools/rollout_streams.py [K]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from citadels_self_play_amd.engine import GameBatch  # noqa: E402

B = 4096
BASE_SEED = 1_000_000_000


def run(K, n_streams):
    batches = [GameBatch(np.arange(BASE_SEED + k * B, BASE_SEED + (k + 1) * B), preset=True, device="cuda")
               for k in range(K)]
    streams = [torch.cuda.Stream() for _ in range(n_streams)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k, gb in enumerate(batches):
        with torch.cuda.stream(streams[k % n_streams]):
            gb.rollout()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    trans = sum(int(gb.steps.sum().item()) for gb in batches)
    return trans / el, trans


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    run(2, 1)                                   # warm-up
    out = {"batches": K, "games_per_batch": B}
    ref = None
    for n in (1, 2, 4, 8, 1, 2, 4, 8, 4, 4):
        v, trans = run(K, n)
        ref = trans if ref is None else ref
        out.setdefault("streams_%d" % n, []).append(v)
        out["same_transitions"] = out.get("same_transitions", True) and trans == ref
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
