"""Sweep games-per-block (lanes per workgroup) and batch size for the fused
rollout kernel; prints one JSON line per configuration (HIP-event timing)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from citadels_self_play_amd.engine import GameBatch  # noqa: E402


def run(B, gpb, reps=3, preset=True):
    best = None
    for r in range(reps):
        b = GameBatch(np.arange(5_000_000 + r * B, 5_000_000 + (r + 1) * B), preset=preset, games_per_block=gpb)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.rollout()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        steps = int(b.steps.sum())
        errs = int((b.errors() != 0).sum())
        rate = steps / (ms * 1e-3)
        if best is None or rate > best["rate"]:
            best = {"B": B, "gpb": gpb, "preset": preset, "ms": ms, "steps": steps, "rate": rate, "errs": errs}
    return best


if __name__ == "__main__":
    bs = [int(x) for x in os.environ.get("BS", "4096").split(",")]
    gs = [int(x) for x in os.environ.get("GS", "1,2,4,8,16,32,64").split(",")]
    for B in bs:
        for g in gs:
            print(json.dumps(run(B, g)), flush=True)
