"""Distribution of carry_out steps per game (config 2) and the tail it puts
on a fixed-size launch: python tools/game_lengths.py [B]  (GPU)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from citadels_self_play_amd.engine import GameBatch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
gb = GameBatch(np.arange(1_000_000_000, 1_000_000_000 + B), preset=True, device="cuda:0")
gb.rollout()
torch.cuda.synchronize()
s = gb.steps.cpu().numpy().astype(np.float64)
q = np.percentile(s, [50, 90, 99, 99.9, 100])
print(json.dumps({"B": B, "mean": s.mean(), "p50": q[0], "p90": q[1], "p99": q[2], "p999": q[3], "max": q[4],
                  "mean_over_max": s.mean() / q[4]}))
