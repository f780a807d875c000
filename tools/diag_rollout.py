"""Game-length distribution of the config-2 batch (tail effect of the
one-game-per-wave rollout: the launch lasts as long as its longest game)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from citadels_self_play_amd.engine import GameBatch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
gb = GameBatch(np.arange(1_000_000_000, 1_000_000_000 + B), preset=True, device="cuda:0")
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
gb.rollout()
e1.record()
torch.cuda.synchronize()
s = gb.steps.cpu().numpy().astype(np.int64)
ms = e0.elapsed_time(e1)
print(json.dumps({"B": B, "ms": ms, "mean": float(s.mean()), "max": int(s.max()), "min": int(s.min()),
                  "p50": float(np.percentile(s, 50)), "p99": float(np.percentile(s, 99)),
                  "us_per_step_longest": ms * 1e3 / s.max(), "mean_over_max": float(s.mean() / s.max())}))
