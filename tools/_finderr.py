import sys, numpy as np, torch, collections
sys.path.insert(0, ".")
from citadels_self_play_amd.engine import GameBatch
B = int(sys.argv[1]); n = int(sys.argv[2]); base = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000_000
cnt = collections.Counter(); steps = 0
for step in range(n):
    s0 = base + step * B
    b = GameBatch(np.arange(s0, s0 + B), preset=True)
    b.rollout()
    e = b.errors().cpu().numpy()
    steps += int(b.steps.sum())
    for l in np.nonzero(e)[0]:
        cnt[hex(e[l])] += 1
        print("seed", s0 + l, "err", hex(e[l]), "steps", int(b.steps[l]), flush=True)
print("games", B * n, "transitions", steps, "errors", dict(cnt))
