"""How much of a config-2 launch (k_rollout_u, 4096 games) is the tail.

`python tools/rollout_clock.py build [flags]` (CPU) compiles cit_hip.hip with
-DROLL_CLOCK into build/rollclock/librollclock.so; `python
tools/rollout_clock.py run` (GPU box) rolls out 4096 preset games and prints:
launch span, per-game duration and steps, busy fraction = sum(game time) /
(games x span), the number of games still running at 25/50/75/90 % of the
span, and per-step time of the longest games (the latency that sets the
launch time) vs the median game."""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build", "rollclock")
LIB = os.path.join(OUT, "librollclock.so")


def build(extra=()):
    import __graft_entry__ as G
    os.makedirs(OUT, exist_ok=True)
    o = os.path.join(OUT, "cit_hip.o")
    subprocess.check_call([G.HIPCC] + G.HIP_FLAGS + ["-DROLL_CLOCK"] + list(extra) +
                          ["-c", os.path.join(G.CSRC, "cit_hip.hip"), "-o", o])
    others = [os.path.join(ROOT, "build", "hip", u.replace(".hip", ".o")) for u in G.HIP_UNITS[1:]]
    subprocess.check_call([G.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", o] + others + ["-o", LIB])
    print(LIB)


def run(lib_path=LIB):
    import torch
    import citadels_self_play_amd._lib as LL
    LL.LIB_PATH = lib_path
    from citadels_self_play_amd import _lib
    from citadels_self_play_amd.engine import GameBatch
    lib = _lib.load()
    lib.cit_roll_clock_read.argtypes = [C.c_void_p, C.c_int]
    B = 4096
    for rep in range(3):
        b = GameBatch(np.arange(1_000_000_000 + rep * B, 1_000_000_000 + (rep + 1) * B), preset=True)
        torch.cuda.synchronize()
        b.rollout()
        torch.cuda.synchronize()
        buf = (C.c_ulonglong * (2 * B))()
        _lib.check(lib.cit_roll_clock_read(buf, B), "cit_roll_clock_read")
        t = np.array(list(buf), dtype=np.float64).reshape(B, 2) / 100.0   # us
        t -= t[:, 0].min()
        dur = t[:, 1] - t[:, 0]
        span = t[:, 1].max()
        steps = b.steps.cpu().numpy().astype(np.float64)
        live = {f: int(((t[:, 0] <= f * span) & (t[:, 1] > f * span)).sum()) for f in (0.25, 0.5, 0.75, 0.9)}
        order = np.argsort(-dur)
        print(json.dumps({"rep": rep, "span_us": span, "game_us": {"mean": dur.mean(), "max": dur.max()},
                          "steps": {"mean": steps.mean(), "max": steps.max()},
                          "busy_frac": float(dur.sum() / (B * span)), "live_games_at": live,
                          "start_spread_us": float(t[:, 0].max()),
                          "us_per_step_median_game": float(np.median(dur / steps)),
                          "longest": [{"us": float(dur[i]), "steps": int(steps[i]), "us_per_step": float(dur[i] / steps[i])}
                                      for i in order[:3]],
                          "most_steps": {"steps": int(steps.max()), "us": float(dur[np.argmax(steps)])}}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        run(*sys.argv[2:])
