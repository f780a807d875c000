"""Diagnostic (GPU box): step the one-game-per-lane rollout kernel
(games_per_block = G, cit_lanes.hip) one carry_out at a time over the golden
trajectories and dump, for each lane's first step whose post-state hash
differs from the reference's, the pre-state (row, CPython stream) and the
GPU post-state row, so the step can be replayed on the host build
(tests/hostcheck.py) and the two rows compared field by field.

    python tools/diag_lanes.py [preset|random] [G] > gpurun_out/diag_lanes.json
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from citadels_self_play_amd import canon  # noqa: E402
from citadels_self_play_amd import layout as L  # noqa: E402
from citadels_self_play_amd.engine import GameBatch  # noqa: E402
from conftest import load_golden  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "random"
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    recs = load_golden("traj_random.json.gz" if kind == "random" else "traj_preset.json.gz")
    b = GameBatch([r["seed"] for r in recs], preset=kind != "random")
    out = {}
    nmax = max(len(r["steps"]) for r in recs)
    for i in range(nmax):
        pre = b.rows()
        mt, idx = b.mt.cpu().numpy().view(np.uint32).copy(), b.mt_idx.cpu().numpy().copy()
        b.rollout(max_steps=1, games_per_block=G)
        post = b.rows()
        for l, r in enumerate(recs):
            if l in out or i >= len(r["steps"]):
                continue
            if canon.hash_obj(canon.canon_game(L.game_from_bytes(post[l]))) != r["steps"][i][5]:
                out[l] = {"lane": l, "seed": r["seed"], "step": i, "golden_step": r["steps"][i],
                          "pre_row": pre[l].tolist(), "pre_mt": mt[:, l].tolist(), "pre_idx": int(idx[l]),
                          "post_row": post[l].tolist()}
        if len(out) == len(recs):
            break
    # at each diverged pre-state: the per-lane enumeration (cit_get_options_lanes)
    # against the wave-uniform one (cit_get_options), options and seer scratch
    from citadels_self_play_amd import _lib
    lib = _lib.load()
    for x in list(out.values())[:8]:
        res = {}
        for name in ("cit_get_options", "cit_get_options_lanes"):
            games = torch.tensor(np.array([x["pre_row"]], np.uint8), device="cuda")
            mt = torch.tensor(np.array(x["pre_mt"], np.uint32).view(np.int32).reshape(L.MT_N, 1), device="cuda")
            idx = torch.tensor([x["pre_idx"]], dtype=torch.int32, device="cuda")
            seer = torch.zeros((1, L.SEER_MAX), dtype=torch.int64, device="cuda")
            opts = torch.zeros((1, 2048, 16), dtype=torch.uint8, device="cuda")
            n = torch.zeros(1, dtype=torch.int32, device="cuda")
            _lib.check(getattr(lib, name)(games.data_ptr(), mt.data_ptr(), idx.data_ptr(), seer.data_ptr(), 1,
                                          opts.data_ptr(), 2048, n.data_ptr(),
                                          torch.cuda.current_stream().cuda_stream), name)
            torch.cuda.synchronize()
            res[name] = (int(n.item()), opts.cpu().numpy(), seer.cpu().numpy(), int(idx.item()), games.cpu().numpy())
        (nw, ow, sw, iw, gw), (nl, ol, sl, il, gl) = res["cit_get_options"], res["cit_get_options_lanes"]
        x["enum_check"] = {"n_wave": nw, "n_lanes": nl, "opts_equal": bool(np.array_equal(ow[0, :nw], ol[0, :nl])),
                           "seer_equal": bool(np.array_equal(sw, sl)), "idx_wave": iw, "idx_lanes": il,
                           "rows_equal": bool(np.array_equal(gw, gl)),
                           "seer_diff_at": np.nonzero(sw[0] != sl[0])[0][:20].tolist(),
                           "seer_wave_head": [hex(int(v)) for v in sw[0, :12]],
                           "seer_lanes_head": [hex(int(v)) for v in sl[0, :12]]}
    print(json.dumps({"kind": kind, "G": G, "lanes": len(recs), "diverged": list(out.values())}))


if __name__ == "__main__":
    main()
