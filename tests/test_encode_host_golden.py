"""encode_game / encode_option restatements (host build of the engine
headers) against the reference's own encodings (tests/golden/encode.json.gz)."""
import numpy as np

from citadels_self_play_amd import canon
from conftest import load_golden
from hostcheck import HostBatch, encode_games, encode_options


def test_encode_game_and_options_host():
    recs = load_golden("encode.json.gz")
    by_game = {}
    for r in recs:
        by_game.setdefault((r["preset"], r["seed"]), []).append(r)
    for (preset, seed), rs in by_game.items():
        hb = HostBatch([seed], preset)
        want = {r["step"]: r for r in rs}
        step = 0
        while True:
            opts, n = hb.get_options(8192)
            g = hb.game(0)
            if step in want:
                r = want[step]
                assert canon.hash_obj(canon.canon_game(g)) == r["state"], (seed, step)
                assert encode_games(hb)[0].astype(int).tolist() == r["encode"], (preset, seed, step)
                for pid in range(6):
                    assert encode_games(hb, pid)[0].astype(int).tolist() == r["encode_pid"][pid], (seed, step, pid)
                k = len(r["options"])
                enc = encode_options(hb.games[0], opts[0, :k])
                for j, (cs, vec) in enumerate(r["options"]):
                    assert canon.canon_option(__import__("citadels_self_play_amd.layout", fromlist=["x"]).opt_from_bytes(opts[0, j]), g) == cs
                    assert enc[j].astype(int).tolist() == vec, (seed, step, cs)
            if g.terminal:
                break
            k = hb.randbelow(0, int(n[0]))
            hb.carry_out(opts[:, k])
            step += 1
            if hb.game(0).terminal:
                break
