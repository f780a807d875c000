"""The oracle's featurizers (oracle/mlp_oracle.py encode_game / encode_option)
against the reference's own encodings (tests/golden/encode.json.gz), replaying
each recorded trajectory in the oracle."""
import citadels_oracle as O
import mlp_oracle as M
from conftest import load_golden


def test_oracle_encoders_match_reference():
    recs = load_golden("encode.json.gz")
    by_game = {}
    for r in recs:
        by_game.setdefault((r["preset"], r["seed"]), {})[r["step"]] = r
    n_opt = 0
    for (preset, seed), want in by_game.items():
        g = O.new_game(seed, preset)
        step = 0
        while step <= max(want):
            opts = g.get_options()
            if step in want:
                r = want[step]
                assert M.encode_game(g).astype(int).tolist() == r["encode"], (seed, step)
                for pid in (0, 5):
                    assert M.encode_game(g, pid).astype(int).tolist() == r["encode_pid"][pid]
                for o, (cs, vec) in zip(opts, r["options"]):
                    assert o.canon() == cs, (seed, step)
                    assert M.encode_option(o).astype(int).tolist() == vec, (seed, step, cs)
                    n_opt += 1
            if g.carry_out(opts[g.rng._randbelow(len(opts))]) is not None:
                break
            step += 1
    assert n_opt > 1000
