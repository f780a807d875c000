"""compare_to_random.play_games (seat 0: run_mccfr with the value net, seat 1:
run_mccfr without, others random) against the reference's own games
(tests/golden/compare.json.gz; searches shrunk to 30 / 60 iterations):
the oracle with the reference's fp32 torch MLP bit for bit, and the host
build of the engine (cit_advance_policy + the device search code) driven by
the fmaf-chain MLP (the device MFMA arithmetic) - same decisions, winner and
final state."""
import numpy as np
import pytest
import torch

import cfr_oracle as CO
import citadels_oracle as O
import mlp_oracle as M
from citadels_self_play_amd import canon, models
from citadels_self_play_amd import layout as L
from conftest import load_golden
from hostcheck import compare_game
from test_mlp_host import load_variant


@pytest.fixture(scope="module")
def setup():
    g = load_golden("compare.json.gz")
    m = load_variant(dict(np.load("tests/golden/mlp.npz")), "bn")
    return g, m, M.FmaMLP(models.fold(m))


@pytest.mark.slow
def test_oracle_compare_matches_reference(setup):
    gold, m, _ = setup

    def torch_model(game):
        with torch.no_grad():
            x = torch.from_numpy(M.encode_game(game))[None]
            return models.square_and_normalize(m(x), dim=1)[0].numpy()

    for r in gold["games"][:1]:
        g, steps, dec = CO.compare_game(r["seed"], torch_model, gold["pred_iters"], gold["train_iters"])
        assert steps == r["steps"] and g.winner == r["winner"], r["seed"]
        assert dec == r["decisions"], r["seed"]
        assert canon.hash_obj(O.canon(g)) == r["final"], r["seed"]


def test_host_compare_matches_reference(setup):
    gold, m, fma = setup
    for r in gold["games"]:
        hb, steps, dec = compare_game(r["seed"], fma, gold["pred_iters"], gold["train_iters"])
        g = hb.game(0)
        got = [[seat, 0, canon.canon_option(L.opt_from_bytes(o), gb)] for seat, o, gb in dec]
        assert [d[::2] for d in got] == [[d[0], d[2]] for d in r["decisions"]], r["seed"]
        assert steps + len(dec) == r["steps"] and g.winner == r["winner"], r["seed"]
        assert canon.hash_obj(canon.canon_game(g)) == r["final"], r["seed"]
