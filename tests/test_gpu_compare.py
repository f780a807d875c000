"""compare_to_random on a real MI355X (citadels_self_play_amd.compare_to_random
.play_games: cit_advance_policy + sub-batch cfr_pred / cfr_decide) against the
reference's games (tests/golden/compare.json.gz, searches of 30 / 60)."""
import numpy as np
import pytest

from citadels_self_play_amd import canon, models
from conftest import load_golden
from test_mlp_host import load_variant

pytestmark = pytest.mark.gpu


def test_gpu_compare_matches_reference():
    from citadels_self_play_amd.compare_to_random import play_games
    gold = load_golden("compare.json.gz")
    m = load_variant(dict(np.load("tests/golden/mlp.npz")), "bn")
    net = models.ValueNet(m, "cuda")
    recs = gold["games"]
    winners, steps, decisions, b = play_games([r["seed"] for r in recs] + [r["seed"] for r in recs], net,
                                              gold["pred_iters"], gold["train_iters"])
    for l, r in enumerate(recs + recs):
        assert int(winners[l]) == r["winner"], r["seed"]
        assert int(steps[l]) + int(decisions[l]) == r["steps"], r["seed"]
        assert int(decisions[l]) == len(r["decisions"]), r["seed"]
        assert canon.hash_obj(b.canon(l)) == r["final"], r["seed"]
