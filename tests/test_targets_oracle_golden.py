"""Training-data path of train_from_scratch (simulate_game: create_a_random_game(100)
-> cfr_train(2000, training=True) -> get_all_targets) in the CPU oracle, against
the reference's own outputs (tests/golden/targets2000.json.gz, made by
tools/gen_golden_targets.py): positions, tree sizes, decisions, RNG end states
and every target tuple bit for bit (regret targets rtol 1e-12, np.exp)."""
import hashlib

import numpy as np
import pytest

import cfr_oracle as CO
import citadels_oracle as O
from conftest import load_golden
from test_cfr_host_golden import hash_obj

RTOL = 1e-12


def check_targets(got, want, tag):
    assert len(got) == len(want), tag
    for k, ((x, opts, nv, dist), w) in enumerate(zip(got, want)):
        assert np.asarray(x).astype(int).tolist() == w["encode"], (tag, k)
        o = np.ascontiguousarray(opts, np.float32).reshape(1, -1, 131)
        assert list(o.shape) == w["opts_shape"], (tag, k)
        assert hashlib.sha256(o.tobytes()).hexdigest()[:32] == w["opts_sha"], (tag, k)
        assert np.asarray(nv, np.float64).tolist() == w["nv"], (tag, k)
        np.testing.assert_allclose(dist, w["dist"], rtol=RTOL, atol=0, err_msg=str((tag, k)))


@pytest.mark.slow
def test_oracle_targets_match_reference():
    for r in load_golden("targets2000.json.gz"):
        pos, chosen, tr, targets = CO.simulate_game(r["seed"], r["iters"])
        assert O.canon(pos) == r["position"], r["seed"]
        assert tr.count == r["nodes"] and tr.carry_outs == r["carry_outs"], r["seed"]
        assert chosen.canon() == r["chosen"], r["seed"]
        g = tr.root.game
        assert hash_obj(list(g.rng.getstate()[1])) == r["rng_after"][0], r["seed"]
        st = g.nprng.get_state()
        assert hash_obj(st[1].tolist()) == r["rng_after"][1] and int(st[2]) == r["rng_after"][2]
        check_targets(targets, r["targets"], r["seed"])

