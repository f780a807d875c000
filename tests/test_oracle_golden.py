"""Pin the CPU oracle against the reference's own outputs (tests/golden, made by
tools/gen_golden.py from /root/reference): every step's option-list digest,
chosen index and post-state digest, plus the full canonical states."""
import hashlib
import json

import pytest

import citadels_oracle as O


def hash_obj(d):
    return hashlib.sha1(json.dumps(d, sort_keys=True, separators=(",", ":")).encode()).hexdigest()[:16]


def hash_opts(opts):
    return hashlib.sha1("\n".join(o.canon() for o in opts).encode()).hexdigest()[:16]


def replay(rec):
    g = O.new_game(rec["seed"], rec["preset"])
    assert O.canon(g) == rec["states"]["0"]
    for i, (st, pid, n, oh, idx, ph) in enumerate(rec["steps"]):
        assert (g.gs.state, g.gs.pid) == (st, pid), i
        opts = g.get_options()
        if str(i) in rec["options"]:
            assert [o.canon() for o in opts] == rec["options"][str(i)], i
        assert len(opts) == n, i
        assert hash_opts(opts) == oh, i
        k = g.rng._randbelow(len(opts))
        assert k == idx, i
        g.carry_out(opts[k])
        d = O.canon(g)
        if str(i + 1) in rec["states"]:
            assert d == rec["states"][str(i + 1)], i
        assert hash_obj(d) == ph, i
    assert O.canon(g) == rec["states"]["final"]
    assert g.winner == rec["winner"]


def test_oracle_preset_trajectories(golden_preset):
    for rec in golden_preset:
        replay(rec)


def test_oracle_random_role_trajectories(golden_random):
    for rec in golden_random:
        replay(rec)
