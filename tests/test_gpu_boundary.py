"""The search's single-game pieces exported through the C ABI (SURVEY.md
§8(b)): cit_count_options (len(get_options_from_state())),
cit_determinize (Game.sample_private_information) and
cit_skip_false_choice (CFRNode.skip_false_choice), each against the oracle
on seeded positions, and the stream positions they leave behind."""
import numpy as np
import pytest
import torch

import cfr_oracle as CO
import citadels_oracle as O
from citadels_self_play_amd import canon
from citadels_self_play_amd import layout as L

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU")
    from citadels_self_play_amd.engine import GameBatch
    return GameBatch


def _positions(engine, seeds, preset=True):
    """config-3 positions: create_game() + randint(0, 300) random steps."""
    b = engine(seeds, preset=preset)
    b.advance_random(0, 300)
    return b


def _oracle_position(seed, preset=True):
    g = O.new_game(seed, preset)
    k = g.rng.randint(0, 300)
    for _ in range(k):
        opts = g.get_options()
        if g.carry_out(opts[g.rng._randbelow(len(opts))]) is not None:
            break
    return g


@pytest.mark.parametrize("preset", [True, False])
def test_gpu_count_options_matches_list(engine, preset):
    seeds = list(range(500, 564))
    a = _positions(engine, seeds, preset)
    b = _positions(engine, seeds, preset)
    n_count = a.count_options().cpu().numpy()
    _, n_list = b.get_options(8192)
    assert np.array_equal(n_count, n_list.cpu().numpy())
    # the same mutations and draws as get_options
    assert np.array_equal(a.rows(), b.rows())
    assert np.array_equal(a.mt_idx.cpu().numpy(), b.mt_idx.cpu().numpy())
    for l, s in enumerate(seeds[:16]):
        og = _oracle_position(s, preset)
        if og.terminal:
            continue
        assert n_count[l] == len(og.get_options()), s


@pytest.mark.parametrize("role_sample", [True, False])
def test_gpu_determinize_matches_oracle(engine, role_sample):
    seeds = list(range(600, 632))
    b = _positions(engine, seeds)
    pids = b.rows()[:, L.CitGame.gs_pid.offset].view(np.int8).astype(np.int32)
    b.determinize(pids, role_sample)
    rows = b.rows()
    assert int((b.errors() != 0).sum()) == 0
    for l, s in enumerate(seeds):
        og = _oracle_position(s)
        if og.terminal:
            continue
        CO.sample_private_information(og, og.players[og.gs.pid], role_sample)
        assert canon.canon_game(L.game_from_bytes(rows[l])) == O.canon(og), s


def test_gpu_skip_false_choice_matches_oracle(engine):
    seeds = list(range(700, 764))
    b = _positions(engine, seeds)
    carried = b.skip_false_choice().cpu().numpy()
    rows = b.rows()
    for l, s in enumerate(seeds):
        og = _oracle_position(s)
        tr = CO.Tree.__new__(CO.Tree)        # only the root Node's skip_forced, no search
        tr.carry_outs, tr.count = 0, 0
        node = CO.Node.__new__(CO.Node)
        node.tree, node.game = tr, og
        node.skip_forced()
        assert carried[l] == tr.carry_outs, s
        assert canon.canon_game(L.game_from_bytes(rows[l])) == O.canon(og), s
    assert (carried > 0).any()
