"""The reference-shaped object API (citadels_self_play_amd/api.py) on a real
MI355X: the random-policy step loop, run_mccfr, the training-target and
test-data harnesses written exactly as the reference's callers write them,
against the oracle and the reference's goldens."""
import numpy as np
import pytest
import torch

import citadels_oracle as O
from citadels_self_play_amd import api, canon
from citadels_self_play_amd import layout as L
from conftest import load_golden
from test_targets_oracle_golden import check_targets

pytestmark = pytest.mark.gpu


def _play_random(game, st, max_steps=10 ** 6):
    """compare_to_random.py:32-35 / run_utils.py:37-41: choice(options).carry_out(game)."""
    steps, winner = 0, None
    while not winner and steps < max_steps:
        options = game.get_options_from_state()
        winner = options[st.randint(0, len(options) - 1)].carry_out(game)
        steps += 1
    return steps, winner


def test_api_random_games_match_oracle():
    st = api.default_stream()
    for s, preset in [(0, True), (1, True), (7, True), (3, False), (11, False)]:
        st.seed(s)
        g = api.Game(preset=preset)
        steps, winner = _play_random(g, st)
        og, n = O.random_rollout(s, preset)
        assert steps == n and winner.id == og.winner, s
        assert canon.canon_game(g.packed()) == O.canon(og), s
        assert g.terminal and g.rewards[og.winner] == 1


def test_api_options_and_copies():
    st = api.default_stream()
    st.seed(5)
    g = api.create_game()
    opts = g.get_options_from_state()
    assert all(o.name == "role_pick" for o in opts) and len(opts) == 7
    assert opts[0] == api.Option(opts[0].desc, g.packed()) and opts[0] != opts[1]
    assert opts[0].encode_option().shape == (1, 131)
    x = g.encode_game()
    assert x.shape == (418,) and x.dtype == torch.float32
    h = __import__("copy").deepcopy(g)
    opts[0].carry_out(h)
    assert canon.canon_game(g.packed()) != canon.canon_game(h.packed())
    assert [p.id for p in g.players] == list(range(6)) and g.players[3].crown


def test_api_run_mccfr_matches_reference():
    st = api.default_stream()
    for r in load_golden("cfr_train200.json.gz")[:4]:
        if r.get("skip"):
            continue
        st.seed(r["seed"])
        g = api.create_game()
        k = st.randint(0, 300)
        for _ in range(k):
            options = g.get_options_from_state()
            if options[st.randint(0, len(options) - 1)].carry_out(g):
                break
        assert canon.canon_game(g.packed()) == r["position"], r["seed"]
        chosen, root = api.run_mccfr(g, max_iterations=r["iters"])
        assert root.node_count == r["nodes"] and root.carry_outs == r["carry_outs"], r["seed"]
        assert canon.canon_game(g.packed()) == r["root_game"], r["seed"]
        assert chosen.name == r["chosen"].split("|")[0]
        assert root.node_value.tolist() == r["root"]["node_value"]
        assert len(root.children) == r["root"]["n_children"]


def test_api_simulate_game_targets_match_reference():
    st = api.default_stream()
    for r in load_golden("targets2000.json.gz")[:3]:
        st.seed(r["seed"])
        game = api.create_a_random_game(100)
        assert canon.canon_game(game.packed()) == r["position"], r["seed"]
        _, root = api.run_mccfr(game, model=None, max_iterations=r["iters"], training=True)
        targets = root.get_all_targets(usefulness_treshold=200)
        got = [(x.numpy(), o.numpy()[0], v.numpy(), d.numpy()) for x, o, v, d in targets]
        check_targets(got, r["targets"], r["seed"])


def test_api_setup_game_matches_reference():
    st = api.default_stream()
    done = 0
    for r in load_golden("testdata500.json.gz"):
        if isinstance(r["result"], str):
            continue
        st.seed(r["seed"])
        game = api.create_game()
        almost = api.create_a_close_to_finished_game(game)
        assert canon.canon_game(almost.packed()) == r["position"], r["seed"]
        x = almost.encode_game()
        _, root = api.run_mccfr(game=almost, max_iterations=r["iters"])
        opts = api.encode_options_from_node(root)
        target = api.create_target_strategy(root)
        check_targets([(x.numpy(), opts.numpy()[0], root.node_value, target.numpy())], [r["result"]], r["seed"])
        done += 1
        if done == 4:
            break


@pytest.mark.parametrize("node_cap", [None, 64])
def test_api_cfrnode_constructor_skip_and_live_false_sampler(node_cap):
    """CFRNode(game) runs skip_false_choice on `game` in the constructor
    (deep_mccfr.py:19-20); after run_mccfr's search, action_choice(live=False)
    draws children with the in-search sampler from the tree's numpy stream
    (:67-91) -- both against the oracle's Tree / Node.choose.  node_cap=64
    forces every search to overflow its pool and be searched again (twice:
    64 -> 256 -> 1024 nodes), so the sampler must read the retry batch's
    tree (a node id past the overflowed tree would be an unallocated block)."""
    import cfr_oracle as CO
    st = api.default_stream()
    done = 0
    for seed in range(300, 340):
        pos = CO.config3_position(seed)
        if pos is None:
            continue
        og, npr = pos
        st.seed(seed)
        g = api.create_game()
        k = st.randint(0, 300)
        for _ in range(k):
            options = g.get_options_from_state()
            if options[st.randint(0, len(options) - 1)].carry_out(g):
                break
        assert canon.canon_game(g.packed()) == O.canon(og), seed
        node = api.CFRNode(g, g.gamestate.player_id, node_cap=node_cap)
        og.nprng = npr
        tr = CO.Tree(og, og.gs.pid, np_rng=npr)          # its root Node runs skip_forced on og
        assert canon.canon_game(g.packed()) == O.canon(og), seed
        node.cfr_train(max_iterations=200)
        tr.cfr_train(200)
        assert node.node_count == tr.count and node.carry_outs == tr.carry_outs, seed
        if node_cap is not None:
            assert node._b._retry is not None and node._b.lane_batch(0)[0] is not node._b, seed
        _, chosen = node.action_choice(live=True)
        _, ochosen = tr.root.choose(live=True)
        assert chosen.name == ochosen.name, seed
        for _ in range(3):
            child, opt = node.action_choice(live=False)
            ochild, oopt = tr.root.choose(live=False)
            assert opt.name == oopt.name, seed
            assert child.node_value.tolist() == np.asarray(ochild.nv, float).tolist(), seed
        done += 1
        if done == 6:
            break
    assert done == 6
