"""HIP engine parity on a real MI355X, through the C ABI (libcitadels_hip.so).

Checks, in order of strength:
  * RNG: the device MT19937 streams equal CPython's / numpy's (golden streams);
  * every golden trajectory step by step through the per-step ABI
    (cit_get_options -> cit_random_choice -> cit_carry_out): option-list
    digest, chosen index, post-state digest, full states — bit-exact;
  * the fused rollout kernel reproduces the golden final states;
  * fresh seeds against the CPU oracle;
  * size-independent properties at the benchmark size (B = 4096):
    determinism, chunked == fused, independence of the workgroup shape.
"""
import numpy as np
import pytest
import torch

from citadels_self_play_amd import canon
from citadels_self_play_amd import layout as L

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU")
    from citadels_self_play_amd.engine import GameBatch
    return GameBatch


def _stream():
    return torch.cuda.current_stream().cuda_stream


def test_gpu_mt_streams(engine, golden_rng):
    from citadels_self_play_amd import _lib
    lib = _lib.load()
    for numpy_style, recs in ((0, golden_rng["cpython"]), (1, golden_rng["numpy"])):
        seeds = torch.tensor([r["seed"] for r in recs], dtype=torch.int64, device="cuda")
        B = len(recs)
        mt = torch.zeros((L.MT_N, B), dtype=torch.int32, device="cuda")
        idx = torch.zeros(B, dtype=torch.int32, device="cuda")
        _lib.check(lib.cit_mt_seed(mt.data_ptr(), idx.data_ptr(), B, seeds.data_ptr(), numpy_style, _stream()), "seed")
        key = "state0" if numpy_style == 0 else "key0"
        got = mt.cpu().numpy().view(np.uint32)
        for l, r in enumerate(recs):
            assert got[:, l].tolist() == r[key][:624]
        if numpy_style == 0:
            n = 1500
            out = torch.zeros((B, n), dtype=torch.int32, device="cuda")
            _lib.check(lib.cit_mt_draw(mt.data_ptr(), idx.data_ptr(), B, n, out.data_ptr(), _stream()), "draw")
            o = out.cpu().numpy().view(np.uint32)
            for l, r in enumerate(recs):
                assert o[l].tolist() == r["getrandbits32"]


def _stepwise(engine, recs, preset, max_opts):
    b = engine([r["seed"] for r in recs], preset=preset)
    rows = b.rows()
    for l, r in enumerate(recs):
        assert canon.canon_game(L.game_from_bytes(rows[l])) == r["states"]["0"], l
    nmax = max(len(r["steps"]) for r in recs)
    for i in range(nmax):
        opts, n = b.get_options(max_opts)
        rows_pre = b.rows()
        opts_h = opts.cpu().numpy()
        n_h = n.cpu().numpy()
        chosen, k = b.random_choice(opts, n)
        b.carry_out(chosen)
        rows = b.rows()
        k_h = k.cpu().numpy()
        for l, r in enumerate(recs):
            if i >= len(r["steps"]):
                continue
            st, pid, cnt, oh, idx, ph = r["steps"][i]
            g = L.game_from_bytes(rows_pre[l])
            assert g.err == 0, (l, i, g.err)
            assert (g.gs_state, g.gs_pid) == (st, pid), (l, i)
            assert n_h[l] == cnt, (l, i)
            descs = [L.opt_from_bytes(opts_h[l, j]) for j in range(min(cnt, max_opts))]
            assert cnt <= max_opts
            if str(i) in r["options"]:
                assert [canon.canon_option(o, g) for o in descs] == r["options"][str(i)], (l, i)
            assert canon.hash_options(descs, g) == oh, (l, i)
            assert k_h[l] == idx, (l, i)
            post = canon.canon_game(L.game_from_bytes(rows[l]))
            if str(i + 1) in r["states"]:
                assert post == r["states"][str(i + 1)], (l, i)
            assert canon.hash_obj(post) == ph, (l, i)


def test_gpu_stepwise_preset(engine, golden_preset):
    _stepwise(engine, golden_preset, True, 64)


def test_gpu_stepwise_random_role(engine, golden_random):
    _stepwise(engine, golden_random, False, 8192)


@pytest.mark.parametrize("preset", [True, False])
def test_gpu_rollout_golden(engine, golden_preset, golden_random, preset):
    recs = golden_preset if preset else golden_random
    for gpb in (1, 16, 64):
        b = engine([r["seed"] for r in recs], preset=preset)
        steps, w = b.rollout(games_per_block=gpb)
        steps, w = steps.cpu().numpy(), w.cpu().numpy()
        rows = b.rows()
        for l, r in enumerate(recs):
            assert steps[l] == r["n_steps"], (gpb, l)
            assert w[l] == r["winner"], (gpb, l)
            assert canon.canon_game(L.game_from_bytes(rows[l])) == r["states"]["final"], (gpb, l)


def test_gpu_rollout_vs_oracle_fresh_seeds(engine):
    import citadels_oracle as O
    seeds = list(range(100000, 100192))
    for preset in (True, False):
        b = engine(seeds, preset=preset)
        steps, w = b.rollout()
        steps, w = steps.cpu().numpy(), w.cpu().numpy()
        rows = b.rows()
        for l, s in enumerate(seeds):
            og, n = O.random_rollout(s, preset)
            assert steps[l] == n, (preset, s)
            assert w[l] == og.winner, (preset, s)
            assert canon.canon_game(L.game_from_bytes(rows[l])) == O.canon(og), (preset, s)


def test_gpu_full_size_properties(engine):
    """B = 4096 (the benchmark configuration): no lane errors, every game ends,
    chunked stepping == fused rollout == other workgroup shapes, deterministic,
    and a sample of lanes equals the oracle."""
    import citadels_oracle as O
    B = 4096
    seeds = np.arange(7_000_000, 7_000_000 + B)
    a = engine(seeds, preset=True)
    steps_a, w_a = a.rollout(games_per_block=16)
    torch.cuda.synchronize()
    assert int((a.errors() != 0).sum()) == 0
    assert bool(a.terminal().all())
    sa = steps_a.cpu().numpy()
    assert sa.min() > 100 and sa.max() < 2000
    rows_a = a.rows()
    b = engine(seeds, preset=True)
    while True:
        b.rollout(max_steps=37, games_per_block=64)
        if bool(b.terminal().all()) or int((b.errors() != 0).sum()):
            break
    assert np.array_equal(b.rows(), rows_a)
    assert np.array_equal(b.steps.cpu().numpy(), sa)
    c = engine(seeds, preset=True)
    c.rollout(games_per_block=4)
    assert np.array_equal(c.rows(), rows_a)
    rng = np.random.default_rng(0)
    for l in rng.choice(B, 12, replace=False):
        og, n = O.random_rollout(int(seeds[l]), True)
        assert sa[l] == n
        assert canon.canon_game(L.game_from_bytes(rows_a[l])) == O.canon(og)
