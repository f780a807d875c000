"""HIP engine parity on a real MI355X, through the C ABI (libcitadels_hip.so).

Checks, in order of strength:
  * RNG: the device MT19937 streams equal CPython's / numpy's (golden streams);
  * every golden trajectory step by step through the per-step ABI
    (cit_get_options -> cit_random_choice -> cit_carry_out): option-list
    digest, chosen index, post-state digest, full states — bit-exact;
  * the fused rollout kernels reproduce the golden final states -- the
    benchmarked one-game-per-workgroup kernel k_rollout_u
    (games_per_block=0) and the one-game-per-lane kernel (cit_lanes.hip);
  * fresh seeds against the CPU oracle;
  * size-independent properties at the benchmark size (B = 4096, k_rollout_u):
    determinism, chunked == fused, k_rollout_u == the lanes kernel, lanes vs
    the oracle;
  * random-role games at B = 1024 through k_rollout_u, whose option lists
    exceed its 64-entry LDS buffer (the cit_pick_option path), every lane vs
    the oracle.
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
    for gpb in (0, 1, 16, 64):     # 0 = k_rollout_u, the benchmarked kernel
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
    """B = 4096 (the benchmark configuration) through k_rollout_u
    (games_per_block=0, the kernel bench.py times): no lane errors, every game
    ends, fused == chunked stepping (k_rollout_u and the lanes kernel) == the
    one-game-per-lane kernel at two shapes, and 256 lanes equal the oracle."""
    import citadels_oracle as O
    B = 4096
    seeds = np.arange(7_000_000, 7_000_000 + B)
    a = engine(seeds, preset=True)
    steps_a, w_a = a.rollout(games_per_block=0)
    torch.cuda.synchronize()
    assert int((a.errors() != 0).sum()) == 0
    assert bool(a.terminal().all())
    sa = steps_a.cpu().numpy()
    wa = w_a.cpu().numpy()
    assert sa.min() > 100 and sa.max() < 2000
    rows_a = a.rows()
    for chunk_gpb in (0, 64):
        b = engine(seeds, preset=True)
        while True:
            b.rollout(max_steps=37, games_per_block=chunk_gpb)
            if bool(b.terminal().all()) or int((b.errors() != 0).sum()):
                break
        assert np.array_equal(b.rows(), rows_a), chunk_gpb
        assert np.array_equal(b.steps.cpu().numpy(), sa), chunk_gpb
    for gpb in (4, 16):
        c = engine(seeds, preset=True)
        sc, wc = c.rollout(games_per_block=gpb)
        assert np.array_equal(c.rows(), rows_a), gpb
        assert np.array_equal(sc.cpu().numpy(), sa) and np.array_equal(wc.cpu().numpy(), wa), gpb
    rng = np.random.default_rng(0)
    for l in rng.choice(B, 256, replace=False):
        og, n = O.random_rollout(int(seeds[l]), True)
        assert sa[l] == n, l
        assert wa[l] == og.winner, l
        assert canon.canon_game(L.game_from_bytes(rows_a[l])) == O.canon(og), l


def test_gpu_rollout_streams_overlap(engine):
    """bench.py --streams: 8 batches of 4096 games launched round-robin on 4
    HIP streams (k_rollout_u launches overlapping) give the same rows, steps
    and winners as each batch rolled out alone on one stream."""
    B, K, S = 4096, 8, 4
    seeds = [np.arange(8_000_000 + k * B, 8_000_000 + (k + 1) * B) for k in range(K)]
    alone = []
    for s in seeds:
        a = engine(s, preset=True)
        st, w = a.rollout(games_per_block=0)
        torch.cuda.synchronize()
        alone.append((a.rows(), st.cpu().numpy().copy(), w.cpu().numpy().copy()))
    batches = [engine(s, preset=True) for s in seeds]
    streams = [torch.cuda.Stream() for _ in range(S)]
    torch.cuda.synchronize()
    for k, gb in enumerate(batches):
        with torch.cuda.stream(streams[k % S]):
            gb.rollout(games_per_block=0)
    torch.cuda.synchronize()
    for k, gb in enumerate(batches):
        assert int((gb.errors() != 0).sum()) == 0, k
        assert np.array_equal(gb.rows(), alone[k][0]), k
        assert np.array_equal(gb.steps.cpu().numpy(), alone[k][1]), k
        assert np.array_equal(gb.winner.cpu().numpy(), alone[k][2]), k


def test_gpu_continuous_loop_with_init(engine):
    """bench.py's e2e loop: K batches re-initialised (cit_init = the LDS-free
    k_mt_seed_cpython + k_init) and rolled out, init + rollout of batch k on
    stream k % 3, so inits run beside earlier batches' rollouts.  Every batch
    equals the same batch initialised and rolled out alone (rows, steps,
    winners, both stream words and positions), and a batch seeded by the
    one-game-per-lane restatement of random.seed (cit_mt_seed, cit_core.h's
    mt_seed_cpython) and dealt by k_init from that stream equals cit_init's."""
    from citadels_self_play_amd import _lib
    lib = _lib.load()
    B, K, S = 4096, 6, 3
    seeds = [np.arange(11_000_000 + k * B, 11_000_000 + (k + 1) * B) for k in range(K)]
    alone = []
    for s in seeds:
        a = engine(s, preset=True)
        init_rows, init_mt = a.rows(), a.mt.cpu().numpy().copy()
        st, w = a.rollout(games_per_block=0)
        torch.cuda.synchronize()
        alone.append((init_rows, init_mt, a.rows(), st.cpu().numpy().copy(), w.cpu().numpy().copy(),
                      a.mt.cpu().numpy().copy(), a.mt_idx.cpu().numpy().copy()))
    # the seeding restated one game per lane, then the deal from that stream
    b = engine(seeds[0], preset=True)
    sd = torch.as_tensor(seeds[0], dtype=torch.int64, device="cuda")
    b.games.zero_()
    _lib.check(lib.cit_mt_seed(b.mt.data_ptr(), b.mt_idx.data_ptr(), B, sd.data_ptr(), 0, _stream()), "seed")
    _lib.check(lib.cit_init(b.games.data_ptr(), b.mt.data_ptr(), b.mt_idx.data_ptr(), B, None, 1, _stream()), "init")
    torch.cuda.synchronize()
    assert np.array_equal(b.rows(), alone[0][0])
    batches = [engine(s, preset=True) for s in seeds]
    for gb in batches:                                  # played-out games, as in the bench before e2e
        gb.rollout(games_per_block=0)
    streams = [torch.cuda.Stream() for _ in range(S)]
    torch.cuda.synchronize()
    for k, gb in enumerate(batches):
        with torch.cuda.stream(streams[k % S]):
            gb.reset()
            gb.rollout(games_per_block=0)
    torch.cuda.synchronize()
    for k, gb in enumerate(batches):
        _, _, rows, st, w, mt, idx = alone[k]
        assert int((gb.errors() != 0).sum()) == 0, k
        assert np.array_equal(gb.rows(), rows), k
        assert np.array_equal(gb.steps.cpu().numpy(), st), k
        assert np.array_equal(gb.winner.cpu().numpy(), w), k
        assert np.array_equal(gb.mt.cpu().numpy(), mt) and np.array_equal(gb.mt_idx.cpu().numpy(), idx), k


def test_gpu_rollout_u_option_overflow(engine):
    """Random-role games (thousands of options per step for the cardinal /
    magician) through k_rollout_u at B = 1024: a draw k >= 64 misses the LDS
    option buffer and takes cit_pick_option (re-enumeration to the k-th
    option).  Every lane equals the oracle and the lanes kernel; the test
    asserts the overflow path was actually taken many times."""
    import citadels_oracle as O
    B = 1024
    seeds = np.arange(9_100_000, 9_100_000 + B)
    a = engine(seeds, preset=False)
    steps_a, w_a = a.rollout(games_per_block=0)
    sa, wa = steps_a.cpu().numpy(), w_a.cpu().numpy()
    assert int((a.errors() != 0).sum()) == 0
    assert bool(a.terminal().all())
    rows_a = a.rows()
    c = engine(seeds, preset=False)
    sc, wc = c.rollout(games_per_block=8)
    rows_c = c.rows()
    bad = np.nonzero((rows_c != rows_a).any(axis=1))[0]
    assert len(bad) == 0, [(int(l), np.nonzero(rows_c[l] != rows_a[l])[0][:12].tolist(),
                            canon.canon_game(L.game_from_bytes(rows_c[l])) == canon.canon_game(L.game_from_bytes(rows_a[l])))
                           for l in bad[:6]]
    assert np.array_equal(sc.cpu().numpy(), sa) and np.array_equal(wc.cpu().numpy(), wa)
    big_draws = 0
    for l, s in enumerate(seeds):
        trace = []
        og, n = O.random_rollout(int(s), False, trace=trace)
        big_draws += sum(1 for t in trace if t[3] >= 64)
        assert sa[l] == n, l
        assert wa[l] == og.winner, l
        assert canon.canon_game(L.game_from_bytes(rows_a[l])) == O.canon(og), l
    assert big_draws >= 50, big_draws


@pytest.mark.parametrize("preset", [True, False])
def test_gpu_fingerprint_matches_reference(engine, preset):
    """SURVEY §6 fingerprint of the reference's own random-policy games
    (tests/golden/fingerprint.json.gz, tools/gen_golden.py): seeds 0..399 preset /
    0..199 random-role through k_rollout_u -- seat win counts, total steps and
    total winner points exact."""
    from conftest import load_golden
    fp = [f for f in load_golden("fingerprint.json.gz") if f["preset"] == preset][0]
    b = engine(list(range(fp["games"])), preset=preset)
    steps, w = b.rollout(games_per_block=0)
    steps, w = steps.cpu().numpy(), w.cpu().numpy()
    assert int((b.errors() != 0).sum()) == fp["errors"] == 0
    assert np.bincount(w, minlength=6).tolist() == fp["wins"]
    assert int(steps.sum()) == fp["steps"]
    off = L.CitGame.points.offset
    pts = b.rows()[:, off:off + 12].copy().view(np.int16).reshape(-1, 6)
    assert int(pts.max(axis=1).sum()) == fp["winner_points"]


def test_gpu_rollout_queue_matches_rollout():
    """cit_rollout_queue (a work queue of one-wave slots) plays every game
    exactly as cit_rollout_random (one workgroup per game): steps, winners,
    final rows and streams, bit for bit, on 12,288 games (more than the
    8,192 slots, so slots take second games)."""
    from citadels_self_play_amd.engine import GameBatch
    seeds = np.arange(1_500_000_000, 1_500_000_000 + 12288)
    a = GameBatch(seeds, preset=True)
    b = GameBatch(seeds, preset=True)
    a.rollout()
    b.rollout_queue()
    torch.cuda.synchronize()
    for x, y in ((a.steps, b.steps), (a.winner, b.winner), (a.games, b.games), (a.mt, b.mt), (a.mt_idx, b.mt_idx)):
        assert torch.equal(x, y)
    assert int((a.errors() != 0).sum()) == 0 and bool(a.terminal().all())
