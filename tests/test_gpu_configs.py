"""The reference's own full-size settings on MI355X.

* Config 5 at cfr_train(200000) per tree (train_from_scratch.py:39,45,58):
  64 simulate_game trees (seeds 30000000..30000063) through
  selfplay.simulate_games' default product path -- the tree queue with
  QUEUE_OVERCOMMIT, ARENA_FRAC and 200k-sized block tables, the slice planner
  pausing trees -- forced by a pool budget that holds 32 trees at ARENA_FRAC
  (the default budget on a 288 GB card holds all 64 at once).  The lanes with
  a reference golden (tests/golden/targets200000.json.gz, generated from the
  reference by tools/gen_golden_targets.py) must match it: node and carry_out
  counts, the live decision, both streams' end states and every target; the
  golden error seeds must end in the reference's ValueError (CIT_ERR_VALUE)
  after the reference's carry_out count, with no targets.
* train_from_scratch's --on-error policy on the error seed 30000012.
* Config 4 at full size: cfr_pred(200, 10) with the value net over 512 and
  4,096 positions per GPU (BASELINE configs[3]: 4096 positions over 8 GPUs):
  deterministic across runs and across time-sliced search launches
  (cit_cfr_pred_slice), a strided sub-batch equals the full batch, and the
  cfr_pred200 golden lanes embedded in the big batch still equal the
  reference."""
import numpy as np
import pytest
import torch

from citadels_self_play_amd import canon
from citadels_self_play_amd import layout as L
from conftest import load_golden
from test_cfr_host_golden import hash_obj
from test_targets_oracle_golden import check_targets

pytestmark = pytest.mark.gpu

CIT_ERR_VALUE = 0x8
CFG5_SEED0, CFG5_TREES, CFG5_ITERS = 30_000_000, 64, 200_000


def _split(t, n):
    t = {k: v.cpu().numpy() for k, v in t.items() if k in ("meta", "feat", "value", "dist", "opt_feat")}
    per = [[] for _ in range(n)]
    for k, (lane, node, pid, nch, c0) in enumerate(t["meta"]):
        per[lane].append((t["feat"][k], t["opt_feat"][c0:c0 + nch], t["value"][k], t["dist"][c0:c0 + nch]))
    return per


@pytest.mark.timeout(900)
@pytest.mark.parametrize("rounds", [1, 2], ids=["one_round", "cross_round_queue"])
def test_gpu_config5_200k_queue_golden(rounds):
    """rounds = 2: the 64 trees as two data rounds of 32 through one
    selfplay.TreeQueue (train_from_scratch.collect's cross-round queue: the
    second round's trees enter the slots the first round's tail frees), each
    round's result checked as simulate_games' would be."""
    from citadels_self_play_amd import selfplay
    from citadels_self_play_amd.engine import pool_bytes, pool_caps
    recs = {r["seed"]: r for r in load_golden("targets200000.json.gz")}
    seeds = np.arange(CFG5_SEED0, CFG5_SEED0 + CFG5_TREES)
    assert set(recs) <= set(seeds.tolist())
    nc, ec = pool_caps(CFG5_ITERS)
    msgs = []
    def log(m):                       # progress on stdout (a long test must not look hung)
        msgs.append(m)
        print(m, flush=True)
    tag = "overcommit %.2f" % selfplay.QUEUE_OVERCOMMIT
    if rounds == 1:
        budget = pool_bytes(32, nc, ec, selfplay.ARENA_FRAC)       # 32 trees at ARENA_FRAC, overcommitted slots
        b, stats, t = selfplay.simulate_games(seeds, CFG5_ITERS, max_pool_bytes=budget, log=log)
        assert selfplay.QUEUE_OVERCOMMIT > 1 and any(tag in m for m in msgs), msgs[-3:]    # the queue ran, overcommitted
        _check_cfg5(recs, seeds, b, stats, t)
        return
    half = len(seeds) // 2
    budget = pool_bytes(32, nc, ec, selfplay.ARENA_FRAC)       # a round's 32 trees at ARENA_FRAC
    q = selfplay.TreeQueue(CFG5_ITERS, half, max_pool_bytes=budget, log=log)
    q.add(seeds[:half])
    q.add(seeds[half:])
    assert q.S == half and q.planner is not None                # both rounds share the slots and arena
    for r in range(2):
        q.run(r)
        b, stats, t = q.result(r)
        _check_cfg5(recs, seeds[r * half:(r + 1) * half], b, stats, t)
    q.close()
    assert any("32 of 32 + " in m for m in msgs), msgs[-3:]        # round 1's trees ran beside round 0's tail


def _check_cfg5(recs, seeds, b, stats, t):
    stats_np, chosen = stats.cpu().numpy(), t["chosen"].cpu().numpy()
    per = _split(t, len(seeds))
    counts = t["counts"].cpu().numpy()
    rows = b.rows()
    mt, idx = b.mt.cpu().numpy().view(np.uint32), b.mt_idx.cpu().numpy()
    npmt, npidx = b.np_mt.cpu().numpy().view(np.uint32), b.np_idx.cpu().numpy()
    assert not bool(t["overflow"].any())
    n_err = 0
    for l, s in enumerate(seeds.tolist()):
        root, n_nodes, n_edges, carry, err = stats_np[l]
        if err:
            n_err += 1
            assert counts[l].tolist() == [0, 0] and not per[l], s           # an error tree yields no targets
        r = recs.get(s)
        if r is None:
            continue
        if r.get("error"):
            assert r["error"] == "ValueError", s
            assert err & CIT_ERR_VALUE, (s, err)
            assert carry == r["carry_outs"], (s, carry, r["carry_outs"])
            continue
        assert err == 0, (s, err)
        assert n_nodes == r["nodes"] and carry == r["carry_outs"], (s, n_nodes, carry)
        g = L.game_from_bytes(rows[l])
        assert canon.canon_option(L.opt_from_bytes(chosen[l]), g) == r["chosen"], s
        assert hash_obj(mt[:, l].tolist() + [int(idx[l])]) == r["rng_after"][0], s
        assert hash_obj(npmt[:, l].tolist()) == r["rng_after"][1] and int(npidx[l]) == r["rng_after"][2], s
        check_targets(per[l], r["targets"], s)
    assert n_err >= sum(1 for r in recs.values() if r.get("error") and r["seed"] in set(seeds.tolist()))


def test_gpu_train_from_scratch_on_error(tmp_path):
    """Seed 30000012 raises the reference's ValueError after one carry_out
    (np.random.choice over an empty list) at any iteration count.  Its round
    (seeds 30000000..30000015): --on-error raise stops the run with a
    ValueError as the reference's get_mccfr_targets does; drop counts the tree
    and goes on."""
    from citadels_self_play_amd import selfplay
    from citadels_self_play_amd import train_from_scratch as T
    _, st, t = selfplay.simulate_games([30_000_012], 300)
    err, carry = int(st[0, 4]), int(st[0, 3])
    assert err & CIT_ERR_VALUE and carry == 1 and int(t["counts"].sum()) == 0
    args = ["--iters", "300", "--games-per-gpu", "16", "--pretrain-targets", "1", "--phases", "0", "--epochs", "1",
            "--seed", str(CFG5_SEED0), "--out", str(tmp_path), "--val", str(tmp_path / "none.pkl")]
    with pytest.raises(ValueError, match="simulate_game raised"):
        T.main(args + ["--on-error", "raise"])
    T.main(args + ["--on-error", "drop"])
    assert T.collect.dropped["value_error"] >= 1 and T.collect.dropped["capacity"] == 0


@pytest.mark.timeout(300)
def test_gpu_collect_lookahead_equals_round_by_round():
    """collect's cross-round queue (up to LOOKAHEAD_DEPTH rounds beyond the
    one it waits for) pools exactly the targets of its rounds searched one
    after another by simulate_games."""
    from types import SimpleNamespace
    from citadels_self_play_amd import train_from_scratch as T
    base = dict(iters=300, games_per_gpu=16, node_cap=None, seed=CFG5_SEED0, on_error="drop", save_tuples=False)
    out = {}
    for la in (False, True):
        f, v, _ = T.collect(0, 1, SimpleNamespace(lookahead=la, **base), 0, 10 ** 15, lambda m: None, max_rounds=4)
        out[la] = (f.numpy(), v.numpy(), dict(T.collect.dropped), T.collect.queue)
    assert out[False][0].shape[0] > 0
    assert np.array_equal(out[False][0], out[True][0]) and np.array_equal(out[False][1], out[True][1])
    assert out[False][2] == out[True][2]
    assert out[True][3]["speculated_rounds"] == 3              # rounds 1-3 entered the queue ahead of collect


@pytest.fixture(scope="module")
def net():
    from citadels_self_play_amd import models
    from test_mlp_host import load_variant
    g = dict(np.load("tests/golden/mlp.npz"))
    return models.ValueNet(load_variant(g, "bn"), "cuda")


@pytest.mark.parametrize("n", [512, 4096])
def test_gpu_config4_full_size(net, n):
    from citadels_self_play_amd import selfplay
    recs = [r for r in load_golden("cfr_pred200.json.gz") if not r.get("skip")]
    seeds = np.arange(8_000_000, 8_000_000 + n, dtype=np.int64)
    where = np.linspace(0, n - 1, len(recs)).astype(np.int64)        # golden lanes spread over the batch
    seeds[where] = [r["seed"] for r in recs]
    from citadels_self_play_amd import engine
    runs = []
    keep = engine.PRED_SLICE_TICKS
    try:
        # in-kernel leaves (one launch, the default); whole leaf rounds, then
        # 30 us time slices (cit_cfr_pred_slice: many more search launches);
        # then a strided sub-batch with in-kernel leaves
        for sel, ticks, fused in ((slice(None), 0, True), (slice(None), 0, False), (slice(None), 3000, False),
                                  (slice(3, None, 37), 0, True)):
            engine.PRED_SLICE_TICKS = ticks
            b, chosen, stats, rounds = selfplay.decide(seeds[sel], 200, net=net, fused=fused)
            torch.cuda.synchronize()
            runs.append((chosen.cpu().numpy(), stats.cpu().numpy(), b.rows(), b.np_mt.cpu().numpy(),
                         b.mt.cpu().numpy(), rounds, b))
    finally:
        engine.PRED_SLICE_TICKS = keep
    (c0, s0, r0, n0, m0, k0, b0), (c1, s1, r1, n1, m1, k1, _), (c3, s3, r3, n3, m3, k3, _), \
        (c2, s2, r2, n2, m2, _, _) = runs
    assert k0 == 0 and k1 > 10 and k3 >= k1
    for x, y, z in ((c0, c1, c3), (s0, s1, s3), (r0, r1, r3), (n0, n1, n3), (m0, m1, m3)):
        assert np.array_equal(x, y) and np.array_equal(x, z)        # mode-, slice-invariant
    for x, y in ((c0[3::37], c2), (s0[3::37, 1:], s2[:, 1:]), (r0[3::37], r2), (n0[:, 3::37], n2), (m0[:, 3::37], m2)):
        assert np.array_equal(x, y)                                  # sub-batch invariant
    assert (s0[:, 4] == 0).mean() > 0.8
    for l, r in zip(where.tolist(), recs):
        root, n_nodes, n_edges, carry, err = s0[l]
        assert err == 0, r["seed"]
        assert n_nodes == r["nodes"] and carry == r["carry_outs"], r["seed"]
        g = L.game_from_bytes(r0[l])
        assert canon.canon_game(g) == r["root_game"], r["seed"]
        assert canon.canon_option(L.opt_from_bytes(c0[l]), g) == r["chosen"], r["seed"]
        nodes, edges, _ = b0.tree(l)
        np.testing.assert_allclose(nodes[root]["nv"], r["root"]["node_value"], rtol=0, atol=2e-6)


def test_gpu_pred_ahead_invariant(net):
    """cfr_pred's batched rounds (engine.PRED_AHEAD launches enqueued per host
    poll) search exactly as a host check after every launch (PRED_AHEAD = 1):
    decisions, stats, rows, leaf rounds and both streams are identical for 1,
    4 (the default) and 8 rounds per poll."""
    from citadels_self_play_amd import engine, selfplay
    seeds = np.arange(8_100_000, 8_100_512, dtype=np.int64)
    keep = engine.PRED_AHEAD
    runs = []
    try:
        for ahead in (1, 4, 8):
            engine.PRED_AHEAD = ahead
            b, chosen, stats, rounds = selfplay.decide(seeds, 200, net=net, fused=False)
            torch.cuda.synchronize()
            runs.append((chosen.cpu().numpy(), stats.cpu().numpy(), b.rows(), b.np_mt.cpu().numpy(),
                         b.np_idx.cpu().numpy(), b.mt.cpu().numpy(), b.mt_idx.cpu().numpy(), rounds))
    finally:
        engine.PRED_AHEAD = keep
    assert runs[0][7] > 10
    for other in runs[1:]:
        for x, y in zip(runs[0][:7], other[:7]):
            assert np.array_equal(x, y)
        assert other[7] == runs[0][7]
