"""Featurizers, value MLP and model-driven MCCFR on a real MI355X through the
C ABI (cit_encode_games / cit_encode_options / cit_mlp_forward /
cit_mlp_forward_wave / cit_cfr_pred_step / cit_cfr_pred_fused).

* encode kernels == the host build of the same headers (itself pinned to the
  reference's encodings, test_encode_host_golden.py), bit for bit;
* the fp32-MFMA MLP and the single-row wave MLP == the fmaf-chain oracle
  (oracle/mlp_fma.c) bit for bit, and within PROB_RTOL/PROB_ATOL of the
  reference's own forward (mlp.npz);
* cfr_pred(200, 10) with the seeded value net, leaves in the search kernel
  and in leaf rounds: trees == the oracle driven by the fmaf-chain MLP bit for bit; node/carry_out counts, root game and
  decisions == the reference (cfr_pred200), root values within VALUE_ATOL."""
import numpy as np
import pytest
import torch

import cfr_oracle as CO
import mlp_oracle as M
from citadels_self_play_amd import canon, models
from citadels_self_play_amd import layout as L
from conftest import load_golden
from hostcheck import HostBatch, HostCfr, encode_games, encode_options
from test_cfr_host_golden import dfs
from test_mlp_host import PROB_ATOL, PROB_RTOL, load_variant

pytestmark = pytest.mark.gpu
VALUE_ATOL = 2e-6


@pytest.fixture(scope="module")
def golden():
    g = dict(np.load("tests/golden/mlp.npz"))
    g["x"] = g["x_int16"].astype(np.float32)
    return g


@pytest.mark.parametrize("fused", [False, True], ids=["layers", "fused"])
@pytest.mark.parametrize("variant", ["init", "bn"])
def test_gpu_mlp_bitwise_vs_fma_oracle(golden, variant, fused):
    m = load_variant(golden, variant)
    net = models.ValueNet(m, "cuda")
    x = np.concatenate([golden["x"], golden["x"][:45] * 0.5])      # ragged last tile (301 rows)
    probs, logits = net.forward(torch.from_numpy(x).cuda(), logits=True, fused=fused)
    probs, logits = probs.cpu().numpy(), logits.cpu().numpy()
    fp, fl = M.FmaMLP(models.fold(m))(x, logits=True)
    assert np.array_equal(logits.view(np.uint32), fl.view(np.uint32))
    assert np.array_equal(probs.view(np.uint32), fp.view(np.uint32))
    np.testing.assert_allclose(probs[:256], golden["%s.probs" % variant], rtol=PROB_RTOL * 50, atol=PROB_ATOL * 10)
    np.testing.assert_allclose(logits[:256], golden["%s.logits" % variant], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("rows", [1, 16, 17, 1024, 1029])
def test_gpu_mlp_layer_split_equals_fused(golden, rows):
    """cit_mlp_forward_packed (fc1 / fc2 spread over the chip) and the one-launch
    k_mlp give bitwise the same probs / logits at every row count, including
    a single row and ragged last tiles; the first rows also equal the oracle."""
    net = models.ValueNet(load_variant(golden, "bn"), "cuda")
    g = torch.Generator().manual_seed(rows)
    x = torch.randint(-3, 6, (rows, 418), generator=g).float() * 0.25
    x[: min(rows, 64)] = torch.from_numpy(golden["x"][: min(rows, 64)])
    pa, la = net.forward(x.cuda(), logits=True)
    pb, lb = net.forward(x.cuda(), logits=True, fused=True)
    assert torch.equal(pa.view(torch.int32), pb.view(torch.int32))
    assert torch.equal(la.view(torch.int32), lb.view(torch.int32))
    k = min(rows, 40)
    fp, fl = M.FmaMLP(models.fold(load_variant(golden, "bn")))(x[:k].numpy(), logits=True)
    assert np.array_equal(la[:k].cpu().numpy().view(np.uint32), fl.view(np.uint32))
    assert np.array_equal(pa[:k].cpu().numpy().view(np.uint32), fp.view(np.uint32))


@pytest.mark.parametrize("variant", ["init", "bn"])
def test_gpu_mlp_wave_bitwise_vs_fma_oracle(golden, variant):
    """The single-row forward the search kernel evaluates its leaves with
    (cit_mlp_forward_wave: one row per wavefront, VALU fmaf chains over the wave
    layout) == the fmaf-chain oracle == the MFMA layer-split path, bit for bit."""
    m = load_variant(golden, variant)
    net = models.ValueNet(m, "cuda")
    x = np.concatenate([golden["x"], golden["x"][:45] * 0.5, -golden["x"][:19] * 3.0])
    xd = torch.from_numpy(x).cuda()
    probs, logits = net.forward(xd, logits=True, wave=True)
    pk, lk = net.forward(xd, logits=True)
    probs, logits = probs.cpu().numpy(), logits.cpu().numpy()
    fp, fl = M.FmaMLP(models.fold(m))(x, logits=True)
    assert np.array_equal(logits.view(np.uint32), fl.view(np.uint32))
    assert np.array_equal(probs.view(np.uint32), fp.view(np.uint32))
    assert np.array_equal(lk.cpu().numpy().view(np.uint32), logits.view(np.uint32))
    assert np.array_equal(pk.cpu().numpy().view(np.uint32), probs.view(np.uint32))


def test_gpu_mlp_packed_rejects_short_workspace(golden):
    from citadels_self_play_amd import _lib
    net = models.ValueNet(load_variant(golden, "init"), "cuda")
    lib = _lib.load()
    x = torch.zeros((40, 418), device="cuda")
    probs = torch.zeros((40, 6), device="cuda")
    need = int(lib.cit_mlp_work_bytes(40))
    assert need == 40 * (512 + 256) * 4
    work = torch.empty(need - 4, dtype=torch.uint8, device="cuda")
    assert lib.cit_mlp_forward_packed(x.data_ptr(), 40, net.packed.data_ptr(), probs.data_ptr(), None,
                                      work.data_ptr(), need - 4, None) == -1


def test_gpu_encode_matches_host():
    from citadels_self_play_amd import _lib
    from citadels_self_play_amd.engine import GameBatch
    lib = _lib.load()
    seeds = list(range(300, 364))
    b = GameBatch(seeds, preset=False)
    hb = HostBatch(seeds, False)
    b.advance_random(0, 120)
    HostCfr(hb, node_cap=16, edge_cap=16).advance(0, 120)
    rows = b.rows()
    assert np.array_equal(rows, hb.games.reshape(len(seeds), -1))
    for pid in (-1, 0, 3, 5):
        feat = torch.zeros((len(seeds), 418), dtype=torch.float32, device="cuda")
        _lib.check(lib.cit_encode_games(b.games.data_ptr(), len(seeds), pid, feat.data_ptr(), None), "enc")
        assert np.array_equal(feat.cpu().numpy(), encode_games(hb, pid)), pid
    opts, n = b.get_options(256)
    opts, n = opts.cpu().numpy(), n.cpu().numpy()
    lane_of = np.concatenate([np.full(min(int(k), 256), l, np.int32) for l, k in enumerate(n)])
    flat = np.concatenate([opts[l, :min(int(k), 256)] for l, k in enumerate(n)])
    out = torch.zeros((len(flat), 131), dtype=torch.float32, device="cuda")
    flat_d, lane_d = torch.from_numpy(flat).cuda(), torch.from_numpy(lane_of).cuda()   # held across the launch
    _lib.check(lib.cit_encode_options(b.games.data_ptr(), flat_d.data_ptr(), lane_d.data_ptr(), len(flat),
                                      out.data_ptr(), None), "enc_opt")
    torch.cuda.synchronize()
    out = out.cpu().numpy()
    i = 0
    for l, k in enumerate(n):
        k = min(int(k), 256)
        assert np.array_equal(out[i:i + k], encode_options(hb.games[l], opts[l, :k])), l
        i += k


@pytest.mark.parametrize("fused", [True, False], ids=["in_kernel_leaves", "leaf_rounds"])
def test_gpu_cfr_pred_golden(golden, fused):
    """Both cfr_pred modes: leaves evaluated inside the search kernel
    (cit_cfr_pred_fused, the default) and rounds of search launches + MFMA
    leaf launches (cit_cfr_pred_slice)."""
    from citadels_self_play_amd.engine import GameBatch
    m = load_variant(golden, "bn")
    net = models.ValueNet(m, "cuda")
    fma = M.FmaMLP(models.fold(m))
    recs = [r for r in load_golden("cfr_pred200.json.gz") if not r.get("skip")]
    b = GameBatch([r["seed"] for r in recs], preset=True)
    b.advance_random(0, 300)
    b.seed_numpy()
    chosen, stats, rounds = b.cfr_pred(200, net, max_depth=10, node_cap=2048, fused=fused)
    torch.cuda.synchronize()
    assert rounds > 10 if not fused else rounds == 0
    chosen, stats, rows = chosen.cpu().numpy(), stats.numpy(), b.rows()
    for l, r in enumerate(recs):
        root, n_nodes, n_edges, carry, err = stats[l]
        assert err == 0, r["seed"]
        g = L.game_from_bytes(rows[l])
        assert n_nodes == r["nodes"] and carry == r["carry_outs"], r["seed"]
        assert canon.canon_game(g) == r["root_game"], r["seed"]
        assert canon.canon_option(L.opt_from_bytes(chosen[l]), g) == r["chosen"], r["seed"]
        nodes, edges, _ = b.tree(l)
        np.testing.assert_allclose(nodes[root]["nv"], r["root"]["node_value"], rtol=0, atol=VALUE_ATOL)
    # bitwise tree comparison vs the fmaf-chain oracle on the first lanes
    for l, r in enumerate(recs[:6]):
        og, npr = CO.config3_position(r["seed"])
        _, tr = CO.run_mccfr(og, npr, 200, model=lambda gm: fma(M.encode_game(gm))[0])
        onodes = CO.dfs(tr.root, [])
        nodes, edges, _ = b.tree(l)
        order = dfs(nodes, edges, int(stats[l][0]), [])
        assert len(order) == len(onodes), r["seed"]
        for i, on in zip(order, onodes):
            assert nodes[i]["nv"].tolist() == np.asarray(on.nv, float).tolist(), r["seed"]


def test_gpu_cfr_pred_rejects_pool_without_pred(golden):
    """A pool reset without pred_node_value room (cit_cfr_arena_reset_fmt pred=0)
    stops every cfr_pred tree with CIT_ERR_UNSUPPORTED instead of writing the
    predictions over other records (both the fused and the resumable kernels)."""
    from citadels_self_play_amd import _lib
    from citadels_self_play_amd.engine import GameBatch
    net = models.ValueNet(load_variant(golden, "bn"), "cuda")
    lib = _lib.load()
    b = GameBatch(list(range(900, 908)), preset=True)
    b.advance_random(0, 300)
    b.seed_numpy()
    for fused in (True, False):
        b._pool(2048, 4 * 2048, pred=False)
        B = b.B
        state = torch.zeros((B, lib.cit_cfr_state_bytes() // 4), dtype=torch.int32, device="cuda")
        chosen = torch.zeros((B, 16), dtype=torch.uint8, device="cuda")
        p = lambda t: t.data_ptr()
        args = (p(b.games), p(b.mt), p(b.mt_idx), p(b.np_mt), p(b.np_idx), p(b.seer), B, 200, 0, None, 10,
                p(b.pool), b.node_cap, b.edge_cap, p(b.optbuf))
        if fused:
            stats = torch.zeros((B, 5), dtype=torch.int32, device="cuda")
            _lib.check(lib.cit_cfr_pred_fused(*args, net.wave.data_ptr(), p(state), p(chosen), p(stats), None), "fused")
            err = stats[:, 4].cpu().numpy()
        else:
            probs = torch.zeros((B, 6), dtype=torch.float32, device="cuda")
            feat = torch.zeros((B, 418), dtype=torch.float32, device="cuda")
            waiting = torch.zeros(2, dtype=torch.int32, device="cuda")
            _lib.check(lib.cit_cfr_pred_step(*args, p(state), p(probs), p(feat), p(chosen), p(waiting), None), "step")
            assert int(waiting[0]) == 0
            err = state[:, 2].cpu().numpy()
        torch.cuda.synchronize()
        assert (err & 0x40).all(), (fused, err)          # CIT_ERR_UNSUPPORTED


def test_gpu_mlp_wave_nonfinite_weight_reads_every_row(golden):
    """A non-finite weight clears the wave layout's flag word (0 * inf is NaN,
    not a no-op), so the single-row forward reads every input row and still
    equals the MFMA path, NaNs and infinities included."""
    m = load_variant(golden, "bn")
    net = models.ValueNet(m, "cuda")
    flag = int(net.wave.view(torch.int32)[-4])           # MLPW_FLAG (then 3 pad words)
    assert flag == 1                                         # finite weights: zero inputs skipped
    with torch.no_grad():
        m.fc3.weight[0, 5] = float("inf")
        m.fc2.weight[3, 7] = float("-inf")
    net = models.ValueNet(m, "cuda")
    assert int(net.wave.view(torch.int32)[-4]) == 0
    x = torch.from_numpy(np.concatenate([golden["x"], golden["x"][:45] * 0.5])).cuda()
    pw, lw = net.forward(x, logits=True, wave=True)
    pk, lk = net.forward(x, logits=True)
    pw, lw, pk, lk = (t.cpu().numpy() for t in (pw, lw, pk, lk))
    assert not np.isfinite(lk).all()                         # the infinities reach the logits somewhere
    np.testing.assert_array_equal(lw, lk)                    # (NaN == NaN here)
    np.testing.assert_array_equal(pw, pk)
