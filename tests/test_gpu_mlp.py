"""Featurizers, value MLP and model-driven MCCFR on a real MI355X through the
C ABI (cit_encode_games / cit_encode_options / cit_mlp_forward /
cit_cfr_pred_step).

* encode kernels == the host build of the same headers (itself pinned to the
  reference's encodings, test_encode_host_golden.py), bit for bit;
* the fp32-MFMA MLP == the fmaf-chain oracle (oracle/mlp_fma.c) bit for bit,
  and within PROB_RTOL/PROB_ATOL of the reference's own forward (mlp.npz);
* cfr_pred(200, 10) with the seeded value net: trees == the oracle driven by
  the fmaf-chain MLP bit for bit; node/carry_out counts, root game and
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


def test_gpu_cfr_pred_golden(golden):
    from citadels_self_play_amd.engine import GameBatch
    m = load_variant(golden, "bn")
    net = models.ValueNet(m, "cuda")
    fma = M.FmaMLP(models.fold(m))
    recs = [r for r in load_golden("cfr_pred200.json.gz") if not r.get("skip")]
    b = GameBatch([r["seed"] for r in recs], preset=True)
    b.advance_random(0, 300)
    b.seed_numpy()
    chosen, stats, rounds = b.cfr_pred(200, net, max_depth=10, node_cap=2048)
    torch.cuda.synchronize()
    assert rounds > 10
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
