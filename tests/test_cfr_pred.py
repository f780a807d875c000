"""Model-driven MCCFR (cfr_pred, max_depth 10; deep_mccfr.py:207-229) with a
seeded ValueOnlyNN(418, 512).

* oracle + torch fp32 MLP == the reference (tests/golden/cfr_pred200) bit for bit;
* oracle + the fmaf-chain MLP (the arithmetic of the device's fp32 MFMA) ==
  the engine's resumable search (host build here, GPU in test_gpu_cfr_pred)
  bit for bit, trees included;
* engine vs the reference: identical search structure and decisions, node
  values within 2e-6 absolute (float32 leaf values summed into float64)."""
import numpy as np
import pytest
import torch

import cfr_oracle as CO
import citadels_oracle as O
import mlp_oracle as M
from citadels_self_play_amd import canon, models
from citadels_self_play_amd import layout as L
from conftest import load_golden
from hostcheck import HostBatch, HostCfr, cfr_pred
from test_cfr_host_golden import compare_node, dfs, hash_obj
from test_mlp_host import load_variant

VALUE_ATOL = 2e-6


@pytest.fixture(scope="module")
def net():
    g = dict(np.load("tests/golden/mlp.npz"))
    m = load_variant(g, "bn")
    return m, M.FmaMLP(models.fold(m))


def torch_infer(m):
    def f(game):
        with torch.no_grad():
            x = torch.from_numpy(M.encode_game(game))[None]
            return models.square_and_normalize(m(x), dim=1)[0].numpy()
    return f


def test_oracle_torch_mlp_matches_reference(net):
    m, _ = net
    for r in load_golden("cfr_pred200.json.gz"):
        if r.get("skip"):
            continue
        g, npr = CO.config3_position(r["seed"])
        chosen, tr = CO.run_mccfr(g, npr, 200, model=torch_infer(m))
        assert tr.count == r["nodes"] and tr.carry_outs == r["carry_outs"]
        assert chosen.canon() == r["chosen"]
        assert tr.root.nv.tolist() == r["root"]["node_value"]
        assert np.asarray(tr.root.R).tolist() == r["root"]["R"]


def test_engine_pred_matches_fma_oracle_and_reference(net):
    m, fma = net
    recs = [r for r in load_golden("cfr_pred200.json.gz") if not r.get("skip")]
    hb = HostBatch([r["seed"] for r in recs], True)
    cf = HostCfr(hb, node_cap=2048, edge_cap=8 * 2048)
    cf.advance(0, 300)
    chosen, stats, rounds = cfr_pred(cf, 200, 10, fma)
    assert rounds > 10
    for l, r in enumerate(recs):
        root, n_nodes, n_edges, carry, err = stats[l]
        assert err == 0, r["seed"]
        g = hb.game(l)
        # vs the reference (torch MLP): same structure, values within tolerance
        assert n_nodes == r["nodes"] and carry == r["carry_outs"], r["seed"]
        assert canon.canon_game(g) == r["root_game"], r["seed"]
        assert canon.canon_option(L.opt_from_bytes(chosen[l]), g) == r["chosen"], r["seed"]
        nodes, edges, rows = cf.tree(l)
        np.testing.assert_allclose(nodes[root]["nv"], r["root"]["node_value"], rtol=0, atol=VALUE_ATOL)
        # vs the oracle with the same (fmaf-chain) MLP: bit for bit
        og, npr = CO.config3_position(r["seed"])
        ochosen, tr = CO.run_mccfr(og, npr, 200, model=lambda gm: fma(M.encode_game(gm))[0])
        onodes = CO.dfs(tr.root, [])
        order = dfs(nodes, edges, root, [])
        assert len(order) == len(onodes)
        for i, on in zip(order, onodes):
            assert nodes[i]["nv"].tolist() == np.asarray(on.nv, float).tolist()
            assert nodes[i]["wp"].tolist() == np.asarray(on.wp, float).tolist()
            if on.pred is not None and nodes[i]["flags"] & 4:
                assert nodes[i]["pred"].tolist() == np.asarray(on.pred, float).tolist()


def test_host_cfr_pred_rejects_pool_without_pred():
    """The host build of cfr_pred on a pool reset without pred_node_value room
    stops every tree with CIT_ERR_UNSUPPORTED (the predictions would
    otherwise overwrite other nodes' rows / edges)."""
    import numpy as np
    from hostcheck import HostBatch, HostCfr, cfr_pred
    hb = HostBatch(list(range(910, 914)), True)
    cf = HostCfr(hb, node_cap=2048, edge_cap=8192, pred=False)
    cf.advance(0, 300)
    calls = []
    chosen, stats, rounds = cfr_pred(cf, 50, 10, lambda f: calls.append(len(f)) or np.full((len(f), 6), 1 / 6, np.float32))
    assert rounds == 0 and not calls
    assert ((stats[:, 4] & 0x40) != 0).all()                  # CIT_ERR_UNSUPPORTED
