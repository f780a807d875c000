"""The value-net trainer (citadels_self_play_amd/train.py) against the
reference's train_node_value_only (algorithms/train.py:13-86) run on the same
seeded targets (tests/golden/trainer.npz, tools/gen_golden_trainer.py): the
per-epoch train / eval losses, learning rates and the returned best eval loss.
CPU, torch.manual_seed(0) before the call as in the generator; the same torch
ops in the same order, so the histories agree to float64 round-off
(tolerance rtol 1e-6 covers a different torch build's kernel choices)."""
import os
import tempfile

import numpy as np
import torch

from conftest import GOLDEN


def test_trainer_matches_reference():
    from citadels_self_play_amd.train import train_node_value_only
    z = np.load(os.path.join(GOLDEN, "trainer.npz"))
    tup = lambda x, v: [(torch.from_numpy(x[i]), None, torch.from_numpy(v[i]), None) for i in range(len(x))]
    torch.manual_seed(0)
    with tempfile.TemporaryDirectory() as d:
        best, model, hist = train_node_value_only(tup(z["xt"], z["vt"]), tup(z["xv"], z["vv"]), epochs=3, lr=0.01,
                                                  hidden_size=64, gamma=0.9, batch_size=32, device="cpu",
                                                  parent_folder=d)
        assert os.path.exists(os.path.join(d, "best_model.pt"))
        sd = torch.load(os.path.join(d, "best_model.pt"), weights_only=True)
        assert set(sd) == set(model.state_dict())
    np.testing.assert_allclose(hist["train"], z["train"], rtol=1e-6, atol=0)
    np.testing.assert_allclose(hist["eval"], z["eval"], rtol=1e-6, atol=0)
    np.testing.assert_allclose(hist["lr"], z["lr"], rtol=0, atol=0)
    np.testing.assert_allclose(best, float(z["best"]), rtol=1e-6, atol=0)
