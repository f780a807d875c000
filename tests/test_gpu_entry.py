"""The three entry points end to end on one MI355X with small settings:
generate_test_data (against the reference's setup_game goldens),
train_from_scratch (data rounds + training + checkpoints), compare_to_random."""
import os
import pickle

import numpy as np
import pytest
import torch

from conftest import load_golden
from test_targets_oracle_golden import check_targets

pytestmark = pytest.mark.gpu


def test_gpu_generate_test_data(tmp_path):
    from citadels_self_play_amd import generate_test_data
    recs = load_golden("testdata500.json.gz")
    out = generate_test_data.main(["--games", str(len(recs)), "--iters", "500", "--out", str(tmp_path)])
    with open(tmp_path / "validation_targets.pkl", "rb") as f:
        val = pickle.load(f)
    assert len(val) == len(out["validation_targets.pkl"])
    want = [r["result"] for r in recs if not isinstance(r["result"], str)]
    got = [(x.numpy(), o.numpy()[0], v.numpy(), d.numpy()) for x, o, v, d in val]
    check_targets(got, want, "generate_test_data")
    assert os.path.exists(tmp_path / "test_targets.pkl")


def test_gpu_train_from_scratch(tmp_path):
    from citadels_self_play_amd import train_from_scratch
    model = train_from_scratch.main(["--iters", "300", "--games-per-gpu", "64", "--pretrain-targets", "40",
                                     "--train-targets", "20", "--phases", "1", "--epochs", "3", "--batch-size", "32",
                                     "--out", str(tmp_path), "--val", str(tmp_path / "none.pkl"), "--save-tuples"])
    for name in ("pretrain", "train0"):
        sd = torch.load(tmp_path / name / "best_model.pt", map_location="cpu", weights_only=True)
        assert set(sd) >= {"fc1.weight", "bn1.running_mean", "fc4.bias"}
        with open(tmp_path / name / "targets_rank0.pkl", "rb") as f:
            t = pickle.load(f)
        assert len(t) >= 20 and t[0][0].shape == (418,) and t[0][1].shape[-1] == 131
        assert all(float(x[2].sum()) >= 15 for x in t)
    assert isinstance(model, torch.nn.Module)


def test_gpu_compare_to_random_main():
    from citadels_self_play_amd import compare_to_random
    counts = compare_to_random.main(["--games", "6", "--pred-iters", "20", "--train-iters", "40"])
    assert sum(counts) == 6
