"""Golden fixture for the value-net trainer from the
reference itself (build container only; writes tests/golden/trainer.npz).

Harness: 256 training and 64 validation targets (synthetic, seeded: encode_game
-like small-int features f32[418], node_value-like counts f64[6]) as the
reference's tuples (x, options, node_value, target); then, on the CPU,
    torch.manual_seed(0)
    algorithms.train.train_node_value_only(train, val, epochs=3, lr=0.01,
        hidden_size=64, gamma=0.9, batch_size=32, device="cpu")      # train.py:13-86
recording the per-epoch train / eval losses and learning rates (captured from
its plot_metrics call, which is stubbed, as is seaborn) and the best eval
loss it returns.  tests/test_trainer_golden.py runs train.py's restatement on
the same data and seed."""
import os
import sys
import tempfile
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "tests", "golden", "trainer.npz")
sys.path.insert(0, REF)
sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))


def data(n, seed):
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 9, size=(n, 418)).astype(np.float32)
    v = rng.integers(0, 40, size=(n, 6)).astype(np.float64)
    v[np.arange(n), rng.integers(0, 6, size=n)] += 1.0       # no all-zero rows
    return x, v


def main():
    import algorithms.train as T
    xt, vt = data(256, 1)
    xv, vv = data(64, 2)
    tup = lambda x, v: [(torch.from_numpy(x[i]), None, torch.from_numpy(v[i]), None) for i in range(len(x))]
    rec = {}

    def capture(train_losses, eval_losses, learning_rates, epochs, folder):
        rec["train"], rec["eval"], rec["lr"] = list(train_losses), list(eval_losses), list(learning_rates)

    T.plot_metrics = capture
    torch.manual_seed(0)
    with tempfile.TemporaryDirectory() as d:
        best = T.train_node_value_only(tup(xt, vt), tup(xv, vv), epochs=3, lr=0.01, hidden_size=64, gamma=0.9,
                                       batch_size=32, device="cpu", parent_folder=d)
    np.savez_compressed(OUT, xt=xt, vt=vt, xv=xv, vv=vv, train=np.array(rec["train"]), eval=np.array(rec["eval"]),
                        lr=np.array(rec["lr"]), best=np.array(best), torch_version=np.array(torch.__version__))
    print(best, rec)


if __name__ == "__main__":
    main()
