"""Golden value-MLP vectors from the reference's own model class
(algorithms/models.py ValueOnlyNN(418, 512), eval mode) and
square_and_normalize (algorithms/train_utils.py:143-145).

Weights: torch.manual_seed(0) init (variant "init") and the same with
seeded random BatchNorm statistics / affine parameters (variant "bn"), saved
as plain float32 arrays (np.savez, no pickle).  Inputs: the first 256
encode_game rows of tests/golden/encode.json.gz.  Outputs: logits and
probabilities from the reference's forward on CPU."""
import gzip
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "tests", "golden")
sys.path.insert(0, REF)
sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))


def main():
    from algorithms.models import ValueOnlyNN
    from algorithms.train_utils import square_and_normalize
    with gzip.open(os.path.join(OUT, "encode.json.gz"), "rt") as f:
        recs = json.load(f)
    x = torch.tensor([r["encode"] for r in recs[:256]], dtype=torch.float32)
    arrays = {"x_int16": x.numpy().astype(np.int16)}     # encode_game rows are small integers
    for variant in ("init", "bn"):
        torch.manual_seed(0)
        m = ValueOnlyNN(418, hidden_size=512)
        if variant == "bn":
            g = torch.Generator().manual_seed(1)
            with torch.no_grad():
                for bn in (m.bn1, m.bn2):
                    n = bn.num_features
                    bn.running_mean.copy_(torch.randn(n, generator=g) * 0.5)
                    bn.running_var.copy_(torch.rand(n, generator=g) * 2 + 0.1)
                    bn.weight.copy_(torch.rand(n, generator=g) + 0.5)
                    bn.bias.copy_(torch.randn(n, generator=g) * 0.1)
        m.eval()
        with torch.no_grad():
            logits = m(x)
            probs = square_and_normalize(logits, dim=1)
        import hashlib
        for k, v in m.state_dict().items():
            if not v.dtype.is_floating_point:
                continue
            a = v.detach().numpy().astype(np.float32)
            if k.startswith("bn"):
                arrays["%s.%s" % (variant, k)] = a            # small: kept verbatim
            else:                                             # fc weights: torch.manual_seed(0) init, by digest
                arrays["%s.%s.sha256" % (variant, k)] = np.frombuffer(
                    hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)
        arrays["%s.logits" % variant] = logits.numpy()
        arrays["%s.probs" % variant] = probs.numpy()
    np.savez_compressed(os.path.join(OUT, "mlp.npz"), **arrays)
    print("wrote", len(arrays), "arrays")


if __name__ == "__main__":
    main()
