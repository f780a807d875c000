"""k_mlp (ValueOnlyNN(418,512) leaf evaluation, fp32 MFMA) throughput on the
GPU box: HIP-event time per call at several row counts, TFLOP/s at 757,248
FLOP per row and the fraction of the 157.3 TF fp32 matrix
peak (MI355X_MICROARCH.md).  Prints one JSON line per row count."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from citadels_self_play_amd import models  # noqa: E402

FLOP_PER_ROW = 757_248
PEAK_TF = 157.3


def main():
    torch.manual_seed(0)
    net = models.ValueNet(models.ValueOnlyNN(418, 512).eval(), "cuda")
    for M in (512, 1024, 2048, 4096, 8192):
        x = torch.randint(0, 4, (M, 418), device="cuda").float()
        for _ in range(3):
            net.forward(x)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            net.forward(x)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        tf = FLOP_PER_ROW * M / (us * 1e-6) / 1e12
        print(json.dumps({"rows": M, "us_per_call": us, "tflops": tf, "frac_fp32_peak": tf / PEAK_TF}), flush=True)


if __name__ == "__main__":
    main()
