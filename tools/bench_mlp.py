"""Value-MLP (ValueOnlyNN(418,512) leaf evaluation, fp32 MFMA) throughput on
the GPU box: HIP-event time per call at several row counts for both
schedules (the layer-split cit_mlp_forward_packed and the one-launch k_mlp),
TFLOP/s at 757,248 FLOP per row and the fraction of the
157.3 TF fp32 matrix peak (MI355X_MICROARCH.md).  Prints one JSON line per
(schedule, row count); run it under rocprofv3 --kernel-trace --stats for the
per-kernel split."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from citadels_self_play_amd import models  # noqa: E402

FLOP_PER_ROW = 757_248
PEAK_TF = 157.3


def wave_latency(net):
    """The single-row forward of the search's leaf evaluation
    (cit_mlp_forward_wave, one row per wavefront): microseconds per launch of
    M rows (M <= 1,024 rows run side by side, so the launch time is one
    wavefront's latency), on encode_game-like sparse rows and on dense rows."""
    for kind in ("sparse", "dense"):
        for M in (1, 64, 512):
            g = torch.Generator().manual_seed(M)
            if kind == "sparse":      # ~80 of 418 features set, small counts (an encode_game row's shape)
                x = (torch.rand((M, 418), generator=g) < 0.2).float() * torch.randint(1, 4, (M, 418), generator=g)
            else:
                x = torch.rand((M, 418), generator=g) + 0.1
            x = x.cuda()
            probs = torch.empty((M, 6), device="cuda")
            call = lambda: net.lib.cit_mlp_forward_wave(x.data_ptr(), M, net.wave.data_ptr(), probs.data_ptr(), None,
                                                       torch.cuda.current_stream().cuda_stream)
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 50
            e0.record()
            for _ in range(n):
                call()
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"schedule": "wave", "rows": M, "input": kind, "nnz_mean": float((x != 0).sum(1).float().mean()),
                              "us_per_call": e0.elapsed_time(e1) * 1e3 / n}), flush=True)


def main():
    torch.manual_seed(0)
    net = models.ValueNet(models.ValueOnlyNN(418, 512).eval(), "cuda")
    wave_latency(net)
    if "--wave-only" in sys.argv:
        return
    for fused in (False, True):
        for M in (512, 1024, 1365, 2048, 4096, 8192):
            x = torch.randint(0, 4, (M, 418), device="cuda").float()
            probs = torch.empty((M, 6), device="cuda")
            work = net.workspace(M)
            ptrs = [t.data_ptr() for t in net.w]

            def call():
                s = torch.cuda.current_stream().cuda_stream
                if fused:
                    net.lib.cit_mlp_forward(x.data_ptr(), M, *ptrs, probs.data_ptr(), None, s)
                else:
                    net.lib.cit_mlp_forward_packed(x.data_ptr(), M, net.packed.data_ptr(), probs.data_ptr(), None,
                                                   work.data_ptr(), work.numel(), s)
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 50
            e0.record()
            for _ in range(n):
                call()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / n
            tf = FLOP_PER_ROW * M / (us * 1e-6) / 1e12
            print(json.dumps({"schedule": "fused" if fused else "layers", "rows": M, "us_per_call": us,
                              "tflops": tf, "frac_fp32_peak": tf / PEAK_TF}), flush=True)


if __name__ == "__main__":
    main()
