"""Cycles per random.shuffle of n elements on one wave with an LDS stream
(tests/testkit.py's k_bench_shuffle): the draws alone, serial LDS swaps,
register swaps and the traced-positions variant.  One JSON line per mode."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import testkit  # noqa: E402
import torch  # noqa: E402

lib = testkit.lib()
blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 64
NS = tuple(int(x) for x in sys.argv[2].split(",")) if len(sys.argv) > 2 else (16, 60, 100)
for n in NS:
    for mode, name in enumerate(("draws_only", "lds_swaps", "reg_swaps", "traced", "draws_queue4", "draws_queue8", "batched",
                                  "batched_draws_only", "batched_draws_lds_swaps")):
        out = torch.zeros(blocks, dtype=torch.int64, device="cuda")
        sink = torch.zeros(blocks, dtype=torch.int32, device="cuda")
        for _ in range(2):
            assert lib.citk_bench_shuffle(mode, n, 32, blocks, out.data_ptr(), sink.data_ptr(),
                                          torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        v = out.cpu().double()
        print(json.dumps({"n": n, "mode": name, "blocks": blocks, "cycles_per_shuffle": float(v.mean()),
                          "cycles_per_step": float(v.mean()) / (n - 1)}), flush=True)
