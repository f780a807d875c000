"""The batched random.shuffle of the wave paths (csrc/cit_engine.h
fy_draws_batched + traced swaps, CIT_SHUFFLE_BATCH) against the serial
_randbelow draws and swaps (Lib/random.py:380-392, 239-249) from the same MT
stream: the same sequences, the same stream position after, the same later
draws.  Test-only kernel (tests/testkit.py).  Lengths under
CIT_SHUFFLE_BATCH_MIN (12) take the serial path in both runs."""
import numpy as np
import pytest

POS0 = (0, 1, 63, 64, 300, 560, 600, 620, 623, 624)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3, 5, 16, 33, 60, 63, 64, 65, 66, 88, 100, 127, 128])
def test_gpu_batched_shuffle_matches_serial(n):
    import torch
    import testkit
    lib = testkit.lib()
    reps = 12                                  # n = 128 crosses the 624-word twist several times
    rs = np.random.default_rng(1000 + n)
    B = 4 * len(POS0)
    words = torch.as_tensor(rs.integers(0, 2 ** 32, size=(B, 624), dtype=np.uint64).astype(np.uint32).view(np.int32),
                            device="cuda")
    pos0 = torch.as_tensor(np.tile(np.asarray(POS0, np.int32), 4), device="cuda")
    out = torch.zeros((2, B, reps, n), dtype=torch.uint8, device="cuda")
    tail = torch.zeros((2, B, 4), dtype=torch.int32, device="cuda")
    assert lib.citk_shuffle_check(n, reps, B, words.data_ptr(), pos0.data_ptr(), out.data_ptr(), tail.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    o, t = out.cpu().numpy(), tail.cpu().numpy()
    assert np.array_equal(o[1], o[0])
    assert np.array_equal(t[1], t[0])
    assert all(sorted(o[0, b, r]) == list(range(n)) for b in range(B) for r in range(reps))
    assert len({o[0, b, r].tobytes() for b in range(B) for r in range(reps)}) > (1 if n > 3 else 0)
