"""cfr_pred's batched rounds (engine.GameBatch._pred_poll, PRED_AHEAD): the
host reads the per-round (waiting, running) slots of a batch once and must
count the same leaf rounds, and stop at the same launch, as a host check
after every launch (the loop of deep_mccfr.py:207-229's batched driver).
Host logic only: the counters are given, no GPU is touched."""
import torch

from citadels_self_play_amd.engine import GameBatch


def poll(slots, n=None):
    b = GameBatch.__new__(GameBatch)
    b._pred = {"waiting": torch.tensor(slots, dtype=torch.int32)}
    return b._pred_poll(len(slots) if n is None else n)


def serial(slots):
    """The one-launch-per-poll loop over the same launches: (done, rounds, lead)."""
    rounds = 0
    for waiting, running in slots:
        if waiting == 0 and running == 0:
            return True, rounds, False
        rounds += waiting > 0
    return False, rounds, slots[-1][0] > 0


def test_poll_counts_rounds_until_done():
    s = [[3, 0], [2, 0], [0, 0], [0, 0]]
    assert poll(s) == (True, 2, False) == serial(s)


def test_poll_not_done_leads_with_leaves():
    s = [[3, 0], [0, 5], [1, 0], [2, 0]]
    assert poll(s) == (False, 3, True) == serial(s)


def test_poll_time_sliced_only_running():
    s = [[0, 4]]
    assert poll(s) == (False, 0, False) == serial(s)


def test_poll_reads_only_the_batch_slots():
    # a short last batch (max_rounds clamp) leaves stale slots past n unread
    s = [[1, 0], [0, 0], [7, 7], [7, 7]]
    assert poll(s, 1) == (False, 1, True)
    assert poll(s, 2) == (True, 1, False)
