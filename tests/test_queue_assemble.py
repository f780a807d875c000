"""Host logic of the tree queue (selfplay._assemble_targets): targets extracted
from trees spread over slot lanes in several slices come back in seed order
with the option rows (CSR over children) re-laid out -- the same dict one
batch extraction gives.  Synthetic targets, CPU tensors."""
import torch

from citadels_self_play_amd.selfplay import _assemble_targets


def _batch(counts_t, nch_of, seed):
    """A cfr_targets-shaped dict over lanes with counts_t[l] targets each."""
    g = torch.Generator().manual_seed(seed)
    meta, feat, value, dist, opt = [], [], [], [], []
    row = 0
    counts = []
    for lane, nt in enumerate(counts_t):
        nc = 0
        for k in range(nt):
            nch = nch_of(lane, k)
            meta.append([lane, 100 * lane + k, -1, nch, row])
            feat.append(torch.rand(418, generator=g))
            value.append(torch.rand(6, generator=g, dtype=torch.float64))
            dist.append(torch.rand(nch, generator=g, dtype=torch.float64))
            opt.append(torch.rand((nch, 131), generator=g))
            row += nch
            nc += nch
        counts.append([nt, nc])
    return {"meta": torch.tensor(meta, dtype=torch.int32).reshape(-1, 5),
            "feat": torch.stack(feat) if feat else torch.zeros((0, 418)),
            "value": torch.stack(value) if value else torch.zeros((0, 6), dtype=torch.float64),
            "dist": torch.cat(dist) if dist else torch.zeros(0, dtype=torch.float64),
            "opt_feat": torch.cat(opt) if opt else torch.zeros((0, 131)),
            "counts": torch.tensor(counts, dtype=torch.int32)}


def _sub(full, lanes, slot_of, n_slots):
    """What one slice's extraction returns: trees `lanes` sitting in slots slot_of."""
    meta, feat, value, dist, opt = [], [], [], [], []
    counts = torch.zeros((n_slots, 2), dtype=torch.int32)
    row = 0
    order = sorted(zip(slot_of, lanes))
    for slot, lane in order:
        sel = (full["meta"][:, 0] == lane).nonzero().flatten()
        for k in sel.tolist():
            m = full["meta"][k].clone()
            nch, c0 = int(m[3]), int(m[4])
            m[0], m[4] = slot, row
            meta.append(m)
            feat.append(full["feat"][k])
            value.append(full["value"][k])
            dist.append(full["dist"][c0:c0 + nch])
            opt.append(full["opt_feat"][c0:c0 + nch])
            row += nch
        counts[slot] = full["counts"][lane]
    t = {"meta": torch.stack(meta) if meta else torch.zeros((0, 5), dtype=torch.int32),
         "feat": torch.stack(feat) if feat else torch.zeros((0, 418)),
         "value": torch.stack(value) if value else torch.zeros((0, 6), dtype=torch.float64),
         "dist": torch.cat(dist) if dist else torch.zeros(0, dtype=torch.float64),
         "opt_feat": torch.cat(opt) if opt else torch.zeros((0, 131)), "counts": counts}
    return t, torch.tensor(slot_of), torch.tensor(lanes)


def test_assemble_targets_seed_order():
    counts_t = [3, 0, 5, 1, 2, 4, 0, 2]
    full = _batch(counts_t, lambda lane, k: 1 + (lane * 7 + k * 3) % 5, 0)
    # 8 trees through 3 slots over 3 slices, finishing out of order
    parts = [_sub(full, [2, 0], [1, 0], 3), _sub(full, [1, 3, 4], [2, 0, 1], 3), _sub(full, [7, 5, 6], [0, 2, 1], 3)]
    t = _assemble_targets(parts, len(counts_t))
    for k in ("meta", "feat", "value", "dist", "opt_feat", "counts"):
        assert torch.equal(t[k], full[k]), k


def test_assemble_targets_excludes_retried_trees():
    counts_t = [2, 3, 1]
    full = _batch(counts_t, lambda lane, k: 2 + k, 1)
    junk = _batch([4, 4, 4], lambda lane, k: 1, 2)        # what the overflowed tree 1 left in its slot
    first = _sub(junk, [1], [0], 2)
    first = (first[0], first[1], torch.tensor([1]))
    parts = [_sub(full, [0, 2], [1, 0], 2), first, _sub(full, [1], [0], 1)]
    t = _assemble_targets(parts, 3, exclude=torch.tensor([1]))
    for k in ("meta", "feat", "value", "dist", "opt_feat", "counts"):
        assert torch.equal(t[k], full[k]), k
