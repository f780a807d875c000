"""ctypes mirror of the packed row layout in csrc/cit_core.h.

`CitGame` rows are CIT_GAME_BYTES wide; tests check `sizeof` and a few field
offsets against the values the native library reports (cit_layout), so the
two definitions cannot drift apart silently.
"""
import ctypes as C

NP = 6
AREA_CAP, BUILD_CAP = 88, 16     # a player's hand | just_drawn | museum share AREA_CAP slots
DECK_CAP, DISCARD_CAP, USED_CAP = 128, 88, 80
KH_MAX, KH_POOL, SEVEN_CAP = 32, 244, 8
GAME_BYTES = 1552
MT_N = 624
SEER_MAX = 5 * AREA_CAP * 3 + AREA_CAP // 8   # CIT_SEER_MAX: seer give-back options (+ their shuffle list) per lane
NO_CARD = 255
ROLE_BEWITCHED, ROLE_NONE = 27, 255

ERR_BITS = {
    0x1: "OverflowError", 0x2: "IndexError", 0x4: "KeyError", 0x8: "ValueError",
    0x10: "IndexError", 0x20: "AttributeError", 0x40: "NotImplementedError", 0x80: "TypeError", 0x100: "StepCap",
}


class CitPlayer(C.Structure):
    """`hand` is the player's card area: the hand at [0, n_hand), then the
    just-drawn cards and the museum (the `jd` / `museum` properties)."""
    _fields_ = [
        ("hand", C.c_uint8 * AREA_CAP), ("build", C.c_uint8 * BUILD_CAP),
        ("n_hand", C.c_uint8), ("n_build", C.c_uint8), ("n_jd", C.c_uint8), ("n_museum", C.c_uint8),
        ("gold", C.c_int16), ("role", C.c_uint8), ("replicas", C.c_int8), ("flags", C.c_uint8),
        ("pad0", C.c_uint8), ("kr", C.c_uint16 * NP), ("pad1", C.c_uint16),
    ]

    @property
    def jd(self):
        return list(self.hand[self.n_hand:self.n_hand + self.n_jd])

    @property
    def museum(self):
        o = self.n_hand + self.n_jd
        return list(self.hand[o:o + self.n_museum])


class CitKH(C.Structure):
    _fields_ = [("owner", C.c_uint8), ("target", C.c_int8), ("conf_flags", C.c_uint8), ("len", C.c_uint8)]


class CitGame(C.Structure):
    _fields_ = [
        ("pl", CitPlayer * NP),
        ("deck", C.c_uint8 * DECK_CAP), ("discard", C.c_uint8 * DISCARD_CAP),
        ("used_cards", C.c_uint8 * USED_CAP), ("kh_pool", C.c_uint8 * KH_POOL), ("kh", CitKH * KH_MAX),
        ("deck_head", C.c_uint8), ("n_deck", C.c_uint8), ("n_discard", C.c_uint8), ("n_used_cards", C.c_uint8),
        ("n_kh", C.c_uint8), ("kh_fill", C.c_uint8), ("preset", C.c_uint8), ("pad2", C.c_uint8),
        ("roles", C.c_uint8 * 8), ("rtc", C.c_uint8), ("n_used_roles", C.c_uint8),
        ("used_roles", C.c_int8 * NP), ("turn", C.c_uint8 * NP), ("rp", C.c_uint8 * 8),
        ("gs_state", C.c_uint8), ("gs_pid", C.c_int8), ("gs_adm", C.c_uint8 * 9), ("gs_intr", C.c_uint8),
        ("nx_valid", C.c_uint8), ("nx_state", C.c_uint8), ("nx_pid", C.c_int8), ("nx_adm", C.c_uint8 * 9),
        ("nx_intr", C.c_uint8), ("nx_alias", C.c_uint8), ("nx_hasnext", C.c_uint8),
        ("ending", C.c_uint8), ("terminal", C.c_uint8), ("winner", C.c_int8), ("has_points", C.c_uint8),
        ("points", C.c_int16 * NP), ("warrant", C.c_uint8), ("n_seer", C.c_uint8), ("seer_from", C.c_uint8 * 5),
        ("seven_kind", C.c_uint8), ("n_seven", C.c_uint8), ("seven", C.c_uint8 * SEVEN_CAP),
        ("n_sch", C.c_uint8), ("sch", C.c_uint8 * SEVEN_CAP),
        ("err", C.c_uint32), ("steps", C.c_uint32),
    ]


class CitOpt(C.Structure):
    _fields_ = [("name", C.c_uint8), ("perp", C.c_uint8), ("target", C.c_int8), ("a", C.c_uint8),
                ("b", C.c_uint8), ("c", C.c_uint8), ("d", C.c_uint8), ("flags", C.c_uint8), ("x", C.c_uint64)]


def expected_layout():
    """The values cit_layout()/cith_layout() must report (see cit_host.cpp)."""
    return [C.sizeof(CitPlayer), CitGame.deck.offset, CitGame.kh.offset, CitGame.roles.offset,
            CitGame.gs_state.offset, CitGame.points.offset, CitGame.err.offset, CitGame.steps.offset,
            C.sizeof(CitOpt)]


def game_from_bytes(b):
    """A CitGame view over one row (bytes / bytearray / numpy uint8 row)."""
    buf = bytes(b)
    assert len(buf) >= C.sizeof(CitGame)
    return CitGame.from_buffer_copy(buf[:C.sizeof(CitGame)])


def opt_from_bytes(b):
    return CitOpt.from_buffer_copy(bytes(b)[:16])


# ---- MCCFR node pools (csrc/cit_cfr.h): B per-tree regions (block tables, base
# row, scratch row), then one arena of node blocks (CFR_NB node records, and
# CFR_NB raw row slots in row_cap-0 pools) and edge blocks (CFR_EB edge slots)
# the trees take as they grow.  Rows are raw game rows (row_cap 0) or diffs
# against the tree's base row with at most row_cap differing dwords, each a
# run of edge slots (CfrNode.row: a CFR_ROW_HDR-word header, then the
# differing dwords).  tests/test_abi.py checks these constants against the
# library (cit_cfr_block_sizes / cit_cfr_sizes).
CFR_NB, CFR_EB, CFR_TBL_MAX = 4096, 16384, 1024
CFR_NODE_BYTES, CFR_PRED_BYTES, CFR_EDGE_BYTES, CFR_ARENA_HDR = 72, 48, 48, 64
NF_BACKED = 8                     # CfrNode flag: backpropagated (winning_probabilities = nv / nv.sum())
CFR_ROW_W, CFR_ROW_HDR, CFR_ROW_MASKW = GAME_BYTES // 4, 14, 13
CFR_ROW_CAP_MAX = CFR_ROW_W


def cfr_nblocks(node_cap):
    return -(-int(node_cap) // CFR_NB)


def cfr_eblocks(edge_cap):
    return -(-int(edge_cap) // CFR_EB)


def cfr_tables_bytes(node_cap, edge_cap):
    """A tree's node- and edge-block tables (int32, -1 = none), padded to 16 B."""
    return (4 * (cfr_nblocks(node_cap) + cfr_eblocks(edge_cap)) + 15) // 16 * 16


def cfr_pool_bytes(node_cap, edge_cap):
    """Bytes per tree ahead of the arena: its tables, base row and scratch row."""
    return cfr_tables_bytes(node_cap, edge_cap) + 2 * GAME_BYTES


def cfr_row_slot_bytes(row_cap=0):
    """A node block's row slot: a raw row; none in diff-row pools (their rows are edge-slot runs)."""
    return 0 if row_cap else GAME_BYTES


def cfr_row_slots(k):
    """Edge slots of a diff row run with k differing dwords."""
    return -(-(CFR_ROW_HDR + int(k)) // (CFR_EDGE_BYTES // 4))


def cfr_node_block_bytes(row_cap=0, pred=True):
    return CFR_NB * (CFR_NODE_BYTES + (CFR_PRED_BYTES if pred else 0) + cfr_row_slot_bytes(row_cap))


def cfr_ring_bytes(n_blocks, e_blocks):
    """The arena's free-block rings (uint32 per block of each kind), padded to 16 B."""
    return (4 * (n_blocks + e_blocks) + 15) // 16 * 16


def cfr_arena_bytes(n_blocks, e_blocks, row_cap=0, pred=True):
    return CFR_ARENA_HDR + cfr_ring_bytes(n_blocks, e_blocks) + n_blocks * cfr_node_block_bytes(row_cap, pred) + \
        e_blocks * CFR_EB * CFR_EDGE_BYTES


def cfr_row_decode(slot, base):
    """A diff row run (uint8, from its first slot on) against the tree's base row -> the game row."""
    import numpy as np
    w = np.asarray(slot).view("<u4")
    mask = np.unpackbits(w[:CFR_ROW_MASKW].view(np.uint8), bitorder="little")[:CFR_ROW_W].astype(bool)
    out = np.array(np.asarray(base).view("<u4"), copy=True)
    out[mask] = w[CFR_ROW_HDR:CFR_ROW_HDR + int(mask.sum())]
    return out.view(np.uint8)


# A node record as the tests and tools read it (round 3's full record): the
# header, node_value, winning_probabilities (derived: nv / nv.sum() once the
# node was backpropagated, else zeros) and pred_node_value (zeros in pools
# without pred).
FULL_NODE_BYTES = 24 + 3 * 48


def _full_nodes(rec, pred):
    import numpy as np
    n = rec.shape[0] // CFR_NODE_BYTES
    rec = rec[:n * CFR_NODE_BYTES].reshape(n, CFR_NODE_BYTES)
    out = np.zeros((n, FULL_NODE_BYTES), np.uint8)
    out[:, :CFR_NODE_BYTES] = rec
    nv = np.ascontiguousarray(rec[:, 24:72]).view("<f8")
    s = np.zeros(n)
    for k in range(6):                           # numpy's order for 6 elements
        s = s + nv[:, k]
    backed = (rec[:, 16] & NF_BACKED) != 0     # flags byte
    with np.errstate(divide="ignore", invalid="ignore"):
        wp = np.where(backed[:, None], nv / s[:, None], 0.0)
    out[:, 72:120] = np.ascontiguousarray(wp).view(np.uint8).reshape(n, 48)
    if pred is not None:
        out[:, 120:168] = pred[:n * CFR_PRED_BYTES].reshape(n, CFR_PRED_BYTES)
    return out.reshape(-1)


def cfr_tree_bytes(read, B, lane, node_cap, edge_cap):
    """(node records, edge slots, game rows) of tree `lane` as uint8 arrays
    gathered from its blocks in id order (node records in FULL_NODE_BYTES
    form); `read(offset, nbytes)` returns pool bytes as a uint8 ndarray (host
    pool or device copy)."""
    import numpy as np
    per = cfr_pool_bytes(node_cap, edge_cap)
    nb, eb = cfr_nblocks(node_cap), cfr_eblocks(edge_cap)
    tbl = np.array(read(lane * per, 4 * (nb + eb))).view("<i4")
    hdr = np.array(read(B * per, 48)).view("<u4")
    n_cap, e_cap, row_cap, has_pred = int(hdr[1]), int(hdr[3]), int(hdr[8]), int(hdr[9])
    slot = cfr_row_slot_bytes(row_cap)
    node_base = B * per + CFR_ARENA_HDR + cfr_ring_bytes(n_cap, e_cap)
    pred_base = node_base + n_cap * CFR_NB * CFR_NODE_BYTES
    row_base = pred_base + (n_cap * CFR_NB * CFR_PRED_BYTES if has_pred else 0)
    edge_base = row_base + n_cap * CFR_NB * slot

    def held(t):
        out = []
        for b in t:
            if b < 0:
                break
            out.append(int(b))
        return out

    def gather(base, size, blocks):
        parts = [np.array(read(base + b * size, size)) for b in blocks]
        return np.concatenate(parts) if parts else np.zeros(0, np.uint8)

    nbl, ebl = held(tbl[:nb]), held(tbl[nb:])
    rec = gather(node_base, CFR_NB * CFR_NODE_BYTES, nbl)
    nodes = _full_nodes(rec, gather(pred_base, CFR_NB * CFR_PRED_BYTES, nbl) if has_pred else None)
    edges = gather(edge_base, CFR_EB * CFR_EDGE_BYTES, ebl)
    if not row_cap:
        rows = gather(row_base, CFR_NB * slot, nbl).reshape(-1, slot)
        return nodes, edges, rows
    # diff rows: node i's run starts at edge slot CfrNode.row (bytes 20..23);
    # node ids without a row (past n_nodes, or an allocation that failed) decode
    # to garbage
    base = np.array(read(lane * per + cfr_tables_bytes(node_cap, edge_cap), GAME_BYTES)).view("<u4")
    run = np.ascontiguousarray(rec.reshape(-1, CFR_NODE_BYTES)[:, 20:24]).view("<i4")[:, 0]
    ew = np.concatenate([np.ascontiguousarray(edges).view("<u4"), np.zeros(CFR_ROW_HDR + CFR_ROW_W, "<u4")])
    start = np.clip(run, 0, max(0, (ew.shape[0] - CFR_ROW_HDR - CFR_ROW_W) // (CFR_EDGE_BYTES // 4)))
    rows = np.empty((run.shape[0], CFR_ROW_W), "<u4")
    for c in range(0, run.shape[0], 4096):                   # bounded temporaries
        w = ew[start[c:c + 4096, None] * (CFR_EDGE_BYTES // 4) + np.arange(CFR_ROW_HDR + CFR_ROW_W)[None, :]]
        bits = np.unpackbits(np.ascontiguousarray(w[:, :CFR_ROW_MASKW]).view(np.uint8), axis=1,
                             bitorder="little")[:, :CFR_ROW_W].astype(bool)
        rank = np.clip(np.cumsum(bits, axis=1) - 1, 0, CFR_ROW_W - 1) + CFR_ROW_HDR
        rows[c:c + 4096] = np.where(bits, np.take_along_axis(w, rank, axis=1), base[None, :])
    return nodes, edges, rows.view(np.uint8)
