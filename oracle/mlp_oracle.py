"""CPU ORACLE (test infrastructure only): ctypes wrapper of oracle/mlp_fma.c
and encode_game restated over the oracle's game model (game/game.py:91-128)."""
import ctypes as C
import os
import subprocess

import numpy as np

import citadels_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "mlp_fma.c")
LIB = os.path.join(HERE, "_ref", "libmlp_fma.so")
_lib = None


def build():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-shared", "-fPIC", SRC, "-o", LIB, "-lm"])
    return LIB


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
    return _lib


class FmaMLP:
    """folded = models.fold(ValueOnlyNN) tensors (w1t, b1, ..., w4t, b4)."""

    def __init__(self, folded):
        self.w = [np.ascontiguousarray(t.numpy() if hasattr(t, "numpy") else t, np.float32) for t in folded]

    def __call__(self, feat, logits=False):
        x = np.ascontiguousarray(np.atleast_2d(feat), np.float32)
        M = x.shape[0]
        probs = np.zeros((M, 6), np.float32)
        lg = np.zeros((M, 6), np.float32)
        p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        lib().mlp_forward(p(x), C.c_int(M), *[p(w) for w in self.w], p(probs), p(lg))
        return (probs, lg) if logits else probs


def encode_game(g, pid=None):
    """game.py:91-128 over citadels_oracle.OGame; pid overrides gamestate.player_id."""
    cur = g.gs.pid if pid is None else pid
    v = np.zeros(418, np.float32)
    for r in range(8):
        v[r * 3 + g.roles[r] % 3] = 1
    for p in g.players:
        if p.role is None or p.role == O.BEWITCHED:
            continue
        if g.players[cur].kr[p.id][1]:
            v[24 + p.id * 8 + p.role // 3] = 1
    for i, p in enumerate(g.players):
        v[72 + i] = O.count_points(p)
        v[78 + i] = p.gold
        v[84 + i] = len(p.hand)
        for c in p.build:
            v[90 + i * 40 + O.ctype(c)] += 1
            v[330 + i * 5 + O.csuit(c)] += 1
    v[360 + cur] = 1
    v[366 + g.gs.state] = 1
    v[377] = 1 if g.ending else 0
    for r in range(8):
        rp = g.rp[r]
        v[378 + r * 5:378 + r * 5 + 5] = [bool(rp[0]), rp[1] is not None, bool(rp[2]), bool(rp[3]), rp[4] is not None]
    return v


# option.py:33-49 (name_to_id order)
OPTION_IDS = {n: i for i, n in enumerate([
    "role_pick", "gold_or_card", "which_card_to_keep", "blackmail_response",
    "reveal_blackmail_as_blackmailer", "reveal_warrant_as_magistrate", "build", "empty_option",
    "finish_round", "ghost_town_color_choice", "smithy_choice", "laboratory_choice",
    "magic_school_choice", "weapon_storage_choice", "lighthouse_choice", "museum_choice",
    "graveyard", "take_gold_for_war", "assassination", "magistrate_warrant", "bewitching",
    "steal", "blackmail", "spy", "magic_hand_change", "discard_and_draw", "look_at_hand",
    "take_from_hand", "seer", "give_back_card", "take_crown_king", "give_crown",
    "take_crown_pat", "bishop", "cardinal_exchange", "abbot_gold_or_card", "abbot_beg",
    "merchant", "alchemist", "trader", "architect", "navigator_gold_card", "scholar",
    "scholar_card_pick", "warlord_desctruction", "marshal_steal", "diplomat_exchange"])}
NAMED = {"gold": 0, "card": 1, "pay": 2, "not_pay": 3, "reveal": 4, "not_reveal": 5, "4gold": 6, "4card": 7,
         "trade": 8, "war": 9, "religion": 10, "lord": 11, "unique": 12}
ROLE_IDS = dict({n: i // 3 for i, n in enumerate(O.ROLE_NAMES)}, Bewitched=-1)   # config.py:93 role_to_role_id


def encode_option(o):
    """option.encode_option (option.py:52-115) over a citadels_oracle.Opt: the
    first matching attribute branch wins, in the reference's order."""
    v = np.zeros(131, np.float32)
    a = o.a
    v[OPTION_IDS[o.name]] = 1
    v[a["perpetrator"] + 47] = 1
    ch = a.get("choice", None)
    if "target" in a:
        v[a["target"] + 53] = 1
    elif "choice" in a and isinstance(ch, str) and ch in ROLE_IDS:
        v[ROLE_IDS[ch] + 60] = 1
    elif "choice" in a and isinstance(ch, str):
        v[NAMED[ch] + 76] = 1
    elif "choice" in a and isinstance(ch, O.Cd):
        v[O.ctype(ch.code) + 89] = 1
    elif "choice" in a and isinstance(ch, list):
        for c in ch:
            v[O.ctype(c.code) + 89] = 1
    elif "built_card" in a:
        v[O.ctype(a["built_card"].code) + 89] = 1
    elif "real_target" in a:
        v[a["real_target"] + 60] = 1
    elif "fake_targets" in a:
        v[a["fake_targets"][0] + 68] = 1
        v[a["fake_targets"][1] + 68] = 1
    elif "fake_target" in a:
        v[a["fake_target"] + 68] = 1
    elif "replica" in a:
        v[129] = a["replica"]
    elif "gold_or_card_combination" in a:
        v[130] = list(a["gold_or_card_combination"]).count("card")
    elif "chosen_card" in a:
        v[O.ctype(a["chosen_card"].code) + 89] = 1
    elif "cards_to_give" in a:
        for c in a["cards_to_give"]:
            v[O.ctype(c.code) + 89] = O.ctype(c.code)      # the type id itself, not 1 (option.py:113)
    return v
