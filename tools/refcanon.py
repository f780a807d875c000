"""Canonical (address-free) serialisation of the *reference's* Python objects.

This module runs only in the build container, where `/root/reference` is
mounted; it is used by `tools/gen_golden.py` to turn reference games and
option lists into the canonical form that `citadels_self_play_amd.canon`
produces from packed engine state.  Both sides must agree byte for byte, so
the format is spelled out here once:

game  -> dict (see `canon_game`), hashed as sha1(json.dumps(d, sort_keys=True,
         separators=(",", ":")))[:16]
option-> "name|key=value;key=value" with keys sorted; values rendered by
         `canon_val` (cards as `c<code>`, booleans `T`/`F`, lists `[..]`,
         dicts `{k:v,..}` in insertion order, GameState `GS(state,pid,adm,intr)`).

Card codes: type_ID for every card whose suit is the table suit; a Magic
School (type 25) re-suited by `carry_out_magic_school`
(option_functions.py:147-153) is 40 + suit index.
"""
import hashlib
import json

SUITS = ["trade", "war", "religion", "lord", "unique"]
ROLE_NAMES = [
    "Assassin", "Witch", "Magistrate",
    "Thief", "Spy", "Blackmailer",
    "Magician", "Wizard", "Seer",
    "King", "Emperor", "Patrician",
    "Bishop", "Abbot", "Cardinal",
    "Merchant", "Alchemist", "Trader",
    "Architect", "Navigator", "Scholar",
    "Warlord", "Diplomat", "Marshal",
    "Queen", "Artist", "Tax Collector",
]
ADM_TOKENS = ["begged", "character_ability", "lab", "magic_school", "museum",
              "non_trade_building", "smithy", "take_gold", "trade_building"]
OPTION_NAMES = [
    "role_pick", "gold_or_card", "which_card_to_keep", "blackmail_response",
    "reveal_blackmail_as_blackmailer", "reveal_warrant_as_magistrate", "build", "empty_option",
    "finish_round", "ghost_town_color_choice", "smithy_choice", "laboratory_choice",
    "magic_school_choice", "weapon_storage_choice", "lighthouse_choice", "museum_choice",
    "graveyard", "take_gold_for_war", "assassination", "magistrate_warrant", "bewitching",
    "steal", "blackmail", "spy", "magic_hand_change", "discard_and_draw", "look_at_hand",
    "take_from_hand", "seer", "give_back_card", "take_crown_king", "give_crown",
    "take_crown_pat", "bishop", "cardinal_exchange", "abbot_gold_or_card", "abbot_beg",
    "merchant", "alchemist", "trader", "architect", "navigator_gold_card", "scholar",
    "scholar_card_pick", "warlord_desctruction", "marshal_steal", "diplomat_exchange",
]


def card_code(c):
    if c.type_ID == 25 and c.suit != "unique":
        return 40 + SUITS.index(c.suit)
    return int(c.type_ID)


def codes(cards):
    return [card_code(c) for c in cards]


def role_idx(name):
    if name is None:
        return -1
    if name == "Bewitched":
        return 27
    return ROLE_NAMES.index(name)


def adm_counts(adm):
    out = [0] * len(ADM_TOKENS)
    for t in adm:
        out[ADM_TOKENS.index(t)] += 1
    return out


_WB = {None: 0, "Real": 1, "Fake": 2}


def _rk_mask(g, rk):
    m = 0
    last = -2
    for k, v in rk.possible_roles.items():
        assert k > last, "possible_roles not ascending"
        last = k
        if k == -1:
            assert v == "Bewitched"
        else:
            assert v == g.roles[k], (k, v)
        m |= 1 << (k + 1)
    return m


def canon_game(g):
    d = {}
    d["deck"] = codes(g.deck.cards)
    d["discard"] = codes(g.discard_deck.cards)
    d["used_cards"] = codes(g.used_cards.cards)
    players = []
    for i, p in enumerate(g.players):
        assert p.id == i
        kr = []
        for j, rk in enumerate(p.known_roles):
            assert rk.player_id == j
            kr.append([_rk_mask(g, rk), int(rk.confirmed)])
        kh = [[int(h.player_id), int(h.confidence), int(bool(h.wizard)), int(bool(h.used)),
               codes(h.hand.cards)] for h in p.known_hands]
        players.append({
            "hand": codes(p.hand.cards), "build": codes(p.buildings.cards),
            "jd": codes(p.just_drawn_cards.cards), "museum": codes(p.museum_cards.cards),
            "gold": int(p.gold), "role": role_idx(p.role), "replicas": int(p.replicas),
            "crown": int(bool(p.crown)), "lh": int(bool(p.can_use_lighthouse)),
            "f7": int(bool(p.first_to_7)), "witch": int(bool(p.witch)),
            "kr": kr, "kh": kh,
        })
    d["players"] = players
    d["roles"] = [role_idx(g.roles[r]) for r in range(8)]
    d["rtc"] = [int(k) for k in g.roles_to_choose_from.keys()] if hasattr(g, "roles_to_choose_from") else None
    d["used_roles"] = [int(r) for r in g.used_roles] if hasattr(g, "used_roles") else None
    d["turn"] = [int(x) for x in g.turn_orders_for_roles]
    d["rp"] = [[int(bool(rp.dead)), _WB[rp.warrant], int(bool(rp.possessed)), int(bool(rp.robbed)),
                _WB[rp.blackmail]] for _, rp in sorted(g.role_properties.items())]
    gs = g.gamestate
    d["gs"] = [gs.state, -1 if gs.player_id is None else gs.player_id,
               adm_counts(gs.already_done_moves), int(bool(gs.interruption))]
    nx = gs.next_gamestate
    if nx is None:
        d["next"] = None
    else:
        d["next"] = [nx.state, nx.player_id, adm_counts(nx.already_done_moves),
                     int(bool(nx.interruption)),
                     int(nx.already_done_moves is gs.already_done_moves),
                     int(nx.next_gamestate is not None)]
    d["ending"] = int(bool(g.ending))
    d["terminal"] = int(bool(g.terminal))
    rw = [float(x) for x in g.rewards]
    d["winner"] = rw.index(1.0) if 1.0 in rw else -1
    assert sum(rw) == (1.0 if d["winner"] >= 0 else 0.0)
    d["points"] = [int(x) for x in g.points] if hasattr(g, "points") else None
    d["warrant"] = card_code(g.warrant_building) if hasattr(g, "warrant_building") else None
    d["seer_from"] = [int(x) for x in g.seer_taken_card_from] if hasattr(g, "seer_taken_card_from") else None
    if hasattr(g, "seven_drawn_cards"):
        s = g.seven_drawn_cards
        d["seven"] = ["list", list(s)] if isinstance(s, list) else ["deck", codes(s.cards)]
    else:
        d["seven"] = None
    return d


def hash_obj(d):
    return hashlib.sha1(json.dumps(d, sort_keys=True, separators=(",", ":")).encode()).hexdigest()[:16]


def canon_val(v):
    # Imports are local so the module can be read without the reference present.
    from game.deck import Card, Deck
    from game.helper_classes import GameState
    if isinstance(v, bool):
        return "T" if v else "F"
    if isinstance(v, Card):
        return "c%d" % card_code(v)
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(canon_val(x) for x in v) + "]"
    if isinstance(v, dict):
        return "{" + ",".join("%s:%s" % (canon_val(k), canon_val(x)) for k, x in v.items()) + "}"
    if isinstance(v, GameState):
        return "GS(%d,%d,%s,%s)" % (v.state, v.player_id,
                                    "".join(str(c) for c in adm_counts(v.already_done_moves)),
                                    "T" if v.interruption else "F")
    if isinstance(v, Deck):
        return "D" + canon_val(v.cards)
    if v is None:
        return "N"
    if isinstance(v, (int,)):
        return str(int(v))
    if isinstance(v, str):
        return v
    raise TypeError(type(v))


def canon_option(o):
    return o.name + "|" + ";".join("%s=%s" % (k, canon_val(o.attributes[k])) for k in sorted(o.attributes))


def hash_options(opts):
    return hashlib.sha1("\n".join(canon_option(o) for o in opts).encode()).hexdigest()[:16]
