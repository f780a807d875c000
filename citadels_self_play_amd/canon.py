"""Canonical, address-free form of a packed game row and of an option
descriptor.  The format is the one tools/refcanon.py produces from the
reference's Python objects, so a packed row can be compared field by field
with the reference's own state (golden fixtures)."""
import hashlib
import json

from .layout import NO_CARD, ROLE_NONE, CitGame
from .rules import ADM_TOKENS, OPTION_NAMES, ROLE_NAMES, SUITS


def _lst(arr, n):
    return [int(arr[i]) for i in range(n)]


def deck_list(g):
    return [int(g.deck[(g.deck_head + i) & 127]) for i in range(g.n_deck)]


def kh_entries(g):
    """[(owner, target, conf, wizard, used, cards)] in list order."""
    out, off = [], 0
    for e in range(g.n_kh):
        k = g.kh[e]
        out.append((k.owner, k.target, k.conf_flags & 15, (k.conf_flags >> 4) & 1, (k.conf_flags >> 5) & 1,
                    [int(c) for c in g.kh_pool[off:off + k.len]]))
        off += k.len
    return out


def canon_game(g: CitGame):
    d = {"deck": deck_list(g), "discard": _lst(g.discard, g.n_discard), "used_cards": _lst(g.used_cards, g.n_used_cards)}
    khs = kh_entries(g)
    players = []
    for i in range(6):
        p = g.pl[i]
        players.append({
            "hand": _lst(p.hand, p.n_hand), "build": _lst(p.build, p.n_build), "jd": _lst(p.jd, p.n_jd),
            "museum": _lst(p.museum, p.n_museum), "gold": int(p.gold),
            "role": -1 if p.role == ROLE_NONE else int(p.role), "replicas": int(p.replicas),
            "crown": p.flags & 1, "lh": (p.flags >> 1) & 1, "f7": (p.flags >> 2) & 1, "witch": (p.flags >> 3) & 1,
            "kr": [[int(p.kr[j]) & 0x1FF, (int(p.kr[j]) >> 15) & 1] for j in range(6)],
            "kh": [[t, c, w, u, cards] for (o, t, c, w, u, cards) in khs if o == i],
        })
    d["players"] = players
    d["roles"] = _lst(g.roles, 8)
    d["rtc"] = [r for r in range(8) if (g.rtc >> r) & 1]
    d["used_roles"] = None if g.n_used_roles == 255 else [int(x) for x in g.used_roles[:g.n_used_roles]]
    d["turn"] = _lst(g.turn, 6)
    d["rp"] = [[v & 1, (v >> 1) & 3, (v >> 3) & 1, (v >> 4) & 1, (v >> 5) & 3] for v in g.rp]
    d["gs"] = [int(g.gs_state), int(g.gs_pid), _lst(g.gs_adm, 9), int(g.gs_intr)]
    d["next"] = None if not g.nx_valid else [int(g.nx_state), int(g.nx_pid), _lst(g.nx_adm, 9), int(g.nx_intr),
                                             int(g.nx_alias), int(g.nx_hasnext)]
    d["ending"] = int(g.ending)
    d["terminal"] = int(g.terminal)
    d["winner"] = int(g.winner)
    d["points"] = [int(x) for x in g.points] if g.has_points else None
    d["warrant"] = None if g.warrant == NO_CARD else int(g.warrant)
    d["seer_from"] = None if g.n_seer == 255 else _lst(g.seer_from, g.n_seer)
    d["seven"] = [None, ["deck", _lst(g.seven, g.n_seven)], ["list", []]][g.seven_kind]
    return d


def hash_obj(d):
    return hashlib.sha1(json.dumps(d, sort_keys=True, separators=(",", ":")).encode()).hexdigest()[:16]


def _c(code):
    return "c%d" % code


def _gs(state, pid, adm, intr):
    return "GS(%d,%d,%s,%s)" % (state, pid, "".join(str(int(x)) for x in adm), "T" if intr else "F")


def option_attrs(o, g: CitGame):
    """The reference's attribute dict for descriptor `o` generated on game `g`,
    rendered as canonical strings (see tools/refcanon.canon_val)."""
    n = OPTION_NAMES[o.name]
    p = o.perp
    a = {"perpetrator": str(p)}
    T = "T"
    F = "F"
    if n == "role_pick":
        a["choice"] = ROLE_NAMES[g.roles[o.a]]
    elif n == "gold_or_card":
        a["choice"] = ["gold", "card"][o.a]
    elif n == "which_card_to_keep":
        a["choice"] = "[" + ",".join(_c(c) for c in ([o.a] if o.b == NO_CARD else [o.a, o.b])) + "]"
    elif n == "blackmail_response":
        a["choice"] = ["pay", "not_pay"][o.a]
    elif n in ("reveal_blackmail_as_blackmailer", "reveal_warrant_as_magistrate"):
        a["choice"] = ["reveal", "not_reveal"][o.a]
        a["target"] = str(o.target)
    elif n == "build":
        a["built_card"] = _c(o.a)
        a["replica"] = str(_s8(o.c))
    elif n == "empty_option":
        if o.a == 0:
            a["next_gamestate"] = _gs(5, p, [0] * 9, False)
        else:
            a["next_gamestate"] = _gs(g.nx_state, g.nx_pid, g.nx_adm, g.nx_intr)
    elif n == "finish_round":
        a["next_witch"] = T if o.flags & 1 else F
        a["crown"] = T if o.flags & 2 else F
    elif n in ("laboratory_choice", "lighthouse_choice", "museum_choice"):
        a["choice"] = _c(o.a)
    elif n == "magic_school_choice":
        a["choice"] = SUITS[o.a]
    elif n in ("weapon_storage_choice", "warlord_desctruction", "marshal_steal"):
        a["target"] = str(o.target)
        a["choice"] = _c(o.a)
    elif n in ("assassination", "bewitching", "steal"):
        a["choice"] = str(o.a)
    elif n == "magistrate_warrant":
        a["real_target"] = str(o.a)
        a["fake_targets"] = "[%d,%d]" % (o.b, o.c)
    elif n == "blackmail":
        a["real_target"] = str(o.a)
        a["fake_target"] = str(o.b)
    elif n == "spy":
        a["target"] = str(o.target)
        a["suit"] = SUITS[o.a]
    elif n in ("magic_hand_change", "look_at_hand"):
        a["target"] = str(o.target)
    elif n == "discard_and_draw":
        hand = g.pl[p].hand
        a["cards"] = "[" + ",".join(_c(hand[i]) for i in range(64) if (o.x >> i) & 1) + "]"
    elif n == "take_from_hand":
        a["target"] = str(o.target)
        if o.flags & 1:
            a["built_card"] = _c(o.a)
            a["build"] = T
            a["replica"] = str(_s8(o.c))
        else:
            a["card"] = _c(o.a)
            a["build"] = F
    elif n == "give_back_card":
        a["card_handouts"] = "{" + ",".join("%d:%s" % (g.seer_from[i], _c((o.x >> (8 * i)) & 0xFF))
                                            for i in range(o.b)) + "}"
    elif n == "give_crown":
        a["target"] = str(o.target)
        a["gold_or_card"] = ["card", "gold", "nothing"][o.a]
    elif n == "cardinal_exchange":
        hand = g.pl[p].hand
        a["target"] = str(o.target)
        a["built_card"] = _c(o.a)
        a["cards_to_give"] = "[" + ",".join(_c(hand[i]) for i in range(64) if (o.x >> i) & 1) + "]"
        a["replica"] = str(_s8(o.c))
        a["factory"] = T if o.flags & 1 else F
    elif n == "abbot_gold_or_card":
        a["gold_or_card_combination"] = "[" + ",".join(["gold"] * (o.a - o.b) + ["card"] * o.b) + "]"
    elif n == "navigator_gold_card":
        a["choice"] = ["4gold", "4card"][o.a]
    elif n == "scholar_card_pick":
        a["choice"] = _c(o.a)
        a["chosen_card"] = _c(o.a)
        a["unchosen_cards"] = "D[" + ",".join(_c(g.seven[i]) for i in range(g.n_seven)) + "]"
    elif n == "diplomat_exchange":
        a["target"] = str(o.target)
        a["choice"] = _c(o.a)
        a["give"] = _c(o.b)
        a["money_owed"] = str(o.c)
    return n, a


def _s8(v):
    return v - 256 if v >= 128 else v


def canon_option(o, g: CitGame):
    n, a = option_attrs(o, g)
    return n + "|" + ";".join("%s=%s" % (k, a[k]) for k in sorted(a))


def hash_options(opts, g: CitGame):
    return hashlib.sha1("\n".join(canon_option(o, g) for o in opts).encode()).hexdigest()[:16]
