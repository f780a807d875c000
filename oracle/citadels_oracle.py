"""CPU ORACLE — test infrastructure only.

A plain-Python restatement of the reference rules engine (davpat108/
CITADELS_self_play, `game/*.py`) used as the *checker* for the HIP engine.
Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg
may import this module; the product path (citadels_self_play_amd) never does.

Pinned against tests/golden/traj_*.json.gz (generated from the reference
itself by tools/gen_golden.py) by tests/test_oracle_golden.py.

Data model (not the reference's object graph): cards are small ints
(type_ID, or 40+suit for a re-suited Magic School), roles are indices into
ROLE_NAMES, a game is an `OGame` whose lists mirror the reference's containers
in order.  Randomness: one `random.Random(seed)` per game stands in for the
reference's module-global CPython stream (same MT19937 + `_randbelow`
algorithm), so a lane of the engine seeded with `s` must equal the reference
run after `random.seed(s)`.
"""
import itertools
import random as _random

# ---- rules tables (game/config.py:2-121) ----------------------------------
SUITS = ["trade", "war", "religion", "lord", "unique"]
TYPE_COST = [1, 2, 4, 2, 5, 3, 2, 3, 5, 1, 2, 3, 1, 4, 3, 5,
             5, 3, 6, 2, 6, 5, 5, 6, 5, 6, 6, 3, 6, 3, 5, 5, 6, 5, 4, 6, 5, 4, 6, 5]
TYPE_SUIT = [0] * 6 + [1] * 4 + [2] * 3 + [3] * 3 + [4] * 24
# building_cards order (config.py:2-52): (type, multiplicity)
BASE_DECK = [t for t, n in [(0, 5), (1, 3), (2, 3), (3, 4), (4, 2), (5, 3), (6, 3), (7, 3), (8, 2),
                            (9, 3), (10, 3), (11, 3), (12, 3), (13, 4), (14, 5), (15, 3)] for _ in range(n)]
UNIQUE_DECK = [16, 17, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34,
               35, 36, 37, 39]                                          # config.py:55-79
ROLE_NAMES = ["Assassin", "Witch", "Magistrate", "Thief", "Spy", "Blackmailer",
              "Magician", "Wizard", "Seer", "King", "Emperor", "Patrician",
              "Bishop", "Abbot", "Cardinal", "Merchant", "Alchemist", "Trader",
              "Architect", "Navigator", "Scholar", "Warlord", "Diplomat", "Marshal",
              "Queen", "Artist", "Tax Collector"]                       # config.py:82-91
BEWITCHED = 27
R = {n: i for i, n in enumerate(ROLE_NAMES)}


def rank(role):
    """role_to_role_id (config.py:93-121); raises KeyError for None like the reference."""
    if role == BEWITCHED:
        return -1
    if role is None or role < 0:
        raise KeyError(None)
    return role // 3


def rprop(g, role):
    """game.role_properties[role_to_role_id[role]]: the dict has keys 0..7 only,
    so a Bewitched (-1) lookup is a KeyError in the reference (game.py:525-534)."""
    r = rank(role)
    if r < 0:
        raise KeyError(r)
    return g.rp[r]


def ctype(c):
    return 25 if c >= 40 else c


def csuit(c):
    return c - 40 if c >= 40 else TYPE_SUIT[c]


def ccost(c):
    return TYPE_COST[ctype(c)]


def has(cards, t):
    return any(ctype(c) == t for c in cards)


def take_like(cards, c):
    """Deck.get_a_card_like_it (deck.py:49-55): first card of the same type, or the argument."""
    t = ctype(c)
    for i, x in enumerate(cards):
        if ctype(x) == t:
            del cards[i]
            return x
    return c


def draw(cards):
    """Deck.draw_card (deck.py:57-60): None stands for the "Deck Empty" sentinel."""
    return cards.pop(0) if cards else None


def put(cards, c):
    """Deck.add_card (deck.py:62-67): non-cards are dropped."""
    if c is not None:
        cards.append(c)


# ---- option values ---------------------------------------------------------
class Cd:
    """A card-valued option attribute; compares by type like Card.__eq__ (deck.py:13-16)."""
    __slots__ = ("code",)

    def __init__(self, code):
        self.code = code

    def __eq__(self, o):
        return isinstance(o, Cd) and ctype(o.code) == ctype(self.code)

    def __hash__(self):
        return ctype(self.code)


class DeckRef:
    """A Deck-valued attribute (scholar `unchosen_cards`): shares its list like copy(Deck)."""
    __slots__ = ("cards",)

    def __init__(self, cards):
        self.cards = cards

    def __eq__(self, o):
        return isinstance(o, DeckRef) and [ctype(c) for c in o.cards] == [ctype(c) for c in self.cards]


class Opt:
    __slots__ = ("name", "a")

    def __init__(self, name, **a):
        self.name = name
        self.a = a

    def __eq__(self, o):
        return self.name == o.name and self.a == o.a

    def canon(self):
        return self.name + "|" + ";".join("%s=%s" % (k, cval(self.a[k])) for k in sorted(self.a))


ADM = ["begged", "character_ability", "lab", "magic_school", "museum",
       "non_trade_building", "smithy", "take_gold", "trade_building"]


def cval(v):
    if isinstance(v, bool):
        return "T" if v else "F"
    if isinstance(v, Cd):
        return "c%d" % v.code
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(cval(x) for x in v) + "]"
    if isinstance(v, dict):
        return "{" + ",".join("%s:%s" % (cval(k), cval(x)) for k, x in v.items()) + "}"
    if isinstance(v, OGS):
        return "GS(%d,%d,%s,%s)" % (v.state, v.pid, "".join(str(v.adm.count(t)) for t in ADM),
                                    "T" if v.intr else "F")
    if isinstance(v, DeckRef):
        return "D[" + ",".join("c%d" % c for c in v.cards) + "]"
    if v is None:
        return "N"
    return str(v)


# ---- state -----------------------------------------------------------------
class OGS:
    """GameState (helper_classes.py:16-34); `adm` is a list object so the
    reference's list aliasing (option_functions.py:127,310,341,496) is kept."""
    __slots__ = ("state", "pid", "adm", "next", "intr")

    def __init__(self, state=0, pid=None, adm=None, nxt=None, intr=False):
        self.state, self.pid = state, pid
        self.adm = adm if adm is not None else []
        self.next, self.intr = nxt, intr


class OKH:
    """HandKnowledge (helper_classes.py:37-43)."""
    __slots__ = ("pid", "conf", "cards", "wizard", "used")

    def __init__(self, pid, cards, conf, wizard=False):
        self.pid, self.cards, self.conf, self.wizard, self.used = pid, cards, conf, wizard, False


class OPlayer:
    """Agent state (agent.py:10-29).  `kr[j]` = [mask over role ids -1..7 (bit id+1), confirmed]."""

    def __init__(self, pid):
        self.id = pid
        self.hand, self.build, self.jd, self.museum = [], [], [], []
        self.role = None
        self.replicas = False
        self.lh = False
        self.crown = False
        self.gold = 2
        self.kh = []
        self.kr = [[0, False] for _ in range(6)]
        self.f7 = False
        self.witch = False


class OGame:
    def __init__(self, seed, preset=True, rng=None):
        """Game.__init__ + set_preset / set_random_game + set_initial_variables (game.py:17-24,420-540).
        `rng` continues an existing stream instead of seeding a new one."""
        self.rng = _random.Random(seed) if rng is None else rng
        if preset:
            deck = BASE_DECK + UNIQUE_DECK
        else:
            deck = BASE_DECK + self.rng.sample(UNIQUE_DECK, 14)
        deck = list(deck)
        self.rng.shuffle(deck)
        self.deck = deck
        self.used_cards = list(deck)
        self.discard = []
        self.players = [OPlayer(i) for i in range(6)]
        if preset:
            hands = [[0, 0, 16, 17, 18, 19], [1, 1, 20, 21, 22, 23], [2, 3, 24, 25, 26, 27],
                     [3, 4, 28, 29, 30, 31], [4, 0, 32, 33, 34, 35], [0, 1, 36, 37, 39, 0]]
            for p, h in zip(self.players, hands):
                for t in h:
                    put(p.hand, take_like(self.deck, t))
            self.players[3].crown = True
            self.roles = [R[n] for n in ["Witch", "Spy", "Wizard", "King", "Abbot", "Alchemist",
                                         "Navigator", "Warlord"]]
            self.turn = [0, 1, 2, 3, 4, 5]
        else:
            for _ in range(4):
                for p in self.players:
                    put(p.hand, draw(self.deck))
            self.roles = [r * 3 + self.rng.choice([0, 1, 2]) for r in range(8)]
            self.turn = [0, 1, 2, 3, 4, 5]
            self.rng.shuffle(self.turn)
            crown = self.rng.randint(0, 5)
            self.players[crown].crown = True
        # set_initial_variables (game.py:522-540)
        self.rp = [[False, None, False, False, None] for _ in range(8)]  # dead, warrant, possessed, robbed, blackmail
        self.gs = OGS()
        self.ending = False
        self.terminal = False
        self.winner = -1
        self.points = None
        self.warrant = None
        self.seer_from = None
        self.seven = None            # None | DeckRef (a Deck) | [] (plain list after scholar put-back)
        self.rtc = None
        self.used_roles = None

    # -- helpers ------------------------------------------------------------
    def cur(self):
        return self.players[self.gs.pid]

    def holder(self, rid):
        """get_player_from_role_id (game.py:403-412)."""
        for p in self.players:
            if (rid == -1 and p.role == BEWITCHED) or (rid != -1 and p.role == self.roles[rid]):
                return p
        return None

    def role_mask_name(self, rid):
        return BEWITCHED if rid == -1 else self.roles[rid]

    # -- round flow ---------------------------------------------------------
    def setup_round(self):
        """game.py:144-171."""
        for rp in self.rp:
            rp[:] = [False, None, False, False, None]
        self.used_roles = []
        pool = list(range(8))
        self.rng.shuffle(pool)
        pool.pop()
        self.rtc = sorted(pool)
        c = next((p.id for p in self.players if p.crown), None)
        self.turn = self.turn[c:] + self.turn[:c]
        self.gs = OGS(0, self.turn[0])
        for p in self.players:
            # agent.py:100-114
            keep = []
            for h in p.kh:
                h.conf -= 1
                h.wizard = False
                h.used = False
                if h.conf != 0:
                    keep.append(h)
            p.kh = keep
            for k in p.kr:
                k[0], k[1] = 0, False

    def refresh_used_roles(self):
        """game.py:349-357."""
        self.used_roles = sorted(rank(p.role) for p in self.players)

    def next_player(self, current=None):
        """setup_next_player (game.py:391-401)."""
        if self.gs.state == 0:
            self.refresh_used_roles()
            self.gs.state = 1
            self.gs.pid = self.holder(self.used_roles[0]).id
        elif current is not None:
            self.gs.state = 1
            i = self.used_roles.index(rank(self.players[current].role))
            self.gs.pid = self.holder(self.used_roles[i + 1]).id
            self.gs.adm = []
        else:
            raise Exception("No current player and not in rolepick state")

    def check_ending(self):
        """game.py:359-368 + Agent.count_points (agent.py:116-143)."""
        if not self.ending:
            return None
        pts = [count_points(p) for p in self.players]
        self.points = pts
        self.terminal = True
        self.winner = pts.index(max(pts))
        return self.winner

    def is_last_round(self):
        """game.py:173-181."""
        if not self.ending:
            for p in self.players:
                if len(p.build) == 7:
                    self.ending = True
                    p.f7 = True

    # -- get_options (agent.py:50-83) -------------------------------------------
    def get_options(self):
        a = self.cur()
        st = self.gs.state
        if st == 0:
            return [Opt("role_pick", perpetrator=a.id, choice=ROLE_NAMES[self.roles[r]]) for r in self.rtc]
        crown = a.role in (R["King"], R["Patrician"])
        if a.role == BEWITCHED or not rprop(self, a.role)[0]:
            if st == 1:
                return gen_gold_or_card(self, a)
            if st == 2:
                return gen_keep(self, a)
            if st == 3:
                return gen_blackmail_response(self, a)
            if st == 4:
                return [Opt("reveal_blackmail_as_blackmailer", choice=c, perpetrator=a.id, target=self.gs.next.pid)
                        for c in ("reveal", "not_reveal")]
            if st == 6:
                if a.gold > 0:
                    return [Opt("graveyard", perpetrator=a.id)]
                return [Opt("empty_option", perpetrator=a.id, next_gamestate=self.gs.next)]
            if st == 7:
                return [Opt("reveal_warrant_as_magistrate", choice=c, perpetrator=a.id, target=self.gs.next.pid)
                        for c in ("reveal", "not_reveal")]
            if a.role == R["Witch"]:
                return [Opt("bewitching", perpetrator=a.id, choice=r) for r in range(1, 8)]
            if not rprop(self, a.role)[2]:
                if st == 5:
                    return gen_main(self, a)
                if st == 8:
                    return gen_seer_give_back(self, a)
                if st == 9:
                    return gen_scholar_pick(self, a)
                if st == 10:
                    return gen_wizard_take(self, a)
                return None
            return [Opt("finish_round", perpetrator=a.id, next_witch=True, crown=crown)]
        if a.role == R["Emperor"] and "character_ability" not in self.gs.adm:
            return gen_emperor(self, a, dead=True)
        return [Opt("finish_round", perpetrator=a.id, next_witch=False, crown=crown)]

    def carry_out(self, o):
        """option.carry_out (option.py:118-122): transition + is_last_round; returns winner id or None."""
        w = TRANSITIONS[o.name](self, o)
        self.is_last_round()
        return w


def count_points(p):
    """agent.py:116-143."""
    pts = 0
    well = has(p.build, 31)
    for c in p.build:
        pts += ccost(c)
        if ctype(c) in (18, 23):
            pts += 2
        if well and csuit(c) == 4:
            pts += 1
    if len(p.build) >= 7:
        pts += 2
    if p.f7:
        pts += 4
    pts += len(p.museum)
    if has(p.build, 37):
        pts += p.gold
    if has(p.build, 39):
        pts += len(p.hand)
    return pts


# ---- option generators (game/agent_functions.py) ---------------------------
def gen_gold_or_card(g, a):
    """agent_functions.py:16-17."""
    if len(g.deck) > 1:
        return [Opt("gold_or_card", perpetrator=a.id, choice="gold"), Opt("gold_or_card", perpetrator=a.id, choice="card")]
    return [Opt("gold_or_card", perpetrator=a.id, choice="gold")]


def gen_keep(g, a):
    """agent_functions.py:19-33."""
    if has(a.build, 20):
        return [Opt("which_card_to_keep", perpetrator=a.id, choice=(Cd(x), Cd(y)))
                for x, y in itertools.combinations(a.jd, 2)]
    out, seen = [], set()
    for c in a.jd:
        if ctype(c) not in seen:
            seen.add(ctype(c))
            out.append(Opt("which_card_to_keep", perpetrator=a.id, choice=[Cd(c)]))
    return out


def gen_blackmail_response(g, a):
    """agent_functions.py:35-38."""
    if rprop(g, a.role)[4]:
        return [Opt("blackmail_response", choice=c, perpetrator=a.id) for c in ("pay", "not_pay")]
    return [Opt("empty_option", perpetrator=a.id, next_gamestate=OGS(5, a.id))]


def build_limit(role):
    """agent.py:87-98."""
    return {R["Architect"]: 3, R["Scholar"]: 2, R["Bishop"]: 0, R["Navigator"]: 0}.get(role, 1)


def gen_builds(g, a, out):
    """get_builds / build_options (agent_functions.py:108-130)."""
    adm = g.gs.adm
    lim = build_limit(a.role)
    n = adm.count("non_trade_building") if a.role == R["Trader"] else \
        adm.count("trade_building") + adm.count("non_trade_building")
    if n >= lim:
        return
    factory = has(a.build, 35)
    for c in a.hand:
        cost = ccost(c) + (1 if factory and csuit(c) == 4 else 0)
        rep = 0
        if has(a.build, ctype(c)) and not a.replicas:
            rep = a.replicas + 1
        o = Opt("build", perpetrator=a.id, built_card=Cd(c), replica=rep)
        if cost <= a.gold and o not in out:
            out.append(o)


def gen_character(g, a):
    """character_options (agent_functions.py:156-209)."""
    out = []
    adm = g.gs.adm
    if "character_ability" not in adm:
        fn = ROLE_GEN.get(ROLE_NAMES[a.role] if 0 <= a.role < 27 else None)
        if fn is not None:
            out = fn(g, a)
    if a.role == R["Abbot"] and "begged" not in adm:
        out = out + [Opt("abbot_beg", perpetrator=a.id)]
    if a.role in (R["Warlord"], R["Marshal"], R["Diplomat"]) and "take_gold" not in adm:
        out = out + [Opt("take_gold_for_war", perpetrator=a.id)]
    return out


def gen_main(g, a):
    """main_round_options (agent_functions.py:133-147)."""
    out = []
    gen_builds(g, a, out)
    out += gen_character(g, a)
    adm = g.gs.adm
    if has(a.build, 21) and a.gold >= 2 and "smithy" not in adm:                     # :54-57
        out.append(Opt("smithy_choice", perpetrator=a.id))
    if has(a.build, 22) and "lab" not in adm:                                         # :59-65
        out += [Opt("laboratory_choice", perpetrator=a.id, choice=Cd(c)) for c in a.hand]
    if "magic_school" not in adm and has(a.build, 25):                                # :67-74
        out += [Opt("magic_school_choice", choice=s, perpetrator=a.id) for s in SUITS]
    if has(a.build, 27):                                                              # :76-83
        for p in g.players:
            if p.id != a.id:
                out += [Opt("weapon_storage_choice", perpetrator=a.id, target=p.id, choice=Cd(c)) for c in p.build]
    if has(a.build, 29) and a.lh:                                                     # :85-94
        seen = set()
        for c in g.deck:
            if ctype(c) not in seen:
                seen.add(ctype(c))
                out.append(Opt("lighthouse_choice", choice=Cd(c), perpetrator=a.id))
    if has(a.build, 34) and "museum" not in adm:                                      # :96-105
        seen = set()
        for c in a.hand:
            if ctype(c) not in seen:
                seen.add(ctype(c))
                out.append(Opt("museum_choice", choice=Cd(c), perpetrator=a.id))
    out.append(Opt("finish_round", perpetrator=a.id, next_witch=False, crown=False))
    return out


def gen_assassin(g, a):
    return [Opt("assassination", perpetrator=a.id, choice=r) for r in range(1, 8)]          # :213-218


def gen_magistrate(g, a):
    """agent_functions.py:221-234."""
    t = list(range(1, 8))
    return [Opt("magistrate_warrant", perpetrator=a.id, real_target=r, fake_targets=list(f))
            for r in t for f in itertools.combinations(t, 2) if r not in f]


def gen_thief(g, a):
    return [Opt("steal", perpetrator=a.id, choice=r) for r in range(2, 8)]                  # :246-253


def gen_blackmailer(g, a):
    """agent_functions.py:255-272."""
    t = list(range(2, 8))
    for rid in range(8):
        if g.rp[rid][2]:
            t.remove(rid)
    out = []
    for x, y in itertools.combinations(t, 2):
        out.append(Opt("blackmail", perpetrator=a.id, real_target=x, fake_target=y))
        out.append(Opt("blackmail", perpetrator=a.id, real_target=y, fake_target=x))
    return out


def gen_spy(g, a):
    return [Opt("spy", perpetrator=a.id, target=p.id, suit=s)
            for p in g.players if p.id != a.id for s in SUITS]                               # :274-281


def _stride(n):
    """max(round(n/1e2), 1) with Python's round-half-even (agent_functions.py:293,416)."""
    return max(round(n / 1e2), 1)


def gen_magician(g, a):
    """agent_functions.py:284-296."""
    out = [Opt("magic_hand_change", perpetrator=a.id, target=p.id) for p in g.players if p.id != a.id]
    for r in range(1, len(a.hand) + 1):
        combos = list(itertools.combinations(a.hand, r))
        for i in range(0, len(combos), _stride(len(combos))):
            out.append(Opt("discard_and_draw", perpetrator=a.id, cards=tuple(Cd(c) for c in combos[i])))
    return out


def gen_wizard_look(g, a):
    return [Opt("look_at_hand", perpetrator=a.id, target=p.id)
            for p in g.players if p.id != a.id and p.hand]                                   # :298-308


def gen_wizard_take(g, a):
    """agent_functions.py:310-326 (sticky `replica`)."""
    hk = next((h for h in a.kh if h.conf == 5 and h.pid != -1 and h.wizard), None)
    out = []
    rep = 0
    factory = has(a.build, 35)
    for c in hk.cards:
        o = Opt("take_from_hand", card=Cd(c), build=False, perpetrator=a.id, target=hk.pid)
        if o not in out:
            out.append(o)
        cost = ccost(c) + (1 if factory and csuit(c) == 4 else 0)
        if has(a.build, ctype(c)):
            rep = a.replicas + 1
        o = Opt("take_from_hand", built_card=Cd(c), build=True, perpetrator=a.id, target=hk.pid, replica=rep)
        if cost <= a.gold and o not in out:
            out.append(o)
    if not out:
        return [Opt("empty_option", perpetrator=a.id, next_gamestate=g.gs.next)]
    return out


def gen_seer(g, a):
    return [Opt("seer", perpetrator=a.id)]


def gen_seer_give_back(g, a):
    """seer_give_back_card (agent_functions.py:332-361): consumes the game RNG."""
    out = []
    k = len(g.seer_from)
    for pos in range(k):
        perms = []
        for c in a.hand:
            rest = [x for x in a.hand if ctype(x) != ctype(c)]
            for _ in range(3):
                g.rng.shuffle(rest)
                pm = list(rest[:k - 1])
                pm.insert(pos, c)
                perms.append(tuple(pm))
        for pm in perms:
            out.append(Opt("give_back_card", perpetrator=a.id,
                           card_handouts={pid: Cd(c) for pid, c in zip(g.seer_from, pm)}))
    return out


def gen_king(g, a):
    return [Opt("take_crown_king", perpetrator=a.id)]


def gen_emperor(g, a, dead=False):
    """agent_functions.py:368-382."""
    out = []
    for p in g.players:
        if p.id != a.id:
            if len(p.hand) and not dead:
                out.append(Opt("give_crown", perpetrator=a.id, target=p.id, gold_or_card="card"))
            if p.gold and not dead:
                out.append(Opt("give_crown", perpetrator=a.id, target=p.id, gold_or_card="gold"))
            if (not p.gold and not len(p.hand)) or dead:
                out.append(Opt("give_crown", perpetrator=a.id, target=p.id, gold_or_card="nothing"))
    return out


def gen_patrician(g, a):
    return [Opt("take_crown_pat", perpetrator=a.id)]


def gen_bishop(g, a):
    return [Opt("bishop", perpetrator=a.id)]


def gen_cardinal(g, a):
    """agent_functions.py:393-419."""
    out = []
    factory_owned = has(a.build, 35)
    for p in g.players:
        for c in a.hand:
            cost = ccost(c)
            factory = False
            rep = 0
            if factory_owned and csuit(c) == 4:
                cost += 1
                factory = True
            if has(a.build, ctype(c)) and not a.replicas:
                rep = a.replicas + 1
            if cost <= p.gold:
                k = max(p.gold - cost, 0)
                if len(a.hand) - 1 >= k:
                    others = [x for x in a.hand if ctype(x) != ctype(c)]
                    combos = list(itertools.combinations(others, k))
                    for i in range(0, len(combos), _stride(len(combos))):
                        out.append(Opt("cardinal_exchange", perpetrator=a.id, target=p.id, built_card=Cd(c),
                                       cards_to_give=tuple(Cd(x) for x in combos[i]), replica=rep, factory=factory))
    return out


def gen_abbot(g, a):
    """agent_functions.py:422-430."""
    n = sum(1 for c in a.hand if csuit(c) == 2)
    if n == 0:
        return []
    return [Opt("abbot_gold_or_card", perpetrator=a.id, gold_or_card_combination=list(cmb))
            for cmb in itertools.combinations_with_replacement(["gold", "card"], n)]


def gen_merchant(g, a):
    return [Opt("merchant", perpetrator=a.id)]


def gen_trader(g, a):
    return [Opt("trader", perpetrator=a.id)]


def gen_architect(g, a):
    return [Opt("architect", perpetrator=a.id)]


def gen_navigator(g, a):
    return [Opt("navigator_gold_card", perpetrator=a.id, choice=c) for c in ("4gold", "4card")]


def gen_scholar(g, a):
    return [Opt("scholar", perpetrator=a.id)] if g.deck else []


def gen_scholar_pick(g, a):
    """scholar_give_back_options (agent_functions.py:462-470): every option shares
    the seven-drawn list and the loop removes from it while iterating."""
    lst = g.seven.cards
    out = []
    i = 0
    while i < len(lst):
        c = lst[i]
        take_like(lst, c)
        out.append(Opt("scholar_card_pick", choice=Cd(c), perpetrator=a.id, unchosen_cards=DeckRef(lst),
                       chosen_card=Cd(c)))
        i += 1
    return out


def gen_warlord(g, a):
    """agent_functions.py:473-482."""
    out = []
    for p in g.players:
        if len(p.build) < 7:
            for b in p.build:
                if ccost(b) - 1 <= a.gold and ctype(b) != 17 and p.role != R["Bishop"]:
                    o = Opt("warlord_desctruction", target=p.id, perpetrator=a.id, choice=Cd(b))
                    if o not in out:
                        out.append(o)
    return out


def gen_marshal(g, a):
    """agent_functions.py:484-492."""
    out = []
    for p in g.players:
        if len(p.build) < 7 and p.id != a.id:
            for b in p.build:
                if ccost(b) <= a.gold and ccost(b) <= 3 and not has(a.build, ctype(b)) and ctype(b) != 17 \
                        and p.role != R["Bishop"]:
                    o = Opt("marshal_steal", target=p.id, perpetrator=a.id, choice=Cd(b))
                    if o not in out:
                        out.append(o)
    return out


def gen_diplomat(g, a):
    """agent_functions.py:494-504."""
    out = []
    for p in g.players:
        if len(p.build) < 7 and p.id != a.id:
            for e in p.build:
                for own in a.build:
                    if ccost(e) - ccost(own) <= a.gold and ctype(e) != 17 and p.role != R["Bishop"] \
                            and not has(a.build, ctype(e)):
                        o = Opt("diplomat_exchange", target=p.id, perpetrator=a.id, choice=Cd(e), give=Cd(own),
                                money_owed=abs(ccost(e) - ccost(own)))
                        if o not in out:
                            out.append(o)
    return out


ROLE_GEN = {
    "Assassin": gen_assassin, "Magistrate": gen_magistrate, "Thief": gen_thief, "Blackmailer": gen_blackmailer,
    "Spy": gen_spy, "Magician": gen_magician, "Wizard": gen_wizard_look, "Seer": gen_seer, "King": gen_king,
    "Emperor": gen_emperor, "Patrician": gen_patrician, "Bishop": gen_bishop, "Cardinal": gen_cardinal,
    "Abbot": gen_abbot, "Merchant": gen_merchant, "Alchemist": lambda g, a: [], "Trader": gen_trader,
    "Architect": gen_architect, "Navigator": gen_navigator, "Scholar": gen_scholar, "Warlord": gen_warlord,
    "Marshal": gen_marshal, "Diplomat": gen_diplomat,
}


# ---- transitions (game/option_functions.py) --------------------------------
def reshuffle_if_empty(g):
    """option_functions.py:564-570."""
    if not g.deck and g.discard:
        g.rng.shuffle(g.discard)
        g.deck = list(g.discard)
        g.discard = []


def draw_into(g, dst, n):
    for _ in range(n):
        reshuffle_if_empty(g)
        put(dst, draw(g.deck))


def _at5(g, p, token=None):
    g.gs.state = 5
    g.gs.pid = p
    if token is not None:
        g.gs.adm.append(token)


def confirm_roles(g, q):
    """confirm_role_knowledges (option_functions.py:608-622); the unconfirmed
    filter keeps every entry whose name differs OR whose id is not below the
    revealed rank — for an entry carrying the revealed name that id IS the rank,
    so the filter is a no-op, as in the reference."""
    rq = rank(q.role)
    lower = [r for r in g.used_roles if r < rq]
    bit_q = 1 << (rq + 1)
    for p in g.players:
        for j, k in enumerate(p.kr):
            if j == q.id:
                k[0], k[1] = bit_q, True
            elif not k[1]:
                m = 0
                for rid in range(-1, 8):
                    if k[0] >> (rid + 1) & 1:
                        if g.role_mask_name(rid) != q.role or rid not in lower:
                            m |= 1 << (rid + 1)
                k[0] = m


def move_crown(g, t):
    """option_functions.py:625-631 + troneroom_owner_gold :588-595."""
    for p in g.players:
        if p.crown:
            p.crown = False
            break
    g.players[t].crown = True
    for p in g.players:
        if has(p.build, 32):
            p.gold += 1
            break


def t_role_pick(g, o):
    """option_functions.py:6-30."""
    a = g.players[o.a["perpetrator"]]
    role = R[o.a["choice"]]
    a.role = role
    rk = rank(role)
    g.rtc.remove(rk)
    rtc_mask = sum(1 << (r + 1) for r in g.rtc)
    all_mask = sum(1 << (r + 1) for r in range(8))
    for p in g.players:
        if p is a:
            continue
        if g.turn.index(p.id) < g.turn.index(a.id):
            a.kr[p.id][0] = all_mask & ~rtc_mask & ~(1 << (rk + 1))
        else:
            a.kr[p.id][0] = rtc_mask
    if a.id != g.turn[-1]:
        g.gs.state = 0
        g.gs.pid = g.turn[g.turn.index(a.id) + 1]
    else:
        g.next_player()


def t_gold_or_card(g, o):
    """option_functions.py:33-55."""
    a = g.players[o.a["perpetrator"]]
    confirm_roles(g, a)
    if rprop(g, a.role)[3]:
        g.holder(1).gold += a.gold
        a.gold = 0
    if o.a["choice"] == "gold":
        a.gold += 2
        g.gs.state, g.gs.pid = 3, a.id
    else:
        draw_into(g, a.jd, 3 if has(a.build, 16) else 2)
        g.gs.state, g.gs.pid = 2, a.id


def t_keep(g, o):
    """carry_out_put_back_card (option_functions.py:58-66)."""
    a = g.players[o.a["perpetrator"]]
    for c in o.a["choice"]:
        put(a.hand, take_like(a.jd, c.code))
    for c in a.jd:
        put(g.deck, c)
    a.jd = []
    g.gs.state, g.gs.pid = 3, a.id


def t_empty(g, o):
    g.gs = o.a["next_gamestate"]                                         # option_functions.py:68-69


def t_blackmail_response(g, o):
    """option_functions.py:71-82."""
    a = g.players[o.a["perpetrator"]]
    if o.a["choice"] == "pay":
        half = int(a.gold / 2)
        g.holder(1).gold += half
        a.gold -= int(a.gold / 2)
        _at5(g, a.id)
    else:
        g.gs.state = 4
        g.gs.pid = g.holder(1).id
        g.gs.intr = True
        g.gs.next = OGS(5, a.id)


def t_reveal_blackmail(g, o):
    """option_functions.py:85-92."""
    a, t = g.players[o.a["perpetrator"]], g.players[o.a["target"]]
    if o.a["choice"] == "reveal" and rprop(g, t.role)[4] == "Real":
        a.gold += t.gold
        t.gold = 0
        for rp in g.rp:
            rp[4] = None
    g.gs = g.gs.next


def t_reveal_warrant(g, o):
    """option_functions.py:94-100."""
    a, t = g.players[o.a["perpetrator"]], g.players[o.a["target"]]
    if o.a["choice"] == "reveal" and rprop(g, t.role)[1] == "Real":
        put(a.build, take_like(t.build, g.warrant))
        t.gold += ccost(g.warrant)
        for rp in g.rp:
            rp[1] = None
    g.gs = g.gs.next


def t_build(g, o):
    """carry_out_building (option_functions.py:102-127)."""
    a = g.players[o.a["perpetrator"]]
    card = o.a["built_card"].code
    put(a.build, take_like(a.hand, card))
    if a.role != R["Alchemist"]:
        a.gold -= ccost(card)
    if o.a["replica"]:
        a.replicas = o.a["replica"]
    g.gs.adm.append("trade_building" if csuit(card) == 0 else "non_trade_building")
    if ctype(card) == 29:
        a.lh = True
    if rprop(g, a.role)[1] is None:
        _at5(g, a.id)
    else:
        g.warrant = card
        g.gs.state = 7
        g.gs.pid = g.holder(0).id
        g.gs.intr = True
        g.gs.next = OGS(5, a.id, g.gs.adm)


def t_smithy(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :131-138
    a.gold -= 2
    draw_into(g, a.jd, 3)
    _at5(g, a.id, "smithy")


def t_lab(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :140-145
    put(g.discard, take_like(a.hand, o.a["choice"].code))
    a.gold += 1
    _at5(g, a.id, "lab")


def t_magic_school(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :147-153
    take_like(a.build, 25)
    s = SUITS.index(o.a["choice"])
    put(a.build, 25 if s == 4 else 40 + s)
    _at5(g, a.id, "magic_school")


def t_ghost_town(g, o):
    raise NotImplementedError("ghost_town_color_choice is never offered (agent_functions.py:47-52)")


def t_museum(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :161-165
    put(a.museum, take_like(a.hand, o.a["choice"].code))
    _at5(g, a.id, "museum")


def t_weapon_storage(g, o):
    a, t = g.players[o.a["perpetrator"]], g.players[o.a["target"]]       # :167-171
    put(g.discard, take_like(a.build, 27))
    put(g.discard, take_like(t.build, o.a["choice"].code))
    _at5(g, a.id)


def t_lighthouse(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :173-180
    a.kh.append(OKH(-1, list(g.deck), 5))
    put(a.hand, take_like(g.deck, o.a["choice"].code))
    a.lh = False
    g.rng.shuffle(g.deck)
    _at5(g, a.id)


def t_graveyard(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :183-187
    put(a.build, g.discard.pop(-1))
    a.gold -= 1
    g.gs = g.gs.next


def t_finish(g, o):
    """finish_main_sequnce_actions (option_functions.py:189-243)."""
    a = g.players[o.a["perpetrator"]]
    if not rprop(g, a.role)[0]:
        if has(a.build, 28) and len(a.hand) == 0:
            draw_into(g, a.jd, 2)
        if has(a.build, 30) and len(a.hand) == 0:
            a.gold += 1
    if o.a["crown"]:
        confirm_roles(g, a)
        move_crown(g, a.id)
    elif rprop(g, a.role)[0]:
        confirm_roles(g, a)
    if o.a["next_witch"]:
        g.gs.state = 5
        g.gs.pid = g.holder(0).id
        w = g.players[g.gs.pid]
        w.role = a.role
        rprop(g, a.role)[2] = False
        a.role = BEWITCHED
        for p in g.players:
            if p.id != w.id:
                p.kr[w.id][0] = 1 << (rank(w.role) + 1)
            if p.id != a.id:
                p.kr[a.id][0] = 1                                       # {-1: "Bewitched"}
        g.gs.adm = []
        return None
    if g.used_roles[-1] == rank(a.role):
        w = g.check_ending()
        if w is None:
            g.setup_round()
        else:
            return w
    else:
        g.next_player(a.id)
    return None


def t_assassination(g, o):
    g.rp[o.a["choice"]][0] = True                                        # :245-249
    _at5(g, o.a["perpetrator"], "character_ability")


def t_warrant(g, o):
    g.rp[o.a["real_target"]][1] = "Real"                                 # :251-257
    g.rp[o.a["fake_targets"][0]][1] = "Fake"
    g.rp[o.a["fake_targets"][1]][1] = "Fake"
    _at5(g, o.a["perpetrator"], "character_ability")


def t_bewitch(g, o):
    g.rp[o.a["choice"]][2] = True                                        # :259-262
    g.players[o.a["perpetrator"]].witch = True
    g.next_player(o.a["perpetrator"])


def t_steal(g, o):
    g.rp[o.a["choice"]][3] = True                                        # :265-269
    _at5(g, o.a["perpetrator"], "character_ability")


def t_blackmail(g, o):
    g.rp[o.a["real_target"]][4] = "Real"                                 # :271-276
    g.rp[o.a["fake_target"]][4] = "Fake"
    _at5(g, o.a["perpetrator"], "character_ability")


def t_spy(g, o):
    """option_functions.py:278-288."""
    a, t = g.players[o.a["perpetrator"]], g.players[o.a["target"]]
    s = SUITS.index(o.a["suit"])
    n = sum(1 for c in t.hand if csuit(c) == s)
    steal = min(n, t.gold)
    a.gold += steal
    t.gold -= steal
    draw_into(g, a.hand, 1)
    _at5(g, a.id, "character_ability")


def t_magic(g, o):
    """carry_out_magicking (option_functions.py:291-303); iterate-while-remove kept."""
    a = g.players[o.a["perpetrator"]]
    if o.name == "magic_hand_change":
        t = g.players[o.a["target"]]
        a.hand, t.hand = t.hand, a.hand
    else:
        i = 0
        while i < len(a.hand):
            put(g.deck, take_like(a.hand, a.hand[i]))
            i += 1
        draw_into(g, a.hand, len(a.hand))
    _at5(g, a.id, "character_ability")


def t_look(g, o):
    """carry_out_wizard_hand_looking (option_functions.py:305-310)."""
    a, t = g.players[o.a["perpetrator"]], g.players[o.a["target"]]
    a.kh.append(OKH(t.id, list(t.hand), 5, wizard=True))
    g.gs.state, g.gs.pid = 10, a.id
    g.gs.adm.append("character_ability")
    g.gs.next = OGS(5, a.id, g.gs.adm)


def t_take(g, o):
    """carry_out_wizard_take_from_hand (option_functions.py:312-328); mutates the
    option's `replica` like the reference."""
    a, t = g.players[o.a["perpetrator"]], g.players[o.a["target"]]
    hk = next((h for h in a.kh if h.wizard), None)
    if o.a["build"]:
        card = o.a["built_card"].code
        put(a.hand, take_like(t.hand, card))
        o.a["replica"] = sum(1 for c in a.build if ctype(c) == ctype(card))
        t_build(g, o)
        take_like(hk.cards, card)
    else:
        card = o.a["card"].code
        put(a.hand, take_like(t.hand, card))
        take_like(hk.cards, card)
    g.gs = g.gs.next


def t_seer(g, o):
    """carry_out_seer_take_a_card (option_functions.py:330-341)."""
    a = g.players[o.a["perpetrator"]]
    g.seer_from = []
    for p in g.players:
        if p.id != a.id and p.hand:
            g.rng.shuffle(p.hand)
            reshuffle_if_empty(g)
            put(a.hand, draw(p.hand))
            g.seer_from.append(p.id)
    g.gs.state, g.gs.pid = 8, a.id
    g.gs.adm.append("character_ability")
    g.gs.next = OGS(5, a.id, g.gs.adm)


def t_give_back(g, o):
    """carry_out_seer_give_back_cards (option_functions.py:343-350)."""
    a = g.players[o.a["perpetrator"]]
    for pid, c in o.a["card_handouts"].items():
        put(g.players[pid].hand, take_like(a.hand, c.code))
        a.kh.append(OKH(pid, [c.code], 5))
    g.seer_from = []
    g.gs = g.gs.next


def _lords(a, suit):
    return sum(1 for c in a.build if csuit(c) == suit)


def t_king(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :354-363
    a.gold += _lords(a, 3)
    if not a.witch:
        move_crown(g, a.id)
    _at5(g, a.id, "character_ability")


def t_patrician(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :365-375
    for c in a.build:
        if csuit(c) == 3:
            draw_into(g, a.hand, 1)
    if not a.witch:
        move_crown(g, a.id)
    _at5(g, a.id, "character_ability")


def t_emperor(g, o):
    """option_functions.py:377-393."""
    a, t = g.players[o.a["perpetrator"]], g.players[o.a["target"]]
    a.gold += _lords(a, 3)
    if o.a["gold_or_card"] == "card":
        g.rng.shuffle(t.hand)
        put(a.hand, draw(t.hand))
    if o.a["gold_or_card"] == "gold":
        a.gold += 1
        t.gold -= 1
    confirm_roles(g, a)
    move_crown(g, t.id)
    _at5(g, a.id, "character_ability")


def t_bishop(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :397-403
    a.gold += _lords(a, 2)
    _at5(g, a.id, "character_ability")


def t_abbot(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :405-412
    cmb = o.a["gold_or_card_combination"]
    a.gold += cmb.count("gold")
    draw_into(g, a.hand, cmb.count("card"))
    _at5(g, a.id, "character_ability")


def t_abbot_beg(g, o):
    """option_functions.py:414-420 (first max)."""
    golds = [p.gold for p in g.players]
    i = golds.index(max(golds))
    g.players[i].gold -= 1
    g.holder(4).gold += 1
    _at5(g, o.a["perpetrator"], "begged")


def t_cardinal(g, o):
    """option_functions.py:422-439."""
    a, t = g.players[o.a["perpetrator"]], g.players[o.a["target"]]
    card = o.a["built_card"].code
    put(a.build, take_like(a.hand, card))
    a.gold -= ccost(card) - int(o.a["factory"])
    a.gold = max(0, a.gold)
    if o.a["replica"]:
        a.replicas = o.a["replica"]
    if o.a["cards_to_give"]:
        t.gold -= len(o.a["cards_to_give"])
        for c in o.a["cards_to_give"]:
            put(t.hand, take_like(a.hand, c.code))
    _at5(g, a.id, "character_ability")


def t_merchant(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :442-449
    a.gold += _lords(a, 0) + 1
    _at5(g, a.id, "character_ability")


def t_alchemist(g, o):
    return None                                                          # :451-452


def t_trader(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :455-461
    a.gold += _lords(a, 0)
    _at5(g, a.id, "character_ability")


def t_architect(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :464-471
    draw_into(g, a.hand, 2)
    _at5(g, a.id, "character_ability")


def t_navigator(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :473-483
    if o.a["choice"] == "4card":
        draw_into(g, a.hand, 4)
    if o.a["choice"] == "4gold":
        a.gold += 4
    _at5(g, a.id, "character_ability")


def t_scholar(g, o):
    """carry_out_scholar_draw (option_functions.py:485-496)."""
    a = g.players[o.a["perpetrator"]]
    seven = DeckRef([])
    g.seven = seven
    for _ in range(min(7, len(g.deck))):
        reshuffle_if_empty(g)
        c = draw(g.deck)
        put(a.hand, c)
        put(seven.cards, c)
    g.gs.state, g.gs.pid = 9, a.id
    g.gs.adm.append("character_ability")
    g.gs.next = OGS(5, a.id, g.gs.adm)


def t_scholar_pick(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :498-502
    for c in o.a["unchosen_cards"].cards:
        put(g.deck, take_like(a.hand, c))
    g.gs = g.gs.next
    g.seven = []


def _settle(g, o, a, t):
    """check_if_building_is_replica + settle_museum + settle_lighthouse (:573-606)."""
    card = o.a["choice"].code
    if has(t.build, ctype(card)) and sum(1 for c in t.build if ctype(c) == ctype(card)) > 1:
        t.replicas -= 1
    if ctype(card) == 34:
        n = len(t.museum)
        for _ in range(n):
            put(g.discard if o.name == "warlord_desctruction" else a.museum, draw(t.museum))
    if ctype(card) == 29 and t.lh:
        t.lh = False
        a.lh = True


def t_marshal(g, o):
    a, t = g.players[o.a["perpetrator"]], g.players[o.a["target"]]       # :505-515
    card = o.a["choice"].code
    a.gold -= ccost(card)
    t.gold += ccost(card)
    put(a.build, take_like(t.build, card))
    _settle(g, o, a, t)
    _at5(g, a.id, "character_ability")


def t_warlord(g, o):
    """option_functions.py:517-535."""
    a, t = g.players[o.a["perpetrator"]], g.players[o.a["target"]]
    card = o.a["choice"].code
    a.gold -= ccost(card) - 1
    put(g.discard, take_like(t.build, card))
    _settle(g, o, a, t)
    _at5(g, a.id, "character_ability")
    owner = next((p for p in g.players if has(p.build, 24)), None)
    if owner is not None and owner is not a:
        g.gs.state = 6
        g.gs.pid = owner.id
        g.gs.intr = True
        g.gs.next = OGS(5, a.id, ["character_ability"])


def t_diplomat(g, o):
    a, t = g.players[o.a["perpetrator"]], g.players[o.a["target"]]       # :538-551
    a.gold -= o.a["money_owed"]
    t.gold += o.a["money_owed"]
    put(a.build, take_like(t.build, o.a["choice"].code))
    put(t.build, take_like(a.build, o.a["give"].code))
    _settle(g, o, a, t)
    _at5(g, a.id, "character_ability")


def t_take_gold(g, o):
    a = g.players[o.a["perpetrator"]]                                    # :553-559
    a.gold += _lords(a, 1)
    _at5(g, a.id, "take_gold")


TRANSITIONS = {
    "role_pick": t_role_pick, "gold_or_card": t_gold_or_card, "which_card_to_keep": t_keep,
    "blackmail_response": t_blackmail_response, "reveal_blackmail_as_blackmailer": t_reveal_blackmail,
    "reveal_warrant_as_magistrate": t_reveal_warrant, "build": t_build, "empty_option": t_empty,
    "finish_round": t_finish, "ghost_town_color_choice": t_ghost_town, "smithy_choice": t_smithy,
    "laboratory_choice": t_lab, "magic_school_choice": t_magic_school, "weapon_storage_choice": t_weapon_storage,
    "lighthouse_choice": t_lighthouse, "museum_choice": t_museum, "graveyard": t_graveyard,
    "take_gold_for_war": t_take_gold, "assassination": t_assassination, "magistrate_warrant": t_warrant,
    "bewitching": t_bewitch, "steal": t_steal, "blackmail": t_blackmail, "spy": t_spy,
    "magic_hand_change": t_magic, "discard_and_draw": t_magic, "look_at_hand": t_look,
    "take_from_hand": t_take, "seer": t_seer, "give_back_card": t_give_back, "take_crown_king": t_king,
    "give_crown": t_emperor, "take_crown_pat": t_patrician, "bishop": t_bishop, "cardinal_exchange": t_cardinal,
    "abbot_gold_or_card": t_abbot, "abbot_beg": t_abbot_beg, "merchant": t_merchant, "alchemist": t_alchemist,
    "trader": t_trader, "architect": t_architect, "navigator_gold_card": t_navigator, "scholar": t_scholar,
    "scholar_card_pick": t_scholar_pick, "warlord_desctruction": t_warlord, "marshal_steal": t_marshal,
    "diplomat_exchange": t_diplomat,
}


# ---- canonical form (shared format with tools/refcanon.py) ------------------
def canon(g):
    adm = lambda l: [l.count(t) for t in ADM]  # noqa: E731
    WB = {None: 0, "Real": 1, "Fake": 2}
    d = {"deck": list(g.deck), "discard": list(g.discard), "used_cards": list(g.used_cards)}
    d["players"] = [{
        "hand": list(p.hand), "build": list(p.build), "jd": list(p.jd), "museum": list(p.museum),
        "gold": p.gold, "role": -1 if p.role is None else p.role, "replicas": int(p.replicas),
        "crown": int(p.crown), "lh": int(p.lh), "f7": int(p.f7), "witch": int(p.witch),
        "kr": [[k[0], int(k[1])] for k in p.kr],
        "kh": [[h.pid, h.conf, int(h.wizard), int(h.used), list(h.cards)] for h in p.kh]}
        for p in g.players]
    d["roles"] = list(g.roles)
    d["rtc"] = None if g.rtc is None else list(g.rtc)
    d["used_roles"] = None if g.used_roles is None else list(g.used_roles)
    d["turn"] = list(g.turn)
    d["rp"] = [[int(r[0]), WB[r[1]], int(r[2]), int(r[3]), WB[r[4]]] for r in g.rp]
    gs = g.gs
    d["gs"] = [gs.state, -1 if gs.pid is None else gs.pid, adm(gs.adm), int(gs.intr)]
    nx = gs.next
    d["next"] = None if nx is None else [nx.state, nx.pid, adm(nx.adm), int(nx.intr), int(nx.adm is gs.adm),
                                         int(nx.next is not None)]
    d["ending"] = int(g.ending)
    d["terminal"] = int(g.terminal)
    d["winner"] = g.winner
    d["points"] = None if g.points is None else list(g.points)
    d["warrant"] = g.warrant
    d["seer_from"] = None if g.seer_from is None else list(g.seer_from)
    if g.seven is None:
        d["seven"] = None
    elif isinstance(g.seven, DeckRef):
        d["seven"] = ["deck", list(g.seven.cards)]
    else:
        d["seven"] = ["list", list(g.seven)]
    return d


def new_game(seed, preset=True, rng=None):
    """run_utils.create_game (run_utils.py:20-27) with a per-game RNG seeded like random.seed(seed)."""
    g = OGame(seed, preset, rng)
    g.setup_round()
    return g


def random_rollout(seed, preset=True, max_steps=None, trace=None):
    """The random-policy step loop (compare_to_random.py:37-39 / run_utils.py:37-41):
    get_options -> random.choice -> carry_out until a winner.  Returns (game, steps)."""
    g = new_game(seed, preset)
    steps = 0
    w = None
    while w is None and (max_steps is None or steps < max_steps):
        opts = g.get_options()
        if not opts:
            raise IndexError("Cannot choose from an empty sequence")
        k = g.rng._randbelow(len(opts))
        if trace is not None:
            trace.append((g.gs.state, g.gs.pid, opts, k))
        w = g.carry_out(opts[k])
        steps += 1
    return g, steps
