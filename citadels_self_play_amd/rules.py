"""Rules tables shared by the host facade (names and codes only; the rules
themselves live in csrc/cit_engine.h).  Values follow game/config.py:2-121
and game/option.py:34-45 of the reference."""

SUITS = ["trade", "war", "religion", "lord", "unique"]
TYPE_COST = [1, 2, 4, 2, 5, 3, 2, 3, 5, 1, 2, 3, 1, 4, 3, 5,
             5, 3, 6, 2, 6, 5, 5, 6, 5, 6, 6, 3, 6, 3, 5, 5, 6, 5, 4, 6, 5, 4, 6, 5]
ROLE_NAMES = ["Assassin", "Witch", "Magistrate", "Thief", "Spy", "Blackmailer",
              "Magician", "Wizard", "Seer", "King", "Emperor", "Patrician",
              "Bishop", "Abbot", "Cardinal", "Merchant", "Alchemist", "Trader",
              "Architect", "Navigator", "Scholar", "Warlord", "Diplomat", "Marshal",
              "Queen", "Artist", "Tax Collector"]
ROLE_ID = {n: i for i, n in enumerate(ROLE_NAMES)}
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
OPTION_ID = {n: i for i, n in enumerate(OPTION_NAMES)}


def card_type(c):
    return 25 if c >= 40 else c


def card_suit(c):
    t = card_type(c)
    if c >= 40:
        return c - 40
    return 0 if t < 6 else 1 if t < 10 else 2 if t < 13 else 3 if t < 16 else 4


def card_cost(c):
    return TYPE_COST[card_type(c)]


def role_rank(role):
    return -1 if role == 27 else role // 3
