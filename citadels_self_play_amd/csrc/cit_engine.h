// The rules engine on one packed game row: get_options (as an enumeration
// into a sink, so a caller can count, pick the k-th, or materialise without a
// per-lane option buffer) and carry_out.  Host+device (CIT_HD).
//
//   cit_get_options  = cit_prepare_options (mutating part) + cit_enum_options
//                      game/agent.py:50-83, game/agent_functions.py:13-509
//   cit_carry_out    = game/option.py:118-122 -> game/option_functions.py:6-631
//   cit_setup_round  = game/game.py:144-171
//   cit_init_game    = game/game.py:17-24,420-540 (+ run_utils.create_game)
#pragma once
#include "cit_core.h"

// =========================================================== list helpers
// Lists of up to 64 entries are scanned one element per lane under CIT_WAVE
// (cit_core.h); longer ones (the deck ring) and the host build loop.
CIT_HD bool has_type(const uint8_t* a, int n, int t) {
#if CIT_WAVE
  if (n <= 64) {
    int i = cit_lane();
    return cit_ballot((i < n) & (card_type(cit_ld(a, i, i < n, 0)) == t)) != 0;
  }
#endif
  for (int i = 0; i < n; i++)
    if (card_type(a[i]) == t) return true;
  return false;
}
CIT_HD int count_type(const uint8_t* a, int n, int t) {
#if CIT_WAVE
  if (n <= 64) {
    int i = cit_lane();
    return __popcll(cit_ballot((i < n) & (card_type(cit_ld(a, i, i < n, 0)) == t)));
  }
#endif
  int k = 0;
  for (int i = 0; i < n; i++) k += card_type(a[i]) == t;
  return k;
}
CIT_HD int count_suit(const uint8_t* a, int n, int s) {
#if CIT_WAVE
  if (n <= 64) {
    int i = cit_lane();
    return __popcll(cit_ballot((i < n) & (card_suit(cit_ld(a, i, i < n, 0)) == s)));
  }
#endif
  int k = 0;
  for (int i = 0; i < n; i++) k += card_suit(a[i]) == s;
  return k;
}
// Deck.get_a_card_like_it (deck.py:49-55): removes the first card of c's type;
// returns it, or c itself when there is none.
CIT_HD int take_like(uint8_t* a, uint8_t& n, int c) {
  int t = card_type(c);
#if CIT_WAVE
  int cnt = n;
  if (cnt <= 64) {
    int j = cit_lane();
    int v = cit_ld(a, j, j < cnt, CIT_NO_CARD);
    uint64_t m = cit_ballot((j < cnt) & (card_type(v) == t));
    if (!m) return c;
    int i = __ffsll((unsigned long long)m) - 1;
    int r = cit_readlane(v, i);
    if (j > i && j < cnt) a[j - 1] = (uint8_t)v;   // every lane loaded before any stores
    n = (uint8_t)(cnt - 1);
    return r;
  }
#endif
  for (int i = 0; i < n; i++) {
    if (card_type(a[i]) == t) {
      int r = a[i];
      for (int j = i + 1; j < n; j++) a[j - 1] = a[j];
      n--;
      return r;
    }
  }
  return c;
}
// Length statistics (host measurement builds only, tools/capstats.cpp): the
// tool defines cit_cap_note and sees every append's resulting length.
#if defined(CIT_CAP_STATS) && !defined(__HIP_DEVICE_COMPILE__)
void cit_cap_note(const CitGame& g, const void* list, int n);
#define CIT_CAP_NOTE(g, a, n) cit_cap_note(g, a, n)
#else
#define CIT_CAP_NOTE(g, a, n) ((void)0)
#endif
// Deck.add_card (deck.py:62-67): the "Deck Empty" sentinel (CIT_NO_CARD) is dropped.
CIT_HD void put_card(CitGame& g, uint8_t* a, uint8_t& n, int cap, int c) {
  if (c == CIT_NO_CARD) return;
  CIT_CAP_NOTE(g, a, n + 1);
  if (n >= cap) { g.err |= CIT_ERR_OVERFLOW; return; }
  a[n++] = (uint8_t)c;
}
CIT_HD int pop_front(uint8_t* a, uint8_t& n) {
  if (!n) return CIT_NO_CARD;
#if CIT_WAVE
  int cnt = n;
  if (cnt <= 64) {
    int j = cit_lane();
    int v = cit_ld(a, j, j < cnt, 0);
    int r = cit_readlane(v, 0);
    if (j >= 1 && j < cnt) a[j - 1] = (uint8_t)v;
    n = (uint8_t)(cnt - 1);
    return r;
  }
#endif
  int r = a[0];
  for (int j = 1; j < n; j++) a[j - 1] = a[j];
  n--;
  return r;
}
// Read-only view of a list of up to 64 bytes for a serial loop: under
// CIT_WAVE lane i holds a[i] (one LDS round trip) and [i] is a readlane.
struct ByteList {
#if CIT_WAVE
  int v;
  CIT_HD ByteList(const uint8_t* a, int n) { int i = cit_lane(); v = cit_ld(a, i, i < n, 0); }
  CIT_HD int operator[](int i) const { return cit_readlane(v, i); }
#else
  const uint8_t* a;
  CIT_HD ByteList(const uint8_t* p, int) : a(p) {}
  CIT_HD int operator[](int i) const { return a[i]; }
#endif
};

#define BUILD(p) (p).build, (p).n_build, CIT_BUILD_CAP

// ------------------------------------------------- a player's card area
// hand | just_drawn_cards | museum_cards back to back in CitPlayer::hand
// (cit_core.h).  A list starts where the lists before it end; every change of
// a list's length goes through the functions below, which move the lists
// after it.  Reads index the area directly (the hand at 0, pl_jd, pl_museum).
enum { AL_HAND = 0, AL_JD = 1, AL_MUSEUM = 2 };
CIT_HD int area_used(const CitPlayer& P) { return P.n_hand + P.n_jd + P.n_museum; }
CIT_HD int area_off(const CitPlayer& P, int L) { return L == AL_HAND ? 0 : L == AL_JD ? P.n_hand : P.n_hand + P.n_jd; }
CIT_HD int area_len(const CitPlayer& P, int L) { return L == AL_HAND ? P.n_hand : L == AL_JD ? P.n_jd : P.n_museum; }
CIT_HD void area_set_len(CitPlayer& P, int L, int n) {
  (L == AL_HAND ? P.n_hand : L == AL_JD ? P.n_jd : P.n_museum) = (uint8_t)n;
}
CIT_HD const uint8_t* pl_jd(const CitPlayer& P) { return P.hand + P.n_hand; }
CIT_HD const uint8_t* pl_museum(const CitPlayer& P) { return P.hand + P.n_hand + P.n_jd; }
#if defined(CIT_CAP_STATS) && !defined(__HIP_DEVICE_COMPILE__)
void cit_area_note(const CitGame& g, const CitPlayer& P);
#define CIT_AREA_NOTE(g, P) cit_area_note(g, P)
#else
#define CIT_AREA_NOTE(g, P) ((void)0)
#endif

// List L of P: its elements [at, at + del) are replaced by src(0), ..,
// src(ins - 1) (the reference's list surgery: append, remove, pop(0), clear,
// reassign); the lists after L move by ins - del.  An area past CIT_AREA_CAP
// sets the overflow bit and changes nothing.  Wave: lane l moves the area
// bytes at l and l + 64 past the cut and writes src(l) and src(l + 64); every
// load precedes every store, so src may read the area.
template <class Src>
CIT_HD void area_splice(CitGame& g, CitPlayer& P, int L, int at, int del, int ins, Src src) {
  const int used = area_used(P), cut = area_off(P, L) + at;
  if (used - del + ins > CIT_AREA_CAP) { g.err |= CIT_ERR_OVERFLOW; return; }
#if CIT_WAVE
  {
    const int l = cit_lane(), j0 = cut + del + l, j1 = j0 + 64;
    // the first halves load on every lane (no branch); the second halves (past
    // lane 64: rarely any lane) keep the branch that skips them
    const int v0 = cit_ld(P.hand, j0, j0 < used, 0), v1 = j1 < used ? P.hand[j1] : 0;
    const int s0 = (int)src(l), s1 = l + 64 < ins ? (int)src(l + 64) : 0;   // (src is safe past ins)
    __asm__ volatile("" ::: "memory");   // every byte loaded before any is stored
    if (j0 < used) P.hand[j0 - del + ins] = (uint8_t)v0;
    if (j1 < used) P.hand[j1 - del + ins] = (uint8_t)v1;
    if (l < ins) P.hand[cut + l] = (uint8_t)s0;
    if (l + 64 < ins) P.hand[cut + l + 64] = (uint8_t)s1;
  }
#else
  {   // serial: the lists after the cut move first, then src fills the gap (src must
      // not read the area here -- no serial caller's does -- so no private copy is needed)
    const int shift = ins - del, from = cut + del, tail = used - from;
    if (shift > 0)
      for (int i = tail - 1; i >= 0; i--) P.hand[from + i + shift] = P.hand[from + i];
    else if (shift < 0)
      for (int i = 0; i < tail; i++) P.hand[from + i + shift] = P.hand[from + i];
    for (int i = 0; i < ins; i++) P.hand[cut + i] = (uint8_t)src(i);
  }
#endif
  area_set_len(P, L, area_len(P, L) - del + ins);
  CIT_AREA_NOTE(g, P);
}
// Deck.add_card on list L (the "Deck Empty" sentinel, CIT_NO_CARD, is dropped)
CIT_HD void pl_put(CitGame& g, CitPlayer& P, int L, int c) {
  if (c == CIT_NO_CARD) return;
  area_splice(g, P, L, area_len(P, L), 0, 1, [c](int) { return c; });
}
// Deck.get_a_card_like_it on list L: removes the first card of c's type and
// returns it, or returns c itself when there is none.  Wave: one load of the
// list and the lists after it, one ballot, one store of the moved bytes.
CIT_HD int pl_take_like(CitGame& g, CitPlayer& P, int L, int c) {
  const int t = card_type(c), off = area_off(P, L), n = area_len(P, L);
#if CIT_WAVE
  {
    const int used = area_used(P), l = cit_lane(), p0 = off + l, p1 = p0 + 64;
    const int v0 = cit_ld(P.hand, p0, p0 < used, 0), v1 = p1 < used ? P.hand[p1] : 0;
    const uint64_t m0 = cit_ballot((l < n) & (card_type(v0) == t)), m1 = cit_ballot((l + 64 < n) & (card_type(v1) == t));
    if (!(m0 | m1)) return c;
    const int i = m0 ? __ffsll((unsigned long long)m0) - 1 : 64 + __ffsll((unsigned long long)m1) - 1;
    const int r = i < 64 ? cit_readlane(v0, i) : cit_readlane(v1, i - 64);
    if (l > i && p0 < used) P.hand[p0 - 1] = (uint8_t)v0;
    if (l + 64 > i && p1 < used) P.hand[p1 - 1] = (uint8_t)v1;
    area_set_len(P, L, n - 1);
    return r;
  }
#endif
  for (int i = 0; i < n; i++) {
    int r = P.hand[off + i];
    if (card_type(r) == t) {
      area_splice(g, P, L, i, 1, 0, [](int) { return 0; });
      return r;
    }
  }
  return c;
}
// list L emptied (`.cards = []`)
CIT_HD void pl_clear(CitGame& g, CitPlayer& P, int L) {
  const int n = area_len(P, L);
  if (area_off(P, L) + n == area_used(P)) area_set_len(P, L, 0);   // nothing after it moves
  else area_splice(g, P, L, 0, n, 0, [](int) { return 0; });
}
// Deck.draw_card (pop(0)) on list L; CIT_NO_CARD when empty
CIT_HD int pl_pop_front(CitGame& g, CitPlayer& P, int L) {
  if (!area_len(P, L)) return CIT_NO_CARD;
  const int r = P.hand[area_off(P, L)];
  area_splice(g, P, L, 0, 1, 0, [](int) { return 0; });
  return r;
}
CIT_HD bool p_has(const CitPlayer& p, int t) { return has_type(p.build, p.n_build, t); }
// bit t set iff a card of type t is in the list
CIT_HD uint64_t type_mask(const uint8_t* a, int n) {
#if CIT_WAVE
  if (n <= 64) {
    int i = cit_lane();
    return cit_wave_or64(i < n ? 1ull << card_type(a[i]) : 0ull);
  }
#endif
  uint64_t m = 0;
  for (int i = 0; i < n; i++) m |= 1ull << card_type(a[i]);
  return m;
}
#define HAS(mask, t) (((mask) >> (t)) & 1)

// the first seat whose buildings hold type t, or -1 (the reference's seat
// loops over p_has: get_graveyard_owner, troneroom_owner_gold).  Wave: lane l
// reads building l % 10 of seat l / 10 (a seat with more than 10 buildings
// falls back to the loop).
CIT_HD int seat_with_type(const CitGame& g, int t) {
#if CIT_WAVE
  {
    int l = cit_lane(), p = l / 10, i = l - 10 * p, ps = p < CIT_NP ? p : 0;
    int nb = g.pl[ps].n_build;
    int c = g.pl[ps].build[i];
    if (!cit_ballot(i == 0 && p < CIT_NP && nb > 10)) {
      uint64_t m = cit_ballot(p < CIT_NP && i < nb && card_type(c) == t);
      return m ? (__ffsll((unsigned long long)m) - 1) / 10 : -1;
    }
  }
#endif
  for (int p = 0; p < CIT_NP; p++)
    if (p_has(g.pl[p], t)) return p;
  return -1;
}

// ------------------------------------------------------------ deck (ring)
CIT_HD int deck_at(const CitGame& g, int i) { return g.deck[(g.deck_head + i) & (CIT_DECK_CAP - 1)]; }
CIT_HD uint8_t& deck_ref(CitGame& g, int i) { return g.deck[(g.deck_head + i) & (CIT_DECK_CAP - 1)]; }
CIT_HD int deck_draw(CitGame& g) {
  if (!g.n_deck) return CIT_NO_CARD;
  int c = g.deck[g.deck_head];
  g.deck_head = (uint8_t)((g.deck_head + 1) & (CIT_DECK_CAP - 1));
  g.n_deck--;
  return c;
}
CIT_HD void deck_put(CitGame& g, int c) {
  if (c == CIT_NO_CARD) return;
  CIT_CAP_NOTE(g, g.deck, g.n_deck + 1);
  if (g.n_deck >= CIT_DECK_CAP - 1) { g.err |= CIT_ERR_OVERFLOW; return; }
  deck_ref(g, g.n_deck) = (uint8_t)c;
  g.n_deck++;
}
CIT_HD int deck_take_like(CitGame& g, int c) {
  int t = card_type(c);
#if CIT_WAVE
  {   // lanes l / 64 + l hold logical positions l / 64 + l; one ballot finds the
      // first match, every lane loads before any lane stores the shifted tail
    const int nd = g.n_deck, head = g.deck_head, l = cit_lane();
    int c0 = cit_ld(g.deck, (head + l) & (CIT_DECK_CAP - 1), l < nd, CIT_NO_CARD);
    int c1 = l + 64 < nd ? g.deck[(head + l + 64) & (CIT_DECK_CAP - 1)] : CIT_NO_CARD;
    uint64_t m0 = cit_ballot((l < nd) & (card_type(c0) == t)), m1 = cit_ballot((l + 64 < nd) & (card_type(c1) == t));
    if (!(m0 | m1)) return c;
    int i = m0 ? __ffsll((unsigned long long)m0) - 1 : 64 + __ffsll((unsigned long long)m1) - 1;
    int r = i < 64 ? cit_readlane(c0, i) : cit_readlane(c1, i - 64);
    if (l > i && l < nd) g.deck[(head + l - 1) & (CIT_DECK_CAP - 1)] = (uint8_t)c0;
    if (l + 64 > i && l + 64 < nd) g.deck[(head + l + 63) & (CIT_DECK_CAP - 1)] = (uint8_t)c1;
    g.n_deck = (uint8_t)(nd - 1);
    return r;
  }
#endif
  for (int i = 0; i < g.n_deck; i++) {
    if (card_type(deck_at(g, i)) == t) {
      int r = deck_at(g, i);
      for (int j = i + 1; j < g.n_deck; j++) deck_ref(g, j - 1) = (uint8_t)deck_at(g, j);
      g.n_deck--;
      return r;
    }
  }
  return c;
}
// random.shuffle (Lib/random.py:380-392) over any indexable sequence.  With
// a coop (LDS) stream under CIT_WAVE the draws come through a register
// window (a readlane each instead of an LDS round trip per draw); the swaps
// stay serial (LDS operations of one wave are in order, so a swap's reads
// never wait on the previous swap's writes).
#ifndef CIT_SHUFFLE_REG
#define CIT_SHUFFLE_REG 0
#endif
#ifndef CIT_SHUFFLE_BATCH
#define CIT_SHUFFLE_BATCH 1
#endif
// below this length the serial draws are faster (tools/bench_shuffle.py: n = 3
// 1.1 k vs 1.9 k cycles, n = 8 2.7 k vs 3.0 k, n = 12 even, n = 16 5.1 k vs 4.6 k)
#ifndef CIT_SHUFFLE_BATCH_MIN
#define CIT_SHUFFLE_BATCH_MIN 12
#endif
#if CIT_WAVE
// The n - 1 draws of random.shuffle from a coop (LDS) stream, a chunk of up to
// 64 stream words at a time instead of one _randbelow after another.  Draw t
// (t = 0 .. n-2) is _randbelow(n - t): getrandbits(k) = word >> (32 - k),
// rejected while >= n - t (Lib/random.py:239-249), so word q of a chunk is
// tried by draw t0 + q - s, where s is the number of rejections before q.
// Per chunk: lane q loads and tempers word q; one ballot per rejection finds
// the next rejected word at the current s (every word before it is an
// accepted draw); a ds_permute moves each accepted draw into lane t & 63 of
// jv0 (t < 64) or jv1.  Same words, same order, same results as the serial
// loop; the stream's position is advanced and its register window dropped.
__device__ __forceinline__ void fy_draws_batched(CitMT& rng, int n, int& jv0, int& jv1) {
  const int l = cit_lane();
  uint32_t pos = rng.pos;
  int t0 = 0;
  while (t0 < n - 1) {
    if (pos >= CIT_MT_N) {
      if (CIT_TWIST_INLINE)
        mt_twist_wave((cit_lds_u32*)rng.mt);
      else
        mt_twist_coop((cit_lds_u32*)rng.mt);
      pos = 0;
    }
    const int L = CIT_MT_N - (int)pos < 64 ? CIT_MT_N - (int)pos : 64;   // words left before the twist
    const int q = (int)pos + l;
    const uint32_t word = mt_temper(((const cit_lds_u32*)rng.mt)[q < CIT_MT_N ? q : 0]);
    uint64_t rej = 0;
    int p = 0, s = 0, c;
    const int n0 = n - t0 - l;   // lane l's bound at shift 0; at shift s it tries draw t0 + l - s, bound n0 + s
    for (;;) {
      const uint32_t N = (uint32_t)(n0 + s);
      const uint64_t R0 = cit_ballot((word >> __builtin_clz(N | 1u)) >= N);   // (N | 1: clz(N) for N >= 2)
      // the live lanes p .. hi: up to the last draw at this shift, or the chunk's end
      const int e = n - 2 - t0 + s, hi = e < L - 1 ? e : L - 1;
      const uint64_t R = R0 & (hi >= 63 ? ~0ull : ((2ull << hi) - 1)) & (~0ull << p);
      if (!R) {   // every live word from p on is accepted
        c = hi + 1;
        break;
      }
      const int r = __ffsll((unsigned long long)R) - 1;
      rej |= 1ull << r;
      p = r + 1;
      s++;
      if (p >= L) {
        c = L;
        break;
      }
    }
    const uint64_t acc = (c >= 64 ? ~0ull : ((1ull << c) - 1)) & ~rej;
    const int nd = __popcll(acc);
    const bool a = (acc >> l) & 1;
    const int sl = __popcll(rej & cit_below());
    const int t = t0 + l - sl;
    const uint32_t N = (uint32_t)(n - t);
    const int j = (int)(word >> __builtin_clz(N | 1u));
    // accepted lane -> relative slot l - sl (its draw); the others fill the
    // slots from nd on, in lane order: a permutation, no two lanes collide
    const int slot = a ? l - sl : nd + __popcll(~acc & cit_below());
    const int recv = __builtin_amdgcn_ds_permute(((t0 + slot) & 63) << 2, j);
    const int k = (l - t0) & 63;   // this lane as a destination: draw t0 + k
    if (k < nd) {
      if (t0 + k < 64)
        jv0 = recv;
      else
        jv1 = recv;
    }
    pos += (uint32_t)c;
    t0 += nd;
  }
  rng.pos = pos;
  rng.win_base = -1;
}
#endif
template <class At>
CIT_HD void shuffle_seq(CitMT& rng, int n, At at) {
#if CIT_WAVE
  if (CIT_SHUFFLE_BATCH && rng.coop && n >= CIT_SHUFFLE_BATCH_MIN && n > 1 && n <= 128) {
    // all draws first (above), then each lane traces its element's final
    // position back through the swaps (swap i is its own inverse, the last one
    // first: a position p equal to i or to j moves to the other, p ^ (i ^ j)),
    // one gather and one store of the sequence.  (Swaps of a one-VGPR sequence
    // by readlane / writelane measured slower: ~117 against ~92 cycles per
    // swap, tools/bench_shuffle.py.)
    const int l = cit_lane();
    int jv0 = 0, jv1 = 0;
    fy_draws_batched(rng, n, jv0, jv1);
    int p0 = l, p1 = l + 64;
    if (n > 65) {
      for (int t = n - 2; t >= 64; t--) {
        const int i = n - 1 - t, j = __builtin_amdgcn_readlane(jv1, t - 64), x = i ^ j;
        p0 = (p0 == i || p0 == j) ? p0 ^ x : p0;
        p1 = (p1 == i || p1 == j) ? p1 ^ x : p1;
      }
    }
    if (n > 64) {
      for (int t = 63; t >= 0; t--) {
        const int i = n - 1 - t, j = __builtin_amdgcn_readlane(jv0, t), x = i ^ j;
        p0 = (p0 == i || p0 == j) ? p0 ^ x : p0;
        p1 = (p1 == i || p1 == j) ? p1 ^ x : p1;
      }
    } else {
#pragma unroll 4
      for (int t = n - 2; t >= 0; t--) {
        const int i = n - 1 - t, j = __builtin_amdgcn_readlane(jv0, t), x = i ^ j;
        p0 = (p0 == i || p0 == j) ? p0 ^ x : p0;
      }
    }
    const int x0 = l < n ? (int)at(l < n ? p0 : 0) : 0;
    const int x1 = l + 64 < n ? (int)at(l + 64 < n ? p1 : 0) : 0;
    __builtin_amdgcn_wave_barrier();
    if (l < n) at(l) = (uint8_t)x0;
    if (l + 64 < n) at(l + 64) = (uint8_t)x1;
    __builtin_amdgcn_wave_barrier();
    return;
  }
  if (CIT_SHUFFLE_REG && rng.coop && n > 1 && n <= 128) {
    // the sequence in two VGPRs (lane l: elements l and 64 + l); a swap is
    // two readlanes at wave-uniform indices and two lane selects, the same
    // draws in the same order, one load and one store of the sequence
    CitMT w = cit_mt_window(rng);
    const int l = cit_lane();
    int v0 = l < n ? (int)at(l) : 0, v1 = l + 64 < n ? (int)at(l + 64) : 0;
    for (int i = n - 1; i > 0; i--) {
      const int j = __builtin_amdgcn_readfirstlane((int)mt_randbelow(w, (uint32_t)(i + 1)));
      const int x = i < 64 ? __builtin_amdgcn_readlane(v0, i) : __builtin_amdgcn_readlane(v1, i - 64);
      const int y = j < 64 ? __builtin_amdgcn_readlane(v0, j) : __builtin_amdgcn_readlane(v1, j - 64);
      v0 = l == i ? y : (l == j ? x : v0);
      v1 = l + 64 == i ? y : (l + 64 == j ? x : v1);
    }
    if (l < n) at(l) = (uint8_t)v0;
    if (l + 64 < n) at(l + 64) = (uint8_t)v1;
    cit_mt_unwindow(rng, w);
    return;
  }
  if (rng.coop && n > 1) {
    CitMT w = cit_mt_window(rng);
    for (int i = n - 1; i > 0; i--) {
      int j = (int)mt_randbelow(w, (uint32_t)(i + 1));
      uint8_t t = at(i);
      at(i) = at(j);
      at(j) = t;
    }
    cit_mt_unwindow(rng, w);
    return;
  }
#endif
  for (int i = n - 1; i > 0; i--) {
    int j = (int)mt_randbelow(rng, (uint32_t)(i + 1));
    uint8_t t = at(i);
    at(i) = at(j);
    at(j) = t;
  }
}
CIT_HD void shuffle_arr(CitMT& rng, uint8_t* a, int n) {
  shuffle_seq(rng, n, [a](int i) -> uint8_t& { return a[i]; });
}
CIT_HD void deck_shuffle(CitGame& g, CitMT& rng) {
  shuffle_seq(rng, g.n_deck, [&g](int i) -> uint8_t& { return deck_ref(g, i); });
}
// reshuffle_deck_if_empty (option_functions.py:564-570)
CIT_HD void reshuffle_if_empty(CitGame& g, CitMT& rng) {
  if (g.n_deck || !g.n_discard) return;
  shuffle_arr(rng, g.discard, g.n_discard);
  g.deck_head = 0;
  for (int i = 0; i < g.n_discard; i++) g.deck[i] = g.discard[i];
  g.n_deck = g.n_discard;
  g.n_discard = 0;
}
// k draws from the deck onto list L of P (each reshuffling the discard pile
// into an empty deck first); wave: when the deck holds k cards and the area has
// room, the k front cards move in one splice.
CIT_HD void pl_draw(CitGame& g, CitMT& rng, CitPlayer& P, int L, int k) {
#if CIT_WAVE
  {
    const int nd = g.n_deck, head = g.deck_head;
    if (k <= 64 && nd >= k && area_used(P) + k <= CIT_AREA_CAP) {
      area_splice(g, P, L, area_len(P, L), 0, k, [&g, head](int i) { return g.deck[(head + i) & (CIT_DECK_CAP - 1)]; });
      g.deck_head = (uint8_t)((head + k) & (CIT_DECK_CAP - 1));
      g.n_deck = (uint8_t)(nd - k);
      return;
    }
  }
#endif
  for (int i = 0; i < k; i++) {
    reshuffle_if_empty(g, rng);
    pl_put(g, P, L, deck_draw(g));
  }
}

// ------------------------------------------------------ hand knowledge pool
CIT_HD int kh_conf(const CitKH& e) { return e.conf_flags & 15; }
CIT_HD int kh_off(const CitGame& g, int e) {
  int o = 0;
  for (int i = 0; i < e; i++) o += g.kh[i].len;
  return o;
}
template <class At>
CIT_HD void kh_append(CitGame& g, int owner, int target, int conf, bool wizard, int n, At card_at) {
  CIT_CAP_NOTE(g, g.kh, g.n_kh + 1);
  CIT_CAP_NOTE(g, g.kh_pool, g.kh_fill + n);
  if (g.n_kh >= CIT_KH_MAX || g.kh_fill + n > CIT_KH_POOL) { g.err |= CIT_ERR_OVERFLOW; return; }
  CitKH& e = g.kh[g.n_kh++];
  e.owner = (uint8_t)owner;
  e.target = (int8_t)target;
  e.conf_flags = (uint8_t)(conf | (wizard ? 0x10 : 0));
  e.len = (uint8_t)n;
#if CIT_WAVE
  if (n <= 64) {
    int f = g.kh_fill, l = cit_lane();
    int v = 0;
    if (l < n) v = (int)card_at(l);
    if (l < n) g.kh_pool[f + l] = (uint8_t)v;
    g.kh_fill = (uint8_t)(f + n);
    return;
  }
#endif
  for (int i = 0; i < n; i++) g.kh_pool[g.kh_fill + i] = (uint8_t)card_at(i);
  g.kh_fill = (uint8_t)(g.kh_fill + n);
}
// get_a_card_like_it on one entry's hand
CIT_HD void kh_take_like(CitGame& g, int e, int c) {
#if CIT_WAVE
  {
    int l = cit_lane();
    int len_l = g.kh[l < CIT_KH_MAX ? l : 0].len;
    int off = (int)__ockl_wfred_add_u32(l < e && l < CIT_KH_MAX ? (unsigned)len_l : 0u);
    int n = cit_readlane(len_l, e < CIT_KH_MAX ? e : 0), fill = g.kh_fill, t = card_type(c);
    if (e >= CIT_KH_MAX || n > 64) goto serial;
    {
      int v = g.kh_pool[off + (l < n ? l : 0)];
      uint64_t m = cit_ballot(l < n && card_type(v) == t);
      if (!m) return;
      int s0 = off + __ffsll((unsigned long long)m);     // first byte after the match
      int cnt = fill - s0;
      int w[4];
#pragma unroll
      for (int k = 0; k < 4; k++) w[k] = k ? (l + 64 * k < cnt ? g.kh_pool[s0 + l + 64 * k] : 0) : cit_ld(g.kh_pool, s0 + l, l < cnt, 0);
      __asm__ volatile("" ::: "memory");   // every byte loaded before any is moved
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (l + 64 * k < cnt) g.kh_pool[s0 - 1 + l + 64 * k] = (uint8_t)w[k];
      g.kh[e].len = (uint8_t)(n - 1);
      g.kh_fill = (uint8_t)(fill - 1);
      return;
    }
  }
serial:
#endif
  int off = kh_off(g, e), n = g.kh[e].len, t = card_type(c);
  for (int i = 0; i < n; i++) {
    if (card_type(g.kh_pool[off + i]) == t) {
      for (int j = off + i + 1; j < g.kh_fill; j++) g.kh_pool[j - 1] = g.kh_pool[j];
      g.kh[e].len--;
      g.kh_fill--;
      return;
    }
  }
}
// substract_from_known_hand_confidences_and_clear_wizard (agent.py:100-109), all owners
CIT_HD void kh_decay(CitGame& g) {
#if CIT_WAVE
  {   // lane e holds entry e; a kept entry's cards move left by one lane-parallel
      // copy (all lanes load before any stores), its record by one compaction store
    const int n = g.n_kh, l = cit_lane();
    CitKH k = g.kh[l < n ? l : 0];
    const int len = l < n ? k.len : 0, conf = kh_conf(k) - 1;
    const bool keep = l < n && conf != 0;
    int ro = 0, wo = 0;
    for (int e = 0; e < n; e++) {
      int le = cit_readlane(len, e);
      if (cit_readlane(conf, e) != 0) {
        if (wo != ro)
          for (int i = l; i < le; i += 64) {
            int v = g.kh_pool[ro + i];
            g.kh_pool[wo + i] = (uint8_t)v;
          }
        wo += le;
      }
      ro += le;
    }
    const uint64_t km = cit_ballot(keep);
    k.conf_flags = (uint8_t)(conf & 15);
    if (keep) g.kh[__popcll(km & cit_below())] = k;
    g.n_kh = (uint8_t)__popcll(km);
    g.kh_fill = (uint8_t)wo;
    return;
  }
#endif
  int w = 0, wo = 0, ro = 0;
  for (int e = 0; e < g.n_kh; e++) {
    CitKH k = g.kh[e];
    int conf = kh_conf(k) - 1;
    int len = k.len;
    if (conf != 0) {
      for (int i = 0; i < len; i++) g.kh_pool[wo + i] = g.kh_pool[ro + i];
      k.conf_flags = (uint8_t)(conf & 15);
      g.kh[w++] = k;
      wo += len;
    }
    ro += len;
  }
  g.n_kh = (uint8_t)w;
  g.kh_fill = (uint8_t)wo;
}

// ------------------------------------------------------------------ roles
// role_to_role_id (config.py:93-121); ROLE_NONE is a KeyError
CIT_HD int role_rank(CitGame& g, int role) {
  if (role == ROLE_BEWITCHED) return -1;
  if (role >= 27) { g.err |= CIT_ERR_KEY; return 0; }
  return role / 3;
}
// role_properties[role_to_role_id[role]]: the dict has keys 0..7 only, so the
// Bewitched (-1) and the rank-8 roles (24..26: Queen, Artist, Tax Collector)
// are KeyErrors
CIT_HD uint8_t& rp_of(CitGame& g, int role) {
  int r = role_rank(g, role);
  if (r < 0 || r >= 8) { g.err |= CIT_ERR_KEY; r = 0; }
  return g.rp[r];
}
CIT_HD int rp_warrant(uint8_t v) { return (v >> RP_WARRANT_SHIFT) & 3; }
CIT_HD int rp_blackmail(uint8_t v) { return (v >> RP_BLACKMAIL_SHIFT) & 3; }
CIT_HD int role_of_id(const CitGame& g, int rid) { return rid < 0 ? ROLE_BEWITCHED : g.roles[rid]; }
// get_player_from_role_id (game.py:403-412); -1 for None
CIT_HD int holder(const CitGame& g, int rid) {
  int want = role_of_id(g, rid);
#if CIT_WAVE
  {
    int i = cit_lane();
    const int ri = g.pl[i < CIT_NP ? i : 0].role;
    uint64_t m = cit_ballot((i < CIT_NP) & (ri == want));
    return m ? __ffsll((unsigned long long)m) - 1 : -1;
  }
#endif
  for (int i = 0; i < CIT_NP; i++)
    if (g.pl[i].role == want) return i;
  return -1;
}
CIT_HD int holder_checked(CitGame& g, int rid) {
  int h = holder(g, rid);
  if (h < 0) { g.err |= CIT_ERR_ATTR; return 0; }
  return h;
}

// ---------------------------------------------------------- game states
CIT_HD void gs_set(CitGame& g, int state, int pid) {
  g.gs_state = (uint8_t)state;
  g.gs_pid = (int8_t)pid;
}
CIT_HD void gs_append(CitGame& g, int tok) {
  g.gs_adm[tok]++;
  if (g.nx_valid && g.nx_alias) g.nx_adm[tok]++;
}
// next_gamestate = GameState(state=5, player_id=pid, already_done_moves=<alias|fresh|[ability]>)
enum { NX_FRESH = 0, NX_ALIAS = 1, NX_ABILITY = 2 };
CIT_HD void gs_make_next(CitGame& g, int pid, int mode) {
  g.nx_valid = 1;
  g.nx_state = 5;
  g.nx_pid = (int8_t)pid;
  for (int i = 0; i < ADM_N; i++) g.nx_adm[i] = mode == NX_ALIAS ? g.gs_adm[i] : 0;
  if (mode == NX_ABILITY) g.nx_adm[ADM_ABILITY] = 1;
  g.nx_intr = 0;
  g.nx_alias = mode == NX_ALIAS;
  g.nx_hasnext = 0;
}
// game.gamestate = game.gamestate.next_gamestate
CIT_HD void gs_goto_next(CitGame& g) {
  if (!g.nx_valid) { g.err |= CIT_ERR_ATTR; return; }
  g.gs_state = g.nx_state;
  g.gs_pid = g.nx_pid;
  for (int i = 0; i < ADM_N; i++) g.gs_adm[i] = g.nx_adm[i];
  g.gs_intr = g.nx_intr;
  g.nx_valid = 0;
  g.nx_alias = 0;
}
// a brand-new GameState(state, pid) replaces the current one
CIT_HD void gs_fresh(CitGame& g, int state, int pid) {
  gs_set(g, state, pid);
  for (int i = 0; i < ADM_N; i++) g.gs_adm[i] = 0;
  g.gs_intr = 0;
  g.nx_valid = 0;
  g.nx_alias = 0;
}
CIT_HD void gs_rebind_adm(CitGame& g) {   // gamestate.already_done_moves = []
  for (int i = 0; i < ADM_N; i++) g.gs_adm[i] = 0;
  g.nx_alias = 0;
}
CIT_HD void at5(CitGame& g, int pid, int tok) {
  gs_set(g, 5, pid);
  if (tok >= 0) gs_append(g, tok);
}

// ================================================================= setup
// refresh_used_roles (game.py:349-357)
CIT_HD void refresh_used_roles(CitGame& g) {
#if CIT_WAVE
  {   // lane i: player i's role rank; its place in the stable sort by counting
    const int l = cit_lane();
    const int role = g.pl[l < CIT_NP ? l : 0].role;
    if (cit_ballot(l < CIT_NP && role != ROLE_BEWITCHED && role >= 27)) g.err |= CIT_ERR_KEY;
    const int v = role == ROLE_BEWITCHED ? -1 : role >= 27 ? 0 : role / 3;
    int pos = 0;
    for (int j = 0; j < CIT_NP; j++) {
      int vj = cit_readlane(v, j);
      pos += (vj < v || (vj == v && j < l)) ? 1 : 0;
    }
    if (l < CIT_NP) g.used_roles[pos] = (int8_t)v;
    g.n_used_roles = CIT_NP;
    return;
  }
#endif
  int8_t v[CIT_NP];
  for (int i = 0; i < CIT_NP; i++) v[i] = (int8_t)role_rank(g, g.pl[i].role);
  for (int i = 1; i < CIT_NP; i++) {     // insertion sort
    int8_t x = v[i];
    int j = i - 1;
    while (j >= 0 && v[j] > x) { v[j + 1] = v[j]; j--; }
    v[j + 1] = x;
  }
  for (int i = 0; i < CIT_NP; i++) g.used_roles[i] = v[i];
  g.n_used_roles = CIT_NP;
}
// setup_next_player (game.py:391-401); current < 0 means "no current player"
CIT_HD void setup_next_player(CitGame& g, int current) {
  if (g.gs_state == 0) {
    refresh_used_roles(g);
    g.gs_state = 1;
    g.gs_pid = (int8_t)holder_checked(g, g.used_roles[0]);
  } else if (current >= 0) {
    g.gs_state = 1;
    int r = role_rank(g, g.pl[current].role);
    int i = -1;
#if CIT_WAVE
    {
      int k = cit_lane(), nu = g.n_used_roles;
      const int uk = g.used_roles[k < CIT_NP ? k : 0];
      uint64_t m = cit_ballot((k < nu) & (k < CIT_NP) & (uk == r));
      if (nu <= CIT_NP) i = m ? __ffsll((unsigned long long)m) - 1 : -1;
      else
        for (int kk = 0; kk < nu; kk++)
          if (g.used_roles[kk] == r) { i = kk; break; }
    }
#else
    for (int k = 0; k < g.n_used_roles; k++)
      if (g.used_roles[k] == r) { i = k; break; }
#endif
    if (i < 0) { g.err |= CIT_ERR_VALUE; return; }
    if (i + 1 >= g.n_used_roles) { g.err |= CIT_ERR_INDEX; return; }
    g.gs_pid = (int8_t)holder_checked(g, g.used_roles[i + 1]);
    gs_rebind_adm(g);
  } else {
    g.err |= CIT_ERR_UNSUPPORTED;
  }
}

CIT_HD void cit_setup_round(CitGame& g, CitMT& rng) {
  for (int r = 0; r < 8; r++) g.rp[r] = 0;
  g.n_used_roles = 0;
  // the 8 ranks shuffled (random.shuffle) as nibbles of one register word
  uint32_t pool = 0x76543210u;
  for (int i = 7; i > 0; i--) {
    int j = (int)mt_randbelow(rng, (uint32_t)(i + 1));
    uint32_t ai = (pool >> (4 * i)) & 15u, aj = (pool >> (4 * j)) & 15u;
    pool &= ~((15u << (4 * i)) | (15u << (4 * j)));
    pool |= (aj << (4 * i)) | (ai << (4 * j));
  }
  uint8_t m = 0;
  for (int r = 0; r < 7; r++) m |= (uint8_t)(1u << ((pool >> (4 * r)) & 15u));   // pool[7] is the face-down role
  g.rtc = m;
  int c = -1;
#if CIT_WAVE
  {
    int i = cit_lane();
    const int fi = g.pl[i < CIT_NP ? i : 0].flags;
    uint64_t m = cit_ballot((i < CIT_NP) & ((fi & PF_CROWN) != 0));
    c = m ? __ffsll((unsigned long long)m) - 1 : -1;
    if (c < 0) { g.err |= CIT_ERR_UNSUPPORTED; return; }
    int v = cit_ld(g.turn, (i + c) % CIT_NP, i < CIT_NP, 0);    // every lane reads before any lane writes
    if (i < CIT_NP) g.turn[i] = (uint8_t)v;
    gs_fresh(g, 0, cit_readlane(v, 0));
    kh_decay(g);
    if (i < CIT_NP * CIT_NP) g.pl[i / CIT_NP].kr[i % CIT_NP] = 0;
    return;
  }
#endif
  for (int i = 0; i < CIT_NP; i++)
    if (g.pl[i].flags & PF_CROWN) { c = i; break; }
  if (c < 0) { g.err |= CIT_ERR_UNSUPPORTED; return; }     // turn order would double (game.py:164-165)
  uint8_t t[CIT_NP];
  for (int i = 0; i < CIT_NP; i++) t[i] = g.turn[(i + c) % CIT_NP];
  for (int i = 0; i < CIT_NP; i++) g.turn[i] = t[i];
  gs_fresh(g, 0, g.turn[0]);
  kh_decay(g);
  for (int i = 0; i < CIT_NP; i++)
    for (int j = 0; j < CIT_NP; j++) g.pl[i].kr[j] = 0;
}

// Game(preset) + set_initial_variables + create_game's setup_round, for a
// game whose CPython stream has just been seeded.
CIT_HD void cit_init_game(CitGame& g, CitMT& rng, bool preset) {
  // building_cards multiplicities per type 0..15, one nibble each (config.py:2-52)
  const uint64_t kBaseCounts = 0x3543333233324335ull;
  uint8_t uniq[24];
  for (int i = 0; i < 24; i++) uniq[i] = (uint8_t)(i == 0 ? 16 : i == 1 || i == 2 ? 17 : i < 23 ? i + 15 : 39);
  int n = 0;
#if CIT_WAVE
  {   // the row zeroed and the 52 base cards (+ the 24 uniques of the preset) laid out by the lanes
    const int l = cit_lane();
    static_assert(sizeof(CitGame) % 4 == 0, "row words");
    for (int i = l; i < (int)(sizeof(CitGame) / 4); i += 64) reinterpret_cast<uint32_t*>(&g)[i] = 0;
    int v0 = 0, v1 = 0, off = 0;
    for (int k = 0; k < 16; k++) {
      int cnt = (int)((kBaseCounts >> (4 * k)) & 15);
      if (l >= off && l < off + cnt) v0 = k;
      if (l + 64 >= off && l + 64 < off + cnt) v1 = k;
      off += cnt;
    }
    n = off;                                        // 52
    if (preset) {
      int u = l - n;
      if (u >= 0 && u < 24) v0 = u == 0 ? 16 : u == 1 || u == 2 ? 17 : u < 23 ? u + 15 : 39;
      int u1 = l + 64 - n;
      if (u1 >= 0 && u1 < 24) v1 = u1 == 0 ? 16 : u1 == 1 || u1 == 2 ? 17 : u1 < 23 ? u1 + 15 : 39;
    }
    int nn = preset ? n + 24 : n;
    if (l < nn) g.deck[l] = (uint8_t)v0;
    if (l + 64 < nn) g.deck[l + 64] = (uint8_t)v1;
    n = nn;
  }
  if (!preset) {
#else
  uint8_t* z = (uint8_t*)&g;
  for (int i = 0; i < (int)sizeof(CitGame); i++) z[i] = 0;
  for (int k = 0; k < 16; k++)
    for (int j = 0; j < (int)((kBaseCounts >> (4 * k)) & 15); j++) g.deck[n++] = (uint8_t)k;
  if (preset) {
    for (int i = 0; i < 24; i++) g.deck[n++] = uniq[i];
  } else {
#endif
    // random.sample(unique_building_cards, 14): pool variant (Lib/random.py:483-490)
    uint8_t pool[24];
    for (int i = 0; i < 24; i++) pool[i] = uniq[i];
    for (int i = 0; i < 14; i++) {
      int j = (int)mt_randbelow(rng, (uint32_t)(24 - i));
      g.deck[n++] = pool[j];
      pool[j] = pool[24 - i - 1];
    }
  }
  g.deck_head = 0;
  g.n_deck = (uint8_t)n;
  deck_shuffle(g, rng);
#if CIT_WAVE
  {
    const int l = cit_lane();
    int d0 = cit_ld(g.deck, l, l < n, 0), d1 = l + 64 < n ? g.deck[l + 64] : 0;
    if (l < n) g.used_cards[l] = (uint8_t)d0;
    if (l + 64 < n && l + 64 < CIT_USED_CAP) g.used_cards[l + 64] = (uint8_t)d1;
  }
#else
  for (int i = 0; i < n; i++) g.used_cards[i] = g.deck[i];
#endif
  g.n_used_cards = (uint8_t)n;
  for (int i = 0; i < CIT_NP; i++) {
    g.pl[i].gold = 2;
    g.pl[i].role = ROLE_NONE;
  }
  if (preset) {
    // set_preset hands (game.py:428-474), one byte per card
    const uint64_t kHands[6] = {0x131211100000ull, 0x171615140101ull, 0x1b1a19180302ull,
                                0x1f1e1d1c0403ull, 0x232221200004ull, 0x002725240100ull};
    for (int p = 0; p < CIT_NP; p++)
      for (int k = 0; k < 6; k++) pl_put(g, g.pl[p], AL_HAND, deck_take_like(g, (int)((kHands[p] >> (8 * k)) & 0xFF)));
    g.pl[3].flags |= PF_CROWN;
    // Witch, Spy, Wizard, King, Abbot, Alchemist, Navigator, Warlord (game.py:479-486)
    const uint64_t kRoles = 0x1513100d09070401ull;
    for (int r = 0; r < 8; r++) g.roles[r] = (uint8_t)((kRoles >> (8 * r)) & 0xFF);
    for (int i = 0; i < CIT_NP; i++) g.turn[i] = (uint8_t)i;
  } else {
    for (int k = 0; k < 4; k++)
      for (int p = 0; p < CIT_NP; p++) pl_put(g, g.pl[p], AL_HAND, deck_draw(g));
    for (int r = 0; r < 8; r++) g.roles[r] = (uint8_t)(r * 3 + (int)mt_randbelow(rng, 3));
    for (int i = 0; i < CIT_NP; i++) g.turn[i] = (uint8_t)i;
    shuffle_arr(rng, g.turn, CIT_NP);
    int crown = (int)mt_randbelow(rng, 6);
    g.pl[crown].flags |= PF_CROWN;
  }
  g.preset = preset;
  g.gs_pid = -1;
  g.winner = -1;
  g.warrant = CIT_NO_CARD;
  g.n_seer = 255;
  g.n_used_roles = 255;
  cit_setup_round(g, rng);
}

// ============================================================ scoring
CIT_HD int count_points(const CitPlayer& p) {           // agent.py:116-143
  int pts = 0;
  bool well = p_has(p, 31);
  for (int i = 0; i < p.n_build; i++) {
    int c = p.build[i], t = card_type(c);
    pts += card_cost(c);
    if (t == 18 || t == 23) pts += 2;
    if (well && card_suit(c) == SUIT_UNIQUE) pts += 1;
  }
  if (p.n_build >= 7) pts += 2;
  if (p.flags & PF_FIRST7) pts += 4;
  pts += p.n_museum;
  if (p_has(p, 37)) pts += p.gold;
  if (p_has(p, 39)) pts += p.n_hand;
  return pts;
}
// check_game_ending (game.py:359-368): winner index or -1
CIT_HD int check_game_ending(CitGame& g) {
  if (!g.ending) return -1;
  int best = 0;
  for (int i = 0; i < CIT_NP; i++) {
    g.points[i] = (int16_t)count_points(g.pl[i]);
    if (g.points[i] > g.points[best]) best = i;
  }
  g.has_points = 1;
  g.terminal = 1;
  g.winner = (int8_t)best;
  return best;
}
// is_last_round (game.py:173-181)
CIT_HD void is_last_round(CitGame& g) {
#if CIT_WAVE
  {
    // both loads issued before either is tested: one LDS round trip
    int i = cit_lane();
    int ending = g.ending;
    int nb = g.pl[i < CIT_NP ? i : 0].n_build;
    if (ending || !cit_ballot(i < CIT_NP && nb == 7)) return;
  }
#endif
  if (g.ending) return;
  for (int i = 0; i < CIT_NP; i++)
    if (g.pl[i].n_build == 7) {
      g.ending = 1;
      g.pl[i].flags |= PF_FIRST7;
    }
}

// ======================================================= option helpers
CIT_HD CitOpt mk(int name, int perp, int target = -1, int a = 0, int b = 0, int c = 0, int flags = 0,
                 uint64_t x = 0) {
  CitOpt o;
  o.name = (uint8_t)name;
  o.perp = (uint8_t)perp;
  o.target = (int8_t)target;
  o.a = (uint8_t)a;
  o.b = (uint8_t)b;
  o.c = (uint8_t)c;
  o.d = 0;
  o.flags = (uint8_t)flags;
  o.x = x;
  return o;
}
enum { OF_TUPLE = 1, OF_NEXT_WITCH = 1, OF_CROWN = 2, OF_BUILD = 1, OF_FACTORY = 1 };

#if CIT_WAVE
// Lane-parallel generation (CIT_WAVE): every lane proposes one option (p, o);
// the proposals are taken in lane order, i.e. lane i plays iteration i of
// the reference's loop.  cit_lane_rank = number of proposing lanes below.
__device__ __forceinline__ int cit_lane_rank(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
__device__ __forceinline__ CitOpt cit_readlane_opt(const CitOpt& o, int src) {
  uint32_t w[4];
  __builtin_memcpy(w, &o, 16);
  for (int j = 0; j < 4; j++) w[j] = (uint32_t)__builtin_amdgcn_readlane((int)w[j], src);
  CitOpt r;
  __builtin_memcpy(&r, w, 16);
  return r;
}
// true on the lowest valid lane of each key (the reference's `seen` sets:
// first occurrence wins).  All lanes must be active.
// One uniform iteration per distinct key: the lowest valid lane left takes its
// key's whole ballot out of the set, so no lane leaves the loop early (no
// exec-mask bookkeeping) and the count is the keys', not the lanes'.
__device__ __forceinline__ bool cit_first_key(bool valid, int key) {
#ifndef CIT_FIRST_KEY_LANES
  uint64_t m = cit_ballot(valid), first = 0;
  while (m) {
    const int j = __ffsll((unsigned long long)m) - 1;
    const int kj = __builtin_amdgcn_readlane(key, j);
    m &= ~cit_ballot(valid && key == kj);   // j and every later lane with its key
    first |= 1ull << j;
  }
  return (first >> cit_lane()) & 1;
#else
  uint64_t m = cit_ballot(valid);
  int me = cit_lane();
  bool dup = false;
  while (m) {
    int j = __ffsll((unsigned long long)m) - 1;
    m &= m - 1;
    if (j >= me) break;
    dup |= key == __builtin_amdgcn_readlane(key, j);
  }
  return valid && !dup;
#endif
}
// list sinks: proposals compacted into buf[n + rank]
#define CIT_WAVE_LIST_EMIT                                        \
  CIT_HD bool wave_emit(bool p, const CitOpt& o) {                \
    uint64_t m = cit_ballot(p);                                   \
    int r = n + cit_lane_rank(m);                                 \
    if (p && r < cap) buf[r] = o;                                 \
    n += __popcll(m);                                             \
    return false;                                                 \
  }
#else
#define CIT_WAVE_LIST_EMIT
#endif
#define WEMIT(p, o)                                \
  do {                                             \
    if (s.wave_emit((p), (o))) return true;        \
  } while (0)

// Sinks: emit() returns true to stop the enumeration.
// PickSink(k) stops at the k-th option (out); PickSink(-1) just counts (n).
// The fused rollout uses this one sink for both passes, so the enumerator is
// instantiated once in that kernel.
struct PickSink {
  int k;
  int n = 0;
  CitOpt out;
  uint32_t err = 0;
  CIT_HD explicit PickSink(int kk) : k(kk) { out = mk(O_NUM_NAMES, 0); }
  CIT_HD bool emit(const CitOpt& o) {
    if (n++ == k) { out = o; return true; }
    return false;
  }
  template <class F> CIT_HD bool block(int cnt, F&& f) {
    if (k >= n && k < n + cnt) { out = f(k - n); n = k + 1; return true; }
    n += cnt;
    return false;
  }
#if CIT_WAVE
  CIT_HD bool wave_emit(bool p, const CitOpt& o) {
    uint64_t m = cit_ballot(p);
    int c = __popcll(m);
    if (k >= n && k < n + c) {
      uint64_t hit = cit_ballot(p && cit_lane_rank(m) == k - n);
      out = cit_readlane_opt(o, __ffsll((unsigned long long)hit) - 1);
      n = k + 1;
      return true;
    }
    n += c;
    return false;
  }
#endif
};
struct ListSink {
  CitOpt* buf;
  int cap;
  int n = 0;
  uint32_t err = 0;
  CIT_HD ListSink(CitOpt* b, int c) : buf(b), cap(c) {}
  CIT_HD bool emit(const CitOpt& o) {
    if (n < cap) buf[n] = o;
    n++;
    return false;
  }
  template <class F> CIT_HD bool block(int cnt, F&& f) {
    int m = cap - n < cnt ? cap - n : cnt;      // materialise up to cap, count the rest
    for (int i = 0; i < m; i++) buf[n + i] = f(i);
    n += cnt;
    return false;
  }
  CIT_WAVE_LIST_EMIT
};
// The step loop's sink: lists the first `cap` options into `buf` (LDS in the
// rollout kernel) while counting all of them.
struct BufSink {
  CitOpt* buf;
  int cap;
  int n = 0;
  uint32_t err = 0;
  CIT_HD BufSink(CitOpt* b, int c) : buf(b), cap(c) {}
  CIT_HD bool emit(const CitOpt& o) {
    if (n < cap) buf[n] = o;
    n++;
    return false;
  }
  template <class F> CIT_HD bool block(int cnt, F&& f) {
    int m = cap - n < cnt ? cap - n : cnt;
    for (int i = 0; i < m; i++) buf[n + i] = f(i);
    n += cnt;
    return false;
  }
  CIT_WAVE_LIST_EMIT
};

#if CIT_WAVE
// BufSink's list held in registers instead of LDS: lane i keeps option i (the
// first 64; more are only counted), so a serial emit is four lane selects
// and the draw four readlanes -- no LDS store per option, no LDS round trip
// for the pick.  A lane-parallel emit moves the proposals to lanes n + rank
// with one ds_permute per word (a bijection: the other lanes go to the
// remaining lanes, which keep their words).
struct RegSink {
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  int n = 0;
  uint32_t err = 0;
  __device__ __forceinline__ void put(const CitOpt& o) {
    uint32_t w[4];
    __builtin_memcpy(w, &o, 16);
    const bool me = (int)__lane_id() == n;
    r0 = me ? w[0] : r0;
    r1 = me ? w[1] : r1;
    r2 = me ? w[2] : r2;
    r3 = me ? w[3] : r3;
  }
  __device__ bool emit(const CitOpt& o) {
    if (n < 64) put(o);
    n++;
    return false;
  }
  template <class F> __device__ bool block(int cnt, F&& f) {
    int m = 64 - n < cnt ? 64 - n : cnt;
    for (int i = 0; i < m; i++) {
      put(f(i));
      n++;
    }
    n += cnt - (m > 0 ? m : 0);
    return false;
  }
  __device__ bool wave_emit(bool p, const CitOpt& o) {
    const uint64_t m = cit_ballot(p);
    const int c = __popcll(m);
    if (c && n < 64) {
      const int ln = (int)__lane_id();
      const int dst = (n + (p ? cit_lane_rank(m) : c + cit_lane_rank(~m))) & 63;
      uint32_t w[4];
      __builtin_memcpy(w, &o, 16);
      const int a = dst << 2;
      const uint32_t q0 = (uint32_t)__builtin_amdgcn_ds_permute(a, (int)w[0]);
      const uint32_t q1 = (uint32_t)__builtin_amdgcn_ds_permute(a, (int)w[1]);
      const uint32_t q2 = (uint32_t)__builtin_amdgcn_ds_permute(a, (int)w[2]);
      const uint32_t q3 = (uint32_t)__builtin_amdgcn_ds_permute(a, (int)w[3]);
      const bool mine = ln >= n && ln < n + c;
      r0 = mine ? q0 : r0;
      r1 = mine ? q1 : r1;
      r2 = mine ? q2 : r2;
      r3 = mine ? q3 : r3;
    }
    n += c;
    return false;
  }
  // option k < 64 (k wave-uniform)
  __device__ __forceinline__ CitOpt at(int k) const {
    uint32_t w[4] = {(uint32_t)__builtin_amdgcn_readlane((int)r0, k), (uint32_t)__builtin_amdgcn_readlane((int)r1, k),
                     (uint32_t)__builtin_amdgcn_readlane((int)r2, k), (uint32_t)__builtin_amdgcn_readlane((int)r3, k)};
    CitOpt o;
    __builtin_memcpy(&o, w, 16);
    return o;
  }
};
#endif

// skip_false_choice only asks whether a state has exactly one option: this
// sink lists like ListSink but, when `stop` is set, ends the enumeration once
// a second option is known (n is then a lower bound >= 2).  Callers clear
// `stop` where the full enumeration may still raise after emitting options
// (cit_enum_late_error), so the error bits are the full enumeration's.
struct Upto2Sink {
  CitOpt* buf;
  int cap;
  int n = 0;
  uint32_t err = 0;
  bool stop;
  CIT_HD Upto2Sink(CitOpt* b, int c, bool s) : buf(b), cap(c), stop(s) {}
  CIT_HD bool emit(const CitOpt& o) {
    if (n < cap) buf[n] = o;
    n++;
    return stop && n >= 2;
  }
  template <class F> CIT_HD bool block(int cnt, F&& f) {
    int m = cap - n < cnt ? cap - n : cnt;
    if (stop && m > 2) m = 2;
    for (int i = 0; i < m; i++) buf[n + i] = f(i);
    n += cnt;
    return stop && n >= 2;
  }
#if CIT_WAVE
  CIT_HD bool wave_emit(bool p, const CitOpt& o) {
    uint64_t m = cit_ballot(p);
    int r = n + cit_lane_rank(m);
    if (p && r < cap) buf[r] = o;
    n += __popcll(m);
    return stop && n >= 2;
  }
#endif
};

#if CIT_WAVE
// Upto2Sink keeping only the first option, wave-uniform (skip_false_choice
// carries it out when it is the only one): no list in LDS.
struct Upto2FirstSink {
  int n = 0;
  uint32_t err = 0;
  bool stop;
  CitOpt first;
  __device__ explicit Upto2FirstSink(bool s) : stop(s) {}
  __device__ bool emit(const CitOpt& o) {
    if (n == 0) first = o;
    n++;
    return stop && n >= 2;
  }
  template <class F> __device__ bool block(int cnt, F&& f) {
    if (n == 0 && cnt > 0) first = f(0);
    n += cnt;
    return stop && n >= 2;
  }
  __device__ bool wave_emit(bool p, const CitOpt& o) {
    const uint64_t m = cit_ballot(p);
    if (n == 0 && m) first = cit_readlane_opt(o, __ffsll((unsigned long long)m) - 1);
    n += __popcll(m);
    return stop && n >= 2;
  }
};
#endif

#define EMIT(...)                                  \
  do {                                             \
    if (s.emit(__VA_ARGS__)) return true;          \
  } while (0)

// Python round(x/1e2) (half to even) on an integer count, floored at 1
// (agent_functions.py:293,416).
CIT_HD long subsample_stride(long c) {
  long q = c / 100, r = c % 100;
  if (r > 50 || (r == 50 && (q & 1))) q++;
  return q < 1 ? 1 : q;
}
CIT_HD long binom(int n, int k) {
  if (k < 0 || k > n) return 0;
  if (k > n - k) k = n - k;
  long r = 1;
  for (int i = 1; i <= k; i++) r = r * (n - k + i) / i;
  return r;
}
// lexicographic combination number `idx` of k items out of n (itertools.combinations order)
CIT_HD uint64_t unrank_comb(int n, int k, long idx) {
  uint64_t m = 0;
  int x = 0;
  for (int i = 0; i < k; i++) {
    while (true) {
      long c = binom(n - x - 1, k - i - 1);
      if (idx < c) break;
      idx -= c;
      x++;
    }
    m |= 1ull << x;
    x++;
  }
  return m;
}

// ================================================== option generators
// build_options / get_builds (agent_functions.py:108-130)
template <class S>
CIT_HD bool gen_builds(const CitGame& g, int a, uint64_t bm, S& s) {
  const CitPlayer& P = g.pl[a];
  const int role = P.role, adm_nt = g.gs_adm[ADM_NON_TRADE], adm_tr = g.gs_adm[ADM_TRADE];
#if CIT_WAVE
  const int nh = P.n_hand, gold = P.gold, reps = P.replicas;   // loaded with the role: one round trip
  __asm__ volatile("" ::"v"(role), "v"(adm_nt), "v"(adm_tr), "v"(nh), "v"(gold), "v"(reps));
#endif
  int lim = role == R_ARCHITECT ? 3 : role == R_SCHOLAR ? 2 : (role == R_BISHOP || role == R_NAVIGATOR) ? 0 : 1;
  int done = adm_nt + (role == R_TRADER ? 0 : adm_tr);
  if (done >= lim) return false;
  bool factory = HAS(bm, 35);
#if CIT_WAVE
  {
    int i = cit_lane();
    int c = 0, t = 0;
    bool q = false;
    if (i < nh) {
      c = P.hand[i];
      t = card_type(c);
      q = card_cost(c) + (factory && card_suit(c) == SUIT_UNIQUE ? 1 : 0) <= gold;
    }
    int rep = (HAS(bm, t) && !reps) ? reps + 1 : 0;
    WEMIT(cit_first_key(q, t), mk(O_BUILD, a, -1, c, 0, rep));
    return false;
  }
#endif
  uint64_t seen = 0;
  for (int i = 0; i < P.n_hand; i++) {
    int c = P.hand[i], t = card_type(c);
    int cost = card_cost(c) + (factory && card_suit(c) == SUIT_UNIQUE ? 1 : 0);
    int rep = (HAS(bm, t) && !P.replicas) ? P.replicas + 1 : 0;
    if (cost <= P.gold && !((seen >> t) & 1)) {
      seen |= 1ull << t;
      EMIT(mk(O_BUILD, a, -1, c, 0, rep));
    }
  }
  return false;
}

template <class S>
CIT_HD bool gen_emperor(const CitGame& g, int a, bool dead, S& s) {   // agent_functions.py:368-382
  for (int p = 0; p < CIT_NP; p++) {
    if (p == a) continue;
    const CitPlayer& Q = g.pl[p];
    if (Q.n_hand && !dead) EMIT(mk(O_GIVE_CROWN, a, p, 0));
    if (Q.gold && !dead) EMIT(mk(O_GIVE_CROWN, a, p, 1));
    if ((!Q.gold && !Q.n_hand) || dead) EMIT(mk(O_GIVE_CROWN, a, p, 2));
  }
  return false;
}

// character_options' per-role generators (agent_functions.py:156-504)
template <class S>
CIT_HD bool gen_role(const CitGame& g, int a, S& s) {
  const CitPlayer& P = g.pl[a];
  switch (P.role) {
    case R_ASSASSIN:
#if CIT_WAVE
      WEMIT(cit_lane() >= 1 && cit_lane() < 8, mk(O_ASSASSINATION, a, -1, cit_lane()));
      return false;
#endif
      for (int r = 1; r < 8; r++) EMIT(mk(O_ASSASSINATION, a, -1, r));
      return false;
    case R_MAGISTRATE:
      for (int r = 1; r < 8; r++)
        for (int f0 = 1; f0 < 8; f0++)
          for (int f1 = f0 + 1; f1 < 8; f1++)
            if (r != f0 && r != f1) EMIT(mk(O_MAGISTRATE_WARRANT, a, -1, r, f0, f1));
      return false;
    case R_THIEF:
#if CIT_WAVE
      WEMIT(cit_lane() >= 2 && cit_lane() < 8, mk(O_STEAL, a, -1, cit_lane()));
      return false;
#endif
      for (int r = 2; r < 8; r++) EMIT(mk(O_STEAL, a, -1, r));
      return false;
    case R_BLACKMAILER: {
      uint8_t t = 0xFC;   // ranks 2..7
      for (int r = 0; r < 8; r++)
        if (g.rp[r] & RP_POSSESSED) {
          if (!((t >> r) & 1)) { s.err |= CIT_ERR_VALUE; return true; }
          t &= (uint8_t)~(1u << r);
        }
      for (int x = 0; x < 8; x++)
        for (int y = x + 1; y < 8; y++)
          if (((t >> x) & 1) && ((t >> y) & 1)) {
            EMIT(mk(O_BLACKMAIL, a, -1, x, y));
            EMIT(mk(O_BLACKMAIL, a, -1, y, x));
          }
      return false;
    }
    case R_SPY:
#if CIT_WAVE
      {
        int i = cit_lane(), p = i / 5;
        WEMIT(i < 5 * CIT_NP && p != a, mk(O_SPY, a, p, i - 5 * p));
        return false;
      }
#endif
      for (int p = 0; p < CIT_NP; p++)
        if (p != a)
          for (int su = 0; su < 5; su++) EMIT(mk(O_SPY, a, p, su));
      return false;
    case R_MAGICIAN: {
      int n = P.n_hand;
      if (n > CIT_HAND_MASK_MAX) { s.err |= CIT_ERR_UNSUPPORTED; return true; }   // (cit_core.h)
      for (int p = 0; p < CIT_NP; p++)
        if (p != a) EMIT(mk(O_MAGIC_HAND_CHANGE, a, p));
      for (int r = 1; r <= n; r++) {
        long C = binom(n, r), st = subsample_stride(C);
        int cnt = (int)((C + st - 1) / st);
        if (s.block(cnt, [&](int i) { return mk(O_DISCARD_AND_DRAW, a, -1, r, 0, 0, 0, unrank_comb(n, r, (long)i * st)); }))
          return true;
      }
      return false;
    }
    case R_WIZARD:
#if CIT_WAVE
      {
        int p = cit_lane();
        const int nhp = g.pl[p < CIT_NP ? p : 0].n_hand;
        WEMIT((p < CIT_NP) & (p != a) & (nhp > 0), mk(O_LOOK_AT_HAND, a, p));
        return false;
      }
#endif
      for (int p = 0; p < CIT_NP; p++)
        if (p != a && g.pl[p].n_hand > 0) EMIT(mk(O_LOOK_AT_HAND, a, p));
      return false;
    case R_SEER:
      EMIT(mk(O_SEER, a));
      return false;
    case R_KING:
      EMIT(mk(O_TAKE_CROWN_KING, a));
      return false;
    case R_EMPEROR:
      return gen_emperor(g, a, false, s);
    case R_PATRICIAN:
      EMIT(mk(O_TAKE_CROWN_PAT, a));
      return false;
    case R_BISHOP:
      EMIT(mk(O_BISHOP, a));
      return false;
    case R_CARDINAL: {
      bool factory_owned = p_has(P, 35);
      int n = P.n_hand;
      if (n > CIT_HAND_MASK_MAX) { s.err |= CIT_ERR_UNSUPPORTED; return true; }   // as the magician's
      for (int p = 0; p < CIT_NP; p++) {
        const CitPlayer& Q = g.pl[p];
        for (int i = 0; i < n; i++) {
          int c = P.hand[i], t = card_type(c);
          int cost = card_cost(c);
          bool factory = false;
          if (factory_owned && card_suit(c) == SUIT_UNIQUE) { cost += 1; factory = true; }
          int rep = (p_has(P, t) && !P.replicas) ? P.replicas + 1 : 0;
          if (cost > Q.gold) continue;
          int k = Q.gold - cost;
          if (k < 0) k = 0;
          if (n - 1 < k) continue;
          uint8_t slot[CIT_HAND_MASK_MAX];
          int m = 0;
          for (int j = 0; j < n; j++)
            if (card_type(P.hand[j]) != t) slot[m++] = (uint8_t)j;
          long C = binom(m, k), st = subsample_stride(C);
          int cnt = (int)((C + st - 1) / st);
          if (s.block(cnt, [&](int ii) {
                uint64_t cm = unrank_comb(m, k, (long)ii * st), hm = 0;
                for (int q = 0; q < m; q++)
                  if ((cm >> q) & 1) hm |= 1ull << slot[q];
                return mk(O_CARDINAL, a, p, c, k, rep, factory ? OF_FACTORY : 0, hm);
              }))
            return true;
        }
      }
      return false;
    }
    case R_ABBOT: {
      int n = count_suit(P.hand, P.n_hand, SUIT_RELIGION);
      for (int j = 0; n > 0 && j <= n; j++) EMIT(mk(O_ABBOT_GOLD_OR_CARD, a, -1, n, j));
      return false;
    }
    case R_MERCHANT:
      EMIT(mk(O_MERCHANT, a));
      return false;
    case R_TRADER:
      EMIT(mk(O_TRADER, a));
      return false;
    case R_ARCHITECT:
      EMIT(mk(O_ARCHITECT, a));
      return false;
    case R_NAVIGATOR:
      EMIT(mk(O_NAVIGATOR, a, -1, 0));
      EMIT(mk(O_NAVIGATOR, a, -1, 1));
      return false;
    case R_SCHOLAR:
      if (g.n_deck) EMIT(mk(O_SCHOLAR, a));
      return false;
    case R_WARLORD:
#if CIT_WAVE
      {
        // all seats at once: lane l = building l % 10 of seat l / 10 (p-major
        // order, as the loops); `seen` is per seat, so the key carries the seat
        int l = cit_lane(), p = l / 10, i = l - 10 * p, ps = p < CIT_NP ? p : 0;
        int nb = g.pl[ps].n_build, role = g.pl[ps].role, gold = P.gold;
        int b = g.pl[ps].build[i];
        if (!cit_ballot(i == 0 && p < CIT_NP && nb > 10)) {
          int t = card_type(b);
          bool q = p < CIT_NP && i < nb && nb < 7 && role != R_BISHOP && card_cost(b) - 1 <= gold && t != 17;
          WEMIT(cit_first_key(q, p * 64 + t), mk(O_WARLORD, a, p, b));
          return false;
        }
      }
#endif
      for (int p = 0; p < CIT_NP; p++) {
        const CitPlayer& Q = g.pl[p];
        if (Q.n_build >= 7 || Q.role == R_BISHOP) continue;
#if CIT_WAVE
        {
          int i = cit_lane(), nb = Q.n_build, gold = P.gold;
          int b = 0, t = 0;
          bool q = false;
          if (i < nb) {
            b = Q.build[i];
            t = card_type(b);
            q = card_cost(b) - 1 <= gold && t != 17;
          }
          WEMIT(cit_first_key(q, t), mk(O_WARLORD, a, p, b));
          continue;
        }
#endif
        uint64_t seen = 0;
        for (int i = 0; i < Q.n_build; i++) {
          int b = Q.build[i], t = card_type(b);
          if (card_cost(b) - 1 <= P.gold && t != 17 && !((seen >> t) & 1)) {
            seen |= 1ull << t;
            EMIT(mk(O_WARLORD, a, p, b));
          }
        }
      }
      return false;
    case R_MARSHAL:
      for (int p = 0; p < CIT_NP; p++) {
        const CitPlayer& Q = g.pl[p];
        if (p == a || Q.n_build >= 7 || Q.role == R_BISHOP) continue;
        uint64_t seen = 0;
        for (int i = 0; i < Q.n_build; i++) {
          int b = Q.build[i], t = card_type(b);
          if (card_cost(b) <= P.gold && card_cost(b) <= 3 && !p_has(P, t) && t != 17 && !((seen >> t) & 1)) {
            seen |= 1ull << t;
            EMIT(mk(O_MARSHAL, a, p, b));
          }
        }
      }
      return false;
    case R_DIPLOMAT:
      for (int p = 0; p < CIT_NP; p++) {
        const CitPlayer& Q = g.pl[p];
        if (p == a || Q.n_build >= 7 || Q.role == R_BISHOP) continue;
        uint64_t seen_e = 0;
        for (int i = 0; i < Q.n_build; i++) {
          int e = Q.build[i], te = card_type(e);
          if (te == 17 || p_has(P, te)) continue;   // whole row fails the condition
          bool dup_e = (seen_e >> te) & 1;
          seen_e |= 1ull << te;
          if (dup_e) continue;
          uint64_t seen_o = 0;
          for (int j = 0; j < P.n_build; j++) {
            int own = P.build[j], to = card_type(own);
            int diff = card_cost(e) - card_cost(own);
            if (diff <= P.gold && !((seen_o >> to) & 1)) {
              seen_o |= 1ull << to;
              EMIT(mk(O_DIPLOMAT, a, p, e, own, diff < 0 ? -diff : diff));
            }
          }
        }
      }
      return false;
    default:
      return false;   // Witch (handled earlier), Alchemist, rank-8 roles: no character options
  }
}

// main_round_options (agent_functions.py:133-147)
template <class S>
CIT_HD bool gen_main(const CitGame& g, int a, S& s) {
  const CitPlayer& P = g.pl[a];
  uint64_t bm;
  {
    CIT_PROF_SCOPE(25);
    bm = type_mask(P.build, P.n_build);
  }
  {
    CIT_PROF_SCOPE(26);
    if (gen_builds(g, a, bm, s)) return true;
  }
  {
    CIT_PROF_SCOPE(27);
    if (!g.gs_adm[ADM_ABILITY])
      if (gen_role(g, a, s)) return true;
  }
  CIT_PROF_SCOPE(28);
  // the fields the remaining tests read, in one round of loads
  const int role = P.role, gold = P.gold, pfl = P.flags;
  const int adm_beg = g.gs_adm[ADM_BEGGED], adm_tg = g.gs_adm[ADM_TAKE_GOLD], adm_sm = g.gs_adm[ADM_SMITHY],
            adm_lab = g.gs_adm[ADM_LAB], adm_ms = g.gs_adm[ADM_MAGIC_SCHOOL], adm_mu = g.gs_adm[ADM_MUSEUM];
#if CIT_WAVE
  __asm__ volatile("" ::"v"(role), "v"(gold), "v"(pfl), "v"(adm_beg), "v"(adm_tg), "v"(adm_sm), "v"(adm_lab),
                   "v"(adm_ms), "v"(adm_mu));
#endif
  if (role == R_ABBOT && !adm_beg) EMIT(mk(O_ABBOT_BEG, a));
  if ((role == R_WARLORD || role == R_MARSHAL || role == R_DIPLOMAT) && !adm_tg)
    EMIT(mk(O_TAKE_GOLD_WAR, a));
  if (HAS(bm, 21) && gold >= 2 && !adm_sm) EMIT(mk(O_SMITHY, a));
  if (HAS(bm, 22) && !adm_lab)
#if CIT_WAVE
  {
    int i = cit_lane(), nh = P.n_hand;
    WEMIT(i < nh, mk(O_LAB, a, -1, cit_ld(P.hand, i, i < nh, 0)));
  }
#else
    for (int i = 0; i < P.n_hand; i++) EMIT(mk(O_LAB, a, -1, P.hand[i]));
#endif
  if (!adm_ms && HAS(bm, 25))
#if CIT_WAVE
    WEMIT(cit_lane() < 5, mk(O_MAGIC_SCHOOL, a, -1, cit_lane()));
#else
    for (int su = 0; su < 5; su++) EMIT(mk(O_MAGIC_SCHOOL, a, -1, su));
#endif
  if (HAS(bm, 27))
    for (int p = 0; p < CIT_NP; p++)
      if (p != a)
#if CIT_WAVE
      {
        int i = cit_lane(), nb = g.pl[p].n_build;
        WEMIT(i < nb, mk(O_WEAPON_STORAGE, a, p, cit_ld(g.pl[p].build, i, i < nb, 0)));
      }
#else
        for (int i = 0; i < g.pl[p].n_build; i++) EMIT(mk(O_WEAPON_STORAGE, a, p, g.pl[p].build[i]));
#endif
  if (HAS(bm, 29) && (pfl & PF_LIGHTHOUSE)) {
    uint64_t seen = 0;
    for (int i = 0; i < g.n_deck; i++) {
      int c = deck_at(g, i), t = card_type(c);
      if (!((seen >> t) & 1)) {
        seen |= 1ull << t;
        EMIT(mk(O_LIGHTHOUSE, a, -1, c));
      }
    }
  }
  if (HAS(bm, 34) && !adm_mu) {
#if CIT_WAVE
    int i = cit_lane(), nh = P.n_hand;
    int c = cit_ld(P.hand, i, i < nh, 0);
    WEMIT(cit_first_key(i < nh, card_type(c)), mk(O_MUSEUM, a, -1, c));
#else
    uint64_t seen = 0;
    for (int i = 0; i < P.n_hand; i++) {
      int c = P.hand[i], t = card_type(c);
      if (!((seen >> t) & 1)) {
        seen |= 1ull << t;
        EMIT(mk(O_MUSEUM, a, -1, c));
      }
    }
#endif
  }
  EMIT(mk(O_FINISH_ROUND, a));
  return false;
}

// wizard_take_from_hand_options (agent_functions.py:310-326)
template <class S>
CIT_HD bool gen_wizard_take(const CitGame& g, int a, S& s) {
  const CitPlayer& P = g.pl[a];
  int e = -1, off = 0, o = 0;
  for (int i = 0; i < g.n_kh; i++) {
    const CitKH& k = g.kh[i];
    if (k.owner == a && kh_conf(k) == 5 && k.target != -1 && (k.conf_flags & 0x10)) { e = i; off = o; break; }
    o += k.len;
  }
  if (e < 0) { s.err |= CIT_ERR_ATTR; return true; }
  int tgt = g.kh[e].target;
  const uint64_t bm = type_mask(P.build, P.n_build);
  bool factory = HAS(bm, 35);
  int rep = 0;
  uint64_t seen_take = 0, seen_b0 = 0, seen_b1 = 0;
  int emitted = 0;
  for (int i = 0; i < g.kh[e].len; i++) {
    int c = g.kh_pool[off + i], t = card_type(c);
    if (!((seen_take >> t) & 1)) {
      seen_take |= 1ull << t;
      emitted++;
      EMIT(mk(O_TAKE_FROM_HAND, a, tgt, c, 0, 0, 0));
    }
    int cost = card_cost(c) + (factory && card_suit(c) == SUIT_UNIQUE ? 1 : 0);
    if (HAS(bm, t)) rep = P.replicas + 1;
    uint64_t& seen = rep == 0 ? seen_b0 : seen_b1;   // rep takes at most one non-zero value
    if (cost <= P.gold && !((seen >> t) & 1)) {
      seen |= 1ull << t;
      emitted++;
      EMIT(mk(O_TAKE_FROM_HAND, a, tgt, c, 0, rep, OF_BUILD));
    }
  }
  if (!emitted) EMIT(mk(O_EMPTY, a, -1, 1));
  return false;
}

// get_options dispatcher (agent.py:50-83) on a prepared game.
template <class S>
CIT_HD bool cit_enum_options(const CitGame& g, S& s, const uint64_t* seer) {
  CIT_PROF_SCOPE(29);
#if CIT_WAVE
  // the mover, the state, every seat's role (lane p) and every role's
  // properties (lane r) in one round of loads: the role and its properties
  // are then readlanes, not loads behind the mover's id
  const int l_ = cit_lane();
  const int prole_ = g.pl[l_ < CIT_NP ? l_ : 0].role, prp_ = g.rp[l_ & 7];
#endif
  int a = g.gs_pid;
  if (a < 0 || a >= CIT_NP) { s.err |= CIT_ERR_UNSUPPORTED; return true; }
  const CitPlayer& P = g.pl[a];
  int st = g.gs_state;
  if (st == 0) {
#if CIT_WAVE
    WEMIT(cit_lane() < 8 && ((g.rtc >> cit_lane()) & 1), mk(O_ROLE_PICK, a, -1, cit_lane()));
    return false;
#endif
    for (int r = 0; r < 8; r++)
      if ((g.rtc >> r) & 1) EMIT(mk(O_ROLE_PICK, a, -1, r));
    return false;
  }
#if CIT_WAVE
  int role = cit_readlane(prole_, a);
#else
  int role = P.role;
#endif
  bool crown = role == R_KING || role == R_PATRICIAN;
  bool bew = role == ROLE_BEWITCHED;
  if (!bew && role >= CIT_RP_ROLES) { s.err |= CIT_ERR_KEY; return true; }
  int rk = bew ? -1 : role / 3;
#if CIT_WAVE
  const int rp_rk = bew ? 0 : cit_readlane(prp_, rk);
#else
  const int rp_rk = bew ? 0 : g.rp[rk];
#endif
  if (bew || !(rp_rk & RP_DEAD)) {
    switch (st) {
      case 1:
        EMIT(mk(O_GOLD_OR_CARD, a, -1, 0));
        if (g.n_deck > 1) EMIT(mk(O_GOLD_OR_CARD, a, -1, 1));
        return false;
      case 2: {
        const uint8_t* jd = pl_jd(P);
        const int nj = P.n_jd;
        if (p_has(P, 20)) {
          for (int i = 0; i < nj; i++)
            for (int j = i + 1; j < nj; j++) EMIT(mk(O_WHICH_CARD, a, -1, jd[i], jd[j], 0, OF_TUPLE));
          return false;
        }
#if CIT_WAVE
        if (nj <= 64) {
          int i = cit_lane();
          int c = cit_ld(jd, i, i < nj, 0);
          WEMIT(cit_first_key(i < nj, card_type(c)), mk(O_WHICH_CARD, a, -1, c, CIT_NO_CARD));
          return false;
        }
#endif
        uint64_t seen = 0;
        for (int i = 0; i < nj; i++) {
          int t = card_type(jd[i]);
          if (!((seen >> t) & 1)) {
            seen |= 1ull << t;
            EMIT(mk(O_WHICH_CARD, a, -1, jd[i], CIT_NO_CARD));
          }
        }
        return false;
      }
      case 3:
        if (bew) { s.err |= CIT_ERR_KEY; return true; }
        if (rp_blackmail(rp_rk)) {
          EMIT(mk(O_BLACKMAIL_RESPONSE, a, -1, 0));
          EMIT(mk(O_BLACKMAIL_RESPONSE, a, -1, 1));
        } else {
          EMIT(mk(O_EMPTY, a, -1, 0));
        }
        return false;
      case 4:
      case 7:
        if (!g.nx_valid) { s.err |= CIT_ERR_ATTR; return true; }
        EMIT(mk(st == 4 ? O_REVEAL_BLACKMAIL : O_REVEAL_WARRANT, a, g.nx_pid, 0));
        EMIT(mk(st == 4 ? O_REVEAL_BLACKMAIL : O_REVEAL_WARRANT, a, g.nx_pid, 1));
        return false;
      case 6:
        if (P.gold > 0) EMIT(mk(O_GRAVEYARD, a));
        else EMIT(mk(O_EMPTY, a, -1, 1));
        return false;
      default:
        break;
    }
    if (role == R_WITCH) {
#if CIT_WAVE
      WEMIT(cit_lane() >= 1 && cit_lane() < 8, mk(O_BEWITCHING, a, -1, cit_lane()));
#else
      for (int r = 1; r < 8; r++) EMIT(mk(O_BEWITCHING, a, -1, r));
#endif
      return false;
    }
    if (bew) { s.err |= CIT_ERR_KEY; return true; }
    if (!(rp_rk & RP_POSSESSED)) {
      switch (st) {
        case 5:
          return gen_main(g, a, s);
        case 8: {
          // seer_give_back_card: the permutations were drawn by cit_prepare_options
          if (!seer) { s.err |= CIT_ERR_UNSUPPORTED; return true; }
          int k = g.n_seer == 255 ? 0 : g.n_seer;
          int cnt = k * P.n_hand * 3;
          if (s.block(cnt, [&](int i) {
                uint64_t v = seer[i];
                return mk(O_GIVE_BACK_CARD, a, -1, 0, (int)(v >> 56), 0, 0, v & 0x00FFFFFFFFFFFFFFull);
              }))
            return true;
          return false;
        }
        case 9:
          for (int i = 0; i < g.n_sch; i++) EMIT(mk(O_SCHOLAR_PICK, a, -1, g.sch[i]));
          return false;
        case 10:
          return gen_wizard_take(g, a, s);
        default:
          s.err |= CIT_ERR_NONE_OPTIONS;
          return true;
      }
    }
    EMIT(mk(O_FINISH_ROUND, a, -1, 0, 0, 0, OF_NEXT_WITCH | (crown ? OF_CROWN : 0)));
    return false;
  }
  if (role == R_EMPEROR && !g.gs_adm[ADM_ABILITY]) return gen_emperor(g, a, true, s);
  EMIT(mk(O_FINISH_ROUND, a, -1, 0, 0, 0, crown ? OF_CROWN : 0));
  return false;
}

// The mutating half of get_options:
//  * state 9: the scholar's iterate-while-remove over the shared seven-drawn
//    list (agent_functions.py:462-470);
//  * state 8: seer_give_back_card's shuffles (agent_functions.py:332-361),
//    which consume the game's CPython stream inside get_options; the drawn
//    permutations go to `seer` (CIT_SEER_MAX packed options per lane:
//    card i in byte i, handout count in byte 7).
// (+ CIT_AREA_CAP bytes after the options: the shuffled `rest` list of the
// give-back draws, kept out of private memory)
#define CIT_SEER_OPTS (5 * CIT_AREA_CAP * 3)
#define CIT_SEER_MAX (CIT_SEER_OPTS + CIT_AREA_CAP / 8)
static_assert(CIT_AREA_CAP % 8 == 0, "seer scratch tail in whole words");
CIT_HD void cit_prepare_options(CitGame& g, CitMT& rng, uint64_t* seer) {
  g.n_sch = 0;
  if ((g.gs_state != 9 && g.gs_state != 8) || g.gs_pid < 0) return;
  const CitPlayer& P = g.pl[g.gs_pid];
  if (P.role >= CIT_RP_ROLES) return;    // the dispatcher reports the error
  if (P.role == R_WITCH || (g.rp[P.role / 3] & (RP_DEAD | RP_POSSESSED))) return;
  if (g.gs_state == 8) {
    if (!seer) return;         // the enumerator reports UNSUPPORTED
    int k = g.n_seer == 255 ? 0 : g.n_seer;
    int n = P.n_hand, o = 0;
    uint8_t* rest = reinterpret_cast<uint8_t*>(seer + CIT_SEER_OPTS);
    for (int pos = 0; pos < k; pos++) {
      for (int j = 0; j < n; j++) {
        int card = P.hand[j], t = card_type(card);
        int m = 0;
        for (int q = 0; q < n; q++)
          if (card_type(P.hand[q]) != t) rest[m++] = P.hand[q];
        for (int rep = 0; rep < 3; rep++) {
          shuffle_arr(rng, rest, m);
          // perm = rest[:k-1]; perm.insert(pos, card)  (list.insert clamps pos)
          uint8_t perm[6];
          int take = k - 1 < m ? k - 1 : m, len = 0;
          int ins = pos < take ? pos : take;
          for (int q = 0; q < take; q++) {
            if (q == ins) perm[len++] = (uint8_t)card;
            perm[len++] = rest[q];
          }
          if (ins == take) perm[len++] = (uint8_t)card;
          int h = len < k ? len : k;
          uint64_t v = (uint64_t)h << 56;
          for (int q = 0; q < h; q++) v |= (uint64_t)perm[q] << (8 * q);
          seer[o++] = v;
        }
      }
    }
    return;
  }
  if (g.seven_kind != 1) { g.err |= CIT_ERR_ATTR; return; }
  int i = 0;
  while (i < g.n_seven) {
    int c = g.seven[i];
    take_like(g.seven, g.n_seven, c);
    g.sch[g.n_sch++] = (uint8_t)c;
    i++;
  }
}

// Whether the enumeration of g may raise after it has emitted options: only
// the blackmailer's character options raise late (gen_role: a possessed rank
// outside 2..7 after the build options were listed), and the magician's and
// cardinal's over a hand past CIT_HAND_MASK_MAX; every other error of
// cit_enum_options comes before the first option of its branch.
CIT_HD bool cit_enum_late_error(const CitGame& g) {
  int a = g.gs_pid;
  if (a < 0 || a >= CIT_NP) return false;
  const int role = g.pl[a].role;
  return role == R_BLACKMAILER ||
         ((role == R_MAGICIAN || role == R_CARDINAL) && g.pl[a].n_hand > CIT_HAND_MASK_MAX);
}

CIT_HD int cit_count_options(const CitGame& g, uint32_t& err, const uint64_t* seer) {
  PickSink s(-1);
  cit_enum_options(g, s, seer);
  err |= s.err;
  return s.n;
}
CIT_HD CitOpt cit_pick_option(const CitGame& g, int k, const uint64_t* seer) {
  PickSink s(k);
  cit_enum_options(g, s, seer);
  return s.out;
}

// ====================================================== transitions
// confirm_role_knowledges (option_functions.py:608-622); the unconfirmed-entry
// filter keeps every entry (the entry named like the revealed role has id
// == its rank, never below it), so only the revealed column changes.
CIT_HD void confirm_roles(CitGame& g, int q) {
  int rq = role_rank(g, g.pl[q].role);
  uint16_t v = (uint16_t)((1u << (rq + 1)) | KR_CONFIRMED);
#if CIT_WAVE
  if (cit_lane() < CIT_NP) g.pl[cit_lane()].kr[q] = v;
  return;
#endif
  for (int p = 0; p < CIT_NP; p++) g.pl[p].kr[q] = v;
}
// move_crown + troneroom_owner_gold (option_functions.py:588-595,625-631)
CIT_HD void move_crown(CitGame& g, int t) {
#if CIT_WAVE
  {
    int l = cit_lane();
    int f = g.pl[l < CIT_NP ? l : 0].flags;
    uint64_t cm = cit_ballot(l < CIT_NP && (f & PF_CROWN));
    if (cm) g.pl[__ffsll((unsigned long long)cm) - 1].flags &= (uint8_t)~PF_CROWN;
    g.pl[t].flags |= PF_CROWN;
    int o = seat_with_type(g, 32);
    if (o >= 0) g.pl[o].gold++;
    return;
  }
#endif
  for (int p = 0; p < CIT_NP; p++)
    if (g.pl[p].flags & PF_CROWN) { g.pl[p].flags &= (uint8_t)~PF_CROWN; break; }
  g.pl[t].flags |= PF_CROWN;
  for (int p = 0; p < CIT_NP; p++)
    if (p_has(g.pl[p], 32)) { g.pl[p].gold++; break; }
}
// carry_out_building (option_functions.py:102-127)
CIT_HD void do_build(CitGame& g, int a, int card, int replica) {
  CitPlayer& P = g.pl[a];
  put_card(g, BUILD(P), pl_take_like(g, P, AL_HAND, card));
  if (P.role != R_ALCHEMIST) P.gold = (int16_t)(P.gold - card_cost(card));
  if (replica) P.replicas = (int8_t)replica;
  gs_append(g, card_suit(card) == SUIT_TRADE ? ADM_TRADE : ADM_NON_TRADE);
  if (card_type(card) == 29) P.flags |= PF_LIGHTHOUSE;
  if (rp_warrant(rp_of(g, P.role)) == WB_NONE) {
    at5(g, a, -1);
  } else {
    g.warrant = (uint8_t)card;
    gs_set(g, 7, holder_checked(g, 0));
    g.gs_intr = 1;
    gs_make_next(g, a, NX_ALIAS);
  }
}
// check_if_building_is_replica + settle_museum + settle_lighthouse (:573-606)
CIT_HD void settle(CitGame& g, int name, int a, int t, int card) {
  CitPlayer& P = g.pl[a];
  CitPlayer& T = g.pl[t];
  int ty = card_type(card);
  if (count_type(T.build, T.n_build, ty) > 1) T.replicas = (int8_t)(T.replicas - 1);
  if (ty == 34) {
    int n = T.n_museum;
    for (int i = 0; i < n; i++) {
      int c = pl_pop_front(g, T, AL_MUSEUM);
      if (name == O_WARLORD) put_card(g, g.discard, g.n_discard, CIT_DISCARD_CAP, c);
      else pl_put(g, P, AL_MUSEUM, c);
    }
  }
  if (ty == 29 && (T.flags & PF_LIGHTHOUSE)) {
    T.flags &= (uint8_t)~PF_LIGHTHOUSE;
    P.flags |= PF_LIGHTHOUSE;
  }
}

// finish_main_sequnce_actions (option_functions.py:189-243); returns winner or -1
CIT_HD int do_finish(CitGame& g, const CitOpt& o, CitMT& rng) {
  int a = o.perp;
  CitPlayer& P = g.pl[a];
#if CIT_WAVE
  // the tests below read one round of loads: the mover's role, hand size
  // and buildings (lane i), every role's properties (lane r), the used roles
  // (lane k) and the error word
  const int l_ = cit_lane();
  const int role_ = P.role, nh_ = P.n_hand, nb_ = P.n_build, bl_ = P.build[l_ & (CIT_BUILD_CAP - 1)];
  const int rpl_ = g.rp[l_ & 7], nu_ = g.n_used_roles, url_ = g.used_roles[l_ < CIT_NP ? l_ : 0];
  const uint32_t err_ = g.err;
  __asm__ volatile("" ::"v"(role_), "v"(nh_), "v"(nb_), "v"(bl_), "v"(rpl_), "v"(nu_), "v"(url_), "v"(err_));
  // rp_of(g, P.role): role_rank's KeyError (role >= 27, not Bewitched) and
  // rp_of's (Bewitched, rank 8) are together "role >= CIT_RP_ROLES", the dict
  // then read at 0 (so role_ / 3 below is a lane < 8)
  const bool key_ = role_ >= CIT_RP_ROLES;
  if (key_) g.err = err_ | CIT_ERR_KEY;
  const bool dead = (cit_readlane(rpl_, key_ ? 0 : role_ / 3) & RP_DEAD) != 0;
  if (err_ || key_) return -1;
  if (!dead && nh_ == 0) {   // (just-drawn cards leave the hand size as it is)
    const bool h28 = cit_ballot((l_ < nb_) & (card_type(bl_) == 28)) != 0;
    const bool h30 = cit_ballot((l_ < nb_) & (card_type(bl_) == 30)) != 0;
    if (h28) pl_draw(g, rng, P, AL_JD, 2);
    if (h30) P.gold++;
  }
  if (o.flags & OF_CROWN) {
    confirm_roles(g, a);
    move_crown(g, a);
  } else if (dead) {
    confirm_roles(g, a);
  }
#else
  bool dead = rp_of(g, P.role) & RP_DEAD;
  if (g.err) return -1;
  if (!dead && P.n_hand == 0) {     // (the reference tests the building first; both tests are pure)
    if (p_has(P, 28) && P.n_hand == 0) pl_draw(g, rng, P, AL_JD, 2);
    if (p_has(P, 30) && P.n_hand == 0) P.gold++;
  }
  if (o.flags & OF_CROWN) {
    confirm_roles(g, a);
    move_crown(g, a);
  } else if (rp_of(g, P.role) & RP_DEAD) {
    confirm_roles(g, a);
  }
#endif
  if (o.flags & OF_NEXT_WITCH) {
    int w = holder_checked(g, 0);
    gs_set(g, 5, w);
    g.pl[w].role = P.role;
    rp_of(g, P.role) &= (uint8_t)~RP_POSSESSED;
    P.role = ROLE_BEWITCHED;
    int wr = role_rank(g, g.pl[w].role);
    for (int p = 0; p < CIT_NP; p++) {
      if (p != w) g.pl[p].kr[w] = (uint16_t)((g.pl[p].kr[w] & KR_CONFIRMED) | (1u << (wr + 1)));
      if (p != a) g.pl[p].kr[a] = (uint16_t)((g.pl[p].kr[a] & KR_CONFIRMED) | 1u);
    }
    gs_rebind_adm(g);
    return -1;
  }
#if CIT_WAVE
  if (nu_ == 0 || nu_ == 255) { g.err |= CIT_ERR_INDEX; return -1; }
  const int last_ = nu_ - 1 < CIT_NP ? cit_readlane(url_, nu_ - 1) : (int)g.used_roles[nu_ - 1];
  if (last_ == role_ / 3) {                      // (role_ < 27 here: role_rank is role / 3)
#else
  if (g.n_used_roles == 0 || g.n_used_roles == 255) { g.err |= CIT_ERR_INDEX; return -1; }
  if (g.used_roles[g.n_used_roles - 1] == role_rank(g, P.role)) {
#endif
    CIT_PROF_SCOPE(30);
    int w = check_game_ending(g);
    if (w < 0) cit_setup_round(g, rng);
    return w;
  }
  CIT_PROF_SCOPE(31);
  setup_next_player(g, a);
  return -1;
}

// option.carry_out (option.py:118-122): transition then is_last_round.
// Returns the winner's index, or -1.
CIT_HD int cit_carry_out(CitGame& g, const CitOpt& o, CitMT& rng) {
  int a = o.perp;
  CitPlayer& P = g.pl[a];
  int w = -1;
  switch (o.name) {
    case O_ROLE_PICK: {                                      // :6-30
      int rk = o.a;
#if CIT_WAVE
      {
        // turn_orders_for_roles is a permutation.  One round of loads: the
        // role id, the roles left, the turn order (lane i) and the mover's
        // role knowledge (lane j: seat j); seat j's place in the turn order
        // then comes from readlanes, so the knowledge is not loaded behind it
        const int i = cit_lane();
        const int rid = g.roles[rk], rtc0 = g.rtc;
        const int p = g.turn[i < CIT_NP ? i : 0], krj = P.kr[i < CIT_NP ? i : 0];
        __asm__ volatile("" ::"v"(rid), "v"(rtc0), "v"(p), "v"(krj));
        P.role = (uint8_t)rid;
        const uint8_t rtc = (uint8_t)(rtc0 & ~(1u << rk));
        g.rtc = rtc;
        const uint16_t rtc_mask = (uint16_t)(rtc << 1);
        const uint16_t before = (uint16_t)(0x1FE & ~rtc_mask & ~(1u << (rk + 1)));
        const uint64_t at = cit_ballot((i < CIT_NP) & (p == a));
        const int pos_a = at ? 63 - __clzll((long long)at) : 0;   // the last match, as the loop's
        int ij = -1;
#pragma unroll
        for (int q = 0; q < CIT_NP; q++) ij = cit_readlane(p, q) == i ? q : ij;
        if (i < CIT_NP && i != a && ij >= 0)
          P.kr[i] = (uint16_t)((krj & KR_CONFIRMED) | (ij < pos_a ? before : rtc_mask));
        const int last = cit_readlane(p, CIT_NP - 1);
        if (a != last) gs_set(g, 0, cit_readlane(p, pos_a + 1 < CIT_NP ? pos_a + 1 : 0));
        else setup_next_player(g, -1);
        break;
      }
#endif
      P.role = g.roles[rk];
      g.rtc &= (uint8_t)~(1u << rk);
      uint16_t rtc_mask = (uint16_t)(g.rtc << 1);
      uint16_t before = (uint16_t)(0x1FE & ~rtc_mask & ~(1u << (rk + 1)));
      int pos_a = 0;
      for (int i = 0; i < CIT_NP; i++)
        if (g.turn[i] == a) pos_a = i;
      for (int i = 0; i < CIT_NP; i++) {
        int p = g.turn[i];
        if (p == a) continue;
        P.kr[p] = (uint16_t)((P.kr[p] & KR_CONFIRMED) | (i < pos_a ? before : rtc_mask));
      }
      if (a != g.turn[CIT_NP - 1]) gs_set(g, 0, g.turn[pos_a + 1]);
      else setup_next_player(g, -1);
      break;
    }
    case O_GOLD_OR_CARD: {                                   // :33-55
#if CIT_WAVE
      {   // one round of loads: role, gold, buildings (lane i), every role's properties (lane r)
        const int l = cit_lane();
        const int role = P.role, gold = P.gold, nb = P.n_build, bl = P.build[l & (CIT_BUILD_CAP - 1)];
        const int rpl = g.rp[l & 7];
        __asm__ volatile("" ::"v"(role), "v"(gold), "v"(nb), "v"(bl), "v"(rpl));
        // confirm_roles(g, a) then rp_of(g, P.role): KeyError iff role >= 27
        const int rq = role == ROLE_BEWITCHED ? -1 : role >= 27 ? 0 : role / 3;
        if (role >= CIT_RP_ROLES) g.err |= CIT_ERR_KEY;
        if (l < CIT_NP) g.pl[l].kr[a] = (uint16_t)((1u << (rq + 1)) | KR_CONFIRMED);
        if (cit_readlane(rpl, role >= CIT_RP_ROLES ? 0 : role / 3) & RP_ROBBED) {
          int th = holder_checked(g, 1);
          g.pl[th].gold = (int16_t)(g.pl[th].gold + gold);
          P.gold = 0;
        }
        if (o.a == 0) {
          P.gold += 2;
          gs_set(g, 3, a);
        } else {
          const bool h16 = cit_ballot((l < nb) & (card_type(bl) == 16)) != 0;
          pl_draw(g, rng, P, AL_JD, h16 ? 3 : 2);
          gs_set(g, 2, a);
        }
        break;
      }
#endif
      confirm_roles(g, a);
      if (rp_of(g, P.role) & RP_ROBBED) {
        int th = holder_checked(g, 1);
        g.pl[th].gold = (int16_t)(g.pl[th].gold + P.gold);
        P.gold = 0;
      }
      if (o.a == 0) {
        P.gold += 2;
        gs_set(g, 3, a);
      } else {
        pl_draw(g, rng, P, AL_JD, p_has(P, 16) ? 3 : 2);
        gs_set(g, 2, a);
      }
      break;
    }
    case O_WHICH_CARD: {                                     // :58-66
      pl_put(g, P, AL_HAND, pl_take_like(g, P, AL_JD, o.a));
      if (o.b != CIT_NO_CARD) pl_put(g, P, AL_HAND, pl_take_like(g, P, AL_JD, o.b));
#if CIT_WAVE
      {
        int i = cit_lane(), nj = P.n_jd, nd = g.n_deck;
        if (nj <= 64 && nd + nj <= CIT_DECK_CAP - 1) {   // no overflow: one store by all lanes
          int c = cit_ld(pl_jd(P), i, i < nj, CIT_NO_CARD);
          bool v = i < nj && c != CIT_NO_CARD;
          uint64_t m = cit_ballot(v);
          if (v) deck_ref(g, nd + cit_lane_rank(m)) = (uint8_t)c;
          g.n_deck = (uint8_t)(nd + __popcll(m));
          pl_clear(g, P, AL_JD);
          gs_set(g, 3, a);
          break;
        }
      }
#endif
      for (int i = 0; i < P.n_jd; i++) deck_put(g, pl_jd(P)[i]);
      pl_clear(g, P, AL_JD);
      gs_set(g, 3, a);
      break;
    }
    case O_BLACKMAIL_RESPONSE: {                             // :71-82
      if (o.a == 0) {
        int bm = holder_checked(g, 1);
        g.pl[bm].gold = (int16_t)(g.pl[bm].gold + P.gold / 2);
        P.gold = (int16_t)(P.gold - P.gold / 2);
        gs_set(g, 5, a);
      } else {
        gs_set(g, 4, holder_checked(g, 1));
        g.gs_intr = 1;
        gs_make_next(g, a, NX_FRESH);
      }
      break;
    }
    case O_REVEAL_BLACKMAIL: {                               // :85-92
      CitPlayer& T = g.pl[o.target];
      if (o.a == 0 && rp_blackmail(rp_of(g, T.role)) == WB_REAL) {
        P.gold = (int16_t)(P.gold + T.gold);
        T.gold = 0;
        for (int r = 0; r < 8; r++) g.rp[r] &= (uint8_t)~(3u << RP_BLACKMAIL_SHIFT);
      }
      gs_goto_next(g);
      break;
    }
    case O_REVEAL_WARRANT: {                                 // :94-100
      CitPlayer& T = g.pl[o.target];
      if (o.a == 0 && rp_warrant(rp_of(g, T.role)) == WB_REAL) {
        if (g.warrant == CIT_NO_CARD) { g.err |= CIT_ERR_ATTR; break; }
        put_card(g, BUILD(P), take_like(T.build, T.n_build, g.warrant));
        T.gold = (int16_t)(T.gold + card_cost(g.warrant));
        for (int r = 0; r < 8; r++) g.rp[r] &= (uint8_t)~(3u << RP_WARRANT_SHIFT);
      }
      gs_goto_next(g);
      break;
    }
    case O_BUILD:
      do_build(g, a, o.a, (int8_t)o.c);
      break;
    case O_EMPTY:                                            // :68-69
      if (o.a == 0) gs_fresh(g, 5, a);
      else gs_goto_next(g);
      break;
    case O_FINISH_ROUND:
      w = do_finish(g, o, rng);
      break;
    case O_SMITHY:                                           // :131-138
      P.gold -= 2;
      pl_draw(g, rng, P, AL_JD, 3);
      at5(g, a, ADM_SMITHY);
      break;
    case O_LAB:                                              // :140-145
      put_card(g, g.discard, g.n_discard, CIT_DISCARD_CAP, pl_take_like(g, P, AL_HAND, o.a));
      P.gold++;
      at5(g, a, ADM_LAB);
      break;
    case O_MAGIC_SCHOOL:                                     // :147-153
      take_like(P.build, P.n_build, 25);
      put_card(g, BUILD(P), o.a == SUIT_UNIQUE ? 25 : 40 + o.a);
      at5(g, a, ADM_MAGIC_SCHOOL);
      break;
    case O_WEAPON_STORAGE: {                                 // :167-171
      CitPlayer& T = g.pl[o.target];
      put_card(g, g.discard, g.n_discard, CIT_DISCARD_CAP, take_like(P.build, P.n_build, 27));
      put_card(g, g.discard, g.n_discard, CIT_DISCARD_CAP, take_like(T.build, T.n_build, o.a));
      at5(g, a, -1);
      break;
    }
    case O_LIGHTHOUSE:                                       // :173-180
      kh_append(g, a, -1, 5, false, g.n_deck, [&g](int i) { return deck_at(g, i); });
      pl_put(g, P, AL_HAND, deck_take_like(g, o.a));
      P.flags &= (uint8_t)~PF_LIGHTHOUSE;
      deck_shuffle(g, rng);
      at5(g, a, -1);
      break;
    case O_MUSEUM:                                           // :161-165
      pl_put(g, P, AL_MUSEUM, pl_take_like(g, P, AL_HAND, o.a));
      at5(g, a, ADM_MUSEUM);
      break;
    case O_GRAVEYARD:                                        // :183-187
      if (!g.n_discard) { g.err |= CIT_ERR_INDEX; break; }
      put_card(g, BUILD(P), g.discard[--g.n_discard]);
      P.gold--;
      gs_goto_next(g);
      break;
    case O_TAKE_GOLD_WAR:                                    // :553-559
      P.gold = (int16_t)(P.gold + count_suit(P.build, P.n_build, SUIT_WAR));
      at5(g, a, ADM_TAKE_GOLD);
      break;
    case O_ASSASSINATION:                                    // :245-249
      g.rp[o.a] |= RP_DEAD;
      at5(g, a, ADM_ABILITY);
      break;
    case O_MAGISTRATE_WARRANT:                               // :251-257
      g.rp[o.a] = (uint8_t)((g.rp[o.a] & ~(3u << RP_WARRANT_SHIFT)) | (WB_REAL << RP_WARRANT_SHIFT));
      g.rp[o.b] = (uint8_t)((g.rp[o.b] & ~(3u << RP_WARRANT_SHIFT)) | (WB_FAKE << RP_WARRANT_SHIFT));
      g.rp[o.c] = (uint8_t)((g.rp[o.c] & ~(3u << RP_WARRANT_SHIFT)) | (WB_FAKE << RP_WARRANT_SHIFT));
      at5(g, a, ADM_ABILITY);
      break;
    case O_BEWITCHING:                                       // :259-262
      g.rp[o.a] |= RP_POSSESSED;
      P.flags |= PF_WITCH;
      setup_next_player(g, a);
      break;
    case O_STEAL:                                            // :265-269
      g.rp[o.a] |= RP_ROBBED;
      at5(g, a, ADM_ABILITY);
      break;
    case O_BLACKMAIL:                                        // :271-276
      g.rp[o.a] = (uint8_t)((g.rp[o.a] & ~(3u << RP_BLACKMAIL_SHIFT)) | (WB_REAL << RP_BLACKMAIL_SHIFT));
      g.rp[o.b] = (uint8_t)((g.rp[o.b] & ~(3u << RP_BLACKMAIL_SHIFT)) | (WB_FAKE << RP_BLACKMAIL_SHIFT));
      at5(g, a, ADM_ABILITY);
      break;
    case O_SPY: {                                            // :278-288
      CitPlayer& T = g.pl[o.target];
      int n = count_suit(T.hand, T.n_hand, o.a);
      int steal = n < T.gold ? n : T.gold;
      P.gold = (int16_t)(P.gold + steal);
      T.gold = (int16_t)(T.gold - steal);
      pl_draw(g, rng, P, AL_HAND, 1);
      at5(g, a, ADM_ABILITY);
      break;
    }
    case O_MAGIC_HAND_CHANGE: {                              // :291-303
      CitPlayer& T = g.pl[o.target];
      const int np = P.n_hand, nt = T.n_hand;
#if CIT_WAVE
      {   // lane l holds both hands' cards l and l + 64 (area_splice calls src(l), src(l + 64) on lane l)
        const int l = cit_lane();
        const int p0 = cit_ld(P.hand, l, l < np, 0), p1 = l + 64 < np ? P.hand[l + 64] : 0;
        const int t0 = cit_ld(T.hand, l, l < nt, 0), t1 = l + 64 < nt ? T.hand[l + 64] : 0;
        area_splice(g, P, AL_HAND, 0, np, nt, [t0, t1](int i) { return i < 64 ? t0 : t1; });
        area_splice(g, T, AL_HAND, 0, nt, np, [p0, p1](int i) { return i < 64 ? p0 : p1; });
      }
#else
      {   // swap the common prefix in place, append the longer hand's rest to the
          // other, then cut it from the longer one in one splice (no private copy
          // of a hand; the bytes left past the area are the wave path's)
        const int m = np < nt ? np : nt, d = (np < nt ? nt : np) - m;
        for (int i = 0; i < m; i++) {
          uint8_t c = P.hand[i];
          P.hand[i] = T.hand[i];
          T.hand[i] = c;
        }
        CitPlayer& A = np < nt ? P : T;     // receives the extra cards
        CitPlayer& Z = np < nt ? T : P;
        if (area_used(A) + d > CIT_AREA_CAP) g.err |= CIT_ERR_OVERFLOW;
        else {
          for (int i = 0; i < d; i++) pl_put(g, A, AL_HAND, Z.hand[m + i]);
          area_splice(g, Z, AL_HAND, m, d, 0, [](int) { return 0; });
        }
      }
#endif
      at5(g, a, ADM_ABILITY);
      break;
    }
    case O_DISCARD_AND_DRAW: {                               // :291-303, iterate-while-remove
      int i = 0;
      while (i < P.n_hand) {
        deck_put(g, pl_take_like(g, P, AL_HAND, P.hand[i]));
        i++;
      }
      pl_draw(g, rng, P, AL_HAND, P.n_hand);
      at5(g, a, ADM_ABILITY);
      break;
    }
    case O_LOOK_AT_HAND: {                                   // :305-310
      const CitPlayer& T = g.pl[o.target];
      kh_append(g, a, o.target, 5, true, T.n_hand, [&T](int i) { return T.hand[i]; });
      gs_set(g, 10, a);
      gs_append(g, ADM_ABILITY);
      gs_make_next(g, a, NX_ALIAS);
      break;
    }
    case O_TAKE_FROM_HAND: {                                 // :312-328
      CitPlayer& T = g.pl[o.target];
      int e = -1;
#if CIT_WAVE
      {
        int l = cit_lane(), nk = g.n_kh;
        CitKH k = g.kh[l < CIT_KH_MAX ? l : 0];
        uint64_t m = cit_ballot(l < nk && l < CIT_KH_MAX && k.owner == a && (k.conf_flags & 0x10));
        e = m ? __ffsll((unsigned long long)m) - 1 : -1;
      }
#else
      for (int i = 0; i < g.n_kh; i++)
        if (g.kh[i].owner == a && (g.kh[i].conf_flags & 0x10)) { e = i; break; }
#endif
      if (e < 0) { g.err |= CIT_ERR_ATTR; break; }
      pl_put(g, P, AL_HAND, pl_take_like(g, T, AL_HAND, o.a));
      if (o.flags & OF_BUILD) {
        int rep = count_type(P.build, P.n_build, card_type(o.a));   // option.attributes['replica'] is overwritten
        do_build(g, a, o.a, rep);
      }
      kh_take_like(g, e, o.a);
      gs_goto_next(g);
      break;
    }
    case O_SEER: {                                           // :330-341
      g.n_seer = 0;
      for (int p = 0; p < CIT_NP; p++) {
        CitPlayer& Q = g.pl[p];
        if (p == a || !Q.n_hand) continue;
        shuffle_arr(rng, Q.hand, Q.n_hand);
        reshuffle_if_empty(g, rng);
        pl_put(g, P, AL_HAND, pl_pop_front(g, Q, AL_HAND));
        g.seer_from[g.n_seer++] = (uint8_t)p;
      }
      gs_set(g, 8, a);
      gs_append(g, ADM_ABILITY);
      gs_make_next(g, a, NX_ALIAS);
      break;
    }
    case O_GIVE_BACK_CARD: {                                 // :343-350
      int k = o.b;
      for (int i = 0; i < k; i++) {
        int pid = g.seer_from[i];
        int c = (int)((o.x >> (8 * i)) & 0xFF);
        pl_put(g, g.pl[pid], AL_HAND, pl_take_like(g, P, AL_HAND, c));
        kh_append(g, a, pid, 5, false, 1, [c](int) { return c; });
      }
      g.n_seer = 0;
      gs_goto_next(g);
      break;
    }
    case O_TAKE_CROWN_KING:                                  // :354-363
      P.gold = (int16_t)(P.gold + count_suit(P.build, P.n_build, SUIT_LORD));
      if (!(P.flags & PF_WITCH)) move_crown(g, a);
      at5(g, a, ADM_ABILITY);
      break;
    case O_TAKE_CROWN_PAT: {                                 // :365-375
      int n = count_suit(P.build, P.n_build, SUIT_LORD);
      pl_draw(g, rng, P, AL_HAND, n);
      if (!(P.flags & PF_WITCH)) move_crown(g, a);
      at5(g, a, ADM_ABILITY);
      break;
    }
    case O_GIVE_CROWN: {                                     // :377-393
      CitPlayer& T = g.pl[o.target];
      P.gold = (int16_t)(P.gold + count_suit(P.build, P.n_build, SUIT_LORD));
      if (o.a == 0) {
        shuffle_arr(rng, T.hand, T.n_hand);
        pl_put(g, P, AL_HAND, pl_pop_front(g, T, AL_HAND));
      } else if (o.a == 1) {
        P.gold++;
        T.gold--;
      }
      confirm_roles(g, a);
      move_crown(g, o.target);
      at5(g, a, ADM_ABILITY);
      break;
    }
    case O_BISHOP:                                           // :397-403
      P.gold = (int16_t)(P.gold + count_suit(P.build, P.n_build, SUIT_RELIGION));
      at5(g, a, ADM_ABILITY);
      break;
    case O_CARDINAL: {                                       // :422-439
      CitPlayer& T = g.pl[o.target];
      uint8_t give[CIT_HAND_MASK_MAX];
      int ng = 0;
      for (int i = 0; i < P.n_hand && i < CIT_HAND_MASK_MAX; i++)
        if ((o.x >> i) & 1) give[ng++] = P.hand[i];
      put_card(g, BUILD(P), pl_take_like(g, P, AL_HAND, o.a));
      P.gold = (int16_t)(P.gold - (card_cost(o.a) - (o.flags & OF_FACTORY ? 1 : 0)));
      if (P.gold < 0) P.gold = 0;
      if ((int8_t)o.c) P.replicas = (int8_t)o.c;
      if (ng) {
        T.gold = (int16_t)(T.gold - ng);
        for (int i = 0; i < ng; i++) pl_put(g, T, AL_HAND, pl_take_like(g, P, AL_HAND, give[i]));
      }
      at5(g, a, ADM_ABILITY);
      break;
    }
    case O_ABBOT_GOLD_OR_CARD:                               // :405-412
      P.gold = (int16_t)(P.gold + (o.a - o.b));
      pl_draw(g, rng, P, AL_HAND, o.b);
      at5(g, a, ADM_ABILITY);
      break;
    case O_ABBOT_BEG: {                                      // :414-420
      int best = 0;
#if CIT_WAVE
      {
        int l = cit_lane();
        int gl = g.pl[l < CIT_NP ? l : 0].gold;
        gl = l < CIT_NP ? gl : -32768;
        int mx = __ockl_wfred_max_i32(gl);
        best = __ffsll((unsigned long long)cit_ballot(l < CIT_NP && gl == mx)) - 1;   // first maximum
      }
#else
      for (int p = 1; p < CIT_NP; p++)
        if (g.pl[p].gold > g.pl[best].gold) best = p;
#endif
      g.pl[best].gold--;
      int ab = holder_checked(g, 4);
      g.pl[ab].gold++;
      at5(g, a, ADM_BEGGED);
      break;
    }
    case O_MERCHANT:                                         // :442-449
      P.gold = (int16_t)(P.gold + count_suit(P.build, P.n_build, SUIT_TRADE) + 1);
      at5(g, a, ADM_ABILITY);
      break;
    case O_ALCHEMIST:                                        // :451-452
      break;
    case O_TRADER:                                           // :455-461
      P.gold = (int16_t)(P.gold + count_suit(P.build, P.n_build, SUIT_TRADE));
      at5(g, a, ADM_ABILITY);
      break;
    case O_ARCHITECT:                                        // :464-471
      pl_draw(g, rng, P, AL_HAND, 2);
      at5(g, a, ADM_ABILITY);
      break;
    case O_NAVIGATOR:                                        // :473-483
      if (o.a == 1) pl_draw(g, rng, P, AL_HAND, 4);
      else P.gold += 4;
      at5(g, a, ADM_ABILITY);
      break;
    case O_SCHOLAR: {                                        // :485-496
      g.seven_kind = 1;
      g.n_seven = 0;
      int n = g.n_deck < 7 ? g.n_deck : 7;
      for (int i = 0; i < n; i++) {
        reshuffle_if_empty(g, rng);
        int c = deck_draw(g);
        pl_put(g, P, AL_HAND, c);
        put_card(g, g.seven, g.n_seven, CIT_SEVEN_CAP, c);
      }
      gs_set(g, 9, a);
      gs_append(g, ADM_ABILITY);
      gs_make_next(g, a, NX_ALIAS);
      break;
    }
    case O_SCHOLAR_PICK:                                     // :498-502
      for (int i = 0; i < g.n_seven; i++) deck_put(g, pl_take_like(g, P, AL_HAND, g.seven[i]));
      gs_goto_next(g);
      g.seven_kind = 2;
      g.n_seven = 0;
      break;
    case O_WARLORD: {                                        // :517-535
      CitPlayer& T = g.pl[o.target];
      P.gold = (int16_t)(P.gold - (card_cost(o.a) - 1));
      put_card(g, g.discard, g.n_discard, CIT_DISCARD_CAP, take_like(T.build, T.n_build, o.a));
      settle(g, O_WARLORD, a, o.target, o.a);
      at5(g, a, ADM_ABILITY);
      int owner = seat_with_type(g, 24);
      if (owner >= 0 && owner != a) {
        gs_set(g, 6, owner);
        g.gs_intr = 1;
        gs_make_next(g, a, NX_ABILITY);
      }
      break;
    }
    case O_MARSHAL: {                                        // :505-515
      CitPlayer& T = g.pl[o.target];
      P.gold = (int16_t)(P.gold - card_cost(o.a));
      T.gold = (int16_t)(T.gold + card_cost(o.a));
      put_card(g, BUILD(P), take_like(T.build, T.n_build, o.a));
      settle(g, O_MARSHAL, a, o.target, o.a);
      at5(g, a, ADM_ABILITY);
      break;
    }
    case O_DIPLOMAT: {                                       // :538-551
      CitPlayer& T = g.pl[o.target];
      P.gold = (int16_t)(P.gold - o.c);
      T.gold = (int16_t)(T.gold + o.c);
      put_card(g, BUILD(P), take_like(T.build, T.n_build, o.a));
      put_card(g, BUILD(T), take_like(P.build, P.n_build, o.b));
      settle(g, O_DIPLOMAT, a, o.target, o.a);
      at5(g, a, ADM_ABILITY);
      break;
    }
    default:
      g.err |= CIT_ERR_UNSUPPORTED;
      break;
  }
  is_last_round(g);
  g.steps++;
  return w;
}

// ================================================= determinization
// remove_role_from_role_knowledge (game.py:298-301) on a copied knowledge row:
// drop `role` (by name, i.e. by role index) from every unconfirmed entry.
CIT_HD void kr_strip(const CitGame& g, uint16_t* kr, int role) {
  for (int j = 0; j < CIT_NP; j++) {
    if (kr[j] & KR_CONFIRMED) continue;
    for (int rid = -1; rid < 8; rid++)
      if (role_of_id(g, rid) == role) kr[j] &= (uint16_t)~(1u << (rid + 1));
  }
}

// bytes of `unk` scratch cit_sample_private needs (880: unknown cards [80],
// removal counts u32[40], per-type lane masks u64[2][40]); the search also
// stages diff rows in it (cit_cfr.h row_load: 64 dwords per 256 bytes)
#ifndef CIT_SAMPLE_SCRATCH
#define CIT_SAMPLE_SCRATCH 1024
#endif
static_assert(CIT_SAMPLE_SCRATCH >= 880 && CIT_SAMPLE_SCRATCH % 16 == 0, "determinization scratch");

#if CIT_WAVE
// Append src(i), i < cnt (<= 128), to dst[base..) skipping CIT_NO_CARD (the
// reference's add_card drops the "Deck Empty" sentinel); returns the count
// appended.  Lanes i and 64 + i move one element each.
template <class Src, class Dst>
CIT_HD int wave_append(Dst dst, int base, int cnt, Src src) {
  const int l = cit_lane();
  const uint64_t below = cit_below();
  // every lane calls src for its first element (each src reads in bounds past cnt): no
  // branch around those loads; the second (past lane 64, rarely any) keeps its branch
  int c0 = src(l), c1 = l + 64 < cnt ? src(l + 64) : CIT_NO_CARD;
  c0 = l < cnt ? c0 : CIT_NO_CARD;
  uint64_t m0 = cit_ballot(c0 != CIT_NO_CARD), m1 = cit_ballot(c1 != CIT_NO_CARD);
  int n0 = __popcll(m0);
  if (c0 != CIT_NO_CARD) dst(base + __popcll(m0 & below)) = (uint8_t)c0;
  if (c1 != CIT_NO_CARD) dst(base + n0 + __popcll(m1 & below)) = (uint8_t)c1;
  return n0 + __popcll(m1);
}

// cit_sample_private for a wave running the game uniformly with a coop (LDS)
// stream: the same draws in the same order (through a register window), the
// list work spread over the lanes.  `unk` holds >= CIT_SAMPLE_SCRATCH bytes:
// the unknown cards [0, 80), the per-type removal counts u32[40] at 80 and
// the per-type lane masks of the used cards u64[2][40] at 240.
CIT_HD void cit_sample_private_wave(CitGame& g, int orig, bool role_sample, CitMT& rng, uint8_t* unk) {
  const int l = cit_lane();
  const uint64_t below = cit_below();
  CitPlayer& PC = g.pl[orig];
  CitMT w = cit_mt_window(rng);
  // lane e: HandKnowledge entry e, its pool offset (exclusive scan of len)
  const int nkh = g.n_kh;
  const int le = l < nkh ? l : 0;
  const int kowner = g.kh[le].owner, ktarget = g.kh[le].target, kflags = g.kh[le].conf_flags;
  const int klen = l < nkh ? (int)g.kh[le].len : 0;   // (le is clamped: an unconditional load)
  int koff = 0;
  for (int j = 0; j < nkh; j++) koff += j < l ? cit_readlane(klen, j) : 0;
  const bool mine = l < nkh && kowner == orig;
  // hk.used with probability (confidence-1)*0.2, entries in order (:217-222)
  uint64_t used = 0;
  {
  CIT_PROF_SCOPE(16);
  for (uint64_t m = cit_ballot(mine); m; m &= m - 1) {
    int e = __ffsll((unsigned long long)m) - 1;
    double r = mt_random(w);
    int conf = cit_readlane(kflags, e) & 15;
    if ((double)(conf - 1) * 0.2 > r) used |= 1ull << e;
  }
  }
  const bool uu = mine && ((used >> l) & 1);
  if (mine) g.kh[l].conf_flags = (uint8_t)((kflags & ~0x20) | (uu ? 0x20 : 0));
  // get_unknown_cards (:183-213): removals per type, then drop the first k_t
  // used cards of each type t
  int nu = 0;
  {
  CIT_PROF_SCOPE(17);
  uint32_t* kt = reinterpret_cast<uint32_t*>(unk + CIT_USED_CAP);
  uint64_t* tm = reinterpret_cast<uint64_t*>(unk + CIT_USED_CAP + 160);   // [2][40]
  if (l < 40) {
    kt[l] = 0;
    tm[l] = 0;
    tm[40 + l] = 0;
  }
  __syncthreads();
  for (int pass = 0; pass < 2; pass++) {
    int p = pass * 4 + (l >> 4), i = l & 15;
    if (p < CIT_NP && i < g.pl[p].n_build) atomicAdd(&kt[card_type(g.pl[p].build[i])], 1u);
  }
  {   // museums (any length): the seats holding one, 64 cards per pass
    const int pl = l < CIT_NP ? l : 0;
    for (uint64_t m = cit_ballot(l < CIT_NP && g.pl[pl].n_museum > 0); m; m &= m - 1) {
      const CitPlayer& M = g.pl[__ffsll((unsigned long long)m) - 1];
      const uint8_t* mu = pl_museum(M);
      for (int i = l; i < M.n_museum; i += 64) atomicAdd(&kt[card_type(mu[i])], 1u);
    }
  }
  if (l < PC.n_hand) atomicAdd(&kt[card_type(PC.hand[l])], 1u);
  for (uint64_t m = cit_ballot(uu); m; m &= m - 1) {
    int e = __ffsll((unsigned long long)m) - 1;
    int off = cit_readlane(koff, e), len = cit_readlane(klen, e);
    for (int i = l; i < len; i += 64) atomicAdd(&kt[card_type(g.kh_pool[off + i])], 1u);
  }
  __syncthreads();
  const int nuc = g.n_used_cards;
  const bool v0 = l < nuc, v1 = l + 64 < nuc;
  const int c0 = cit_ld(g.used_cards, l, v0, 0), c1 = v1 ? g.used_cards[l + 64] : 0;
  const int t0 = card_type(c0), t1 = card_type(c1);
  // rank among the earlier used cards of the same type: per-type masks of
  // the lanes holding that type (LDS atomic OR), popcount below this lane
  if (v0) atomicOr(reinterpret_cast<unsigned long long*>(&tm[t0]), 1ull << l);
  if (v1) atomicOr(reinterpret_cast<unsigned long long*>(&tm[40 + t1]), 1ull << l);
  __syncthreads();
  const int rk0 = __popcll(tm[t0] & below), rk1 = __popcll(tm[t1]) + __popcll(tm[40 + t1] & below);
  const bool k0 = v0 && rk0 >= (int)kt[t0], k1 = v1 && rk1 >= (int)kt[t1];
  const uint64_t km0 = cit_ballot(k0), km1 = cit_ballot(k1);
  const int nk0 = __popcll(km0);
  __syncthreads();
  if (k0) unk[__popcll(km0 & below)] = (uint8_t)c0;
  if (k1) unk[nk0 + __popcll(km1 & below)] = (uint8_t)c1;
  nu = nk0 + __popcll(km1);
  __syncthreads();
  }
  int head = 0;                                  // unk[head..nu): the undealt unknown cards
  auto deck_slot = [&g](int i) -> uint8_t& { return g.deck[i & (CIT_DECK_CAP - 1)]; };
  // sample_deck (:245-262): lighthouse knowledge first, then shuffled unknowns
  {
    CIT_PROF_SCOPE(18);
    int n = g.n_deck, nd = 0;
    uint64_t lm = cit_ballot(uu && ktarget == -1);
    g.n_deck = 0;
    g.deck_head = 0;
    int lo = 0, kk = 0;
    if (lm) {
      int e = __ffsll((unsigned long long)lm) - 1;
      int ll = cit_readlane(klen, e);
      lo = cit_readlane(koff, e);
      kk = ll < n ? ll : n;
      n -= kk;
    }
    shuffle_arr(w, unk, nu);
    __syncthreads();
    int m = n < nu ? n : nu;
    // the known cards, then the shuffled unknowns: one compaction pass
    nd = wave_append(deck_slot, 0, kk + m,
                     [&g, unk, lo, kk](int i) {
                       const int a = g.kh_pool[i < kk ? lo + i : 0], b = unk[i < kk ? 0 : i - kk];
                       return i < kk ? a : b;
                     });
    head = m;
    g.n_deck = (uint8_t)nd;
  }
  // sample_warrants_and_blackmails (:321-336): the marked roles (<= 8) as
  // nibbles of one word, shuffled; the first is the real one
  for (int which = 0; which < 2; which++) {
    CIT_PROF_SCOPE(19);
    int shift = which == 0 ? RP_BLACKMAIL_SHIFT : RP_WARRANT_SHIFT;
    uint32_t pk = 0;
    int nk = 0;
    for (int r = 0; r < 8; r++)
      if ((g.rp[r] >> shift) & 3) pk |= (uint32_t)r << (4 * nk++);
    if (!nk) continue;
    for (int i = nk - 1; i > 0; i--) {
      int j = (int)mt_randbelow(w, (uint32_t)(i + 1));
      uint32_t ai = (pk >> (4 * i)) & 15, aj = (pk >> (4 * j)) & 15;
      pk &= ~((15u << (4 * i)) | (15u << (4 * j)));
      pk |= (aj << (4 * i)) | (ai << (4 * j));
    }
    int real = (int)(pk & 15);
    for (int i = 0; i < nk; i++) {
      int r = (int)((pk >> (4 * i)) & 15);
      g.rp[r] = (uint8_t)((g.rp[r] & ~(3u << shift)) | ((r == real ? WB_REAL : WB_FAKE) << shift));
    }
  }
  CIT_PROF_SCOPE(20);
  uint16_t kr[CIT_NP];
  for (int j = 0; j < CIT_NP; j++) kr[j] = PC.kr[j];
  // kr_strip: the role ids holding `role` as one ballot over lane r = roles[r]
  const int rl = cit_ld(g.roles, l, l < 8, ROLE_NONE);
  auto strip = [&](int role) {
    uint16_t m = (uint16_t)(((uint32_t)cit_ballot(l < 8 && rl == role) << 1) | (role == ROLE_BEWITCHED ? 1u : 0u));
    for (int j = 0; j < CIT_NP; j++)
      if (!(kr[j] & KR_CONFIRMED)) kr[j] &= (uint16_t)~m;
  };
  if (role_sample) {   // remove_role_and_smaller_id_roles_from_role_knowledge_if_unconfirmed (:304-310)
    int role = g.pl[g.gs_pid].role;
    strip(role);
    if (role != ROLE_NONE) {
      int rr = role_rank(g, role);
      for (int rid = 0; rid < 8; rid++)
        if (rid < rr) strip(cit_readlane(rl, rid));
    }
  }
  for (int p = 0; p < CIT_NP; p++) {
    CitPlayer& Q = g.pl[p];
    if (p != orig) {   // sample_cards_for_opponent (:264-280): known cards, then unknowns, one pass
      int n = Q.n_hand, ho = 0, kk = 0;
      uint64_t hm = cit_ballot(uu && ktarget == p);
      if (hm) {
        int e = __ffsll((unsigned long long)hm) - 1;
        int hl = cit_readlane(klen, e);
        ho = cit_readlane(koff, e);
        kk = hl < n ? hl : n;
        n -= kk;
      }
      int m = n < nu - head ? n : nu - head;
      // the new hand overwrites the old one in place (it is never longer: the
      // unknown cards may run out); a shorter hand pulls the lists after it in
      const int n_old = Q.n_hand;
      int nh = wave_append([&Q](int i) -> uint8_t& { return Q.hand[i < CIT_AREA_CAP ? i : 0]; }, 0, kk + m,
                           [&g, unk, ho, kk, head](int i) {
                             const int a = g.kh_pool[i < kk ? ho + i : 0], b = unk[i < kk ? 0 : head + i - kk];
                             return i < kk ? a : b;
                           });
      head += m;
      if (nh < n_old) area_splice(g, Q, AL_HAND, nh, n_old - nh, 0, [](int) { return 0; });
    }
    // sample_roles_for_opponent (:283-295)
    if (role_sample && p != orig && p != g.gs_pid && g.gs_state != 0) {
      int cnt = 0;
      for (int rid = -1; rid < 8; rid++) cnt += (kr[p] >> (rid + 1)) & 1;
      int k = (int)mt_randbelow(w, (uint32_t)cnt);
      if (cnt) {
        int rid = -1;
        for (int q = -1; q < 8; q++)
          if ((kr[p] >> (q + 1)) & 1) {
            if (k == 0) { rid = q; break; }
            k--;
          }
        Q.role = (uint8_t)(rid < 0 ? ROLE_BEWITCHED : cit_readlane(rl, rid));
        strip(Q.role);
      } else {   // the IndexError band-aid: first role id not in used_roles
        int pick = -1;
        for (int rid = 0; rid < 8 && pick < 0; rid++) {
          bool in = false;
          for (int u = 0; u < g.n_used_roles && u < CIT_NP; u++) in |= g.used_roles[u] == rid;
          if (!in) pick = rid;
        }
        if (pick < 0) { g.err |= CIT_ERR_INDEX; cit_mt_unwindow(rng, w); return; }   // StopIteration
        Q.role = g.roles[pick];
      }
    }
  }
  if (role_sample && g.gs_state != 0) refresh_used_roles(g);
  cit_mt_unwindow(rng, w);
}
#endif

// Game.sample_private_information(players[orig], role_sample) (game.py:215-339):
// resample everything `orig` cannot see.  `unk` is >= CIT_SAMPLE_SCRATCH
// bytes of scratch (LDS on the device).
CIT_HD void cit_sample_private(CitGame& g, int orig, bool role_sample, CitMT& rng, uint8_t* unk) {
#if CIT_WAVE
  if (rng.coop) {
    cit_sample_private_wave(g, orig, role_sample, rng, unk);
    return;
  }
#endif
  CitPlayer& PC = g.pl[orig];
  // hk.used with probability (confidence-1)*0.2 (:217-222)
  for (int e = 0; e < g.n_kh; e++) {
    CitKH& k = g.kh[e];
    if (k.owner != orig) continue;
    double r = mt_random(rng);
    bool used = (double)(kh_conf(k) - 1) * 0.2 > r;
    k.conf_flags = (uint8_t)((k.conf_flags & ~0x20) | (used ? 0x20 : 0));
  }
  // get_unknown_cards (:183-213): used_cards minus every visible / known card,
  // each removal taking the first remaining card of its type.  Removals of one
  // type never move another type's first occurrence, so the sequence of
  // get_a_card_like_it calls equals dropping the first k_t cards of each type t
  // (k_t = removals of type t) in one ordered pass.
  uint8_t* kt = unk + CIT_USED_CAP;
  for (int t = 0; t < 40; t++) kt[t] = 0;
  for (int p = 0; p < CIT_NP; p++)
    for (int i = 0; i < g.pl[p].n_build; i++) kt[card_type(g.pl[p].build[i])]++;
  for (int p = 0; p < CIT_NP; p++)
    for (int i = 0; i < g.pl[p].n_museum; i++) kt[card_type(pl_museum(g.pl[p])[i])]++;
  for (int i = 0; i < PC.n_hand; i++) kt[card_type(PC.hand[i])]++;
  {
    int off = 0;
    for (int e = 0; e < g.n_kh; e++) {
      const CitKH& k = g.kh[e];
      if (k.owner == orig && (k.conf_flags & 0x20))
        for (int i = 0; i < k.len; i++) kt[card_type(g.kh_pool[off + i])]++;
      off += k.len;
    }
  }
  uint8_t nu = 0;
  for (int i = 0; i < g.n_used_cards; i++) {
    int c = g.used_cards[i], t = card_type(c);
    if (kt[t]) kt[t]--;
    else unk[nu++] = (uint8_t)c;
  }
  int head = 0;                                  // unk[head..nu): the undealt unknown cards
  // sample_deck (:245-262): lighthouse knowledge first, then shuffled unknowns
  {
    int n = g.n_deck;
    int lo = -1, ll = 0, off = 0;
    for (int e = 0; e < g.n_kh; e++) {
      const CitKH& k = g.kh[e];
      if (k.owner == orig && k.target == -1 && (k.conf_flags & 0x20)) { lo = off; ll = k.len; break; }
      off += k.len;
    }
    g.n_deck = 0;
    g.deck_head = 0;
    if (lo >= 0) {
      int kk = ll < n ? ll : n;
      for (int i = 0; i < kk; i++) deck_put(g, g.kh_pool[lo + i]);
      n -= kk;
    }
    shuffle_arr(rng, unk, nu);
    for (int i = 0; i < n; i++) deck_put(g, head < nu ? unk[head++] : CIT_NO_CARD);
  }
  // sample_warrants_and_blackmails (:321-336)
  for (int which = 0; which < 2; which++) {
    int shift = which == 0 ? RP_BLACKMAIL_SHIFT : RP_WARRANT_SHIFT;
    uint8_t ks[8];
    int nk = 0;
    for (int r = 0; r < 8; r++)
      if ((g.rp[r] >> shift) & 3) ks[nk++] = (uint8_t)r;
    if (!nk) continue;
    shuffle_arr(rng, ks, nk);
    for (int i = 0; i < nk; i++) {
      int r = ks[i];
      g.rp[r] = (uint8_t)((g.rp[r] & ~(3u << shift)) | ((r == ks[0] ? WB_REAL : WB_FAKE) << shift));
    }
  }
  uint16_t kr[CIT_NP];
  for (int j = 0; j < CIT_NP; j++) kr[j] = PC.kr[j];
  if (role_sample) {   // remove_role_and_smaller_id_roles_from_role_knowledge_if_unconfirmed (:304-310)
    int role = g.pl[g.gs_pid].role;
    kr_strip(g, kr, role);
    if (role != ROLE_NONE) {
      int rr = role_rank(g, role);
      for (int rid = 0; rid < 8; rid++)
        if (rid < rr) kr_strip(g, kr, g.roles[rid]);
    }
  }
  for (int p = 0; p < CIT_NP; p++) {
    CitPlayer& Q = g.pl[p];
    if (p != orig) {   // sample_cards_for_opponent (:264-280)
      int n = Q.n_hand, ho = -1, hl = 0, off = 0;
      for (int e = 0; e < g.n_kh; e++) {
        const CitKH& k = g.kh[e];
        if (k.owner == orig && k.target == p && (k.conf_flags & 0x20)) { ho = off; hl = k.len; break; }
        off += k.len;
      }
      // the new hand overwrites the old one in place (never longer: the
      // unknown cards may run out, add_card drops "Deck Empty"); a shorter
      // hand pulls the lists after it in
      const int n_old = n;
      int w = 0;
      if (ho >= 0) {
        int kk = hl < n ? hl : n;
        for (int i = 0; i < kk; i++) Q.hand[w++] = g.kh_pool[ho + i];
        n -= kk;
      }
      for (int i = 0; i < n && head < nu; i++) Q.hand[w++] = unk[head++];
      if (w < n_old) area_splice(g, Q, AL_HAND, w, n_old - w, 0, [](int) { return 0; });
    }
    // sample_roles_for_opponent (:283-295)
    if (role_sample && p != orig && p != g.gs_pid && g.gs_state != 0) {
      int cnt = 0;
      for (int rid = -1; rid < 8; rid++) cnt += (kr[p] >> (rid + 1)) & 1;
      int k = (int)mt_randbelow(rng, (uint32_t)cnt);
      if (cnt) {
        int rid = -1;
        for (int q = -1; q < 8; q++)
          if ((kr[p] >> (q + 1)) & 1) {
            if (k == 0) { rid = q; break; }
            k--;
          }
        Q.role = (uint8_t)role_of_id(g, rid);
        kr_strip(g, kr, Q.role);
      } else {   // the IndexError band-aid: first role id not in used_roles
        int pick = -1;
        for (int rid = 0; rid < 8 && pick < 0; rid++) {
          bool in = false;
          for (int u = 0; u < g.n_used_roles && u < CIT_NP; u++) in |= g.used_roles[u] == rid;
          if (!in) pick = rid;
        }
        if (pick < 0) { g.err |= CIT_ERR_INDEX; return; }   // StopIteration
        Q.role = g.roles[pick];
      }
    }
  }
  if (role_sample && g.gs_state != 0) refresh_used_roles(g);
}

// ============================================================ featurizers
#define CIT_FEAT 418
#define CIT_OPT_FEAT 131
// Game.encode_game (game.py:91-128), written as 418 floats into `out`.
// pid >= 0 replaces gamestate.player_id (expand_role_pick does that, :120-123).
// zero = false: `out` is already zeroed.
template <class F, bool zero = true>
CIT_HD void cit_encode_game(const CitGame& g, F* out, int pid = -1) {
  if (zero)
    for (int i = 0; i < CIT_FEAT; i++) out[i] = 0;
  int cur = pid >= 0 ? pid : g.gs_pid;
  for (int r = 0; r < 8; r++) out[r * 3 + g.roles[r] % 3] = 1;                 // [8,3] role variants
  for (int p = 0; p < CIT_NP; p++) {                                              // [6,8] confirmed roles
    int role = g.pl[p].role;
    if (role >= 27) continue;
    if (g.pl[cur].kr[p] & KR_CONFIRMED) out[24 + p * 8 + role / 3] = 1;
  }
  for (int p = 0; p < CIT_NP; p++) {
    const CitPlayer& P = g.pl[p];
    out[72 + p] = (F)count_points(P);                                             // points
    out[78 + p] = (F)P.gold;                                                      // gold
    out[84 + p] = (F)P.n_hand;                                                    // hand size
    for (int i = 0; i < P.n_build; i++) {
      out[90 + p * 40 + card_type(P.build[i])] += 1;                              // [6,40] built types
      out[330 + p * 5 + card_suit(P.build[i])] += 1;                              // [6,5] built suits
    }
  }
  out[360 + cur] = 1;                                                             // current player
  out[366 + g.gs_state] = 1;                                                      // state one-hot [11]
  out[377] = g.ending ? 1 : 0;
  for (int r = 0; r < 8; r++) {                                                   // [8,5] role properties
    uint8_t v = g.rp[r];
    out[378 + r * 5 + 0] = (v & RP_DEAD) ? 1 : 0;
    out[378 + r * 5 + 1] = rp_warrant(v) ? 1 : 0;
    out[378 + r * 5 + 2] = (v & RP_POSSESSED) ? 1 : 0;
    out[378 + r * 5 + 3] = (v & RP_ROBBED) ? 1 : 0;
    out[378 + r * 5 + 4] = rp_blackmail(v) ? 1 : 0;
  }
}

// option.encode_option (option.py:52-115) for descriptor `o` generated on `g`
// (hand-slot masks resolve against g).  Only the first matching branch of the
// reference's elif chain writes: a tuple choice, an int role choice, `cards`,
// `card_handouts` and next_gamestate encode nothing beyond name + perpetrator.
template <class F>
CIT_HD void cit_encode_option(const CitOpt& o, const CitGame& g, F* out) {
  for (int i = 0; i < CIT_OPT_FEAT; i++) out[i] = 0;
  out[o.name] = 1;
  out[47 + o.perp] = 1;
  switch (o.name) {
    case O_REVEAL_BLACKMAIL: case O_REVEAL_WARRANT: case O_WEAPON_STORAGE: case O_SPY: case O_MAGIC_HAND_CHANGE:
    case O_LOOK_AT_HAND: case O_TAKE_FROM_HAND: case O_GIVE_CROWN: case O_CARDINAL: case O_WARLORD: case O_MARSHAL:
    case O_DIPLOMAT:
      out[53 + o.target] = 1;
      break;
    case O_ROLE_PICK:
      out[60 + o.a] = 1;
      break;
    case O_GOLD_OR_CARD:
      out[76 + o.a] = 1;                       // gold 0, card 1
      break;
    case O_BLACKMAIL_RESPONSE:
      out[76 + 2 + o.a] = 1;                   // pay 2, not_pay 3
      break;
    case O_NAVIGATOR:
      out[76 + 6 + o.a] = 1;                   // 4gold 6, 4card 7
      break;
    case O_MAGIC_SCHOOL:
      out[76 + 8 + o.a] = 1;                   // trade..unique 8..12
      break;
    case O_LAB: case O_LIGHTHOUSE: case O_MUSEUM: case O_SCHOLAR_PICK: case O_BUILD:
      out[89 + card_type(o.a)] = 1;
      break;
    case O_WHICH_CARD:
      if (!(o.flags & OF_TUPLE)) out[89 + card_type(o.a)] = 1;   // [card]; a tuple matches no branch
      break;
    case O_MAGISTRATE_WARRANT: case O_BLACKMAIL:
      out[60 + o.a] = 1;                       // real_target
      break;
    case O_ABBOT_GOLD_OR_CARD:
      out[130] = (F)o.b;                       // number of "card"
      break;
    default:
      break;
  }
}

// cit_random_step with one enumeration pass in the common case: the options
// are listed into `buf` while counted and the draw indexes the buffer; only a
// list longer than `cap` is enumerated again up to the drawn index.
CIT_HD int cit_random_step_buf(CitGame& g, CitMT& rng, uint64_t* seer, CitOpt* buf, int cap) {
  cit_prepare_options(g, rng, seer);
  BufSink s(buf, cap);
  cit_enum_options(g, s, seer);
  if (s.err) { g.err |= s.err; return 1; }
  int n = s.n;
  if (n == 0) { g.err |= CIT_ERR_EMPTY; return 1; }
  int k = (int)mt_randbelow(rng, (uint32_t)n);
  CitOpt o = k < cap ? buf[k] : cit_pick_option(g, k, seer);
  int w = cit_carry_out(g, o, rng);
  return (w >= 0 || g.err || g.terminal) ? 1 : 0;
}

#if CIT_WAVE
// cit_random_step_buf with the list in registers (RegSink, at most 64 listed)
__device__ __forceinline__ int cit_random_step_reg(CitGame& g, CitMT& rng, uint64_t* seer) {
  cit_prepare_options(g, rng, seer);
  RegSink s;
  cit_enum_options(g, s, seer);
  if (s.err) { g.err |= s.err; return 1; }
  int n = s.n;
  if (n == 0) { g.err |= CIT_ERR_EMPTY; return 1; }
  int k = (int)mt_randbelow(rng, (uint32_t)n);
  CitOpt o = k < 64 ? s.at(k) : cit_pick_option(g, k, seer);
  int w = cit_carry_out(g, o, rng);
  return (w >= 0 || g.err || g.terminal) ? 1 : 0;
}
#elif defined(__HIPCC__)
__device__ int cit_random_step_reg(CitGame& g, CitMT& rng, uint64_t* seer);   // (host pass: kernels only)
#endif

// One random-policy step (compare_to_random.py:37-39): get_options ->
// random.choice -> carry_out.  Returns 1 when the lane is done (winner or error).
CIT_HD int cit_random_step(CitGame& g, CitMT& rng, uint64_t* seer) {
  cit_prepare_options(g, rng, seer);
  uint32_t err = 0;
  int n = cit_count_options(g, err, seer);
  if (err) { g.err |= err; return 1; }
  if (n == 0) { g.err |= CIT_ERR_EMPTY; return 1; }
  int k = (int)mt_randbelow(rng, (uint32_t)n);
  CitOpt o = cit_pick_option(g, k, seer);
  int w = cit_carry_out(g, o, rng);
  return (w >= 0 || g.err || g.terminal) ? 1 : 0;
}

// skip_false_choice (deep_mccfr.py:37-49) on its own, for CFRNode(game)
// constructed by the facade: auto-plays single-option steps (at most 101) and
// stops at a winner.  Returns the number of carry_outs.
CIT_HD int cit_skip_false_choice(CitGame& g, CitMT& py, uint64_t* seer) {
  uint32_t e = 0;
  cit_prepare_options(g, py, seer);
  int n = cit_count_options(g, e, seer);
  int i = 0;
  bool done = false;
  while (n == 1 && !done && !e && !g.err) {
    i++;
    CitOpt o = cit_pick_option(g, 0, seer);
    done = cit_carry_out(g, o, py) >= 0;
    cit_prepare_options(g, py, seer);
    n = cit_count_options(g, e, seer);
    if (i > 100) done = true;
  }
  g.err |= e;
  return i;
}

// compare_to_random.play_games' step loop (compare_to_random.py:16-35) up to
// the next searched decision.  Seats in `search_mask` decide by search when
// they have more than one option; that test is one get_options call, and a
// searched seat with <= 1 option falls through to the else branch, which calls
// get_options again before random.choice.  Other seats make one call.
// Returns the deciding seat, -1 when the game is over (or max_steps random
// steps were taken), -2 on a lane error.
CIT_HD int cit_advance_policy(CitGame& g, CitMT& rng, uint64_t* seer, int search_mask, int max_steps, int& steps) {
  int s = 0;
  while (!g.terminal && !g.err && s < max_steps) {
    int pid = g.gs_pid;
    uint32_t e = 0;
    cit_prepare_options(g, rng, seer);
    int n = cit_count_options(g, e, seer);
    if (e) { g.err |= e; break; }
    if (pid >= 0 && ((search_mask >> pid) & 1)) {
      if (n > 1) { steps += s; return pid; }
      cit_prepare_options(g, rng, seer);
      n = cit_count_options(g, e, seer);
      if (e) { g.err |= e; break; }
    }
    if (n == 0) { g.err |= CIT_ERR_EMPTY; break; }
    int k = (int)mt_randbelow(rng, (uint32_t)n);
    CitOpt o = cit_pick_option(g, k, seer);
    cit_carry_out(g, o, rng);
    s++;
  }
  steps += s;
  return g.err ? -2 : -1;
}

// create_a_random_game(max_move) (run_utils.py:55-73) on a lane whose CPython
// stream is already seeded: k = randint(1, max_move); create_game(); a random
// playout to the winner keeping the game after every step (deepcopy ->
// `ring`, the last max_move snapshots, CIT_GAME_BYTES each); the result is
// games[-k] while the stream stays where the playout left it.  Returns the
// number of steps into the game of the returned position (-1 on error:
// games[-k] past the front raises IndexError in the reference).
CIT_HD int cit_random_position(CitGame& g, CitMT& rng, uint64_t* seer, uint32_t* ring, int max_move) {
  const int W = CIT_GAME_BYTES / 4;
  int k = 1 + (int)mt_randbelow(rng, (uint32_t)max_move);
  cit_init_game(g, rng, true);
  uint32_t* gw = reinterpret_cast<uint32_t*>(&g);
  int n = 0;                                   // snapshots taken
  for (int i = 0; i < W; i++) ring[i] = gw[i];
  n = 1;
  while (!g.terminal && !g.err) {
    if (n > CIT_ROLLOUT_CAP) { g.err |= CIT_ERR_STEP_CAP; break; }
    cit_random_step(g, rng, seer);
    uint32_t* d = ring + (long)(n % max_move) * W;
    for (int i = 0; i < W; i++) d[i] = gw[i];
    n++;
  }
  if (g.err) return -1;
  if (k > n) { g.err |= CIT_ERR_INDEX; return -1; }
  const uint32_t* src = ring + (long)((n - k) % max_move) * W;
  for (int i = 0; i < W; i++) gw[i] = src[i];
  return n - k;
}

// create_a_close_to_finished_game(game) (run_utils.py:29-53) on the lane's
// created game: k = randint(1, max_back); a random playout to the winner with
// a deep copy before the first and after every step; then, at most `limit`
// times while the examined game has < 2 options: examine games[-k] (its
// get_options may mutate it and draw from the stream, as in the reference),
// k -= 1.  Python indexing: games[-0] is games[0], games[-(-j)] is games[j].
// `store` holds CIT_CLOSE_ROWS rows: the first `limit` snapshots and a ring of
// the last max_back (close_slot: a snapshot held in both is always read and
// written through the ring).  Returns the index of the position (-1 on error).
#define CIT_CLOSE_LIMIT 100
#define CIT_CLOSE_BACK 30
#define CIT_CLOSE_ROWS (CIT_CLOSE_LIMIT + CIT_CLOSE_BACK)
CIT_HD uint32_t* close_slot(uint32_t* store, int j, int n) {
  const int W = CIT_GAME_BYTES / 4;
  if (j >= n - CIT_CLOSE_BACK) return store + (long)(CIT_CLOSE_LIMIT + j % CIT_CLOSE_BACK) * W;
  return j < CIT_CLOSE_LIMIT ? store + (long)j * W : nullptr;
}
CIT_HD int cit_close_position(CitGame& g, CitMT& rng, uint64_t* seer, uint32_t* store) {
  const int W = CIT_GAME_BYTES / 4;
  int k = 1 + (int)mt_randbelow(rng, (uint32_t)CIT_CLOSE_BACK);
  uint32_t* gw = reinterpret_cast<uint32_t*>(&g);
  int n = 0;
  for (;;) {                                   // snapshot n, then step
    if (n < CIT_CLOSE_LIMIT)
      for (int i = 0; i < W; i++) store[(long)n * W + i] = gw[i];
    uint32_t* t = store + (long)(CIT_CLOSE_LIMIT + n % CIT_CLOSE_BACK) * W;
    for (int i = 0; i < W; i++) t[i] = gw[i];
    n++;
    if (g.terminal || g.err) break;
    if (n > CIT_ROLLOUT_CAP) { g.err |= CIT_ERR_STEP_CAP; break; }
    cit_random_step(g, rng, seer);
  }
  if (g.err) return -1;
  int cnt = 0, limit = 0, idx = -1;
  while (cnt < 2 && limit < CIT_CLOSE_LIMIT) {
    int m = k;
    idx = m > 0 ? n - m : -m;
    if (idx < 0 || idx >= n) { g.err |= CIT_ERR_INDEX; return -1; }
    uint32_t* src = close_slot(store, idx, n);
    if (!src) { g.err |= CIT_ERR_UNSUPPORTED; return -1; }
    for (int i = 0; i < W; i++) gw[i] = src[i];
    cit_prepare_options(g, rng, seer);
    uint32_t e = 0;
    cnt = cit_count_options(g, e, seer);
    g.err |= e;
    for (int i = 0; i < W; i++) src[i] = gw[i];   // the examined snapshot keeps get_options' mutation
    if (g.err) return -1;
    k--;
    limit++;
  }
  return idx;
}
