// Self-test driver for the card-area list operations (cit_engine.h:
// area_splice, pl_put, pl_take_like, pl_pop_front, pl_clear, pl_draw), run
// by the host build (serial loops) and by a one-wave kernel (the lane-parallel
// CIT_WAVE paths) on the same pseudo-random operation sequence; the tests
// compare the resulting rows byte for byte and check the host result against
// a Python-list model (tests/test_area_ops.py).  The sequence drives player
// areas up to the full CIT_AREA_CAP, where the second byte per lane (l + 64)
// and the overflow check are exercised -- lengths no golden game reaches.
#pragma once
#include "cit_engine.h"

// xorshift64*: the operation stream (host and device alike)
CIT_HD uint64_t area_test_next(uint64_t& s) {
  s ^= s >> 12;
  s ^= s << 25;
  s ^= s >> 27;
  return s * 2685821657736338717ull;
}

// Op k of the sequence on game g (deck refilled from a counter so draws never
// run dry; the MT stream is only used by a draw that reshuffles).  Returns the
// op code, for the model in the test: 0 put, 1 take_like, 2 pop_front,
// 3 clear, 4 draw, 5 hand swap with player (p + 1) % 6.
CIT_HD int area_test_op(CitGame& g, CitMT& rng, uint64_t& s, uint32_t* log) {
  const uint64_t r = area_test_next(s);
  const int op = (int)(r % 6), p = (int)((r >> 8) % CIT_NP), L = (int)((r >> 16) % 3), c = (int)((r >> 24) % 45);
  const int k = 1 + (int)((r >> 32) % 5);
  CitPlayer& P = g.pl[p];
  int res = -1;
  // bias towards growth so areas fill up: puts and draws outnumber removals
  switch (op) {
    case 0: pl_put(g, P, L, c); break;
    case 1: res = pl_take_like(g, P, L, c); break;
    case 2: res = pl_pop_front(g, P, L); break;
    case 3:
      if (((r >> 40) & 7) == 0) pl_clear(g, P, L);
      else pl_put(g, P, L, c);
      break;
    case 4:
      while (g.n_deck < k + 2) deck_put(g, (g.n_deck * 7 + k) % 40);
      pl_draw(g, rng, P, L, k);
      break;
    case 5: {
      CitPlayer& T = g.pl[(p + 1) % CIT_NP];
      const int np = P.n_hand, nt = T.n_hand;
#if CIT_WAVE
      const int l = cit_lane();
      const int p0 = l < np ? P.hand[l] : 0, p1 = l + 64 < np ? P.hand[l + 64] : 0;
      const int t0 = l < nt ? T.hand[l] : 0, t1 = l + 64 < nt ? T.hand[l + 64] : 0;
      area_splice(g, P, AL_HAND, 0, np, nt, [t0, t1](int i) { return i < 64 ? t0 : t1; });
      area_splice(g, T, AL_HAND, 0, nt, np, [p0, p1](int i) { return i < 64 ? p0 : p1; });
#else
      uint8_t hp[CIT_AREA_CAP], ht[CIT_AREA_CAP];
      for (int i = 0; i < np; i++) hp[i] = P.hand[i];
      for (int i = 0; i < nt; i++) ht[i] = T.hand[i];
      area_splice(g, P, AL_HAND, 0, np, nt, [&ht](int i) { return ht[i]; });
      area_splice(g, T, AL_HAND, 0, nt, np, [&hp](int i) { return hp[i]; });
#endif
      break;
    }
  }
  if (log) *log = (uint32_t)(op | (p << 4) | (L << 8) | (c << 12) | (k << 20) | ((res & 0xFF) << 24));
  return op;
}
