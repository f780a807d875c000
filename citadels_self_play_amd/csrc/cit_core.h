// Packed game state, rules tables and the CPython/numpy MT19937 restatement.
//
// One game = one fixed-width `CitGame` row (CIT_GAME_BYTES).  Rows live in HBM
// as [B][CIT_GAME_BYTES] and are staged into LDS, one row per lane, by the
// kernels in cit_hip.hip.  Everything here is plain C++ usable from host code
// too (the test-only host build, cit_host.cpp); CIT_HD marks it for both.
//
// Reference correspondence (davpat108/CITADELS_self_play):
//   CitPlayer            Agent state            game/agent.py:10-29
//   CitGame              Game state             game/game.py:420-540
//   gs_* / nx_*          GameState + next       game/helper_classes.py:16-34
//   kh*                  HandKnowledge lists    game/helper_classes.py:37-43
//   CitPlayer::kr        RoleKnowlage           game/helper_classes.py:45-70
//   CitMT                CPython `random` / numpy RandomState (MT19937)
#pragma once
#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define CIT_HD __host__ __device__ __forceinline__
#define CIT_HDI __host__ __device__ inline
#else
#define CIT_HD inline
#define CIT_HDI inline
#endif

// ------------------------------------------------------------ wave helpers
// CIT_WAVE: device code in a translation unit whose engine callers run the
// game on all 64 lanes of a wavefront with uniform control flow (every lane
// computes the same values; cit_hip.hip's uniform kernels and the MCCFR
// kernels).  The list scans of the engine then read one element per lane
// (one LDS round trip instead of one per element) and combine with ballots
// and readlanes; results are identical to the serial loops, which the host
// build and the one-game-per-lane kernels (CIT_NO_WAVE units) keep.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(CIT_NO_WAVE)
#define CIT_WAVE 1
__device__ __forceinline__ int cit_lane() { return (int)__lane_id(); }
__device__ __forceinline__ uint64_t cit_ballot(bool p) { return (uint64_t)__ballot(p); }
__device__ __forceinline__ int cit_readlane(int v, int i) { return __builtin_amdgcn_readlane(v, i); }
__device__ __forceinline__ int cit_writelane(int v, int val, int i) { return (int)__lane_id() == i ? val : v; }
__device__ __forceinline__ uint64_t cit_below() { return (1ull << __lane_id()) - 1; }   // lanes under this one
// a[i] where ok, else z: every lane loads (a lane that is not ok reads a[0],
// which every list the engine scans has), so no exec-mask branch is built
// around the load -- `ok ? a[i] : z` is a divergent branch to the compiler.
template <class T>
__device__ __forceinline__ int cit_ld(const T* a, int i, bool ok, int z) {
  const int v = (int)a[ok ? i : 0];
  return ok ? v : z;
}
extern "C" __device__ __attribute__((const)) unsigned int __ockl_wfred_or_u32(unsigned int);
__device__ __forceinline__ uint64_t cit_wave_or64(uint64_t v) {
  return ((uint64_t)__ockl_wfred_or_u32((unsigned int)(v >> 32)) << 32) | __ockl_wfred_or_u32((unsigned int)v);
}
#else
#define CIT_WAVE 0
#endif

// ---------------------------------------------------------------- capacities
// A player's hand, just-drawn cards and museum share one card area of
// CIT_AREA_CAP slots (CitPlayer::hand, back to back in that order): the
// reference's lists have no caps, and one player can only hold more than 88
// cards if the game has more cards than the 76 it deals (66 in random-role
// games) -- a reference game gains cards only through get_a_card_like_it's
// fallback (deck.py:49-55), one at a time.  Buildings stay a list of their own
// (the rules end the game a round after 7).  (#ifndef: tools/capstats.cpp
// builds the host engine with wider lists to measure how long they get.)
#define CIT_NP 6
#ifndef CIT_AREA_CAP
#define CIT_AREA_CAP 88
#endif
#ifndef CIT_BUILD_CAP
#define CIT_BUILD_CAP 16
#endif
// the wave paths load a player's buildings one per lane with the lane index
// masked by CIT_BUILD_CAP - 1 (cit_engine.h: do_finish, gold_or_card, ...)
static_assert(CIT_BUILD_CAP > 0 && (CIT_BUILD_CAP & (CIT_BUILD_CAP - 1)) == 0 && CIT_BUILD_CAP <= 64,
              "CIT_BUILD_CAP: a power of two of at most 64");
// roles with a role_properties entry (game.py:525-534: rank ids 0..7); the
// rank-8 roles 24..26 and the Bewitched (>= 27) are KeyErrors there
#define CIT_RP_ROLES 24
#define CIT_DECK_CAP 128          // ring buffer, power of two
#define CIT_DISCARD_CAP 88        // >= the 76 cards a game deals
#define CIT_USED_CAP 80
#define CIT_KH_MAX 32
#define CIT_KH_POOL 244          // cards held by HandKnowledge entries (88 at most in 1,920 cfr_train(200000) trees)
#define CIT_SEVEN_CAP 8
// magician / cardinal options over hands of at most this many cards (their
// hand-slot masks and slot tables); the reference lists every combination of
// the hand there (itertools: 2^33 tuples at 33 cards), a search it cannot run
#define CIT_HAND_MASK_MAX 32

// ------------------------------------------------------------------- errors
// A lane whose reference run would raise (or that overflows a fixed capacity)
// stops with one of these bits set in CitGame::err.
#define CIT_ERR_OVERFLOW 0x1u      // a fixed-capacity container overflowed
#define CIT_ERR_EMPTY 0x2u         // random.choice([]) -> IndexError
#define CIT_ERR_KEY 0x4u           // role_properties[-1] / role_to_role_id[None] -> KeyError
#define CIT_ERR_VALUE 0x8u         // list.remove / list.index of a missing item -> ValueError
#define CIT_ERR_INDEX 0x10u        // used_roles[i+1] past the end -> IndexError
#define CIT_ERR_ATTR 0x20u         // get_player_from_role_id(..) is None -> AttributeError
#define CIT_ERR_UNSUPPORTED 0x40u  // a branch this build does not implement
#define CIT_ERR_NONE_OPTIONS 0x80u // get_options fell through and returned None
#define CIT_ERR_STEP_CAP 0x100u    // rollout hit its hard step cap (the reference has no cap)
// With CIT_ERR_OVERFLOW, which MCCFR node-pool capacity ran out (a search run
// again with more room gives the reference's tree; an overflow without these
// bits is an engine list capacity that no retry fixes: a player holding more
// than CIT_AREA_CAP cards in hand + just-drawn + museum, or more than
// CIT_KH_MAX HandKnowledge entries):
#define CIT_ERR_POOL_ARENA 0x1000u // the shared block arena was exhausted
#define CIT_ERR_POOL_CAP 0x2000u   // the tree reached its node / edge caps
#define CIT_ERR_POOL_ROW 0x4000u   // a node row differs from the base row in more dwords than a diff slot holds
#define CIT_ERR_POOL (CIT_ERR_POOL_ARENA | CIT_ERR_POOL_CAP | CIT_ERR_POOL_ROW)
#define CIT_ROLLOUT_CAP 20000      // max_steps < 0 means "to terminal", bounded by this

// --------------------------------------------------------------- card codes
// code < 40: type_ID with its table suit; 40..44: Magic School (type 25)
// re-suited to suit code-40 (option_functions.py:147-153).
enum { SUIT_TRADE = 0, SUIT_WAR, SUIT_RELIGION, SUIT_LORD, SUIT_UNIQUE };
#define CIT_NO_CARD 255

CIT_HD int card_type(int c) { return c >= 40 ? 25 : c; }
CIT_HD int type_suit(int t) { return t < 6 ? 0 : t < 10 ? 1 : t < 13 ? 2 : t < 16 ? 3 : 4; }
CIT_HD int card_suit(int c) { return c >= 40 ? c - 40 : type_suit(c); }
// config.py costs, 3 bits per type (types 0..19 / 20..39).
#define CIT_COST_LO 0x059dae168d69d511ull
#define CIT_COST_HI 0x0ba5d2eb5e7b5d6eull
CIT_HD int type_cost(int t) {
  return t < 20 ? (int)((CIT_COST_LO >> (3 * t)) & 7) : (int)((CIT_COST_HI >> (3 * (t - 20))) & 7);
}
CIT_HD int card_cost(int c) { return type_cost(card_type(c)); }

// -------------------------------------------------------------------- roles
// role index = rank*3 + variant (config.py:82-91); 27 = "Bewitched", 255 = None.
#define ROLE_BEWITCHED 27
#define ROLE_NONE 255
enum {
  R_ASSASSIN = 0, R_WITCH, R_MAGISTRATE, R_THIEF, R_SPY, R_BLACKMAILER, R_MAGICIAN, R_WIZARD,
  R_SEER, R_KING, R_EMPEROR, R_PATRICIAN, R_BISHOP, R_ABBOT, R_CARDINAL, R_MERCHANT, R_ALCHEMIST,
  R_TRADER, R_ARCHITECT, R_NAVIGATOR, R_SCHOLAR, R_WARLORD, R_DIPLOMAT, R_MARSHAL, R_QUEEN,
  R_ARTIST, R_TAXCOLLECTOR
};

// ------------------------------------------------------------ option names
// ids follow option.py:34-45 (generate_name_to_id_map)
enum {
  O_ROLE_PICK = 0, O_GOLD_OR_CARD, O_WHICH_CARD, O_BLACKMAIL_RESPONSE, O_REVEAL_BLACKMAIL,
  O_REVEAL_WARRANT, O_BUILD, O_EMPTY, O_FINISH_ROUND, O_GHOST_TOWN, O_SMITHY, O_LAB,
  O_MAGIC_SCHOOL, O_WEAPON_STORAGE, O_LIGHTHOUSE, O_MUSEUM, O_GRAVEYARD, O_TAKE_GOLD_WAR,
  O_ASSASSINATION, O_MAGISTRATE_WARRANT, O_BEWITCHING, O_STEAL, O_BLACKMAIL, O_SPY,
  O_MAGIC_HAND_CHANGE, O_DISCARD_AND_DRAW, O_LOOK_AT_HAND, O_TAKE_FROM_HAND, O_SEER,
  O_GIVE_BACK_CARD, O_TAKE_CROWN_KING, O_GIVE_CROWN, O_TAKE_CROWN_PAT, O_BISHOP, O_CARDINAL,
  O_ABBOT_GOLD_OR_CARD, O_ABBOT_BEG, O_MERCHANT, O_ALCHEMIST, O_TRADER, O_ARCHITECT,
  O_NAVIGATOR, O_SCHOLAR, O_SCHOLAR_PICK, O_WARLORD, O_MARSHAL, O_DIPLOMAT, O_NUM_NAMES
};

// already_done_moves tokens, counted (only `in` / `.count` are ever asked of the list)
enum { ADM_BEGGED = 0, ADM_ABILITY, ADM_LAB, ADM_MAGIC_SCHOOL, ADM_MUSEUM, ADM_NON_TRADE, ADM_SMITHY,
       ADM_TAKE_GOLD, ADM_TRADE, ADM_N };

// ------------------------------------------------------------- option desc
// 16-byte option descriptor; field meaning per name is documented in
// include/citadels.h (CitOption).
struct CitOpt {
  uint8_t name, perp;
  int8_t target;
  uint8_t a, b, c, d, flags;
  uint64_t x;
};

// ------------------------------------------------------------- packed game
struct CitPlayer {                 // 128 B
  uint8_t hand[CIT_AREA_CAP];      // card area: hand [0, n_hand) | just_drawn_cards
                                   // [n_hand, +n_jd) | museum_cards [.., +n_museum)
  uint8_t build[CIT_BUILD_CAP];
  uint8_t n_hand, n_build, n_jd, n_museum;
  int16_t gold;
  uint8_t role;                    // role index / ROLE_BEWITCHED / ROLE_NONE
  int8_t replicas;                 // False/True/int semantics of agent.replicas
  uint8_t flags;                   // PF_*
  uint8_t pad0;
  uint16_t kr[CIT_NP];             // RoleKnowlage: bits 0..8 = ids -1..7, bit 15 confirmed
  uint16_t pad1;
};
enum { PF_CROWN = 1, PF_LIGHTHOUSE = 2, PF_FIRST7 = 4, PF_WITCH = 8 };
#define KR_CONFIRMED 0x8000u

struct CitKH {                     // one HandKnowledge entry, 4 B
  uint8_t owner;                   // whose known_hands list
  int8_t target;                   // player_id (-1 = deck)
  uint8_t conf_flags;              // conf (bits 0..3) | wizard 0x10 | used 0x20
  uint8_t len;                     // cards are kh_pool[off..off+len), off = running sum
};

struct CitGame {
  CitPlayer pl[CIT_NP];            // 768
  uint8_t deck[CIT_DECK_CAP];      // ring: logical i at (deck_head+i) & (CAP-1)
  uint8_t discard[CIT_DISCARD_CAP];
  uint8_t used_cards[CIT_USED_CAP];
  uint8_t kh_pool[CIT_KH_POOL];
  CitKH kh[CIT_KH_MAX];            // ordered as appended; per-owner order = list order
  uint8_t deck_head, n_deck, n_discard, n_used_cards;
  uint8_t n_kh, kh_fill, preset, pad2;
  uint8_t roles[8];                // role index per rank
  uint8_t rtc;                     // roles_to_choose_from: rank bitmask (ascending)
  uint8_t n_used_roles;            // 255 = attribute absent
  int8_t used_roles[CIT_NP];       // sorted role ids
  uint8_t turn[CIT_NP];            // turn_orders_for_roles
  uint8_t rp[8];                   // RolePropery: RP_* bits
  // current GameState
  uint8_t gs_state;
  int8_t gs_pid;                   // -1 = None (before the first setup_round)
  uint8_t gs_adm[ADM_N];
  uint8_t gs_intr;
  // next_gamestate (always a fresh GameState(state=5,...) in the reference)
  uint8_t nx_valid, nx_state;
  int8_t nx_pid;
  uint8_t nx_adm[ADM_N];
  uint8_t nx_intr, nx_alias, nx_hasnext;
  uint8_t ending, terminal;
  int8_t winner;
  uint8_t has_points;
  int16_t points[CIT_NP];
  uint8_t warrant;                 // warrant_building card, CIT_NO_CARD = absent
  uint8_t n_seer;                  // 255 = seer_taken_card_from absent
  uint8_t seer_from[5];
  uint8_t seven_kind;              // 0 absent, 1 Deck, 2 plain [] (after put-back)
  uint8_t n_seven;
  uint8_t seven[CIT_SEVEN_CAP];
  uint8_t n_sch;                   // scholar picks prepared by get_options (state 9)
  uint8_t sch[CIT_SEVEN_CAP];
  uint32_t err;
  uint32_t steps;                  // carry_out calls applied to this game
};
enum { RP_DEAD = 1, RP_WARRANT_SHIFT = 1, RP_POSSESSED = 8, RP_ROBBED = 16, RP_BLACKMAIL_SHIFT = 5 };
enum { WB_NONE = 0, WB_REAL = 1, WB_FAKE = 2 };

#ifndef CIT_GAME_BYTES
#define CIT_GAME_BYTES 1552
#endif
static_assert(sizeof(CitGame) <= CIT_GAME_BYTES, "CitGame grew past its row size");
static_assert(CIT_AREA_CAP <= 128, "card area: at most two bytes per lane");
static_assert(CIT_GAME_BYTES % 16 == 0, "row must be 16-byte aligned");

// Optional per-function cycle accounting (build with -DCIT_PROF; profiling
// only, tools/prof_cfr.py; scopes 0..15: the search in cit_cfr.h, 16..31:
// engine internals).  Each tree accumulates its scopes' cycles in LDS
// (one wave per tree: plain adds by lane 0, no atomics inside the search, so
// the accounting does not perturb the memory traffic it measures); the
// kernel adds the totals to g_cit_prof once per tree (cfr_prof_flush).
// Scopes nest: a scope's cycles include those of the scopes it calls.
#if defined(CIT_PROF) && defined(__HIPCC__)
__device__ unsigned long long g_cit_prof[64];
#endif
#if defined(CIT_PROF) && defined(__HIP_DEVICE_COMPILE__)
__shared__ unsigned long long cit_prof_lds[64];
struct CitProf {
  int id;
  unsigned long long t0;
  __device__ explicit CitProf(int i) : id(i), t0(clock64()) {}
  __device__ ~CitProf() {
    unsigned long long dt = clock64() - t0;
    if (threadIdx.x == 0) {
      cit_prof_lds[id] += dt;
      cit_prof_lds[32 + id] += 1ull;
    }
  }
};
// CIT_PROF_MASK selects the scopes that are timed (bit i = scope i), so a
// profile can time a few scopes at a time with little perturbation.
#ifndef CIT_PROF_MASK
#define CIT_PROF_MASK 0xffffffffull
#endif
struct CitProfOff {
  __device__ explicit CitProfOff(int) {}
};
#define CIT_PROF_SCOPE(i)                                                         \
  typename cit_prof_sel<((CIT_PROF_MASK >> (i)) & 1ull) != 0>::type _cit_prof_scope(i)
template <bool On> struct cit_prof_sel { typedef CitProf type; };
template <> struct cit_prof_sel<false> { typedef CitProfOff type; };
__device__ inline void cfr_prof_reset() {
  cit_prof_lds[threadIdx.x] = 0;   // 64 lanes, 64 slots
  __syncthreads();
}
__device__ inline void cfr_prof_flush() {
  __syncthreads();
  atomicAdd(&g_cit_prof[threadIdx.x], cit_prof_lds[threadIdx.x]);
}
#else
#define CIT_PROF_SCOPE(i) ((void)0)
#define cfr_prof_reset() ((void)0)
#define cfr_prof_flush() ((void)0)
#endif

// ----------------------------------------------------------------- MT19937
// Per-lane MT19937 laid out structure-of-arrays: word i of lane l at
// mt[i*stride + l].  The stream position lives in a register while a kernel
// runs (`pos`); callers load it from / store it to the mt_idx array.
#define CIT_MT_N 624
struct CitMT {
  uint32_t* mt;
  int stride;
  uint32_t pos;   // 624 = twist next
  int coop;       // device: every lane of the wave runs this stream's owner
                  // uniformly, so the twist is done lane-parallel (stride 1);
                  // CIT_MT_WINDOW: also draw through `win` (below)
  // CIT_MT_WINDOW streams (a CitMT held in registers, never in memory): lane
  // i of `win` holds the TEMPERED word win_base + i, so a draw is a readlane
  // and the LDS block is read once per 64 draws (all lanes at once).
  uint32_t win;
  int win_base;   // -1: empty
};
#define CIT_MT_COOP 1
#define CIT_MT_WINDOW 2

CIT_HD uint32_t mt_word(const CitMT& r, int i) { return r.mt[(long)i * r.stride]; }
CIT_HD void mt_set(const CitMT& r, int i, uint32_t v) { r.mt[(long)i * r.stride] = v; }

// init_genrand (numpy legacy `RandomState.seed(int)`)
CIT_HDI void mt_init_genrand(CitMT& r, uint32_t s) {
  mt_set(r, 0, s);
  for (int i = 1; i < CIT_MT_N; i++) {
    s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i;
    mt_set(r, i, s);
  }
  r.pos = CIT_MT_N;
}

// CPython random.seed(int): init_by_array(key = 32-bit little-endian words of |seed|)
CIT_HDI void mt_seed_cpython(CitMT& r, uint64_t seed) {
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  int klen = (seed >> 32) ? 2 : 1;
  mt_init_genrand(r, 19650218u);
  int i = 1, j = 0;
  uint32_t prev = mt_word(r, 0);
  for (int k = (CIT_MT_N > klen ? CIT_MT_N : klen); k; k--) {
    uint32_t v = (mt_word(r, i) ^ ((prev ^ (prev >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
    mt_set(r, i, v);
    prev = v;
    i++;
    j++;
    if (i >= CIT_MT_N) { mt_set(r, 0, v); i = 1; }
    if (j >= klen) j = 0;
  }
  for (int k = CIT_MT_N - 1; k; k--) {
    uint32_t v = (mt_word(r, i) ^ ((prev ^ (prev >> 30)) * 1566083941u)) - (uint32_t)i;
    mt_set(r, i, v);
    prev = v;
    i++;
    if (i >= CIT_MT_N) { mt_set(r, 0, v); i = 1; }
  }
  mt_set(r, 0, 0x80000000u);
  r.pos = CIT_MT_N;
}

#if defined(CIT_PROF_ROLLOUT) && defined(__HIPCC__)
__device__ unsigned long long g_roll_prof[160];
#endif
#if defined(CIT_PROF_ROLLOUT) && defined(__HIP_DEVICE_COMPILE__)
struct CitTwistProf {
  unsigned long long t0 = clock64();
  __device__ ~CitTwistProf() {
    if (__lane_id() == 0) {
      atomicAdd(&g_roll_prof[6], clock64() - t0);
      atomicAdd(&g_roll_prof[7], 1ull);
    }
  }
};
#define CIT_TWIST_PROF() CitTwistProf _twist_prof
#else
#define CIT_TWIST_PROF() ((void)0)
#endif

// genrand's twist in chunks of 16 words: every load of a chunk is issued
// before its stores, so one memory round trip covers 16 words.  Within a
// chunk [c, c+16) the loads are mt[c..c+16] (old, or the rewritten mt[0] for
// the last word) and mt[i+397 mod 624] (old for i < 227, rewritten by an
// earlier chunk for i >= 227, since 227 > 16): the serial recurrence exactly.
#define CIT_TWIST_CHUNK 16
#ifdef CIT_TWIST_NOINLINE
#define CIT_TWIST_ATTR __attribute__((noinline))
#else
#define CIT_TWIST_ATTR
#endif
CIT_HDI CIT_TWIST_ATTR void mt_twist(const CitMT& r) {
  CIT_TWIST_PROF();
  for (int c = 0; c < CIT_MT_N; c += CIT_TWIST_CHUNK) {
    uint32_t w[CIT_TWIST_CHUNK + 1], f[CIT_TWIST_CHUNK];
#pragma unroll
    for (int j = 0; j <= CIT_TWIST_CHUNK; j++) w[j] = mt_word(r, c + j < CIT_MT_N ? c + j : 0);
#pragma unroll
    for (int j = 0; j < CIT_TWIST_CHUNK; j++) {
      int m = c + j + 397;
      f[j] = mt_word(r, m < CIT_MT_N ? m : m - CIT_MT_N);
    }
#pragma unroll
    for (int j = 0; j < CIT_TWIST_CHUNK; j++) {
      uint32_t y = (w[j] & 0x80000000u) | (w[j + 1] & 0x7fffffffu);
      mt_set(r, c + j, f[j] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u));
    }
  }
}
static_assert(CIT_MT_N % CIT_TWIST_CHUNK == 0 && CIT_TWIST_CHUNK < 227, "twist chunking");

#if defined(__HIP_DEVICE_COMPILE__)
// The twist by all 64 lanes of a wave that runs the stream's owner uniformly
// (CitMT::coop), in place over an LDS block (stride 1).  New word i reads old
// i, i+1 and (i+397) mod 624; the serial recurrence makes (i+397) mod 624 a
// NEW word for i >= 227 and word 0 new for i = 623.  Hence three phases,
// [0,227) from old words, [227,454) reading phase 1, [454,624) reading phase
// 2 (and new word 0); within a phase every lane reads before any lane writes.
typedef __attribute__((address_space(3))) uint32_t cit_lds_u32;
__device__ __attribute__((noinline)) void mt_twist_coop(cit_lds_u32* m) {
  CIT_TWIST_PROF();
  const int ln = (int)__lane_id();
  const int bounds[4] = {0, 227, 454, CIT_MT_N};
#pragma unroll
  for (int ph = 0; ph < 3; ph++) {
    for (int i0 = bounds[ph]; i0 < bounds[ph + 1]; i0 += 64) {
      int i = i0 + ln;
      bool on = i < bounds[ph + 1];
      uint32_t v = 0;
      if (on) {
        uint32_t y = (m[i] & 0x80000000u) | (m[i + 1 < CIT_MT_N ? i + 1 : 0] & 0x7fffffffu);
        int k = i + 397;
        v = m[k < CIT_MT_N ? k : k - CIT_MT_N] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      __syncthreads();
      if (on) m[i] = v;
      __syncthreads();
    }
  }
}
// The same twist inline, for a unit whose search functions are out of line
// (cit_cfr.hip): a call to mt_twist_coop makes its caller a non-leaf function,
// which must save its return address through a callee-saved VGPR spilled to
// scratch and reload it before returning (a scratch round trip on every call of
// eng_carry, eng_prepare, eng_sample, cfr_choose, ...), for a twist that runs
// once per 624 draws.  One wave owns the stream, so ten 64-word chunks in
// order need no barrier (LDS operations of one wave are in order): in chunk c
// word i reads old words i and i + 1 (or the new word 0 for i = 623) and word
// (i + 397) mod 624, which is old for i < 227 (a later chunk) and new for
// i >= 227 (i - 227 lies in an earlier chunk) -- the serial recurrence.
__device__ __forceinline__ void mt_twist_wave(cit_lds_u32* m) {
  const int ln = (int)__lane_id();
#pragma unroll 1
  for (int c = 0; c < CIT_MT_N; c += 64) {
    const int i = c + ln;
    const int ic = i < CIT_MT_N ? i : 0;
    const int i1 = ic + 1 < CIT_MT_N ? ic + 1 : 0;
    const int k = ic + 397 < CIT_MT_N ? ic + 397 : ic + 397 - CIT_MT_N;
    const uint32_t y = (m[ic] & 0x80000000u) | (m[i1] & 0x7fffffffu);
    const uint32_t v = m[k] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    if (i < CIT_MT_N) m[i] = v;
  }
}
#ifndef CIT_TWIST_INLINE
#define CIT_TWIST_INLINE 1
#endif
#endif

CIT_HD uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

CIT_HD uint32_t mt_next(CitMT& r) {
  uint32_t i = r.pos;
  if (i >= CIT_MT_N) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(CIT_MT_COOP_ONLY)
    // a unit whose every stream is an LDS coop stream
    if (CIT_TWIST_INLINE)
      mt_twist_wave((cit_lds_u32*)r.mt);
    else
      mt_twist_coop((cit_lds_u32*)r.mt);
    r.win_base = -1;
#elif defined(__HIP_DEVICE_COMPILE__)
    if (r.coop) {
      // (coop streams belong to one-wave workgroups: uniform_game launches 64 threads)
      if (CIT_TWIST_INLINE)
        mt_twist_wave((cit_lds_u32*)r.mt);
      else
        mt_twist_coop((cit_lds_u32*)r.mt);
      r.win_base = -1;
    } else {
      mt_twist(r);
    }
#else
    mt_twist(r);
#endif
    i = 0;
  }
  r.pos = i + 1;
#if defined(__HIP_DEVICE_COMPILE__)
  if (r.coop == CIT_MT_WINDOW) {
    int b = (int)(i & ~63u);
    if (b != r.win_base) {
      int j = b + (int)__lane_id();
      const uint32_t wj = ((const cit_lds_u32*)r.mt)[j < CIT_MT_N ? j : 0];   // every lane loads (no branch)
      r.win = mt_temper(j < CIT_MT_N ? wj : 0u);
      r.win_base = b;
    }
    return (uint32_t)__builtin_amdgcn_readlane((int)r.win, (int)(i & 63u));
  }
#if defined(CIT_MT_COOP_ONLY)
  return mt_temper(((const cit_lds_u32*)r.mt)[i]);
#else
  if (r.coop) return mt_temper(((const cit_lds_u32*)r.mt)[i]);   // coop streams live in LDS (stride 1)
#endif
#endif
  return mt_temper(mt_word(r, (int)i));
}

CIT_HD int bit_length(uint32_t n) { return n ? 32 - __builtin_clz(n) : 0; }

// random._randbelow_with_getrandbits (Lib/random.py:239-249)
CIT_HD uint32_t mt_randbelow(CitMT& r, uint32_t n) {
  if (!n) return 0;
  int k = bit_length(n);
  uint32_t v = mt_next(r) >> (32 - k);
  while (v >= n) v = mt_next(r) >> (32 - k);
  return v;
}

// random.random() / numpy random_sample(): 53-bit double from two draws
CIT_HD double mt_random(CitMT& r) {
  uint32_t a = mt_next(r) >> 5, b = mt_next(r) >> 6;
  return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

#if CIT_WAVE
// A burst of draws from an LDS stream through a register window (CitMT
// CIT_MT_WINDOW): a copy of the stream whose draws are readlanes of 64
// tempered words; cit_mt_unwindow() hands the position (and, for a stream
// that already was a window, the window) back.  Only for coop streams
// (r.coop != 0: the words are in LDS and the whole wave runs the owner).
CIT_HD CitMT cit_mt_window(const CitMT& r) {
  CitMT w = r;
  if (w.coop != CIT_MT_WINDOW) {
    w.coop = CIT_MT_WINDOW;
    w.win = 0;
    w.win_base = -1;
  }
  return w;
}
CIT_HD void cit_mt_unwindow(CitMT& r, const CitMT& w) {
  r.pos = w.pos;
  if (r.coop == CIT_MT_WINDOW) {
    r.win = w.win;
    r.win_base = w.win_base;
  }
}
#endif
