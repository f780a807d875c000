// HIP kernels + C ABI (include/citadels.h) of the MI355X Citadels engine.
//
// Execution model: one game per 64-lane workgroup with wave-uniform code
// (uniform_game below): the lanes stage the game's packed row (CIT_GAME_BYTES)
// and, for multi-step kernels, its 624 CPython-MT19937 words from HBM into
// LDS; lane 0 runs the engine with every address derived from blockIdx.x, so
// the game's scalars live in SGPRs and its branches are scalar; the lanes
// write back.  MT19937 streams are stored structure-of-arrays ([624][B]) in
// HBM.  k_rollout (games_per_block > 0) keeps the one-game-per-lane layout for
// sweeps.
#include <hip/hip_runtime.h>

// random.shuffle over a sequence of up to 128 in two VGPRs (cit_engine.h
// shuffle_seq): the rollout's one batch 0.92 -> 0.94 G, the overlapped
// headline unchanged (profiles/r04/rollout_waves/summary_shuffle.txt); the
// search unit keeps the LDS swaps (8 % slower there: its registers are full)
#ifndef CIT_SHUFFLE_REG
#define CIT_SHUFFLE_REG 1
#endif

#include "../../include/citadels.h"
#include "cit_engine.h"
#include "cit_lanes.h"

static_assert(sizeof(CitOpt) == sizeof(CitOption), "descriptor layouts differ");

#define ROW_W (CIT_GAME_BYTES / 4)
#ifndef ROLLOUT_BUF
#define ROLLOUT_BUF 64   // options listed per step; 64 measured 1.3-1.5 % over 32 (preset max 56)
#endif
#ifndef ROLLOUT_REG
#define ROLLOUT_REG 1   // the step's option list in registers (RegSink) instead of buf
#endif

namespace {

__device__ __forceinline__ CitMT lane_mt(uint32_t* mt, const uint32_t* idx, int B, long l) {
  CitMT r;
  r.mt = mt + l;
  r.stride = B;
  r.pos = idx[l];
  r.coop = 0;
  return r;
}

// One game per 64-lane workgroup with wave-uniform code: the game index is
// blockIdx.x (never threadIdx.x), so the compiler keeps the game's scalars in
// SGPRs and branches with s_cbranch instead of exec masks (measured: +27 %
// transitions/s at B = 4096 over one game per lane, and no scratch spills).
// The 64 lanes stage the row (and, for multi-step kernels, the 624 MT19937
// words) into LDS and run `body(game, stream, l)` together: every lane
// computes the same values (LDS reads at uniform addresses are uniform), so
// control flow never diverges, and the lanes are there for lane-parallel
// pieces such as the MT19937 twist (CitMT::coop).  CIT_LANE0_BODY restores
// the lane-0-only body for A/B runs.  The lanes then write back.
#ifndef CIT_LANE0_BODY
#define CIT_LANE0_BODY 0
#endif
template <bool MT_LDS, bool STAGE_ROW, class F>
__device__ __forceinline__ void uniform_game_at(long l, uint32_t* games, uint32_t* mt, uint32_t* idx, int B,
                                                F&& body) {
  __shared__ __attribute__((aligned(16))) uint32_t row[ROW_W];
  __shared__ uint32_t mts[MT_LDS ? CIT_MT_N : 1];
  if (STAGE_ROW)
    for (int i = threadIdx.x; i < ROW_W; i += blockDim.x) row[i] = games[l * ROW_W + i];
  if (MT_LDS)
    for (int i = threadIdx.x; i < CIT_MT_N; i += blockDim.x) mts[i] = mt[(long)i * B + l];
  __syncthreads();
  if (!CIT_LANE0_BODY || threadIdx.x == 0) {
    CitGame& g = *reinterpret_cast<CitGame*>(row);
    CitMT r;
    if (MT_LDS) {
      r.mt = mts;
      r.stride = 1;
    } else {
      r.mt = mt + l;
      r.stride = B;
    }
    r.pos = idx[l];
    r.coop = MT_LDS && !CIT_LANE0_BODY ? CIT_MT_WINDOW : 0;
    r.win = 0;
    r.win_base = -1;
    body(g, r, l);
    if (threadIdx.x == 0) idx[l] = r.pos;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ROW_W; i += blockDim.x) games[l * ROW_W + i] = row[i];
  if (MT_LDS)
    for (int i = threadIdx.x; i < CIT_MT_N; i += blockDim.x) mt[(long)i * B + l] = mts[i];
}
template <bool MT_LDS, bool STAGE_ROW, class F>
__device__ __forceinline__ void uniform_game(uint32_t* games, uint32_t* mt, uint32_t* idx, int B, F&& body) {
  uniform_game_at<MT_LDS, STAGE_ROW>((long)blockIdx.x, games, mt, idx, B, body);
}

// init_genrand(19650218), the first step of CPython's init_by_array, is the
// same for every seed: a compile-time table.
struct CitMTInitTable {
  uint32_t w[CIT_MT_N];
};
constexpr CitMTInitTable cit_mt_init_table() {
  CitMTInitTable t{};
  uint32_t s = 19650218u;
  t.w[0] = s;
  for (int i = 1; i < CIT_MT_N; i++) {
    s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i;
    t.w[i] = s;
  }
  return t;
}
__constant__ CitMTInitTable c_mt_init = cit_mt_init_table();

// CPython random.seed(int) (init_by_array) for 64 games per workgroup, one
// game per lane: each game's recurrence is serial, so the parallelism is
// across games.  The first pass reads the constant table and writes its words
// straight to the games' HBM streams (structure of arrays [624][B]: a wave's
// 64 lanes store one coalesced 256-byte line per step); the second pass reads
// them back from there (L2-resident: written by the same lanes moments
// before), loads issued a window ahead of the serial chain.  No LDS, so the
// seeding of the next batch co-resides with rollout waves of the previous
// ones (bench.py e2e).  Same stream as mt_seed_cpython (cit_core.h).
#define MT_SEED_AHEAD 16
__global__ __launch_bounds__(64) void k_mt_seed_cpython(uint32_t* mt, uint32_t* idx, int B, const uint64_t* seeds) {
  const long g0 = (long)blockIdx.x * 64 + threadIdx.x;
  const bool on = g0 < B;
  const long g = on ? g0 : (long)B - 1;   // an idle lane recomputes the last game and stores nothing
  const uint64_t seed = seeds[g];
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const int klen = k1 ? 2 : 1;
  uint32_t* m = mt + g;                   // word i at m[i * B]
  uint32_t prev = c_mt_init.w[0];
  int j = 0;
  // pass 1 (k = 624 steps): i = 1..623 read the table, the 624th (i = 1 again) its own output
  uint32_t w1 = 0;
  for (int i = 1; i < CIT_MT_N; i++) {
    uint32_t v = (c_mt_init.w[i] ^ ((prev ^ (prev >> 30)) * 1664525u)) + (j ? k1 : k0) + (uint32_t)j;
    if (i == 1) w1 = v;
    else if (on) m[(long)i * B] = v;
    prev = v;
    j = j + 1 >= klen ? 0 : j + 1;
  }
  {
    uint32_t v = (w1 ^ ((prev ^ (prev >> 30)) * 1664525u)) + (j ? k1 : k0) + (uint32_t)j;
    w1 = v;
    prev = v;
  }
  // pass 2 (623 steps): i = 2..623, then i = 1; words 2..623 come back from HBM / L2
  __threadfence_block();
  uint32_t ahead[MT_SEED_AHEAD];
#pragma unroll
  for (int k = 0; k < MT_SEED_AHEAD; k++) ahead[k] = m[(long)(2 + k) * B];
  for (int i0 = 2; i0 < CIT_MT_N; i0 += MT_SEED_AHEAD) {
#pragma unroll
    for (int k = 0; k < MT_SEED_AHEAD; k++) {
      const int i = i0 + k;
      if (i < CIT_MT_N) {
        uint32_t v = (ahead[k] ^ ((prev ^ (prev >> 30)) * 1566083941u)) - (uint32_t)i;
        const int ni = i + MT_SEED_AHEAD;
        if (ni < CIT_MT_N) ahead[k] = m[(long)ni * B];
        if (on) m[(long)i * B] = v;
        prev = v;
      }
    }
  }
  w1 = (w1 ^ ((prev ^ (prev >> 30)) * 1566083941u)) - 1u;
  if (on) {
    m[0] = 0x80000000u;
    m[B] = w1;
    idx[g] = CIT_MT_N;
  }
}

__global__ void k_mt_seed(uint32_t* mt, uint32_t* idx, int B, const uint64_t* seeds, int numpy_style) {
  long l = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= B) return;
  CitMT r = lane_mt(mt, idx, B, l);
  if (numpy_style) mt_init_genrand(r, (uint32_t)seeds[l]);
  else mt_seed_cpython(r, seeds[l]);
  idx[l] = r.pos;
}

__global__ void k_mt_draw(uint32_t* mt, uint32_t* idx, int B, int n, uint32_t* out) {
  long l = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= B) return;
  CitMT r = lane_mt(mt, idx, B, l);
  for (int i = 0; i < n; i++) out[l * n + i] = mt_next(r);
  idx[l] = r.pos;
}

__global__ void k_randbelow(uint32_t* mt, uint32_t* idx, int B, uint32_t bound, int32_t* out) {
  long l = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= B) return;
  CitMT r = lane_mt(mt, idx, B, l);
  out[l] = (int32_t)mt_randbelow(r, bound);
  idx[l] = r.pos;
}

__global__ __launch_bounds__(64) void k_init(uint32_t* games, uint32_t* mt, uint32_t* idx, int B,
                                            const uint64_t* seeds, int preset) {
  uniform_game<true, false>(games, mt, idx, B, [&](CitGame& g, CitMT& r, long l) {
    if (seeds) mt_seed_cpython(r, seeds[l]);          // NULL: continue the lane's stream
    cit_init_game(g, r, preset != 0);
  });
}

__global__ __launch_bounds__(64) void k_get_options(uint32_t* games, uint32_t* mt, uint32_t* idx, uint64_t* seer,
                                                   int B, CitOpt* opts, int max_opts, int32_t* n_opts) {
  uniform_game<false, true>(games, mt, idx, B, [&](CitGame& g, CitMT& r, long l) {
    uint64_t* sc = seer + l * CIT_SEER_MAX;
    cit_prepare_options(g, r, sc);
    ListSink s(opts + l * max_opts, max_opts);
    cit_enum_options(g, s, sc);
    g.err |= s.err;
    n_opts[l] = s.n;
  });
}

// Agent.get_options' count only (get_options may mutate the game: state 9
// scholar picks, state 8 seer draws), nothing materialised.
__global__ __launch_bounds__(64) void k_count_options(uint32_t* games, uint32_t* mt, uint32_t* idx, uint64_t* seer,
                                                     int B, int32_t* n_opts) {
  uniform_game<false, true>(games, mt, idx, B, [&](CitGame& g, CitMT& r, long l) {
    uint64_t* sc = seer + l * CIT_SEER_MAX;
    cit_prepare_options(g, r, sc);
    uint32_t e = 0;
    n_opts[l] = cit_count_options(g, e, sc);
    g.err |= e;
  });
}

// Game.sample_private_information(players[orig[l]], role_sample) per lane.
__global__ __launch_bounds__(64) void k_determinize(uint32_t* games, uint32_t* mt, uint32_t* idx, int B,
                                                   const int32_t* orig, int role_sample) {
  __shared__ __attribute__((aligned(16))) uint8_t unk[CIT_SAMPLE_SCRATCH];
  uniform_game<true, true>(games, mt, idx, B, [&](CitGame& g, CitMT& r, long l) {   // MT in LDS: the wave path
    int o = orig[l];
    if (o < 0 || o >= CIT_NP) {
      g.err |= CIT_ERR_INDEX;
      return;
    }
    cit_sample_private(g, o, role_sample != 0, r, unk);
  });
}

// CFRNode.skip_false_choice (deep_mccfr.py:37-49) per lane; carried[l] = steps played.
__global__ __launch_bounds__(64) void k_skip_false_choice(uint32_t* games, uint32_t* mt, uint32_t* idx,
                                                         uint64_t* seer, int B, int32_t* carried) {
  uniform_game<true, true>(games, mt, idx, B, [&](CitGame& g, CitMT& r, long l) {
    int n = cit_skip_false_choice(g, r, seer + l * CIT_SEER_MAX);
    if (carried) carried[l] = n;
  });
}

__global__ __launch_bounds__(64) void k_carry_out(uint32_t* games, uint32_t* mt, uint32_t* idx, int B,
                                                 const CitOpt* chosen, int32_t* winner) {
  uniform_game<false, true>(games, mt, idx, B,
                            [&](CitGame& g, CitMT& r, long l) { winner[l] = cit_carry_out(g, chosen[l], r); });
}

__global__ void k_random_choice(uint32_t* games, uint32_t* mt, uint32_t* idx, int B, const CitOpt* opts,
                                int max_opts, const int32_t* n_opts, CitOpt* chosen, int32_t* k_out) {
  long l = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= B) return;
  CitGame* g = reinterpret_cast<CitGame*>(games + l * ROW_W);
  int n = n_opts[l];
  if (n <= 0) {
    g->err |= CIT_ERR_EMPTY;
    k_out[l] = -1;
    return;
  }
  CitMT r = lane_mt(mt, idx, B, l);
  int k = (int)mt_randbelow(r, (uint32_t)n);
  idx[l] = r.pos;
  k_out[l] = k;
  if (k >= max_opts) {
    g->err |= CIT_ERR_OVERFLOW;
    return;
  }
  chosen[l] = opts[l * max_opts + k];
}

#ifdef CIT_PROF_ROLLOUT
// Phase cycle accounting of the rollout step (profiling builds only:
// tools/prof_rollout.py).  [0..4] prepare / enumerate / randbelow / pick /
// carry_out cycles, [5] steps, [16+s] enumerate+carry cycles in state s,
// [32+s] steps in state s, [64+o] carry_out cycles of option name o, [112+o] their count.
// s_memtime stamps (clock64): reading one waits for the wave's outstanding LDS
// operations, so a phase is also charged the drain of the previous phase's
// LDS stores.  (HW_REG_SHADER_CYCLES reads 0 on gfx950.)
__device__ __forceinline__ unsigned long long prof_clk() { return clock64(); }
__device__ __forceinline__ unsigned long long prof_d(unsigned long long a, unsigned long long b) { return b - a; }
__device__ __forceinline__ int prof_step(CitGame& g, CitMT& rng, uint64_t* seer, CitOpt* buf, int cap, unsigned long long* acc) {
  int st = g.gs_state;
  unsigned long long t0c = prof_clk();
  cit_prepare_options(g, rng, seer);
  unsigned long long t1 = prof_clk();
#if CIT_WAVE
  RegSink s;                               // the default step's sink (ROLLOUT_REG)
  (void)buf;
  (void)cap;
#else
  BufSink s(buf, cap);
#endif
  cit_enum_options(g, s, seer);
  unsigned long long t2 = prof_clk();
  if (s.err) { g.err |= s.err; return 1; }
  int n = s.n;
  if (n == 0) { g.err |= CIT_ERR_EMPTY; return 1; }
  int k = (int)mt_randbelow(rng, (uint32_t)n);
  unsigned long long t3 = prof_clk();
#if CIT_WAVE
  CitOpt o = k < 64 ? s.at(k) : cit_pick_option(g, k, seer);
#else
  CitOpt o = k < cap ? buf[k] : cit_pick_option(g, k, seer);
#endif
  unsigned long long t4 = prof_clk();
  int w = cit_carry_out(g, o, rng);
  unsigned long long t5 = prof_clk();
  acc[0] += prof_d(t0c, t1); acc[1] += prof_d(t1, t2); acc[2] += prof_d(t2, t3); acc[3] += prof_d(t3, t4);
  acc[4] += prof_d(t4, t5); acc[5] += 1;
  if (st < 11) { acc[16 + st] += prof_d(t1, t2) + prof_d(t4, t5); acc[32 + st] += 1; }
  if (o.name < 47) { acc[64 + o.name] += prof_d(t4, t5); acc[112 + o.name] += 1; }
  return (w >= 0 || g.err || g.terminal) ? 1 : 0;
}
#endif

#ifdef ROLL_CLOCK
// Per-game start / end wall clock (100 MHz) of k_rollout_u (measurement builds
// only: tools/rollout_clock.py).
__device__ unsigned long long g_roll_clock[2 * 65536];
#endif

// The hot loop (default): one game per workgroup (uniform_game), row and
// MT19937 words in LDS for the whole rollout.  ROLL_WAVES_PER_EU bounds the
// register budget: 8 -> 64 VGPRs (some spilled to scratch), 8 games resident
// per SIMD, so a second batch in flight fills the slots.
#ifndef ROLL_WAVES_PER_EU
#define ROLL_WAVES_PER_EU 8
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(ROLL_WAVES_PER_EU))) void k_rollout_u(uint32_t* games, uint32_t* mt, uint32_t* idx, uint64_t* seer, int B,
                                                 int max_steps, int32_t* steps_out, int32_t* winner) {
  __shared__ __attribute__((aligned(16))) CitOpt buf[ROLLOUT_BUF ? ROLLOUT_BUF : 1];
#ifdef ROLL_CLOCK
  unsigned long long rc0 = wall_clock64();
#endif
  cfr_prof_reset();                         // (CIT_PROF builds: the engine scopes of this game)
  uniform_game<true, true>(games, mt, idx, B, [&](CitGame& g, CitMT& r, long l) {
    uint64_t* sc = seer + l * CIT_SEER_MAX;
    int cap = max_steps < 0 ? CIT_ROLLOUT_CAP : max_steps;
    int s = 0;
#ifdef CIT_PROF_ROLLOUT
    unsigned long long acc[160] = {};
    while (!g.terminal && !g.err && s < cap) {
      prof_step(g, r, sc, buf, ROLLOUT_BUF, acc);
      s++;
    }
    if (threadIdx.x == 0)
      for (int i = 0; i < 160; i++) atomicAdd(&g_roll_prof[i], acc[i]);
#else
    while (!g.terminal && !g.err && s < cap) {
      if (ROLLOUT_REG) cit_random_step_reg(g, r, sc);
      else if (ROLLOUT_BUF) cit_random_step_buf(g, r, sc, buf, ROLLOUT_BUF);
      else cit_random_step(g, r, sc);
      s++;
    }
#endif
    if (max_steps < 0 && s >= cap && !g.terminal && !g.err) g.err |= CIT_ERR_STEP_CAP;
    steps_out[l] += s;
    winner[l] = g.winner;
  });
#ifdef ROLL_CLOCK
  if (threadIdx.x == 0 && blockIdx.x < 65536) {
    g_roll_clock[2 * blockIdx.x] = rc0;
    g_roll_clock[2 * blockIdx.x + 1] = wall_clock64();
  }
#endif
  cfr_prof_flush();
}

// The same rollout as a work queue (cit_rollout_queue): a grid of as many
// one-wave workgroups as the GPU holds at once, each taking the next game
// index from `next` (a vector atomic by lane 0) until all B games are played,
// so a finished game's slot takes the next game at once instead of idling
// until the launch's longest game ends.  Every game is played exactly as by
// k_rollout_u (the same body on the same row and stream).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(ROLL_WAVES_PER_EU))) void k_rollout_q(
    uint32_t* games, uint32_t* mt, uint32_t* idx, uint64_t* seer, int B, int max_steps, int32_t* steps_out,
    int32_t* winner, int32_t* next) {
  __shared__ __attribute__((aligned(16))) CitOpt buf[ROLLOUT_BUF ? ROLLOUT_BUF : 1];
  for (;;) {
    int g = 0;
    if (threadIdx.x == 0) g = atomicAdd(next, 1);
    g = __builtin_amdgcn_readfirstlane(g);
    if (g >= B) break;                      // every wave reaches this: the grid drains
    uniform_game_at<true, true>((long)g, games, mt, idx, B, [&](CitGame& gm, CitMT& r, long l) {
      uint64_t* sc = seer + l * CIT_SEER_MAX;
      int cap = max_steps < 0 ? CIT_ROLLOUT_CAP : max_steps;
      int s = 0;
      while (!gm.terminal && !gm.err && s < cap) {
        if (ROLLOUT_REG) cit_random_step_reg(gm, r, sc);
        else if (ROLLOUT_BUF) cit_random_step_buf(gm, r, sc, buf, ROLLOUT_BUF);
        else cit_random_step(gm, r, sc);
        s++;
      }
      if (max_steps < 0 && s >= cap && !gm.terminal && !gm.err) gm.err |= CIT_ERR_STEP_CAP;
      steps_out[l] += s;
      winner[l] = gm.winner;
    });
    __syncthreads();
  }
}

// config-3 position harness: k = random.randint(lo, hi) random steps per lane.
__global__ __launch_bounds__(64) void k_advance(uint32_t* games, uint32_t* mt, uint32_t* idx, uint64_t* seer, int B,
                                               int lo, int hi, int32_t* steps_out) {
  uniform_game<true, true>(games, mt, idx, B, [&](CitGame& g, CitMT& r, long l) {
    uint64_t* sc = seer + l * CIT_SEER_MAX;
    int k = lo + (int)mt_randbelow(r, (uint32_t)(hi - lo + 1));
    int s = 0;
    while (s < k && !g.terminal && !g.err) {
      cit_random_step(g, r, sc);
      s++;
    }
    steps_out[l] = s;
  });
}

// compare_to_random's step loop to the next searched decision per lane.
__global__ __launch_bounds__(64) void k_advance_policy(uint32_t* games, uint32_t* mt, uint32_t* idx, uint64_t* seer,
                                                      int B, int search_mask, int max_steps, int32_t* status,
                                                      int32_t* steps_out) {
  uniform_game<true, true>(games, mt, idx, B, [&](CitGame& g, CitMT& r, long l) {
    int st = steps_out[l];
    status[l] = cit_advance_policy(g, r, seer + l * CIT_SEER_MAX, search_mask, max_steps, st);
    steps_out[l] = st;
  });
}

// create_a_random_game(max_move) per lane (train_from_scratch data generation).
__global__ __launch_bounds__(64) void k_random_position(uint32_t* games, uint32_t* mt, uint32_t* idx, uint64_t* seer,
                                                       int B, int max_move, uint32_t* ring, int32_t* steps_out) {
  uniform_game<true, false>(games, mt, idx, B, [&](CitGame& g, CitMT& r, long l) {
    steps_out[l] = cit_random_position(g, r, seer + l * CIT_SEER_MAX, ring + l * (long)max_move * ROW_W, max_move);
  });
}

// create_a_close_to_finished_game per lane (generate_test_data positions).
__global__ __launch_bounds__(64) void k_close_position(uint32_t* games, uint32_t* mt, uint32_t* idx, uint64_t* seer,
                                                      int B, uint32_t* store, int32_t* index) {
  uniform_game<true, true>(games, mt, idx, B, [&](CitGame& g, CitMT& r, long l) {
    index[l] = cit_close_position(g, r, seer + l * CIT_SEER_MAX, store + l * (long)CIT_CLOSE_ROWS * ROW_W);
  });
}

}  // namespace

#define CHECK_LAUNCH()                       \
  do {                                       \
    hipError_t _e = hipGetLastError();       \
    return _e == hipSuccess ? 0 : (int)_e;   \
  } while (0)

extern "C" {

#ifdef CIT_PROF_ROLLOUT
int cit_roll_prof_read(unsigned long long* out) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_roll_prof), sizeof(unsigned long long) * 160);
  unsigned long long z[160] = {};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_roll_prof), z, sizeof(z));
  return (int)e;
}
#endif

#ifdef CIT_PROF
// the engine's CIT_PROF_SCOPE sums of this unit's rollouts (then cleared):
// [i] cycles, [32 + i] calls of scope i (tools/prof_rollout_scopes.py)
int cit_hip_prof_read(unsigned long long* out) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cit_prof), sizeof(unsigned long long) * 64);
  unsigned long long z[64] = {};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_cit_prof), z, sizeof(z));
  return (int)e;
}
#endif

#ifdef ROLL_CLOCK
int cit_roll_clock_read(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_roll_clock), sizeof(unsigned long long) * 2 * n);
}
#endif

int cit_abi_version(void) { return 9; }
int cit_game_bytes(void) { return CIT_GAME_BYTES; }
int cit_seer_scratch_words(void) { return CIT_SEER_MAX; }

int cit_layout(int* out, int n) {
  int v[] = {(int)sizeof(CitPlayer),          (int)offsetof(CitGame, deck),   (int)offsetof(CitGame, kh),
             (int)offsetof(CitGame, roles),   (int)offsetof(CitGame, gs_state), (int)offsetof(CitGame, points),
             (int)offsetof(CitGame, err),     (int)offsetof(CitGame, steps),  (int)sizeof(CitOpt)};
  int k = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < k && i < n; i++) out[i] = v[i];
  return k;
}

int cit_mt_seed(uint32_t* mt, uint32_t* mt_idx, int B, const uint64_t* seeds, int numpy_style, hipStream_t stream) {
  if (B <= 0 || !mt || !mt_idx || !seeds) return -1;
  hipLaunchKernelGGL(k_mt_seed, dim3((B + 63) / 64), dim3(64), 0, stream, mt, mt_idx, B, seeds, numpy_style);
  CHECK_LAUNCH();
}

int cit_mt_draw(uint32_t* mt, uint32_t* mt_idx, int B, int n, uint32_t* out, hipStream_t stream) {
  if (B <= 0 || n < 0 || !mt || !mt_idx || !out) return -1;
  hipLaunchKernelGGL(k_mt_draw, dim3((B + 63) / 64), dim3(64), 0, stream, mt, mt_idx, B, n, out);
  CHECK_LAUNCH();
}

int cit_randbelow(uint32_t* mt, uint32_t* mt_idx, int B, int bound, int32_t* out, hipStream_t stream) {
  if (B <= 0 || bound <= 0 || !mt || !mt_idx || !out) return -1;
  hipLaunchKernelGGL(k_randbelow, dim3((B + 63) / 64), dim3(64), 0, stream, mt, mt_idx, B, (uint32_t)bound, out);
  CHECK_LAUNCH();
}

int cit_init(void* games, uint32_t* mt, uint32_t* mt_idx, int B, const uint64_t* seeds, int preset,
             hipStream_t stream) {
  if (B <= 0 || !games || !mt || !mt_idx) return -1;
  if (seeds) {   // random.seed(s) for every lane (one game per lane), then the deal continues the streams
    hipLaunchKernelGGL(k_mt_seed_cpython, dim3((B + 63) / 64), dim3(64), 0, stream, mt, mt_idx, B, seeds);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(k_init, dim3(B), dim3(64), 0, stream, (uint32_t*)games, mt, mt_idx, B,
                     (const uint64_t*)nullptr, preset);
  CHECK_LAUNCH();
}

int cit_get_options(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, CitOption* opts,
                    int max_opts, int32_t* n_opts, hipStream_t stream) {
  if (B <= 0 || max_opts < 0 || !games || !mt || !mt_idx || !seer || !n_opts || (max_opts && !opts)) return -1;
  hipLaunchKernelGGL(k_get_options, dim3(B), dim3(64), 0, stream, (uint32_t*)games, mt,
                     mt_idx, seer, B, (CitOpt*)opts, max_opts, n_opts);
  CHECK_LAUNCH();
}

int cit_count_options(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int32_t* n_opts,
                      hipStream_t stream) {
  if (B <= 0 || !games || !mt || !mt_idx || !seer || !n_opts) return -1;
  hipLaunchKernelGGL(k_count_options, dim3(B), dim3(64), 0, stream, (uint32_t*)games, mt, mt_idx, seer, B, n_opts);
  CHECK_LAUNCH();
}

int cit_determinize(void* games, uint32_t* mt, uint32_t* mt_idx, int B, const int32_t* orig_player, int role_sample,
                    hipStream_t stream) {
  if (B <= 0 || !games || !mt || !mt_idx || !orig_player) return -1;
  hipLaunchKernelGGL(k_determinize, dim3(B), dim3(64), 0, stream, (uint32_t*)games, mt, mt_idx, B, orig_player,
                     role_sample);
  CHECK_LAUNCH();
}

int cit_skip_false_choice(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int32_t* carried,
                          hipStream_t stream) {
  if (B <= 0 || !games || !mt || !mt_idx || !seer) return -1;
  hipLaunchKernelGGL(k_skip_false_choice, dim3(B), dim3(64), 0, stream, (uint32_t*)games, mt, mt_idx, seer, B,
                     carried);
  CHECK_LAUNCH();
}

int cit_random_choice(void* games, uint32_t* mt, uint32_t* mt_idx, int B, const CitOption* opts, int max_opts,
                      const int32_t* n_opts, CitOption* chosen, int32_t* k_out, hipStream_t stream) {
  if (B <= 0 || max_opts < 0 || !games || !mt || !mt_idx || !n_opts || !chosen || !k_out || (max_opts && !opts))
    return -1;
  hipLaunchKernelGGL(k_random_choice, dim3((B + 63) / 64), dim3(64), 0, stream, (uint32_t*)games, mt, mt_idx, B,
                     (const CitOpt*)opts, max_opts, n_opts, (CitOpt*)chosen, k_out);
  CHECK_LAUNCH();
}

int cit_carry_out(void* games, uint32_t* mt, uint32_t* mt_idx, int B, const CitOption* chosen, int32_t* winner,
                  hipStream_t stream) {
  if (B <= 0 || !games || !mt || !mt_idx || !chosen || !winner) return -1;
  hipLaunchKernelGGL(k_carry_out, dim3(B), dim3(64), 0, stream, (uint32_t*)games, mt,
                     mt_idx, B, (const CitOpt*)chosen, winner);
  CHECK_LAUNCH();
}

int cit_rollout_random(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int max_steps,
                       int games_per_block, int32_t* steps, int32_t* winner, hipStream_t stream) {
  if (B <= 0 || !games || !mt || !mt_idx || !seer || !steps || !winner) return -1;
  if (games_per_block > CIT_LANES_MAX_G) return -1;
  // 0 = auto: one game per workgroup, wave-uniform code (k_rollout_u)
  if (games_per_block <= 0) {
    hipLaunchKernelGGL(k_rollout_u, dim3(B), dim3(64), 0, stream, (uint32_t*)games, mt, mt_idx, seer, B, max_steps,
                       steps, winner);
    CHECK_LAUNCH();
  }
  // G lanes = G games per workgroup (one wavefront), per-lane code (cit_lanes.hip)
  return cit_rollout_lanes((uint32_t*)games, mt, mt_idx, seer, B, max_steps, games_per_block, steps, winner, stream);
}

int cit_rollout_queue(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int max_steps, int grid,
                      int32_t* steps, int32_t* winner, int32_t* next, hipStream_t stream) {
  if (B <= 0 || grid <= 0 || !games || !mt || !mt_idx || !seer || !steps || !winner || !next) return -1;
  hipError_t e = hipMemsetAsync(next, 0, sizeof(int32_t), stream);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(k_rollout_q, dim3(grid < B ? grid : B), dim3(64), 0, stream, (uint32_t*)games, mt, mt_idx, seer,
                     B, max_steps, steps, winner, next);
  CHECK_LAUNCH();
}

int cit_advance_random(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int lo, int hi,
                       int32_t* steps, hipStream_t stream) {
  if (B <= 0 || hi < lo || lo < 0 || !games || !mt || !mt_idx || !seer || !steps) return -1;
  hipLaunchKernelGGL(k_advance, dim3(B), dim3(64), 0, stream, (uint32_t*)games, mt, mt_idx,
                     seer, B, lo, hi, steps);
  CHECK_LAUNCH();
}

int cit_random_position(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int max_move,
                        uint32_t* ring, int32_t* steps, hipStream_t stream) {
  if (B <= 0 || max_move <= 0 || !games || !mt || !mt_idx || !seer || !ring || !steps) return -1;
  hipLaunchKernelGGL(k_random_position, dim3(B), dim3(64), 0, stream, (uint32_t*)games, mt,
                     mt_idx, seer, B, max_move, ring, steps);
  CHECK_LAUNCH();
}

int cit_close_rows(void) { return CIT_CLOSE_ROWS; }

int cit_close_position(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, uint32_t* store,
                       int32_t* index, hipStream_t stream) {
  if (B <= 0 || !games || !mt || !mt_idx || !seer || !store || !index) return -1;
  hipLaunchKernelGGL(k_close_position, dim3(B), dim3(64), 0, stream, (uint32_t*)games, mt,
                     mt_idx, seer, B, store, index);
  CHECK_LAUNCH();
}

int cit_advance_policy(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int search_mask,
                       int max_steps, int32_t* status, int32_t* steps, hipStream_t stream) {
  if (B <= 0 || !games || !mt || !mt_idx || !seer || !status || !steps) return -1;
  hipLaunchKernelGGL(k_advance_policy, dim3(B), dim3(64), 0, stream, (uint32_t*)games, mt,
                     mt_idx, seer, B, search_mask, max_steps < 0 ? CIT_ROLLOUT_CAP : max_steps, status, steps);
  CHECK_LAUNCH();
}

}  // extern "C"
