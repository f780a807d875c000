// Host build of the engine headers (g++, no HIP).  Two uses, neither on the
// product path (the Python package only ever loads libcitadels_hip.so and has
// no CPU fallback):
//  * the CPU test suite checks the engine logic against the golden fixtures in
//    this (GPU-less) container;
//  * bench.py's cpu_baseline leg times cith_rollout_timed, the C++ CPU
//    restatement SURVEY.md §8(d) asks for, on 1 and on all host cores.
//
// Same argument conventions as the HIP C-ABI in include/citadels.h, minus the
// stream, with host pointers; names are prefixed cith_.
#include <stddef.h>
#include <string.h>

#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "cit_area_test.h"
#include "cit_cfr.h"

extern "C" {

int cith_game_bytes() { return CIT_GAME_BYTES; }
int cith_sizeof_game() { return (int)sizeof(CitGame); }
int cith_seer_max() { return CIT_SEER_MAX; }

// cit_area_test.h's operation sequence on B zeroed games (lane l: seeds[l]),
// the scalar paths of the card-area list operations; ops[l * n_ops + i] logs
// op i.  Returns 0.
int cith_area_test(CitGame* g, int B, const uint64_t* seeds, int n_ops, uint32_t* log) {
  for (int l = 0; l < B; l++) {
    CitMT r;
    r.mt = nullptr;   // never drawn from: the sequence keeps the deck stocked
    r.stride = 1;
    r.pos = 0;
    r.coop = 0;
    uint64_t s = seeds[l] | 1ull;
    for (int i = 0; i < n_ops && !g[l].err; i++) area_test_op(g[l], r, s, log + (long)l * n_ops + i);
  }
  return 0;
}

// field offsets, checked against the Python mirror in layout.py
int cith_layout(int* out, int n) {
  int v[] = {(int)sizeof(CitPlayer),
             (int)offsetof(CitGame, deck),
             (int)offsetof(CitGame, kh),
             (int)offsetof(CitGame, roles),
             (int)offsetof(CitGame, gs_state),
             (int)offsetof(CitGame, points),
             (int)offsetof(CitGame, err),
             (int)offsetof(CitGame, steps),
             (int)sizeof(CitOpt)};
  int k = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < k && i < n; i++) out[i] = v[i];
  return k;
}

static CitMT lane_rng(uint32_t* mt, uint32_t* idx, int B, int l) {
  CitMT r;
  r.mt = mt + l;
  r.stride = B;
  r.pos = idx[l];
  r.coop = 0;
  return r;
}
#define SAVE(r) idx[l] = (r).pos

void cith_mt_seed(uint32_t* mt, uint32_t* idx, int B, const uint64_t* seeds, int numpy_style) {
  for (int l = 0; l < B; l++) {
    CitMT r = lane_rng(mt, idx, B, l);
    if (numpy_style) mt_init_genrand(r, (uint32_t)seeds[l]);
    else mt_seed_cpython(r, seeds[l]);
    SAVE(r);
  }
}

void cith_mt_draw(uint32_t* mt, uint32_t* idx, int B, int lane, int n, uint32_t* out) {
  int l = lane;
  CitMT r = lane_rng(mt, idx, B, l);
  for (int i = 0; i < n; i++) out[i] = mt_next(r);
  SAVE(r);
}

void cith_mt_randbelow(uint32_t* mt, uint32_t* idx, int B, int lane, uint32_t bound, int n, uint32_t* out) {
  int l = lane;
  CitMT r = lane_rng(mt, idx, B, l);
  for (int i = 0; i < n; i++) out[i] = mt_randbelow(r, bound);
  SAVE(r);
}

void cith_mt_random(uint32_t* mt, uint32_t* idx, int B, int lane, int n, double* out) {
  int l = lane;
  CitMT r = lane_rng(mt, idx, B, l);
  for (int i = 0; i < n; i++) out[i] = mt_random(r);
  SAVE(r);
}

void cith_init(CitGame* g, uint32_t* mt, uint32_t* idx, int B, const uint64_t* seeds, int preset) {
  for (int l = 0; l < B; l++) {
    CitMT r = lane_rng(mt, idx, B, l);
    if (seeds) mt_seed_cpython(r, seeds[l]);
    cit_init_game(g[l], r, preset != 0);
    SAVE(r);
  }
}

void cith_get_options(CitGame* g, uint32_t* mt, uint32_t* idx, uint64_t* seer, int B, CitOpt* out, int max_opts,
                      int* n_opts) {
  for (int l = 0; l < B; l++) {
    CitMT r = lane_rng(mt, idx, B, l);
    uint64_t* sc = seer + (long)l * CIT_SEER_MAX;
    cit_prepare_options(g[l], r, sc);
    ListSink s(out + (long)l * max_opts, max_opts);
    cit_enum_options(g[l], s, sc);
    g[l].err |= s.err;
    n_opts[l] = s.n;
    SAVE(r);
  }
}

void cith_carry_out(CitGame* g, uint32_t* mt, uint32_t* idx, int B, const CitOpt* chosen, int* winner) {
  for (int l = 0; l < B; l++) {
    CitMT r = lane_rng(mt, idx, B, l);
    winner[l] = cit_carry_out(g[l], chosen[l], r);
    SAVE(r);
  }
}

void cith_rollout(CitGame* g, uint32_t* mt, uint32_t* idx, uint64_t* seer, int B, int max_steps, int* steps,
                  int* winner) {
  for (int l = 0; l < B; l++) {
    CitMT r = lane_rng(mt, idx, B, l);
    int s = 0;
    int cap = max_steps < 0 ? CIT_ROLLOUT_CAP : max_steps;
    while (!g[l].terminal && !g[l].err && s < cap) {
      cit_random_step(g[l], r, seer + (long)l * CIT_SEER_MAX);
      s++;
    }
    steps[l] = s;
    winner[l] = g[l].winner;
    SAVE(r);
  }
}

// config-3 position harness: k = random.randint(lo, hi) random-policy steps
// from the lane's own stream (stops at a winner)
void cith_advance_random(CitGame* g, uint32_t* mt, uint32_t* idx, uint64_t* seer, int B, int lo, int hi, int* steps) {
  for (int l = 0; l < B; l++) {
    CitMT r = lane_rng(mt, idx, B, l);
    int k = lo + (int)mt_randbelow(r, (uint32_t)(hi - lo + 1));
    int s = 0;
    while (s < k && !g[l].terminal && !g[l].err) {
      cit_random_step(g[l], r, seer + (long)l * CIT_SEER_MAX);
      s++;
    }
    steps[l] = s;
    SAVE(r);
  }
}

int64_t cith_cfr_pool_bytes(int node_cap, int edge_cap) { return cfr_pool_bytes(node_cap, edge_cap); }
int64_t cith_cfr_arena_bytes(int node_blocks, int edge_blocks) { return cfr_arena_bytes(node_blocks, edge_blocks); }
int64_t cith_cfr_arena_bytes_rows(int node_blocks, int edge_blocks, int row_cap) {
  return cfr_row_cap_ok(row_cap) ? cfr_arena_bytes(node_blocks, edge_blocks, row_cap) : -1;
}
void cith_cfr_arena_reset_fmt(uint8_t* pool, int B, int node_cap, int edge_cap, int node_blocks, int edge_blocks,
                              int row_cap, int pred) {
  int64_t tb = cfr_pool_bytes(node_cap, edge_cap) * (int64_t)B;
  memset(pool, 0xff, (size_t)tb);
  CfrArena* a = reinterpret_cast<CfrArena*>(pool + tb);
  memset(a, 0, sizeof(CfrArena));
  a->n_cap = (uint32_t)node_blocks;
  a->e_cap = (uint32_t)edge_blocks;
  a->row_cap = (uint32_t)row_cap;
  a->pred = pred != 0;
}
void cith_cfr_arena_reset_rows(uint8_t* pool, int B, int node_cap, int edge_cap, int node_blocks, int edge_blocks,
                               int row_cap) {
  cith_cfr_arena_reset_fmt(pool, B, node_cap, edge_cap, node_blocks, edge_blocks, row_cap, 1);
}
int64_t cith_cfr_arena_bytes_fmt(int node_blocks, int edge_blocks, int row_cap, int pred) {
  return cfr_row_cap_ok(row_cap) ? cfr_arena_bytes(node_blocks, edge_blocks, row_cap, pred != 0) : -1;
}
void cith_cfr_arena_reset(uint8_t* pool, int B, int node_cap, int edge_cap, int node_blocks, int edge_blocks) {
  cith_cfr_arena_reset_rows(pool, B, node_cap, edge_cap, node_blocks, edge_blocks, 0);
}

void cith_count_options(CitGame* g, uint32_t* mt, uint32_t* idx, uint64_t* seer, int B, int* n_opts) {
  for (int l = 0; l < B; l++) {
    CitMT r = lane_rng(mt, idx, B, l);
    uint64_t* sc = seer + (long)l * CIT_SEER_MAX;
    cit_prepare_options(g[l], r, sc);
    uint32_t e = 0;
    n_opts[l] = cit_count_options(g[l], e, sc);
    g[l].err |= e;
    SAVE(r);
  }
}

void cith_determinize(CitGame* g, uint32_t* mt, uint32_t* idx, int B, const int* orig, int role_sample) {
  uint8_t unk[CIT_SAMPLE_SCRATCH];
  for (int l = 0; l < B; l++) {
    CitMT r = lane_rng(mt, idx, B, l);
    cit_sample_private(g[l], orig[l], role_sample != 0, r, unk);
    SAVE(r);
  }
}

void cith_skip_false_choice(CitGame* g, uint32_t* mt, uint32_t* idx, uint64_t* seer, int B, int* carried) {
  for (int l = 0; l < B; l++) {
    CitMT r = lane_rng(mt, idx, B, l);
    carried[l] = cit_skip_false_choice(g[l], r, seer + (long)l * CIT_SEER_MAX);
    SAVE(r);
  }
}

int cith_cfr_sizes(int* out) {
  out[0] = (int)sizeof(CfrNode);
  out[1] = (int)sizeof(CfrEdge);
  out[2] = CFR_OPT_CAP;
  out[3] = CFR_NB;
  out[4] = CFR_EB;
  return 5;
}

// run_mccfr(game, max_iterations=iters) without a model for every lane; pool
// = B per-tree block tables + the arena (cit_cfr.h), header reset by the caller.
// stats[l] = {root, n_nodes, n_edges, carry_outs, err}
void cith_cfr_decide(CitGame* g, uint32_t* mt, uint32_t* idx, uint32_t* npmt, uint32_t* npidx, uint64_t* seer, int B,
                     int iters, int flags, uint8_t* pool, int node_cap, int edge_cap, CitOpt* optbuf, CitOpt* chosen, int* stats) {
  CitGame* w0 = (CitGame*)aligned_alloc(16, CIT_GAME_BYTES);
  CitGame* w1 = (CitGame*)aligned_alloc(16, CIT_GAME_BYTES);
  uint8_t tmp[CIT_SAMPLE_SCRATCH];
  CitOpt lbuf[CFR_LBUF];
  for (int l = 0; l < B; l++) {
    CfrTree T;
    cfr_tree_bind(T, pool, B, l, node_cap, edge_cap);
    T.n_eblk = 0;
    T.n_nodes = T.n_edges = 0;
    T.orig = g[l].gs_pid;
    T.training = false;
    T.py = lane_rng(mt, idx, B, l);
    T.np = lane_rng(npmt, npidx, B, l);
    T.seer = seer + (long)l * CIT_SEER_MAX;
    T.optbuf = optbuf + (long)l * CFR_OPT_CAP;
    T.w0 = w0;
    T.w1 = w1;
    T.tmp = tmp;
    T.lbuf = lbuf;
    T.err = 0;
    T.carry_outs = 0;
    memcpy(w0, &g[l], CIT_GAME_BYTES);
    int root = cfr_train(T, iters, (flags & 1) != 0);
    CitOpt c = mk(O_NUM_NAMES, 0);
    if (root >= 0 && !T.err) c = cfr_live_choice(T, root);
    chosen[l] = c;
    if (root >= 0) row_load(T, reinterpret_cast<uint32_t*>(&g[l]), root);
    idx[l] = T.py.pos;
    npidx[l] = T.np.pos;
    stats[5 * l + 0] = root;
    stats[5 * l + 1] = T.n_nodes;
    stats[5 * l + 2] = T.n_edges;
    stats[5 * l + 3] = (int)T.carry_outs;
    stats[5 * l + 4] = (int)T.err;
  }
  free(w0);
  free(w1);
}

// cit_cfr_train_slice with an iteration budget per slice (slice_iters, 0 =
// none) instead of the wall clock; st = B CfrState (zero before the first
// call).  Returns the number of trees still running.
int cith_cfr_train_slice(CitGame* g, uint32_t* mt, uint32_t* idx, uint32_t* npmt, uint32_t* npidx, uint64_t* seer,
                         int B, int iters, int flags, uint8_t* pool, int node_cap, int edge_cap, CitOpt* optbuf,
                         CfrState* st, int slice_iters, CitOpt* chosen, int* stats) {
  CitGame* w0 = (CitGame*)aligned_alloc(16, CIT_GAME_BYTES);
  CitGame* w1 = (CitGame*)aligned_alloc(16, CIT_GAME_BYTES);
  uint8_t tmp[CIT_SAMPLE_SCRATCH];
  CitOpt lbuf[CFR_LBUF];
  int running = 0;
  for (int l = 0; l < B; l++) {
    CfrState& S = st[l];
    if (S.phase == CP_DONE) continue;
    CfrTree T;
    cfr_tree_bind(T, pool, B, l, node_cap, edge_cap);
    T.n_eblk = 0;
    T.training = false;
    T.py = lane_rng(mt, idx, B, l);
    T.np = lane_rng(npmt, npidx, B, l);
    T.seer = seer + (long)l * CIT_SEER_MAX;
    T.optbuf = optbuf + (long)l * CFR_OPT_CAP;
    T.w0 = w0;
    T.w1 = w1;
    T.tmp = tmp;
    T.lbuf = lbuf;
    if (S.phase == CP_INIT) {
      T.n_nodes = T.n_edges = 0;
      T.err = 0;
      T.carry_outs = 0;
      memcpy(w0, &g[l], CIT_GAME_BYTES);
      T.orig = S.orig = g[l].gs_pid;
    } else {
      cfr_state_load(T, S);
    }
    CfrBudget bud = {0, 0, slice_iters};
    int r = cfr_train_slice(T, S, iters, (flags & 1) != 0, bud);
    cfr_state_save(T, S);
    idx[l] = T.py.pos;
    npidx[l] = T.np.pos;
    if (r) {
      running++;
      continue;
    }
    int root = S.root;
    CitOpt c = mk(O_NUM_NAMES, 0);
    if (root >= 0 && !T.err) c = cfr_live_choice(T, root);
    chosen[l] = c;
    if (root >= 0) row_load(T, reinterpret_cast<uint32_t*>(&g[l]), root);
    idx[l] = T.py.pos;
    npidx[l] = T.np.pos;
    stats[5 * l + 0] = root;
    stats[5 * l + 1] = T.n_nodes;
    stats[5 * l + 2] = T.n_edges;
    stats[5 * l + 3] = (int)T.carry_outs;
    stats[5 * l + 4] = (int)T.err;
  }
  free(w0);
  free(w1);
  return running;
}

// cit_cfr_arena_release: the blocks of trees lanes[0..n) back to the rings.
void cith_cfr_arena_release(uint8_t* pool, int B, int node_cap, int edge_cap, const int* lanes, int n) {
  int64_t per = cfr_pool_bytes(node_cap, edge_cap);
  CfrArena* a = reinterpret_cast<CfrArena*>(pool + per * (int64_t)B);
  uint32_t* ring = reinterpret_cast<uint32_t*>(a + 1);
  if (a->n_head > a->n_tail) a->n_head = a->n_tail;
  if (a->e_head > a->e_tail) a->e_head = a->e_tail;
  int nb = cfr_nblocks(node_cap), eb = cfr_eblocks(edge_cap);
  for (int k = 0; k < n; k++) {
    int32_t* t = reinterpret_cast<int32_t*>(pool + per * (int64_t)lanes[k]);
    for (int i = 0; i < nb + eb; i++) {
      if (t[i] < 0) continue;
      if (i < nb) ring[a->n_tail++ % a->n_cap] = (uint32_t)t[i];
      else ring[a->n_cap + a->e_tail++ % a->e_cap] = (uint32_t)t[i];
      t[i] = -1;
    }
  }
}

void cith_encode_games(const CitGame* g, int B, int pid, float* out) {
  for (int l = 0; l < B; l++) cit_encode_game(g[l], out + (long)l * CIT_FEAT, pid);
}
void cith_encode_options(const CitGame* g, const CitOpt* opts, int n, float* out) {
  for (int i = 0; i < n; i++) cit_encode_option(opts[i], *g, out + (long)i * CIT_OPT_FEAT);
}

// One resumption of cfr_pred for every lane (see cfr_pred_run); returns the
// number of lanes now waiting for an evaluation (features in feat[l]).
int cith_cfr_pred_step(CitGame* g, uint32_t* mt, uint32_t* idx, uint32_t* npmt, uint32_t* npidx, uint64_t* seer,
                       int B, int iters, int max_depth, uint8_t* pool, int node_cap, int edge_cap, CitOpt* optbuf,
                       CfrState* st, const float* probs, float* feat, CitOpt* chosen) {
  CitGame* w0 = (CitGame*)aligned_alloc(16, CIT_GAME_BYTES);
  CitGame* w1 = (CitGame*)aligned_alloc(16, CIT_GAME_BYTES);
  uint8_t tmp[CIT_SAMPLE_SCRATCH];
  CitOpt lbuf[CFR_LBUF];
  int waiting = 0;
  for (int l = 0; l < B; l++) {
    CfrState& S = st[l];
    if (S.phase == CP_DONE) continue;
    CfrTree T;
    cfr_tree_bind(T, pool, B, l, node_cap, edge_cap);
    T.n_eblk = 0;
    T.training = false;
    T.py = lane_rng(mt, idx, B, l);
    T.np = lane_rng(npmt, npidx, B, l);
    T.seer = seer + (long)l * CIT_SEER_MAX;
    T.optbuf = optbuf + (long)l * CFR_OPT_CAP;
    T.w0 = w0;
    T.w1 = w1;
    T.tmp = tmp;
    T.lbuf = lbuf;
    if (S.phase == CP_INIT) {
      T.n_nodes = T.n_edges = 0;
      T.err = 0;
      T.carry_outs = 0;
      T.orig = g[l].gs_pid;
      memcpy(w0, &g[l], CIT_GAME_BYTES);
    } else {
      cfr_state_load(T, S);
    }
    CitOpt c;
    int r = cfr_pred_run(T, S, iters, max_depth, probs + 6L * l, feat + (long)CIT_FEAT * l, c);
    cfr_state_save(T, S);
    waiting += r;
    if (!r) {
      chosen[l] = c;
      if (S.root >= 0) row_load(T, reinterpret_cast<uint32_t*>(&g[l]), S.root);
    }
    idx[l] = T.py.pos;
    npidx[l] = T.np.pos;
  }
  free(w0);
  free(w1);
  return waiting;
}

void cith_advance_policy(CitGame* g, uint32_t* mt, uint32_t* idx, uint64_t* seer, int B, int search_mask,
                         int max_steps, int* status, int* steps) {
  for (int l = 0; l < B; l++) {
    CitMT r = lane_rng(mt, idx, B, l);
    status[l] = cit_advance_policy(g[l], r, seer + (long)l * CIT_SEER_MAX, search_mask,
                                   max_steps < 0 ? CIT_ROLLOUT_CAP : max_steps, steps[l]);
    SAVE(r);
  }
}

void cith_random_position(CitGame* g, uint32_t* mt, uint32_t* idx, uint64_t* seer, int B, int max_move,
                          uint32_t* ring, int* steps) {
  for (int l = 0; l < B; l++) {
    CitMT r = lane_rng(mt, idx, B, l);
    steps[l] = cit_random_position(g[l], r, seer + (long)l * CIT_SEER_MAX, ring, max_move);
    SAVE(r);
  }
}

void cith_close_position(CitGame* g, uint32_t* mt, uint32_t* idx, uint64_t* seer, int B, uint32_t* store,
                         int* index) {
  for (int l = 0; l < B; l++) {
    CitMT r = lane_rng(mt, idx, B, l);
    index[l] = cit_close_position(g[l], r, seer + (long)l * CIT_SEER_MAX, store);
    SAVE(r);
  }
}

void cith_cfr_target_count(uint8_t* pool, int B, int node_cap, int edge_cap, const int* roots, int mode, int* counts) {
  for (int l = 0; l < B; l++) {
    CfrTree T = cfr_tree_view(pool, B, l, node_cap, edge_cap);
    cfr_count_targets(T, roots[l], mode, counts[2 * l], counts[2 * l + 1]);
  }
}

void cith_cfr_targets(uint8_t* pool, int B, int node_cap, int edge_cap, const int* roots, int mode, uint32_t* mt,
                      uint32_t* idx, const int* offsets, int* meta, float* feat, double* value, double* dist, float* opt_feat) {
  for (int l = 0; l < B; l++) {
    CfrTree T = cfr_tree_view(pool, B, l, node_cap, edge_cap);
    CitMT r = lane_rng(mt, idx, B, l);
    cfr_emit_targets(T, r, roots[l], mode, l, offsets[2 * l], offsets[2 * l + 1], meta, feat, value, dist, opt_feat);
    SAVE(r);
  }
}

// CPU baseline: `threads` host threads each play preset /
// random-role games seeded seed0, seed0+1, ... (an atomic counter hands out
// seeds) with the uniform random policy to terminal -- the step loop of
// compare_to_random.py:37-39 / run_utils.py:37-41 -- until `seconds` have
// elapsed.  Returns the finished games, their carry_out transitions and the
// wall time (the last game of each thread runs to its end).
int cith_rollout_timed(int preset, uint64_t seed0, double seconds, int threads, long long* out_games,
                       long long* out_steps, double* out_wall) {
  if (threads <= 0 || seconds < 0) return -1;
  std::atomic<uint64_t> next(seed0);
  std::atomic<long long> games(0), steps(0), errs(0);
  auto t0 = std::chrono::steady_clock::now();
  auto deadline = t0 + std::chrono::duration<double>(seconds);
  auto work = [&]() {
    CitGame* g = (CitGame*)aligned_alloc(16, CIT_GAME_BYTES);
    std::vector<uint32_t> mt(CIT_MT_N);
    std::vector<uint64_t> seer(CIT_SEER_MAX);
    long long my_games = 0, my_steps = 0, my_errs = 0;
    while (std::chrono::steady_clock::now() < deadline) {
      uint64_t seed = next.fetch_add(1);
      CitMT r;
      r.mt = mt.data();
      r.stride = 1;
      r.pos = 0;
      r.coop = 0;
      mt_seed_cpython(r, seed);
      cit_init_game(*g, r, preset != 0);
      int s = 0;
      while (!g->terminal && !g->err && s < CIT_ROLLOUT_CAP) {
        cit_random_step(*g, r, seer.data());
        s++;
      }
      my_games++;
      my_steps += s;
      my_errs += g->err != 0;
    }
    games += my_games;
    steps += my_steps;
    errs += my_errs;
    free(g);
  };
  std::vector<std::thread> pool;
  for (int i = 1; i < threads; i++) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  *out_wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  *out_games = games;
  *out_steps = steps;
  return (int)errs.load();
}

// The value net's forward for one feature row on the host (ValueOnlyNN,
// algorithms/models.py:17-24, eval mode, BatchNorm folded as models.fold
// does: w = [w1t, b1, w2t, b2, w3t, b3, w4t, b4], [in][out] fp32) followed by
// square_and_normalize (train_utils.py:143-145).  Timing only: no bitwise
// claim against the MFMA kernel (the fmaf-chain oracle makes that one).
static void host_value_net(const float* const* w, const float* x, float* probs) {
  static const int dims[5] = {CIT_FEAT, 512, 256, 128, 6};
  float a[512], b[512];
  const float* in = x;
  float* bufs[2] = {a, b};
  for (int layer = 0; layer < 4; layer++) {
    int ni = dims[layer], no = dims[layer + 1];
    const float* wt = w[2 * layer];
    const float* bias = w[2 * layer + 1];
    float* out = layer == 3 ? probs : bufs[layer & 1];
    for (int o = 0; o < no; o++) out[o] = bias[o];
    for (int i = 0; i < ni; i++) {
      float v = in[i];
      if (v == 0.0f) continue;
      const float* row = wt + (long)i * no;
      for (int o = 0; o < no; o++) out[o] += v * row[o];
    }
    if (layer < 3)
      for (int o = 0; o < no; o++) out[o] = out[o] > 0.0f ? out[o] : 0.0f;
    in = out;
  }
  float s = 0.0f;
  for (int o = 0; o < 6; o++) s += probs[o] * probs[o];
  for (int o = 0; o < 6; o++) probs[o] = probs[o] * probs[o] / s;
}

// CPU baseline of the MCCFR workloads (BASELINE.json configs 3-5, bench.py's
// cfr legs): `threads` host threads each take seeds seed0, seed0+1, ... (an
// atomic counter) and run one reference decision per seed until `seconds`
// have elapsed, with the engine headers built for the host:
//   config 3: random.seed(s); create_game(); randint(0, 300) random steps;
//             np.random.seed(s); run_mccfr(game, None, iters)  (cfr_train)
//   config 4: the same position, run_mccfr(game, model, iters): cfr_pred(iters,
//             depth 10) with host_value_net leaves (weights w, models.fold)
//   config 5: random.seed(s); create_a_random_game(100); np.random.seed(s);
//             run_mccfr(iters, training=True) + get_all_targets(200)
// Each thread owns one tree pool of (node_cap, edge_cap).  Out: decisions
// (trees), carry_outs inside the searches, error lanes, wall time.
int cith_cfr_timed(int config, int iters, uint64_t seed0, double seconds, int threads, int node_cap, int edge_cap,
                   const float* const* w, long long* out_decisions, long long* out_carry, long long* out_errs,
                   double* out_wall) {
  if (threads <= 0 || seconds < 0 || config < 3 || config > 5 || (config == 4 && !w)) return -1;
  std::atomic<uint64_t> next(seed0);
  std::atomic<long long> decisions(0), carry(0), errs(0);
  auto t0 = std::chrono::steady_clock::now();
  auto deadline = t0 + std::chrono::duration<double>(seconds);
  const int nb = cfr_nblocks(node_cap), eb = cfr_eblocks(edge_cap);
  const int64_t pool_bytes = cfr_pool_bytes(node_cap, edge_cap) + cfr_arena_bytes(nb, eb);
  auto work = [&]() {
    CitGame* g = (CitGame*)aligned_alloc(16, CIT_GAME_BYTES);
    uint8_t* pool = (uint8_t*)malloc((size_t)pool_bytes);
    std::vector<uint32_t> mt(CIT_MT_N), npmt(CIT_MT_N);
    std::vector<uint64_t> seer(CIT_SEER_MAX);
    std::vector<CitOpt> optbuf(CFR_OPT_CAP);
    std::vector<uint32_t> ring(config == 5 ? 100 * (CIT_GAME_BYTES / 4) : 1);
    float feat[CIT_FEAT], probs[6] = {};
    long long my_dec = 0, my_carry = 0, my_errs = 0;
    while (pool && std::chrono::steady_clock::now() < deadline) {
      uint64_t seed = next.fetch_add(1);
      uint32_t idx = 0, npidx = 0;
      CitMT r;
      r.mt = mt.data();
      r.stride = 1;
      r.pos = 0;
      r.coop = 0;
      mt_seed_cpython(r, seed);
      int pos_ok;
      if (config == 5) {
        pos_ok = cit_random_position(*g, r, seer.data(), ring.data(), 100) >= 0;
      } else {
        cit_init_game(*g, r, true);
        int k = (int)mt_randbelow(r, 301u), s = 0;
        while (s < k && !g->terminal && !g->err) {
          cit_random_step(*g, r, seer.data());
          s++;
        }
        pos_ok = !g->err;
      }
      idx = r.pos;
      CitMT q;
      q.mt = npmt.data();
      q.stride = 1;
      q.pos = 0;
      q.coop = 0;
      mt_init_genrand(q, (uint32_t)seed);
      npidx = q.pos;
      cith_cfr_arena_reset(pool, 1, node_cap, edge_cap, nb, eb);
      int st[5] = {-1, 0, 0, 0, 1};
      CitOpt chosen;
      if (pos_ok && config == 4) {
        CfrState S;
        memset(&S, 0, sizeof(S));
        while (cith_cfr_pred_step(g, mt.data(), &idx, npmt.data(), &npidx, seer.data(), 1, iters, 10, pool, node_cap,
                                  edge_cap, optbuf.data(), &S, probs, feat, &chosen))
          host_value_net(w, feat, probs);
        st[3] = S.carry_outs;
        st[4] = S.err;
      } else if (pos_ok) {
        cith_cfr_decide(g, mt.data(), &idx, npmt.data(), &npidx, seer.data(), 1, iters, 0, pool, node_cap, edge_cap,
                        optbuf.data(), &chosen, st);
        if (config == 5 && st[0] >= 0 && !st[4]) {
          int counts[2] = {0, 0}, offs[2] = {0, 0};
          cith_cfr_target_count(pool, 1, node_cap, edge_cap, &st[0], CFR_TGT_TREE | CFR_TGT_PRUNE, counts);
          std::vector<int> meta(5 * (size_t)counts[0] + 5);
          std::vector<float> tf((size_t)CIT_FEAT * counts[0] + 1), of((size_t)CIT_OPT_FEAT * counts[1] + 1);
          std::vector<double> tv(6 * (size_t)counts[0] + 1), td((size_t)counts[1] + 1);
          cith_cfr_targets(pool, 1, node_cap, edge_cap, &st[0], CFR_TGT_TREE | CFR_TGT_PRUNE, mt.data(), &idx, offs,
                           meta.data(), tf.data(), tv.data(), td.data(), of.data());
        }
      }
      my_dec++;
      my_carry += st[3];
      my_errs += (!pos_ok || st[4] != 0);
    }
    decisions += my_dec;
    carry += my_carry;
    errs += my_errs;
    free(pool);
    free(g);
  };
  std::vector<std::thread> pool;
  for (int i = 1; i < threads; i++) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  *out_wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  *out_decisions = decisions;
  *out_carry = carry;
  *out_errs = errs;
  return 0;
}

}  // extern "C"
