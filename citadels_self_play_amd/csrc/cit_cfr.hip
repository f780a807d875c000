// MCCFR kernel + C ABI (include/citadels.h, "MCCFR" section): one tree per
// 64-lane workgroup; see cit_cfr.h for the search itself.
// Every MT19937 stream of this unit is an LDS stream run by the whole team.
#define CIT_MT_COOP_ONLY 1
#include <hip/hip_runtime.h>

#include <mutex>
#include <unordered_map>

#include "../../include/citadels.h"
#include "cit_cfr.h"

#define ROW_W (CIT_GAME_BYTES / 4)

#ifdef CFR_TREE_CLOCK
// Per-tree start / end wall clock (100 MHz) of k_cfr_decide (measurement
// builds only: tools/cfr_tree_clock.py).
__device__ unsigned long long g_tree_clock[2 * 65536];
#endif

namespace {

// The tree's two streams (CPython `random`, numpy `np.random`) live in LDS for
// the whole launch: every draw of the search is an LDS access instead of a
// strided HBM one, and a twist is done by the 64 lanes together.
__device__ __forceinline__ CitMT mt_stage_in(uint32_t* dst, const uint32_t* mt, const uint32_t* idx, int B, long l) {
  for (int i = threadIdx.x; i < CIT_MT_N; i += blockDim.x) dst[i] = mt[(long)i * B + l];
  __syncthreads();
  CitMT r;
  r.mt = dst;
  r.stride = 1;
  r.pos = idx[l];
  r.coop = 1;     // the team runs the search in lockstep: lane-parallel twist
  r.win = 0;
  r.win_base = -1;
  return r;
}
__device__ __forceinline__ void mt_stage_out(const uint32_t* src, uint32_t* mt, int B, long l) {
  __syncthreads();
  for (int i = threadIdx.x; i < CIT_MT_N; i += blockDim.x) mt[(long)i * B + l] = src[i];
}

// The tree's LDS block (cit_cfr.h, cfr_ls): pool binding (block tables in LDS),
// streams, working rows.  False when the pool stores diff rows but the launch
// reserved no dynamic LDS for the base row (base_off < 0: the library's record
// of the pool's row format disagrees with the arena header); the kernel then
// stops the tree with CIT_ERR_UNSUPPORTED instead of addressing cfr_dyn[-1].
__device__ __forceinline__ bool tree_setup(uint32_t* mt, uint32_t* idx, uint32_t* npmt, uint32_t* npidx,
                                           uint64_t* seer, int B, long l, uint8_t* pool, int node_cap, int edge_cap,
                                           CitOpt* optbuf, int flags, int base_off) {
  CfrTree& T = cfr_ls.T;
  cfr_ls.cnode = -1;
  cfr_ls.base_off = base_off;
  cfr_ls.sbuf_on = (flags & CIT_CFR_STRATEGY_HBM) ? 0 : 1;
  cfr_tree_bind(T, pool, B, l, node_cap, edge_cap);
  T.nbt = nullptr;          // the tables live in dynamic LDS (cfr_nbt_at / cfr_ebt_at)
  T.ebt = nullptr;
  T.n_eblk = 0;
  T.training = false;
  T.py = mt_stage_in(cfr_ls.py, mt, idx, B, l);
  T.np = mt_stage_in(cfr_ls.np, npmt, npidx, B, l);
  T.seer = seer + l * CIT_SEER_MAX;
  T.optbuf = optbuf + l * CFR_OPT_CAP;
  T.w0 = reinterpret_cast<CitGame*>(cfr_ls.w[0]);
  T.w1 = reinterpret_cast<CitGame*>(cfr_ls.w[1]);
  T.tmp = cfr_ls.tmp;
  T.lbuf = cfr_ls.lbuf;
  return !(T.row_cap != 0 && base_off < 0);
}

// The block tables (and, for diff row slots, the base row) of a resumed tree
// from its pool into dynamic LDS (n node / e edge blocks), and the tables back.
__device__ __forceinline__ void tables_load(const CfrTree& T, int n_nodes, int n_edges) {
  int nb = (n_nodes + CFR_NB - 1) >> CFR_NB_SHIFT, eb = (n_edges + CFR_EB - 1) >> CFR_EB_SHIFT;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) cfr_nbt_at(T, i) = T.nbt_hbm[i];
  for (int i = threadIdx.x; i < eb; i += blockDim.x) cfr_ebt_at(T, i) = T.ebt_hbm[i];
  if (T.row_cap)
    for (int i = threadIdx.x; i < CFR_ROW_W; i += blockDim.x) cfr_base_w(T)[i] = T.base_hbm[i];
  __syncthreads();
}
__device__ __forceinline__ void tables_store(const CfrTree& T) {
  __syncthreads();
  int nb = (T.n_nodes + CFR_NB - 1) >> CFR_NB_SHIFT;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) T.nbt_hbm[i] = cfr_nbt_at(T, i);
  for (int i = threadIdx.x; i < T.n_eblk; i += blockDim.x) T.ebt_hbm[i] = cfr_ebt_at(T, i);
}

// CFR_WAVES_PER_EU (compile-time) bounds the search kernels' VGPRs so that
// many trees share a SIMD (the search is latency-bound, one tree per wave);
// 0 leaves the register budget to the compiler.  3 (<= 168 VGPRs, no
// spills) with the 13 KB LDS block = 12 trees per CU instead of 7: config 4
// 98.4 k -> 102.2 k decisions/s, config 3 unchanged (profiles/r03/occupancy/).
#ifndef CFR_WAVES_PER_EU
#define CFR_WAVES_PER_EU 3
#endif
#if CFR_WAVES_PER_EU
#define CFR_OCC __attribute__((amdgpu_waves_per_eu(CFR_WAVES_PER_EU)))
#else
#define CFR_OCC
#endif

// One MCCFR decision per workgroup: a 64-lane team runs the search on its
// tree (node pool in HBM, working state in LDS).
__global__ __launch_bounds__(64) CFR_OCC void k_cfr_decide(uint32_t* games, uint32_t* mt, uint32_t* idx, uint32_t* npmt,
                                                   uint32_t* npidx, uint64_t* seer, int B, int iters, int flags,
                                                   const int32_t* orig, uint8_t* pool,
                                                   int node_cap, int edge_cap, CitOpt* optbuf, CitOpt* chosen,
                                                   int32_t* stats, int base_off) {
  long l = blockIdx.x;
  if (l >= B) return;
#ifdef CFR_TREE_CLOCK
  unsigned long long tc0 = wall_clock64();
#endif
  cfr_prof_reset();
  CfrTree& T = cfr_ls.T;
  if (!tree_setup(mt, idx, npmt, npidx, seer, B, l, pool, node_cap, edge_cap, optbuf, flags, base_off)) {
    if (threadIdx.x == 0) {
      chosen[l] = mk(O_NUM_NAMES, 0);
      stats[5 * l + 0] = -1;
      stats[5 * l + 1] = stats[5 * l + 2] = stats[5 * l + 3] = 0;
      stats[5 * l + 4] = (int)CIT_ERR_UNSUPPORTED;
    }
    return;
  }
  T.n_nodes = T.n_edges = 0;
  T.err = 0;
  T.carry_outs = 0;
  copy_row(T, cfr_ls.w[0], games + l * ROW_W);
  T.orig = orig ? orig[l] : cfr_w(T, 0).gs_pid;
  int root = cfr_train(T, iters, (flags & CIT_CFR_ROOT_SKIPPED) != 0);
  CitOpt c = mk(O_NUM_NAMES, 0);
  if (root >= 0 && !T.err) c = cfr_uopt(cfr_live_choice(T, root));
  if (root >= 0) row_load(T, games + l * ROW_W, root);
  tables_store(T);
  mt_stage_out(cfr_ls.py, mt, B, l);
  mt_stage_out(cfr_ls.np, npmt, B, l);
  if (threadIdx.x == 0) {
    chosen[l] = c;
    idx[l] = T.py.pos;
    npidx[l] = T.np.pos;
    stats[5 * l + 0] = root;
    stats[5 * l + 1] = T.n_nodes;
    stats[5 * l + 2] = T.n_edges;
    stats[5 * l + 3] = (int)T.carry_outs;
    stats[5 * l + 4] = (int)T.err;
#ifdef CFR_TREE_CLOCK
    if (l < 65536) {
      g_tree_clock[2 * l] = tc0;
      g_tree_clock[2 * l + 1] = wall_clock64();
    }
#endif
  }
  cfr_prof_flush();
}

// One resumption of cfr_pred (cit_cfr.h: cfr_pred_run) per tree; lane 0 adds
// 1 to *waiting when the tree suspends for a leaf evaluation, 1 to *running
// when `ticks` of the wall clock (0 = no limit) ran out first.
__global__ __launch_bounds__(64) CFR_OCC void k_cfr_pred_step(uint32_t* games, uint32_t* mt, uint32_t* idx, uint32_t* npmt,
                                                      uint32_t* npidx, uint64_t* seer, int B, int iters, int flags,
                                                      const int32_t* orig, int max_depth, uint8_t* pool, int node_cap, int edge_cap, CitOpt* optbuf,
                                                      CfrState* state, const float* probs, float* feat,
                                                      CitOpt* chosen, int32_t* waiting, uint64_t ticks,
                                                      int32_t* running, int base_off) {
  long l = blockIdx.x;
  if (l >= B) return;
  CfrBudget bud;
  bud.t0 = wall_clock64();
  bud.ticks = ticks;
  bud.iters_left = 0;
  CfrState& S = cfr_ls.S;
  S = state[l];             // every lane stores the same value
  if (S.phase == CP_DONE) return;
  CfrTree& T = cfr_ls.T;
  if (!tree_setup(mt, idx, npmt, npidx, seer, B, l, pool, node_cap, edge_cap, optbuf, flags, base_off)) {
    if (threadIdx.x == 0) {
      S.err |= (int)CIT_ERR_UNSUPPORTED;
      S.root = -1;
      S.phase = CP_DONE;
      state[l] = S;
      chosen[l] = mk(O_NUM_NAMES, 0);
    }
    return;
  }
  if (S.phase == CP_INIT) {
    T.n_nodes = T.n_edges = 0;
    T.err = 0;
    T.carry_outs = 0;
    copy_row(T, cfr_ls.w[0], games + l * ROW_W);
    T.orig = orig ? orig[l] : cfr_w(T, 0).gs_pid;
  } else {
    cfr_state_load(T, S);
    tables_load(T, T.n_nodes, T.n_edges);
  }
  CitOpt c;
  int r = cfr_pred_run(T, S, iters, max_depth, probs + 6 * l, feat + (long)CIT_FEAT * l, c,
                       (flags & CIT_CFR_ROOT_SKIPPED) != 0, ticks ? &bud : nullptr);
  r = cfr_u(r);
  cfr_state_save(T, S);
  if (!r && S.root >= 0) row_load(T, games + l * ROW_W, S.root);
  tables_store(T);
  mt_stage_out(cfr_ls.py, mt, B, l);
  mt_stage_out(cfr_ls.np, npmt, B, l);
  if (threadIdx.x == 0) {
    state[l] = S;
    if (!r) chosen[l] = c;
    idx[l] = T.py.pos;
    npidx[l] = T.np.pos;
    if (r == 1) atomicAdd(waiting, 1);
    if (r == 2) atomicAdd(running, 1);
  }
}

// cfr_pred + the live choice per tree in ONE launch (cit_cfr_pred_fused):
// leaves are evaluated inside the kernel (cfr_leaf_eval: the single-row MLP
// over the wave-layout weights), so no tree waits for another tree's leaf or
// for a host round; outputs as k_cfr_decide, plus the final CfrState.
__global__ __launch_bounds__(64) CFR_OCC void k_cfr_pred_fused(uint32_t* games, uint32_t* mt, uint32_t* idx, uint32_t* npmt,
                                                       uint32_t* npidx, uint64_t* seer, int B, int iters, int flags,
                                                       const int32_t* orig, int max_depth, uint8_t* pool, int node_cap,
                                                       int edge_cap, CitOpt* optbuf, const float* wave_w,
                                                       CfrState* state, CitOpt* chosen, int32_t* stats, int base_off) {
  long l = blockIdx.x;
  if (l >= B) return;
#ifdef CFR_TREE_CLOCK
  unsigned long long tc0 = wall_clock64();
#endif
  cfr_prof_reset();
  CfrState& S = cfr_ls.S;
  S = CfrState{};           // CP_INIT (every lane stores the same value)
  CfrTree& T = cfr_ls.T;
  if (!tree_setup(mt, idx, npmt, npidx, seer, B, l, pool, node_cap, edge_cap, optbuf, flags, base_off)) {
    if (threadIdx.x == 0) {
      S.err = (int)CIT_ERR_UNSUPPORTED;
      S.root = -1;
      S.phase = CP_DONE;
      if (state) state[l] = S;
      chosen[l] = mk(O_NUM_NAMES, 0);
      stats[5 * l + 0] = -1;
      stats[5 * l + 1] = stats[5 * l + 2] = stats[5 * l + 3] = 0;
      stats[5 * l + 4] = (int)CIT_ERR_UNSUPPORTED;
    }
    return;
  }
  T.n_nodes = T.n_edges = 0;
  T.err = 0;
  T.carry_outs = 0;
  copy_row(T, cfr_ls.w[0], games + l * ROW_W);
  T.orig = orig ? orig[l] : cfr_w(T, 0).gs_pid;
  CitOpt c;
  cfr_pred_run(T, S, iters, max_depth, nullptr, nullptr, c, (flags & CIT_CFR_ROOT_SKIPPED) != 0, nullptr, wave_w);
  cfr_state_save(T, S);
  int root = cfr_u(S.root);
  if (root >= 0) row_load(T, games + l * ROW_W, root);
  tables_store(T);
  mt_stage_out(cfr_ls.py, mt, B, l);
  mt_stage_out(cfr_ls.np, npmt, B, l);
  if (threadIdx.x == 0) {
    if (state) state[l] = S;
    chosen[l] = c;
    idx[l] = T.py.pos;
    npidx[l] = T.np.pos;
    stats[5 * l + 0] = root;
    stats[5 * l + 1] = T.n_nodes;
    stats[5 * l + 2] = T.n_edges;
    stats[5 * l + 3] = (int)T.carry_outs;
    stats[5 * l + 4] = (int)T.err;
#ifdef CFR_TREE_CLOCK
    if (l < 65536) {
      g_tree_clock[2 * l] = tc0;
      g_tree_clock[2 * l + 1] = wall_clock64();
    }
#endif
  }
  cfr_prof_flush();
}

// One slice of cfr_train per tree (the tree queue of simulate_games): the
// tree resumes from its CfrState and runs until `ticks` of the wall clock
// have passed (then lane 0 adds 1 to *running) or it is done (then as
// k_cfr_decide: live choice, root game back into games[l], chosen, stats).
__global__ __launch_bounds__(64) CFR_OCC void k_cfr_train_slice(uint32_t* games, uint32_t* mt, uint32_t* idx, uint32_t* npmt,
                                                        uint32_t* npidx, uint64_t* seer, int B, int iters, int flags,
                                                        const int32_t* orig, uint8_t* pool, int node_cap, int edge_cap,
                                                        CitOpt* optbuf, CfrState* state, uint64_t ticks,
                                                        CitOpt* chosen, int32_t* stats, int32_t* running,
                                                        int base_off) {
  long l = blockIdx.x;
  if (l >= B) return;
  CfrBudget bud;
  bud.t0 = wall_clock64();
  bud.ticks = ticks;
  bud.iters_left = 0;
  CfrState& S = cfr_ls.S;
  S = state[l];
  if (S.phase == CP_DONE) return;
  CfrTree& T = cfr_ls.T;
  if (!tree_setup(mt, idx, npmt, npidx, seer, B, l, pool, node_cap, edge_cap, optbuf, flags, base_off)) {
    if (threadIdx.x == 0) {
      S.err |= (int)CIT_ERR_UNSUPPORTED;
      S.root = -1;
      S.phase = CP_DONE;
      state[l] = S;
      chosen[l] = mk(O_NUM_NAMES, 0);
      stats[5 * l + 0] = -1;
      stats[5 * l + 1] = stats[5 * l + 2] = stats[5 * l + 3] = 0;
      stats[5 * l + 4] = (int)CIT_ERR_UNSUPPORTED;
    }
    return;
  }
  if (S.phase == CP_INIT) {
    T.n_nodes = T.n_edges = 0;
    T.err = 0;
    T.carry_outs = 0;
    copy_row(T, cfr_ls.w[0], games + l * ROW_W);
    T.orig = orig ? orig[l] : cfr_w(T, 0).gs_pid;
    S.orig = T.orig;
  } else {
    cfr_state_load(T, S);
    tables_load(T, T.n_nodes, T.n_edges);
  }
  int r = cfr_u(cfr_train_slice(T, S, iters, (flags & CIT_CFR_ROOT_SKIPPED) != 0, bud));
  int root = cfr_u(S.root);
  CitOpt c = mk(O_NUM_NAMES, 0);
  if (!r) {
    if (root >= 0 && !T.err) c = cfr_uopt(cfr_live_choice(T, root));
    if (root >= 0) row_load(T, games + l * ROW_W, root);
  }
  cfr_state_save(T, S);
  tables_store(T);
  mt_stage_out(cfr_ls.py, mt, B, l);
  mt_stage_out(cfr_ls.np, npmt, B, l);
  if (threadIdx.x == 0) {
    state[l] = S;
    idx[l] = T.py.pos;
    npidx[l] = T.np.pos;
    if (r) {
      atomicAdd(running, 1);
    } else {
      chosen[l] = c;
      stats[5 * l + 0] = root;
      stats[5 * l + 1] = T.n_nodes;
      stats[5 * l + 2] = T.n_edges;
      stats[5 * l + 3] = (int)T.carry_outs;
      stats[5 * l + 4] = (int)T.err;
    }
  }
}

// Releasing trees' blocks (between launches): first pull each ring's head
// back to its tail (takes past an empty ring overshoot it), then one
// workgroup per released tree appends its blocks to the rings and clears its
// tables.
__global__ void k_arena_clamp(CfrArena* a) {
  if (threadIdx.x == 0) {
    if (a->n_head > a->n_tail) a->n_head = a->n_tail;
    if (a->e_head > a->e_tail) a->e_head = a->e_tail;
  }
}
__global__ void k_arena_release(int32_t* tables, long per_words, int nb, int eb, CfrArena* a, const int32_t* lanes) {
  int32_t* t = tables + (long)lanes[blockIdx.x] * per_words;
  uint32_t* ring = reinterpret_cast<uint32_t*>(a + 1);
  for (int i = threadIdx.x; i < nb + eb; i += blockDim.x) {
    int b = t[i];
    if (b < 0) continue;
    if (i < nb) {
      uint32_t pos = atomicAdd(&a->n_tail, 1u);
      ring[pos % a->n_cap] = (uint32_t)b;
    } else {
      uint32_t pos = atomicAdd(&a->e_tail, 1u);
      ring[a->n_cap + pos % a->e_cap] = (uint32_t)b;
    }
    t[i] = -1;
  }
}

// A pool before its trees start: every block-table entry -1, the arena
// header with no blocks handed out and the given capacities.
// Only the tables of each tree's region are set (its base / scratch rows are
// written before they are read).
__global__ void k_arena_reset(int32_t* pool, long per_words, long tbl_words, int B, CfrArena* a, uint32_t n_cap,
                              uint32_t e_cap, uint32_t row_cap, uint32_t pred) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < tbl_words * B) pool[(i / tbl_words) * per_words + i % tbl_words] = -1;
  if (blockIdx.x == 0 && threadIdx.x < sizeof(CfrArena) / 4)
    reinterpret_cast<uint32_t*>(a)[threadIdx.x] = threadIdx.x == 1 ? n_cap : threadIdx.x == 3 ? e_cap
                                                 : threadIdx.x == 8 ? row_cap : threadIdx.x == 9 ? pred : 0u;
}

// Row slot format of each pool this library reset (cit_cfr_arena_reset_rows),
// so a search launch reserves dynamic LDS for the base row only when the pool
// stores diff rows; a pool not reset here gets the room (diff rows or not).
std::mutex g_pool_rows_mu;
std::unordered_map<const void*, int> g_pool_rows;
void pool_rows_set(const void* pool, int row_cap) {
  std::lock_guard<std::mutex> lk(g_pool_rows_mu);
  g_pool_rows[pool] = row_cap;
}
struct DynLds {
  size_t bytes;
  int base_off;     // dwords from cfr_dyn to the base row; -1: no room (raw rows)
};
DynLds dyn_lds(const void* pool, int node_cap, int edge_cap) {
  bool base = true;
  {
    std::lock_guard<std::mutex> lk(g_pool_rows_mu);
    auto it = g_pool_rows.find(pool);
    if (it != g_pool_rows.end()) base = it->second != 0;
  }
  return {(size_t)cfr_dyn_lds_bytes(node_cap, edge_cap, base),
          base ? (int)cfr_dyn_base_off(node_cap, edge_cap) : -1};
}

}  // namespace

#define CHECK_LAUNCH()                       \
  do {                                       \
    hipError_t _e = hipGetLastError();       \
    return _e == hipSuccess ? 0 : (int)_e;   \
  } while (0)

extern "C" {

int cit_cfr_arena_reset_fmt(void* pool, int B, int node_cap, int edge_cap, int node_blocks, int edge_blocks,
                            int row_cap, int pred, hipStream_t stream);

int64_t cit_cfr_pool_bytes(int node_cap, int edge_cap) {
  if (node_cap <= 0 || edge_cap <= 0 || cfr_nblocks(node_cap) > CFR_TBL_MAX || cfr_eblocks(edge_cap) > CFR_TBL_MAX)
    return -1;
  return cfr_pool_bytes(node_cap, edge_cap);
}
int64_t cit_cfr_arena_bytes(int node_blocks, int edge_blocks) {
  if (node_blocks < 0 || edge_blocks < 0) return -1;
  return cfr_arena_bytes(node_blocks, edge_blocks);
}
int64_t cit_cfr_arena_bytes_rows(int node_blocks, int edge_blocks, int row_cap) {
  if (node_blocks < 0 || edge_blocks < 0 || !cfr_row_cap_ok(row_cap)) return -1;
  return cfr_arena_bytes(node_blocks, edge_blocks, row_cap);
}
int64_t cit_cfr_arena_bytes_fmt(int node_blocks, int edge_blocks, int row_cap, int pred) {
  if (node_blocks < 0 || edge_blocks < 0 || !cfr_row_cap_ok(row_cap)) return -1;
  return cfr_arena_bytes(node_blocks, edge_blocks, row_cap, pred != 0);
}
int cit_cfr_block_sizes(int32_t* out) {
  if (!out) return -1;
  out[0] = CFR_NB;
  out[1] = CFR_EB;
  out[2] = CFR_TBL_MAX;
  return 0;
}
int cit_cfr_arena_reset_rows(void* pool, int B, int node_cap, int edge_cap, int node_blocks, int edge_blocks,
                             int row_cap, hipStream_t stream) {
  return cit_cfr_arena_reset_fmt(pool, B, node_cap, edge_cap, node_blocks, edge_blocks, row_cap, 1, stream);
}
int cit_cfr_arena_reset_fmt(void* pool, int B, int node_cap, int edge_cap, int node_blocks, int edge_blocks,
                            int row_cap, int pred, hipStream_t stream) {
  if (!pool || B <= 0 || cit_cfr_pool_bytes(node_cap, edge_cap) < 0 || node_blocks < 0 || edge_blocks < 0 ||
      !cfr_row_cap_ok(row_cap))
    return -1;
  pool_rows_set(pool, row_cap);
  long per_words = (long)(cfr_pool_bytes(node_cap, edge_cap) / 4);
  long tbl_words = (long)(cfr_tables_bytes(node_cap, edge_cap) / 4);
  uint8_t* a = (uint8_t*)pool + per_words * 4 * B;
  long n = tbl_words * B;
  hipLaunchKernelGGL(k_arena_reset, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, (int32_t*)pool,
                     per_words, tbl_words, B, reinterpret_cast<CfrArena*>(a), (uint32_t)node_blocks,
                     (uint32_t)edge_blocks, (uint32_t)row_cap, (uint32_t)(pred != 0));
  CHECK_LAUNCH();
}
int cit_cfr_arena_reset(void* pool, int B, int node_cap, int edge_cap, int node_blocks, int edge_blocks,
                        hipStream_t stream) {
  return cit_cfr_arena_reset_rows(pool, B, node_cap, edge_cap, node_blocks, edge_blocks, 0, stream);
}
int cit_cfr_arena_release(void* pool, int B, int node_cap, int edge_cap, const int32_t* lanes, int n_lanes,
                          hipStream_t stream) {
  if (!pool || B <= 0 || n_lanes < 0 || (n_lanes && !lanes) || cit_cfr_pool_bytes(node_cap, edge_cap) < 0) return -1;
  int64_t per = cfr_pool_bytes(node_cap, edge_cap);
  CfrArena* a = reinterpret_cast<CfrArena*>((uint8_t*)pool + per * (int64_t)B);
  hipLaunchKernelGGL(k_arena_clamp, dim3(1), dim3(64), 0, stream, a);
  if (n_lanes)
    hipLaunchKernelGGL(k_arena_release, dim3(n_lanes), dim3(256), 0, stream, (int32_t*)pool, (long)(per / 4),
                       cfr_nblocks(node_cap), cfr_eblocks(edge_cap), a, lanes);
  CHECK_LAUNCH();
}
int cit_cfr_opt_cap(void) { return CFR_OPT_CAP; }

int cit_cfr_decide(void* games, uint32_t* mt, uint32_t* mt_idx, uint32_t* np_mt, uint32_t* np_idx, uint64_t* seer,
                   int B, int iters, int flags, const int32_t* orig_player, void* pool, int node_cap, int edge_cap,
                   CitOption* optbuf, CitOption* chosen, int32_t* stats, hipStream_t stream) {
  if (B <= 0 || iters < 0 || cit_cfr_pool_bytes(node_cap, edge_cap) < 0 || !games || !mt || !mt_idx || !np_mt ||
      !np_idx || !seer || !pool || !optbuf || !chosen || !stats)
    return -1;
  DynLds d = dyn_lds(pool, node_cap, edge_cap);
  hipLaunchKernelGGL(k_cfr_decide, dim3(B), dim3(64), d.bytes, stream, (uint32_t*)games, mt, mt_idx, np_mt, np_idx, seer,
                     B, iters, flags, orig_player, (uint8_t*)pool, node_cap, edge_cap, (CitOpt*)optbuf, (CitOpt*)chosen, stats,
                     d.base_off);
  CHECK_LAUNCH();
}

int cit_cfr_state_bytes(void) { return (int)sizeof(CfrState); }

int cit_cfr_train_slice(void* games, uint32_t* mt, uint32_t* mt_idx, uint32_t* np_mt, uint32_t* np_idx, uint64_t* seer,
                        int B, int iters, int flags, const int32_t* orig_player, void* pool, int node_cap, int edge_cap,
                        CitOption* optbuf, void* state, int64_t slice_ticks, CitOption* chosen, int32_t* stats,
                        int32_t* running, hipStream_t stream) {
  if (B <= 0 || iters < 0 || slice_ticks < 0 || cit_cfr_pool_bytes(node_cap, edge_cap) < 0 || !games || !mt ||
      !mt_idx || !np_mt || !np_idx || !seer || !pool || !optbuf || !state || !chosen || !stats || !running)
    return -1;
  DynLds d = dyn_lds(pool, node_cap, edge_cap);
  hipLaunchKernelGGL(k_cfr_train_slice, dim3(B), dim3(64), d.bytes, stream, (uint32_t*)games, mt, mt_idx, np_mt, np_idx,
                     seer, B, iters, flags, orig_player, (uint8_t*)pool, node_cap, edge_cap, (CitOpt*)optbuf,
                     (CfrState*)state, (uint64_t)slice_ticks, (CitOpt*)chosen, stats, running, d.base_off);
  CHECK_LAUNCH();
}

int cit_cfr_pred_step(void* games, uint32_t* mt, uint32_t* mt_idx, uint32_t* np_mt, uint32_t* np_idx, uint64_t* seer,
                      int B, int iters, int flags, const int32_t* orig_player, int max_depth, void* pool,
                      int node_cap, int edge_cap, CitOption* optbuf, void* state, const float* probs, float* feat,
                      CitOption* chosen, int32_t* waiting, hipStream_t stream) {
  if (B <= 0 || iters < 0 || cit_cfr_pool_bytes(node_cap, edge_cap) < 0 || !games || !mt || !mt_idx || !np_mt ||
      !np_idx || !seer || !pool || !optbuf || !state || !probs || !feat || !chosen || !waiting)
    return -1;
  DynLds d = dyn_lds(pool, node_cap, edge_cap);
  hipLaunchKernelGGL(k_cfr_pred_step, dim3(B), dim3(64), d.bytes, stream, (uint32_t*)games, mt, mt_idx, np_mt, np_idx,
                     seer, B, iters, flags, orig_player, max_depth, (uint8_t*)pool, node_cap, edge_cap, (CitOpt*)optbuf,
                     (CfrState*)state, probs, feat, (CitOpt*)chosen, waiting, (uint64_t)0, (int32_t*)nullptr, d.base_off);
  CHECK_LAUNCH();
}

int cit_cfr_pred_slice(void* games, uint32_t* mt, uint32_t* mt_idx, uint32_t* np_mt, uint32_t* np_idx, uint64_t* seer,
                       int B, int iters, int flags, const int32_t* orig_player, int max_depth, void* pool,
                       int node_cap, int edge_cap, CitOption* optbuf, void* state, const float* probs, float* feat,
                       CitOption* chosen, int64_t slice_ticks, int32_t* waiting, int32_t* running,
                       hipStream_t stream) {
  if (B <= 0 || iters < 0 || slice_ticks < 0 || cit_cfr_pool_bytes(node_cap, edge_cap) < 0 || !games || !mt ||
      !mt_idx || !np_mt || !np_idx || !seer || !pool || !optbuf || !state || !probs || !feat || !chosen ||
      !waiting || (slice_ticks && !running))
    return -1;
  DynLds d = dyn_lds(pool, node_cap, edge_cap);
  hipLaunchKernelGGL(k_cfr_pred_step, dim3(B), dim3(64), d.bytes, stream,
                     (uint32_t*)games, mt, mt_idx, np_mt, np_idx, seer, B, iters, flags, orig_player, max_depth,
                     (uint8_t*)pool, node_cap, edge_cap, (CitOpt*)optbuf, (CfrState*)state, probs, feat,
                     (CitOpt*)chosen, waiting, (uint64_t)slice_ticks, running, d.base_off);
  CHECK_LAUNCH();
}

int cit_cfr_pred_fused(void* games, uint32_t* mt, uint32_t* mt_idx, uint32_t* np_mt, uint32_t* np_idx, uint64_t* seer,
                       int B, int iters, int flags, const int32_t* orig_player, int max_depth, void* pool,
                       int node_cap, int edge_cap, CitOption* optbuf, const void* wave_weights, void* state,
                       CitOption* chosen, int32_t* stats, hipStream_t stream) {
  if (B <= 0 || iters < 0 || cit_cfr_pool_bytes(node_cap, edge_cap) < 0 || !games || !mt || !mt_idx || !np_mt ||
      !np_idx || !seer || !pool || !optbuf || !wave_weights || !chosen || !stats)
    return -1;
  DynLds d = dyn_lds(pool, node_cap, edge_cap);
  hipLaunchKernelGGL(k_cfr_pred_fused, dim3(B), dim3(64), d.bytes, stream, (uint32_t*)games, mt, mt_idx, np_mt,
                     np_idx, seer, B, iters, flags, orig_player, max_depth, (uint8_t*)pool, node_cap, edge_cap,
                     (CitOpt*)optbuf, (const float*)wave_weights, (CfrState*)state, (CitOpt*)chosen, stats,
                     d.base_off);
  CHECK_LAUNCH();
}

#ifdef CFR_TREE_CLOCK
int cit_tree_clock_read(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tree_clock), sizeof(unsigned long long) * 2 * n);
}
#endif

#if defined(CIT_PROF)
int cit_prof_read(unsigned long long* out) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cit_prof), sizeof(unsigned long long) * 64);
  unsigned long long z[64] = {0};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_cit_prof), z, sizeof(z));
  return (int)e;
}
#endif

}  // extern "C"
