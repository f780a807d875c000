// One-game-per-lane kernels (CIT_NO_WAVE: lanes hold different games, so the
// engine's wave-uniform list scans are compiled out of this unit):
//   * k_rollout: the random-policy step loop with G games per wavefront
//     (games_per_block = G > 0 of cit_rollout_random; kept for sweeps and as
//     an independent execution model in the parity tests: divergence across
//     a 47-way option switch makes it slower than k_rollout_u at every B
//     measured).  Rows in LDS at an odd-dword stride, MT19937 words in HBM
//     (structure of arrays).
//   * k_cfr_target_count / k_cfr_targets: pre-order walks of finished MCCFR
//     trees, one tree per lane (CFR_WALK_TPW trees per wave).
#define CIT_NO_WAVE 1
#include <hip/hip_runtime.h>

#include "../../include/citadels.h"
#include "cit_cfr.h"
#include "cit_lanes.h"

#define ROW_W (CIT_GAME_BYTES / 4)
#define LDS_W (ROW_W + 1)

namespace {

__device__ __forceinline__ void stage_in(uint32_t* lds, const uint32_t* __restrict__ gm, long g0, int nrows) {
  for (int i = threadIdx.x; i < nrows * ROW_W; i += blockDim.x) {
    int r = i / ROW_W, w = i - r * ROW_W;
    lds[r * LDS_W + w] = gm[(g0 + r) * ROW_W + w];
  }
}
__device__ __forceinline__ void stage_out(const uint32_t* lds, uint32_t* __restrict__ gm, long g0, int nrows) {
  for (int i = threadIdx.x; i < nrows * ROW_W; i += blockDim.x) {
    int r = i / ROW_W, w = i - r * ROW_W;
    gm[(g0 + r) * ROW_W + w] = lds[r * LDS_W + w];
  }
}
__device__ __forceinline__ CitMT lane_mt(uint32_t* mt, const uint32_t* idx, int B, long l) {
  CitMT r;
  r.mt = mt + l;
  r.stride = B;
  r.pos = idx[l];
  r.coop = 0;
  return r;
}

__global__ void k_rollout(uint32_t* games, uint32_t* mt, uint32_t* idx, uint64_t* seer, int B, int max_steps,
                          int32_t* steps_out, int32_t* winner) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  long g0 = (long)blockIdx.x * blockDim.x;
  int nrows = (int)min((long)blockDim.x, (long)B - g0);
  stage_in(lds, games, g0, nrows);
  __syncthreads();
  if (threadIdx.x < nrows) {
    long l = g0 + threadIdx.x;
    CitGame& g = *reinterpret_cast<CitGame*>(lds + threadIdx.x * LDS_W);
    CitMT r = lane_mt(mt, idx, B, l);
    uint64_t* sc = seer + l * CIT_SEER_MAX;
    int cap = max_steps < 0 ? CIT_ROLLOUT_CAP : max_steps;
    int s = 0;
    while (!g.terminal && !g.err && s < cap) {
      cit_random_step(g, r, sc);
      s++;
    }
    if (max_steps < 0 && s >= cap && !g.terminal && !g.err) g.err |= CIT_ERR_STEP_CAP;
    steps_out[l] += s;
    winner[l] = g.winner;
    idx[l] = r.pos;
  }
  __syncthreads();
  stage_out(lds, games, g0, nrows);
}

// Trees per wavefront of the two walks: lanes walking different trees diverge
// (their pre-orders have different shapes), so a wave of 64 trees costs about
// the sum of its trees' walks, and B / 64 waves leave most of the chip idle;
// with one tree per wave the B walks run side by side (CFR_WALK_TPW=64: the
// packed launch, for A/B).
#ifndef CFR_WALK_TPW
#define CFR_WALK_TPW 1
#endif
static_assert(CFR_WALK_TPW >= 1 && CFR_WALK_TPW <= 64, "trees per wave of the walks");
__device__ __forceinline__ long walk_tree() {
  return threadIdx.x < CFR_WALK_TPW ? (long)blockIdx.x * CFR_WALK_TPW + threadIdx.x : -1;
}

__global__ void k_cfr_target_count(uint8_t* pool, int B, int node_cap, int edge_cap, const int32_t* roots, int mode,
                                   int32_t* counts) {
  long l = walk_tree();
  if (l < 0 || l >= B) return;
  if (roots[l] < 0) {
    counts[2 * l] = counts[2 * l + 1] = 0;
    return;
  }
  CfrTree T = cfr_tree_view(pool, B, l, node_cap, edge_cap);
  cfr_count_targets(T, roots[l], mode, counts[2 * l], counts[2 * l + 1]);
}

__global__ void k_cfr_targets(uint8_t* pool, int B, int node_cap, int edge_cap, const int32_t* roots, int mode,
                              uint32_t* mt,
                              uint32_t* idx, const int32_t* offsets, int32_t* meta, float* feat, double* value,
                              double* dist, float* opt_feat) {
  long l = walk_tree();
  // a lane without a tree touches nothing: the tree queue walks finished trees while
  // the other lanes' searches run (and write their own stream positions) on another stream
  if (l < 0 || l >= B || roots[l] < 0) return;
  CfrTree T = cfr_tree_view(pool, B, l, node_cap, edge_cap);
  CitMT r = lane_mt(mt, idx, B, l);
  cfr_emit_targets(T, r, roots[l], mode, (int)l, offsets[2 * l], offsets[2 * l + 1], meta, feat, value, dist, opt_feat);
  idx[l] = r.pos;
}

// CFRNode.action_choice(live=False) (deep_mccfr.py:67-91) at node[l] of tree
// l: the child's edge index (np.random.choice from the tree's numpy stream),
// -1 with err[l] set when numpy would raise.
__global__ void k_cfr_choose(uint8_t* pool, int B, int node_cap, int edge_cap, const int32_t* node, uint32_t* npmt,
                             uint32_t* npidx, int32_t* edge_out, int32_t* err_out) {
  long l = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= B) return;
  CfrTree T = cfr_tree_view(pool, B, l, node_cap, edge_cap);
  T.np = lane_mt(npmt, npidx, B, l);
  T.err = 0;
  int n = node[l];
  int a = -1;
  // a node id the tree does not hold (past its node count: an unallocated
  // block) is rejected before its record is read
  bool ok = n >= 0 && n < node_cap && T.nbt[n >> CFR_NB_SHIFT] >= 0;
  if (ok) {   // and an edge run inside the tree's edge blocks
    const CfrNode& N = cfr_node(T, n);
    int f = N.first_edge, span = (N.flags & NF_ROLE_PICK) ? CFR_ROLE_EDGE_SLOTS : N.n_children;
    ok = N.n_children > 0 && f >= 0 && (int64_t)f + span <= edge_cap && T.ebt[f >> CFR_EB_SHIFT] >= 0 &&
         T.ebt[(f + span - 1) >> CFR_EB_SHIFT] >= 0;
  }
  if (!ok) T.err |= CIT_ERR_VALUE;   // choice over []
  else a = cfr_choose(T, n);
  edge_out[l] = T.err ? -1 : a;
  err_out[l] = (int32_t)T.err;
  npidx[l] = T.np.pos;
}

// get_options one game per lane (the per-lane execution model of the
// enumeration, for parity checks against the wave-uniform k_get_options):
// rows and streams stay in HBM.
__global__ void k_get_options_lanes(uint32_t* games, uint32_t* mt, uint32_t* idx, uint64_t* seer, int B, CitOpt* opts,
                                    int max_opts, int32_t* n_opts) {
  long l = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= B) return;
  CitGame& g = *reinterpret_cast<CitGame*>(games + l * ROW_W);
  CitMT r = lane_mt(mt, idx, B, l);
  uint64_t* sc = seer + l * CIT_SEER_MAX;
  cit_prepare_options(g, r, sc);
  ListSink s(opts + l * max_opts, max_opts);
  cit_enum_options(g, s, sc);
  g.err |= s.err;
  n_opts[l] = s.n;
  idx[l] = r.pos;
}

size_t lds_bytes(int G) { return (size_t)G * LDS_W * 4; }

bool g_attrs_done = false;
int ensure_attrs() {
  if (g_attrs_done) return 0;
  int e = (int)hipFuncSetAttribute((const void*)k_rollout, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds_bytes(CIT_LANES_MAX_G));
  if (!e) g_attrs_done = true;
  return e;
}

}  // namespace

#define CHECK_LAUNCH()                       \
  do {                                       \
    hipError_t _e = hipGetLastError();       \
    return _e == hipSuccess ? 0 : (int)_e;   \
  } while (0)

int cit_rollout_lanes(uint32_t* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int max_steps, int G,
                      int32_t* steps, int32_t* winner, hipStream_t stream) {
  if (G <= 0 || G > CIT_LANES_MAX_G) return -1;
  if (int e = ensure_attrs()) return e;
  hipLaunchKernelGGL(k_rollout, dim3((B + G - 1) / G), dim3(G), lds_bytes(G), stream, games, mt, mt_idx, seer, B,
                     max_steps, steps, winner);
  CHECK_LAUNCH();
}

extern "C" {

int cit_get_options_lanes(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, CitOption* opts,
                          int max_opts, int32_t* n_opts, hipStream_t stream) {
  if (B <= 0 || max_opts < 0 || !games || !mt || !mt_idx || !seer || !n_opts || (max_opts && !opts)) return -1;
  hipLaunchKernelGGL(k_get_options_lanes, dim3((B + 63) / 64), dim3(64), 0, stream, (uint32_t*)games, mt, mt_idx,
                     seer, B, (CitOpt*)opts, max_opts, n_opts);
  CHECK_LAUNCH();
}

int cit_cfr_target_count(void* pool, int B, int node_cap, int edge_cap, const int32_t* roots, int mode,
                         int32_t* counts, hipStream_t stream) {
  if (B <= 0 || node_cap <= 0 || edge_cap <= 0 || !pool || !roots || !counts || mode < 0 || mode > 3) return -1;
  hipLaunchKernelGGL(k_cfr_target_count, dim3((B + CFR_WALK_TPW - 1) / CFR_WALK_TPW), dim3(64), 0, stream, (uint8_t*)pool, B, node_cap,
                     edge_cap, roots, mode, counts);
  CHECK_LAUNCH();
}

int cit_cfr_targets(void* pool, int B, int node_cap, int edge_cap, const int32_t* roots, int mode, uint32_t* mt,
                    uint32_t* mt_idx, const int32_t* offsets, int32_t* meta, float* feat, double* value, double* dist,
                    float* opt_feat, hipStream_t stream) {
  if (B <= 0 || node_cap <= 0 || edge_cap <= 0 || !pool || !roots || !mt || !mt_idx || !offsets || mode < 0 ||
      mode > 3)
    return -1;
  hipLaunchKernelGGL(k_cfr_targets, dim3((B + CFR_WALK_TPW - 1) / CFR_WALK_TPW), dim3(64), 0, stream, (uint8_t*)pool, B, node_cap, edge_cap,
                     roots, mode, mt, mt_idx, offsets, meta, feat, value, dist, opt_feat);
  CHECK_LAUNCH();
}

int cit_cfr_action_choice(void* pool, int B, int node_cap, int edge_cap, const int32_t* node, uint32_t* np_mt,
                          uint32_t* np_idx, int32_t* edge, int32_t* err, hipStream_t stream) {
  if (B <= 0 || node_cap <= 0 || edge_cap <= 0 || !pool || !node || !np_mt || !np_idx || !edge || !err) return -1;
  hipLaunchKernelGGL(k_cfr_choose, dim3((B + 63) / 64), dim3(64), 0, stream, (uint8_t*)pool, B, node_cap, edge_cap,
                     node, np_mt, np_idx, edge, err);
  CHECK_LAUNCH();
}

}  // extern "C"
