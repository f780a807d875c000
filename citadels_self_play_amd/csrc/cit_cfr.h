// MCCFR search on packed rows (algorithms/deep_mccfr.py), host+device.
//
// One tree per workgroup on the device.  The tree lives in HBM as a node
// pool: CfrNode headers, CfrEdge records (option + child + regret/strategy
// rows) and one packed game row per node (the reference's `deepcopy(game)`
// becomes a 1552-byte row copy done by the whole 64-lane team).  Every lane
// of the team runs the same scalar search code on the same data (uniform
// control flow, identical writes), so row copies and other data-parallel
// pieces can be split across lanes without divergence.
//
//   CfrNode / cfr_node       CFRNode.__init__ + skip_false_choice   deep_mccfr.py:8-49
//   cfr_update_strategy      update_strategy                        :292-319
//   cfr_choose / cfr_live    action_choice, weighted_average_...   :51-91, game.py:312-317
//   cfr_expand_*             expand / expand_role_pick / _for_original_player / _for_opponents  :93-179
//   cfr_backprop             backpropagate + update_regrets          :231-256, 276-290
//   cfr_train                cfr_train                               :187-205
// fp64 follows numpy's operation order: np.sum = pairwise (8 accumulators,
// blocks of <= 128), axis-0 sums and cumsum sequential, choice(p) = kahan
// check + cumsum + cdf/cdf[-1] + searchsorted(right) on a 53-bit double.
// np.exp is the only op not restated bit for bit (libm/ocml exp; both within
// 1 ulp of numpy's SIMD exp): strategies agree to ~1e-15 relative.
#pragma once
#include <math.h>

#include "cit_engine.h"
#include "cit_mlp_wave.h"

#define CFR_OPP_CHILDREN 10
#define CFR_ROLE_CHILDREN 10
#define CFR_OPT_CAP 512
// options listed into LDS per search step
#ifndef CFR_LBUF
#define CFR_LBUF 32
#endif
// update_strategy's LDS copies of S / CS (CfrLds.sbuf / cbuf) hold the nodes
// with up to CFR_SBUF children (at most 55 seen in 64 cfr_train(2000) trees);
// a node with more runs the host build's loop over its edge records in HBM
// (the same arithmetic in the same order; CIT_CFR_STRATEGY_HBM forces that
// path for every node, so a test can compare the two).
#ifndef CFR_SBUF
#define CFR_SBUF 96
#endif
#define CFR_LN13 0x1.0ca937be1b9dcp-2   // np.log(1.3)
#define CFR_ATOL 1.4901161193847656e-08  // sqrt(finfo(float64).eps), numpy choice's p check

// NF_BACKED: backpropagate has run on the node (winning_probabilities is then
// node_value / node_value.sum(), else its initial zeros)
enum { NF_ROLE_PICK = 1, NF_TERMINAL = 2, NF_PRED = 4, NF_BACKED = 8 };

// A node record: the header and node_value.  winning_probabilities is derived
// (cfr_wp: backpropagate sets it to node_value / node_value.sum() whenever it
// touches node_value); pred_node_value lives in a side array that only pools
// of cfr_pred searches have (cfr_pred_of).  72 B instead of round 3's 168.
struct CfrNode {                       // 72 B
  int32_t parent, first_edge;
  int16_t n_children, edge_cap, depth;
  int8_t player, gs_state;
  uint8_t flags;
  int8_t winner;
  int16_t sib;                         // index among the parent's children (-1: root)
  int32_t row;                         // diff-row pools: edge index of the node's row run (else unused)
  double nv[6];
};
#define CFR_PRED_BYTES 48              // pred_node_value f64[6] per node (cfr_pred pools)
// node_value.sum() in numpy's order (pairwise_sum below 8 elements: sequential)
CIT_HD double cfr_nv_sum(const double* nv) {
  double s = 0.0;
  for (int k = 0; k < 6; k++) s += nv[k];
  return s;
}
// winning_probabilities[p] of a node with node_value nv, flags f (s = cfr_nv_sum(nv))
CIT_HD double cfr_wp(const double* nv, double s, int f, int p) { return (f & NF_BACKED) ? nv[p] / s : 0.0; }
// An edge = (option, child) and the parent's regret / strategy / cumulative
// strategy entries for it.  A normal node's arrays are [nch] (one double per
// edge).  A role-pick node's are [6 players, 10]: it reserves
// CFR_ROLE_CHILDREN edges followed by CFR_ROLE_CHILDREN CfrWide records
// (3 edge slots each) holding the per-player columns, so a normal edge stays
// 48 B (the pool of a cfr_train(200000) tree is ~1M edges).
struct CfrEdge {                       // 48 B
  CitOpt opt;
  int32_t child, pad;
  double R, S, CS;
};
struct CfrWide {                       // 144 B = 3 edge slots
  double R[6], S[6], CS[6];
};
static_assert(sizeof(CfrNode) == 72, "CfrNode layout");
static_assert(sizeof(CfrEdge) == 48, "CfrEdge layout");
static_assert(sizeof(CfrWide) == 3 * sizeof(CfrEdge), "CfrWide layout");
#define CFR_ROLE_EDGE_SLOTS (CFR_ROLE_CHILDREN * 4)   // 10 edges + 10 wide records

// Node pool of B trees, allocated in blocks from one arena as the trees grow
// (a tree takes what it uses, not its worst case: a cfr_train(200000) tree
// averages ~270k nodes against a ~650k-node maximum):
//   per tree l (cfr_pool_bytes each): int32 node-block table [nblocks(node_cap)]
//     | int32 edge-block table [eblocks(edge_cap)] | pad to 16 B | base row
//     (CIT_GAME_BYTES) | scratch row (CIT_GAME_BYTES)
//   arena (at B * cfr_pool_bytes): CfrArena header (64 B) | free-block rings
//     uint32 [n_cap] + [e_cap] (padded to 16 B) | node records [n_cap
//     blocks][CFR_NB] | node row slots [n_cap blocks][CFR_NB] (16-byte
//     aligned) | edges [e_cap blocks][CFR_EB]
// Node rows (the arena's row_cap): row_cap 0 stores each node's game row raw
// (CIT_GAME_BYTES) in a row slot of its node block.  row_cap K > 0 stores it
// as a diff against the tree's base row (its root game as first created), of
// the length it has, in the tree's edge space: a run of cfr_row_slots(k) edge
// slots (CfrNode.row) holding a header of CFR_ROW_HDR words (bit d of the
// 388-bit mask in words 0..12 = dword d differs from the base; word 13 the
// count k) and then the k differing dwords in index order; node blocks then
// hold records only.  A cfr_train(200000) node differs from its root in ~70
// of 388 dwords (~7 edge slots, 336 B, against a fixed 128-dword slot's 576 B
// and a raw row's 1,552 B).  A row with more than K differing dwords stops the
// tree with CIT_ERR_OVERFLOW | CIT_ERR_POOL_ROW and the tree is searched again
// with raw rows (engine.py's retry; K = 388, the product's, never overflows):
// the format never changes a result.
// A block is taken from its free ring (blocks released by finished trees,
// cit_cfr_arena_release) or, when that is empty, from the never-used rest.
// Node id n lives in block nbt[n >> CFR_NB_SHIFT] at slot n & (CFR_NB - 1);
// edge index e likewise through ebt.  An edge run (a node's children) never
// straddles an edge block.  Sizes are 64-bit.
#define CFR_NB_SHIFT 12
#define CFR_NB (1 << CFR_NB_SHIFT)            // nodes (records + rows) per block: 7 MB
#define CFR_EB_SHIFT 14
#define CFR_EB (1 << CFR_EB_SHIFT)            // edge slots per block: 768 KB
#define CFR_TBL_MAX 1024                      // table entries a device tree keeps in LDS
struct CfrArena {                             // 64 B, written by cit_cfr_arena_reset
  uint32_t n_next, n_cap, e_next, e_cap;      // never-used blocks handed out / capacity
  uint32_t n_head, n_tail, e_head, e_tail;    // free rings: taken / released counts (mod cap)
  uint32_t row_cap;                           // row slot format (0: raw rows)
  uint32_t pred;                              // 1: node blocks carry pred_node_value (cfr_pred pools)
  uint32_t pad[6];
};
#define CFR_ROW_W (CIT_GAME_BYTES / 4)        // 388 dwords
#define CFR_ROW_HDR 14                        // header words of a diff row run (mask, count)
#define CFR_ROW_MASKW 13                      // mask words (388 bits)
#define CFR_ROW_CAP_MAX CFR_ROW_W             // every dword may differ
static_assert(sizeof(CfrArena) == 64, "CfrArena layout");

struct CfrTree {
  uint8_t* node_base;                  // arena node records
  uint8_t* pred_base;                  // arena pred_node_value arrays (pools with pred)
  uint8_t* row_base;                   // arena node rows
  uint8_t* edge_base;                  // arena edges
  CfrArena* arena;
  int32_t* nbt;                        // node-block table (LDS copy on the device)
  int32_t* ebt;                        // edge-block table (LDS copy on the device)
  int32_t* nbt_hbm;                    // the tree's tables in the pool
  int32_t* ebt_hbm;
  int node_cap, edge_cap;
  int row_cap;                         // the arena's row slot format (0: raw rows)
  int64_t row_slot;                    // bytes per row slot
  uint32_t* base_hbm;                  // the tree's base row (diff rows) in the pool
  uint32_t* scratch_hbm;               // one row of scratch per tree in the pool
  int n_nodes, n_edges;
  int n_eblk;                          // edge blocks held
  int orig;
  bool training;
  CitMT py;                            // the games' CPython stream
  CitMT np;                            // numpy's global RandomState
  uint64_t* seer;
  CitOpt* optbuf;                      // CFR_OPT_CAP descriptors
  CitGame* w0;                         // working rows (LDS on the device)
  CitGame* w1;
  uint8_t* tmp;                        // >= CIT_USED_CAP bytes scratch
  CitOpt* lbuf;                        // CFR_LBUF descriptors (LDS on the device)
  uint32_t err;
  uint32_t carry_outs;
  // The search's current node (the one cfr_update_strategy last read): its
  // header fields, so the choice, the step to the chosen child and the
  // child's expansion (which asks for its parent's player and state) do not
  // read the record from HBM again.  cur_node -1: nothing cached.
  int cur_node, cur_fe, cur_nch, cur_flags, cur_player, cur_state;
  // Diff-row pools: the row run of node rn_node (read with its header by
  // cfr_expand / cfr_update_strategy, so row_load needs no read of the
  // record), and the run and its capacity (in differing dwords) of the row
  // row_load or row_store last handled (rl_node), which a re-store of that
  // node reuses when the new diff fits.  -1: none.
  int rn_node, rn_run;
  int rl_node, rl_run, rl_k;
};

CIT_HD int cfr_nblocks(int node_cap) { return (node_cap + CFR_NB - 1) >> CFR_NB_SHIFT; }
CIT_HD int cfr_eblocks(int edge_cap) { return (edge_cap + CFR_EB - 1) >> CFR_EB_SHIFT; }
CIT_HD int64_t cfr_tables_bytes(int node_cap, int edge_cap) {   // a tree's two block tables, padded
  return ((int64_t)4 * (cfr_nblocks(node_cap) + cfr_eblocks(edge_cap)) + 15) & ~(int64_t)15;
}
CIT_HD int64_t cfr_pool_bytes(int node_cap, int edge_cap) {   // per tree: tables, base row, scratch row
  return cfr_tables_bytes(node_cap, edge_cap) + 2 * (int64_t)CIT_GAME_BYTES;
}
CIT_HD int cfr_row_cap_ok(int row_cap) { return row_cap == 0 || (row_cap > 0 && row_cap <= CFR_ROW_CAP_MAX && !(row_cap & 3)); }
// bytes of a node block's row slot: a raw row, none for diff rows (they live in edge space)
CIT_HD int64_t cfr_row_slot_bytes(int row_cap) { return row_cap > 0 ? 0 : (int64_t)CIT_GAME_BYTES; }
// edge slots of a diff row run with k differing dwords
CIT_HD int cfr_row_slots(int k) {
  return (CFR_ROW_HDR + k + (int)(sizeof(CfrEdge) / 4) - 1) / (int)(sizeof(CfrEdge) / 4);
}
CIT_HD int64_t cfr_node_block_bytes(int row_cap = 0, int pred = 1) {
  return (int64_t)CFR_NB * ((int64_t)sizeof(CfrNode) + (pred ? CFR_PRED_BYTES : 0) + cfr_row_slot_bytes(row_cap));
}
CIT_HD int64_t cfr_ring_bytes(int64_t n_blocks, int64_t e_blocks) { return (4 * (n_blocks + e_blocks) + 15) & ~(int64_t)15; }
CIT_HD int64_t cfr_arena_bytes(int n_blocks, int e_blocks, int row_cap = 0, int pred = 1) {
  return (int64_t)sizeof(CfrArena) + cfr_ring_bytes(n_blocks, e_blocks) +
         (int64_t)n_blocks * cfr_node_block_bytes(row_cap, pred) + (int64_t)e_blocks * CFR_EB * (int64_t)sizeof(CfrEdge);
}
// Binds tree l of a B-tree pool; the arena's capacities come from its header.
CIT_HD void cfr_tree_bind(CfrTree& T, uint8_t* pool, int B, long l, int node_cap, int edge_cap) {
  int64_t per = cfr_pool_bytes(node_cap, edge_cap);
  int32_t* tbl = reinterpret_cast<int32_t*>(pool + per * (int64_t)l);
  T.nbt_hbm = tbl;
  T.ebt_hbm = tbl + cfr_nblocks(node_cap);
  T.nbt = T.nbt_hbm;
  T.ebt = T.ebt_hbm;
  T.base_hbm = reinterpret_cast<uint32_t*>(pool + per * (int64_t)l + cfr_tables_bytes(node_cap, edge_cap));
  T.scratch_hbm = T.base_hbm + CFR_ROW_W;
  uint8_t* a = pool + per * (int64_t)B;
  T.arena = reinterpret_cast<CfrArena*>(a);
  int64_t ncap = T.arena->n_cap, ecap = T.arena->e_cap;
  T.row_cap = (int)T.arena->row_cap;
  T.row_slot = cfr_row_slot_bytes(T.row_cap);
  T.node_base = a + sizeof(CfrArena) + cfr_ring_bytes(ncap, ecap);
  T.pred_base = T.node_base + ncap * CFR_NB * (int64_t)sizeof(CfrNode);
  T.row_base = T.pred_base + (T.arena->pred ? ncap * CFR_NB * (int64_t)CFR_PRED_BYTES : 0);
  T.edge_base = T.row_base + ncap * CFR_NB * T.row_slot;
  T.node_cap = node_cap;
  T.edge_cap = edge_cap;
  T.cur_node = -1;
  T.rn_node = T.rl_node = -1;
}
// Resumable cfr_pred state of one tree (see cfr_pred_run below): 64 B,
// persists in HBM between launches.
enum { CP_INIT = 0, CP_RUN = 1, CP_WAIT = 2, CP_DONE = 3 };
struct CfrState {
  int32_t n_nodes, n_edges, err, carry_outs;
  int32_t cur, it, phase, pending;
  int32_t root, orig, pad[6];
};
static_assert(sizeof(CfrState) == 64, "CfrState layout");

// The 64 lanes of a tree's workgroup (one wavefront) run the search in
// lockstep on shared state; row copies are split across them.
#if defined(__HIP_DEVICE_COMPILE__)
#define CFR_SYNC() __syncthreads()
#define CFR_LANE ((int)threadIdx.x)
#define CFR_TEAM ((int)blockDim.x)
#else
#define CFR_SYNC() ((void)0)
#define CFR_LANE 0
#define CFR_TEAM 1
#endif

// ------------------------------------------------ uniformity, address spaces
// Every lane of a search team holds the same values, but a value that crosses
// a call boundary (an argument, a return value) arrives in a VGPR, and the
// compiler then treats everything derived from it as divergent: vector ALU
// for scalar work, exec-masked branches, and flat memory instructions (which
// wait on both the LDS and the vector-memory counters).  The search therefore
// (1) keeps its working state in one namespace-scope LDS block (cfr_ls, fixed
// addresses), (2) re-uniformises arguments and returns with readfirstlane
// (cfr_u) and (3) reaches the HBM node pool through pointers cast to the
// global address space (cfr_glb: global_* instructions with scalar bases).
#if CIT_WAVE
#define CFR_GAS __attribute__((address_space(1)))
__device__ __forceinline__ int cfr_u(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t cfr_u(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
template <class X>
__device__ __forceinline__ X* cfr_glb(X* q) {
  uint64_t a = (uint64_t)(uintptr_t)q;
  uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  return (X*)(CFR_GAS X*)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ CitOpt cfr_uopt(const CitOpt& o) {
  uint32_t w[4];
  __builtin_memcpy(w, &o, 16);
  for (int i = 0; i < 4; i++) w[i] = cfr_u(w[i]);
  CitOpt r;
  __builtin_memcpy(&r, w, 16);
  return r;
}
#else
CIT_HD int cfr_u(int v) { return v; }
CIT_HD uint32_t cfr_u(uint32_t v) { return v; }
template <class X>
CIT_HD X* cfr_glb(X* p) { return p; }
CIT_HD CitOpt cfr_uopt(const CitOpt& o) { return o; }
#endif

// The search's working state.  Device (CIT_WAVE): one LDS block per
// workgroup at namespace scope (the tree, the resumable pred state, the two
// working rows w0 / w1, the two MT19937 streams, the option list buffer and
// the determinization scratch); the CfrTree / CfrState references the
// functions receive are then only the host build's.  Host: the pointers
// bound in CfrTree.
#if defined(__HIPCC__)
// Invariant (cfr_leaf_eval): the in-kernel leaf evaluation's scratch overlays
// w[0..1], lbuf, sbuf and cbuf, so nothing may read those after a leaf
// evaluation before writing them again: the working rows are reloaded by the
// next expansion, the list buffer refilled by the next listing, and the
// strategy copies are valid only for node `cnode`, which the evaluation
// resets to -1.  CFR_DEBUG_POISON builds overwrite all four with a pattern
// after each evaluation so that a reader that breaks this fails the
// fused-vs-rounds and golden tests.
struct CfrLds {
  uint32_t w[2][CIT_GAME_BYTES / 4];
  CitOpt lbuf[CFR_LBUF];
  double sbuf[CFR_SBUF], cbuf[CFR_SBUF];         // update_strategy: S, CS of node `cnode`
  uint32_t py[CIT_MT_N], np[CIT_MT_N];
  CfrTree T;
  CfrState S;
  int cnode, cnch;                                // node (and its child count) whose normalised CS is in cbuf (-1: none)
  int sbuf_on;                                    // 0 under CIT_CFR_STRATEGY_HBM
  int base_off;                                   // dwords from cfr_dyn to the base row (diff-row pools)
  // cit_sample_private's scratch is read and written 16 bytes at a time:
  // keep it 16-byte aligned whatever the fields above add up to
  __attribute__((aligned(16))) uint8_t tmp[CIT_SAMPLE_SCRATCH];
};
static __shared__ __attribute__((aligned(16))) CfrLds cfr_ls;
// Dynamic LDS of a search launch (sized per launch, cfr_dyn_lds_bytes): the
// tree's two block tables interleaved (node-block entry i at [2i], edge-block
// entry i at [2i + 1]) so both start at a fixed address whatever the
// capacities; a tree's tables hold max(nblocks, eblocks) entries each (2 at
// configs 3/4, 172 at cfr_train(200000)) instead of a fixed CFR_TBL_MAX.
// Then, for a pool with diff row slots only, the tree's base row at
// cfr_dyn_base_off dwords (CfrLds.base_off): a raw-row launch (configs 3/4)
// takes 16 B of dynamic LDS instead of 1.6 KB.
extern __shared__ __attribute__((aligned(16))) uint32_t cfr_dyn[];
#endif
CIT_HD int64_t cfr_dyn_base_off(int node_cap, int edge_cap) {
  int nb = cfr_nblocks(node_cap), eb = cfr_eblocks(edge_cap);
  return (2 * (int64_t)(nb > eb ? nb : eb) + 3) & ~(int64_t)3;      // 16-byte aligned: rows move as 16-B words
}
CIT_HD int64_t cfr_dyn_lds_bytes(int node_cap, int edge_cap, bool base_row) {
  return 4 * (cfr_dyn_base_off(node_cap, edge_cap) + (base_row ? (int64_t)CFR_ROW_W : 0));
}
#if CIT_WAVE
#define CFR_T(T_in) (cfr_ls.T)
#define CFR_S(S_in) (cfr_ls.S)
__device__ __forceinline__ CitGame& cfr_w(const CfrTree&, int which) {
  return *reinterpret_cast<CitGame*>(cfr_ls.w[which]);
}
__device__ __forceinline__ CitOpt* cfr_lbuf(const CfrTree&) { return cfr_ls.lbuf; }
__device__ __forceinline__ uint8_t* cfr_tmp(const CfrTree&) { return cfr_ls.tmp; }
#else
#define CFR_T(T_in) (T_in)
#define CFR_S(S_in) (S_in)
CIT_HD CitGame& cfr_w(const CfrTree& T, int which) { return which ? *T.w1 : *T.w0; }
CIT_HD CitOpt* cfr_lbuf(const CfrTree& T) { return T.lbuf; }
CIT_HD uint8_t* cfr_tmp(const CfrTree& T) { return T.tmp; }
#endif
// One block for a tree (edge = 0: a node block, 1: an edge block): lane 0
// takes the next entry of the free ring, or a never-used block when the ring
// is empty; -1 when the arena is full.  Takes run concurrently (atomics);
// releases only between launches, so the ring's tail is fixed meanwhile and
// a head that overshoots it is pulled back by the next release.
CIT_HD int cfr_take_block(CfrArena* A, int edge) {
  uint32_t* ring = reinterpret_cast<uint32_t*>(A + 1) + (edge ? A->n_cap : 0);
  uint32_t cap = edge ? A->e_cap : A->n_cap;
  uint32_t* head = edge ? &A->e_head : &A->n_head;
  uint32_t tail = edge ? A->e_tail : A->n_tail;
  uint32_t* next = edge ? &A->e_next : &A->n_next;
  int r = -1;
#if CIT_WAVE
  if (__lane_id() == 0) {
    if (*head < tail) {
      uint32_t h = atomicAdd(head, 1u);
      if (h < tail) r = (int)ring[h % cap];
    }
    if (r < 0) {
      uint32_t v = atomicAdd(next, 1u);
      r = v < cap ? (int)v : -1;
    }
  }
  r = cfr_u(r);
#else
  if (*head < tail) r = (int)ring[(*head)++ % cap];
  if (r < 0) {
    uint32_t v = (*next)++;
    r = v < cap ? (int)v : -1;
  }
#endif
  return r;
}

// The block tables: LDS (fixed addresses, cfr_dyn) in a device search, else
// the pool's.  Entry i of the node- / edge-block table.
#if CIT_WAVE
__device__ __forceinline__ int32_t& cfr_nbt_at(const CfrTree&, int i) {
  return reinterpret_cast<int32_t*>(cfr_dyn)[2 * i];
}
__device__ __forceinline__ int32_t& cfr_ebt_at(const CfrTree&, int i) {
  return reinterpret_cast<int32_t*>(cfr_dyn)[2 * i + 1];
}
__device__ __forceinline__ const uint32_t* cfr_base(const CfrTree&) {
  return cfr_dyn + __builtin_amdgcn_readfirstlane(cfr_ls.base_off);
}
__device__ __forceinline__ uint32_t* cfr_base_w(const CfrTree&) {
  return cfr_dyn + __builtin_amdgcn_readfirstlane(cfr_ls.base_off);
}
#else
CIT_HD int32_t& cfr_nbt_at(const CfrTree& T, int i) { return T.nbt[i]; }
CIT_HD int32_t& cfr_ebt_at(const CfrTree& T, int i) { return T.ebt[i]; }
CIT_HD const uint32_t* cfr_base(const CfrTree& T) { return T.base_hbm; }
CIT_HD uint32_t* cfr_base_w(const CfrTree& T) { return T.base_hbm; }
#endif

// node n's record, edge e (a run of edges continues from it), node n's row slot
CIT_HD int64_t cfr_node_slot(const CfrTree& T, int n) {
  return (int64_t)cfr_nbt_at(T, n >> CFR_NB_SHIFT) * CFR_NB + (n & (CFR_NB - 1));
}
CIT_HD CfrNode& cfr_node(const CfrTree& T, int n) {
  return *reinterpret_cast<CfrNode*>(cfr_glb(T.node_base) + cfr_node_slot(T, n) * (int64_t)sizeof(CfrNode));
}
// node n's pred_node_value (pools with pred only)
CIT_HD double* cfr_pred_of(const CfrTree& T, int n) {
  return reinterpret_cast<double*>(cfr_glb(T.pred_base) + cfr_node_slot(T, n) * (int64_t)CFR_PRED_BYTES);
}
CIT_HD CfrEdge* cfr_edge(const CfrTree& T, int e) {
  int64_t slot = (int64_t)cfr_ebt_at(T, e >> CFR_EB_SHIFT) * CFR_EB + (e & (CFR_EB - 1));
  return reinterpret_cast<CfrEdge*>(cfr_glb(T.edge_base) + slot * (int64_t)sizeof(CfrEdge));
}
// the [6]-wide regret / strategy columns of role-pick child a
CIT_HD CfrWide* cfr_wide(const CfrTree& T, int first_edge) {
  return reinterpret_cast<CfrWide*>(cfr_edge(T, first_edge) + CFR_ROLE_CHILDREN);
}
CIT_HD uint32_t* row_of(const CfrTree& T, int id) {
  return reinterpret_cast<uint32_t*>(cfr_glb(T.row_base) + cfr_node_slot(T, id) * T.row_slot);
}
// A run of n edge slots (a node's children, or a diff row) inside one edge block.
CIT_HD int alloc_edges(CfrTree& T, int n) {
  int f = T.n_edges;
  if ((f & (CFR_EB - 1)) + n > CFR_EB) f = (f | (CFR_EB - 1)) + 1;
  if (f + n > T.edge_cap) { T.err |= CIT_ERR_OVERFLOW | CIT_ERR_POOL_CAP; return -1; }
  while (((f + n - 1) >> CFR_EB_SHIFT) >= T.n_eblk) {
    int b = cfr_take_block(cfr_glb(T.arena), 1);
    if (b < 0) { T.err |= CIT_ERR_OVERFLOW | CIT_ERR_POOL_ARENA; return -1; }
    cfr_ebt_at(T, T.n_eblk++) = b;
  }
  T.n_edges = f + n;
  return f;
}
CIT_HD uint32_t* w_row(const CfrTree& T, int which) { return reinterpret_cast<uint32_t*>(&cfr_w(T, which)); }

// One out-of-line copy of each engine entry point for the search: the
// engine is force-inlined by default (the rollout kernel wants that), and
// inlining it at every call site of the search multiplies code size and
// compile time.  Arguments are small values (a working-row selector, an
// option, an index); the state is reached through cfr_ls.
#if defined(__HIPCC__)
#define CIT_NOINLINE __host__ __device__ inline __attribute__((noinline))
#else
#define CIT_NOINLINE inline
#endif
// CFR_INLINE_LEVEL: which of the search's wrappers are inlined into their
// callers instead of called.  An out-of-line call on gfx950 waits for all of
// the caller's memory operations at entry (s_waitcnt vmcnt(0) lgkmcnt(0)),
// saves the VGPR that holds its spilled SGPRs to scratch and reloads it --
// a scratch round trip -- before it returns; the search makes several such
// calls per carry_out.  Inlining costs code size (each inlined wrapper is
// copied to each call site).
//   1: eng_prepare, eng_first_upto2 (per node, few call sites), cfr_update_regrets
//      (per backprop level, one call site)
//   2: + eng_carry, eng_list_reg (per carry_out / per listing)
//   3: + cfr_node, eng_sample, eng_list
//   4: + cfr_update_strategy, cfr_choose
#ifndef CFR_INLINE_LEVEL
#define CFR_INLINE_LEVEL 3
#endif
#if defined(__HIPCC__)
#define CFR_INLINED __host__ __device__ inline __attribute__((always_inline))
#else
#define CFR_INLINED inline
#endif
#if CFR_INLINE_LEVEL >= 1
#define CFR_INL1 CFR_INLINED
#else
#define CFR_INL1 CIT_NOINLINE
#endif
#if CFR_INLINE_LEVEL >= 2
#define CFR_INL2 CFR_INLINED
#else
#define CFR_INL2 CIT_NOINLINE
#endif
#if CFR_INLINE_LEVEL >= 3
#define CFR_INL3 CFR_INLINED
#else
#define CFR_INL3 CIT_NOINLINE
#endif
#if CFR_INLINE_LEVEL >= 4
#define CFR_INL4 CFR_INLINED
#else
#define CFR_INL4 CIT_NOINLINE
#endif

// The search's two streams sit in its LDS block (CfrTree::py / np, device);
// an engine call or a numpy draw works on a register copy of the stream's
// state (word pointer, position, register window) and hands it back once,
// so no draw reads and writes the position through LDS.
template <class F>
CIT_HD auto cfr_with_np(CfrTree& T, F f) {
  CitMT r = T.np;
  auto v = f(r);
  T.np = r;
  return v;
}

// option.carry_out on working row `which`, counted; returns the winner (-1: none)
CFR_INL2 int eng_carry(CfrTree& T_in, int which, CitOpt o_in) {
  CIT_PROF_SCOPE(0);
  CfrTree& T = CFR_T(T_in);
  CitOpt o = cfr_uopt(o_in);
  T.carry_outs++;
  CitMT py = T.py;               // (a register copy for the call: see cfr_with_np)
  const int w = cit_carry_out(cfr_w(T, cfr_u(which)), o, py);
  T.py = py;
  return w;
}
CFR_INL1 void eng_prepare(CfrTree& T_in, int which) {
  CIT_PROF_SCOPE(1);
  CfrTree& T = CFR_T(T_in);
  CitMT py = T.py;
  cit_prepare_options(cfr_w(T, cfr_u(which)), py, cfr_glb(T.seer));
  T.py = py;
}
CIT_NOINLINE CitOpt eng_pick(CfrTree& T_in, int which, int k) {
  CIT_PROF_SCOPE(3);
  CfrTree& T = CFR_T(T_in);
  return cit_pick_option(cfr_w(T, cfr_u(which)), cfr_u(k), cfr_glb(T.seer));
}
// An option count and the enumeration's error bits (returned, not written
// through a pointer: an out-parameter of a call lives in scratch memory).
struct CfrCnt {
  int n;
  uint32_t err;
};
CIT_HD CfrCnt cfr_ucnt(CfrCnt c) { return {cfr_u(c.n), cfr_u(c.err)}; }
// Every option of working row `which` into T.optbuf (HBM, CFR_OPT_CAP).
CFR_INL3 CfrCnt eng_list(CfrTree& T_in, int which) {
  CIT_PROF_SCOPE(4);
  CfrTree& T = CFR_T(T_in);
  ListSink s(cfr_glb(T.optbuf), CFR_OPT_CAP);
  cit_enum_options(cfr_w(T, cfr_u(which)), s, cfr_glb(T.seer));
  return {s.n, s.err};
}
// A search step's option list: the first CFR_LBUF options land in the LDS
// list buffer while all are counted, so one enumeration serves both the count
// and the draw (eng_pick re-enumerates only for an index past the buffer).
CIT_NOINLINE CfrCnt eng_list_lds(CfrTree& T_in, int which) {
  CIT_PROF_SCOPE(2);
  CfrTree& T = CFR_T(T_in);
  ListSink s(cfr_lbuf(T), CFR_LBUF);
  cit_enum_options(cfr_w(T, cfr_u(which)), s, cfr_glb(T.seer));
  return {s.n, s.err};
}
// skip_false_choice's question (exactly one option?): the options of working
// row `which` into the LDS list buffer until a second one is known (n is then
// a lower bound >= 2), unless the enumeration may still raise (Upto2Sink).
CIT_NOINLINE CfrCnt eng_list_upto2(CfrTree& T_in, int which) {
  CIT_PROF_SCOPE(2);
  CfrTree& T = CFR_T(T_in);
  const CitGame& g = cfr_w(T, cfr_u(which));
  Upto2Sink s(cfr_lbuf(T), CFR_LBUF, cfr_u(cit_enum_late_error(g) ? 0 : 1) != 0);
  cit_enum_options(g, s, cfr_glb(T.seer));
  return {s.n, s.err};
}
#if CIT_WAVE
// eng_list_upto2 without the list: the count (a lower bound >= 2 once a second
// option is known) and the first option, in registers.
struct CfrFirst {
  int n;
  uint32_t err;
  CitOpt o;
};
CFR_INL1 CfrFirst eng_first_upto2(CfrTree& T_in, int which) {
  CIT_PROF_SCOPE(2);
  CfrTree& T = CFR_T(T_in);
  const CitGame& g = cfr_w(T, cfr_u(which));
  Upto2FirstSink s(cfr_u(cit_enum_late_error(g) ? 0 : 1) != 0);
  cit_enum_options(g, s, cfr_glb(T.seer));
  return {s.n, s.err, s.first};
}
// eng_list_lds with the list in registers (RegSink: lane i holds option i of
// the first 64); the draw reads its option with readlanes.
struct CfrRegList {
  int n;
  uint32_t err;
  uint32_t r0, r1, r2, r3;
};
CFR_INL2 CfrRegList eng_list_reg(CfrTree& T_in, int which) {
  CIT_PROF_SCOPE(2);
  CfrTree& T = CFR_T(T_in);
  RegSink s;
  cit_enum_options(cfr_w(T, cfr_u(which)), s, cfr_glb(T.seer));
  return {s.n, s.err, s.r0, s.r1, s.r2, s.r3};
}
__device__ __forceinline__ CitOpt cfr_reg_opt(const CfrRegList& L, int k) {
  RegSink s;
  s.r0 = L.r0;
  s.r1 = L.r1;
  s.r2 = L.r2;
  s.r3 = L.r3;
  return s.at(k);
}
#endif
CFR_INL3 void eng_sample(CfrTree& T_in, int which, int orig, int role_sample) {
  CIT_PROF_SCOPE(5);
  CfrTree& T = CFR_T(T_in);
  CitMT py = T.py;
  cit_sample_private(cfr_w(T, cfr_u(which)), cfr_u(orig), cfr_u(role_sample) != 0, py, cfr_tmp(T));
  T.py = py;
}

// deepcopy(game): the team copies one row (inlined, so each call site's
// source and destination address spaces are known)
CIT_HD void copy_row(const CfrTree& T, uint32_t* dst, const uint32_t* src) {
  (void)T;
  CIT_PROF_SCOPE(6);
  CFR_SYNC();
#if CIT_WAVE
  {   // 97 16-byte words: lanes 0..63, then 0..32; both loads issued before the stores
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    const int l = CFR_LANE, hi = l + 64 < CIT_GAME_BYTES / 16;
    uint4 a = s4[l], b = hi ? s4[l + 64] : a;
    d4[l] = a;
    if (hi) d4[l + 64] = b;
  }
#else
  for (int i = CFR_LANE; i < CIT_GAME_BYTES / 4; i += CFR_TEAM) dst[i] = src[i];
#endif
  CFR_SYNC();
}

// Node row slots (see the pool layout above): row_load = the node's game row
// into dst (a working row in LDS, a scratch row, or a games[] row in HBM);
// row_store = working row src into the node's slot (diff rows: against the
// tree's base row; more than row_cap differing dwords -> CIT_ERR_OVERFLOW).
#if CIT_WAVE
__device__ __forceinline__ uint32_t cfr_mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
#endif
// The row run of node id (diff-row pools): the cached one when id's header was
// just read, else from its record.
CIT_HD int row_run_of(const CfrTree& T, int id) {
  return cfr_u(T.rn_node) == id ? cfr_u(T.rn_run) : cfr_node(T, id).row;
}
CIT_HD uint32_t* row_run_ptr(const CfrTree& T, int run) { return reinterpret_cast<uint32_t*>(cfr_edge(T, run)); }
CIT_HD void row_load(CfrTree& T, uint32_t* dst, int id) {
  CIT_PROF_SCOPE(23);
  if (cfr_u(T.row_cap) == 0) {
    copy_row(T, dst, row_of(T, id));
    return;
  }
  const int run = cfr_u(row_run_of(T, id));
  const uint32_t* s = row_run_ptr(T, run);
  const uint32_t* base = cfr_base(T);
  uint32_t k;
  CFR_SYNC();
#if CIT_WAVE
  {
    // one round of loads: up to STG dwords per lane from the run on (not past
    // its edge block: a run never straddles one), which hold the whole row
    // when it has at most 64 * STG - CFR_ROW_HDR differing dwords, staged in
    // the LDS scratch so each lane can read its dwords' values by rank; lanes
    // 0..12 hold the mask words, lane 13 the count; chunk j = dwords 64j..64j+63
    constexpr int STG = CIT_SAMPLE_SCRATCH / 256 < 4 ? CIT_SAMPLE_SCRATCH / 256 : 4;
    static_assert(STG >= 1 && 64 * STG > CFR_ROW_HDR, "row staging fits the scratch");
    const int l = CFR_LANE;
    const int left = (CFR_EB - (run & (CFR_EB - 1))) * (int)(sizeof(CfrEdge) / 4);
    const int nw = left < STG * 64 ? left : STG * 64;
    uint32_t* stg = reinterpret_cast<uint32_t*>(cfr_ls.tmp);
    uint32_t v[STG];
#pragma unroll
    for (int q = 0; q < STG; q++) v[q] = l + 64 * q < nw ? s[l + 64 * q] : 0u;
    const uint32_t mw = v[0];
    k = (uint32_t)cfr_u((int)__builtin_amdgcn_readlane((int)mw, CFR_ROW_MASKW));
    const bool staged = CFR_ROW_HDR + (int)k <= nw;
    if (staged) {
#pragma unroll
      for (int q = 0; q < STG; q++)
        if (l + 64 * q < CFR_ROW_HDR + (int)k) stg[l + 64 * q] = v[q];
    }
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < (CFR_ROW_W + 63) / 64; j++) {
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)mw, 2 * j);
      const uint32_t hi = 2 * j + 1 < CFR_ROW_MASKW ? (uint32_t)__builtin_amdgcn_readlane((int)mw, 2 * j + 1) : 0u;
      const uint64_t m = ((uint64_t)hi << 32) | lo;
      const int d = 64 * j + l;
      if (d < CFR_ROW_W)
        dst[d] = ((m >> l) & 1) ? (staged ? stg[CFR_ROW_HDR + acc + cfr_mbcnt(m)] : s[CFR_ROW_HDR + acc + cfr_mbcnt(m)])
                                : base[d];
      acc += (uint32_t)__popcll(m);
    }
  }
#else
  {
    k = s[CFR_ROW_MASKW];
    uint32_t q = 0;
    for (int d = 0; d < CFR_ROW_W; d++)
      dst[d] = ((s[d >> 5] >> (d & 31)) & 1) ? s[CFR_ROW_HDR + q++] : base[d];
  }
#endif
  T.rl_node = id;
  T.rl_run = run;
  T.rl_k = (int)k;
  CFR_SYNC();
}
// Working row src as node id's row.  Raw rows: into the node's slot (returns
// -1).  Diff rows: a new run (or, given reuse_run, that run when the diff
// fits its reuse_k dwords) -- returns the run, -1 with T.err set when the
// diff is past row_cap or edge space ran out.
CIT_HD int row_store(CfrTree& T, int id, const uint32_t* src, int reuse_run = -1, int reuse_k = 0) {
  if (cfr_u(T.row_cap) == 0) {
    copy_row(T, row_of(T, id), src);
    return -1;
  }
  reuse_run = cfr_u(reuse_run);
  reuse_k = cfr_u(reuse_k);
  const uint32_t* base = cfr_base(T);
  int run = -1;
  CFR_SYNC();
#if CIT_WAVE
  {
    const int l = CFR_LANE;
    constexpr int NJ = (CFR_ROW_W + 63) / 64;
    uint32_t v[NJ];
    uint64_t m[NJ];
    uint32_t tot = 0;
#pragma unroll
    for (int j = 0; j < NJ; j++) {
      const int d = 64 * j + l;
      v[j] = d < CFR_ROW_W ? src[d] : 0u;
      m[j] = __ballot(d < CFR_ROW_W && v[j] != base[d]);
      tot += (uint32_t)__popcll(m[j]);
    }
    if (tot > (uint32_t)cfr_u(T.row_cap)) {
      T.err |= CIT_ERR_OVERFLOW | CIT_ERR_POOL_ROW;
    } else {
      const bool reuse = reuse_run >= 0 && cfr_row_slots((int)tot) <= cfr_row_slots(reuse_k);
      run = reuse ? reuse_run : cfr_u(alloc_edges(T, cfr_row_slots((int)tot)));
      if (run >= 0) {
        uint32_t* s = row_run_ptr(T, run);
        uint32_t acc = 0;
#pragma unroll
        for (int j = 0; j < NJ; j++) {
          if ((m[j] >> l) & 1) s[CFR_ROW_HDR + acc + cfr_mbcnt(m[j])] = v[j];
          acc += (uint32_t)__popcll(m[j]);
        }
        uint32_t h = l == CFR_ROW_MASKW ? tot : 0u;
#pragma unroll
        for (int w = 0; w < CFR_ROW_MASKW; w++) h = l == w ? (uint32_t)(m[w >> 1] >> (32 * (w & 1))) : h;
        if (l < CFR_ROW_HDR) s[l] = h;
        T.rl_node = id;
        T.rl_run = run;
        T.rl_k = reuse && reuse_k > (int)tot ? reuse_k : (int)tot;
      }
    }
  }
#else
  {
    uint32_t mask[CFR_ROW_MASKW] = {0};
    uint32_t k = 0;
    for (int d = 0; d < CFR_ROW_W; d++)
      if (src[d] != base[d]) {
        mask[d >> 5] |= 1u << (d & 31);
        k++;
      }
    if (k > (uint32_t)T.row_cap) {
      T.err |= CIT_ERR_OVERFLOW | CIT_ERR_POOL_ROW;
    } else {
      const bool reuse = reuse_run >= 0 && cfr_row_slots((int)k) <= cfr_row_slots(reuse_k);
      run = reuse ? reuse_run : alloc_edges(T, cfr_row_slots((int)k));
      if (run >= 0) {
        uint32_t* s = row_run_ptr(T, run);
        uint32_t q = 0;
        for (int d = 0; d < CFR_ROW_W; d++)
          if ((mask[d >> 5] >> (d & 31)) & 1) s[CFR_ROW_HDR + q++] = src[d];
        for (int w = 0; w < CFR_ROW_HDR; w++) s[w] = w < CFR_ROW_MASKW ? mask[w] : k;
        T.rl_node = id;
        T.rl_run = run;
        T.rl_k = reuse && reuse_k > (int)k ? reuse_k : (int)k;
      }
    }
  }
#endif
  CFR_SYNC();
  return run;
}
// Node id's row := working row src for a node that has one (its game changed:
// get_options' lazy state, a live choice): in place when row_load / row_store
// last handled id and the diff fits its run, else in a new run the record
// then points to.
CIT_HD void row_restore(CfrTree& T, int id, const uint32_t* src) {
  if (cfr_u(T.row_cap) == 0) {
    row_store(T, id, src);
    return;
  }
  const bool have = cfr_u(T.rl_node) == id;
  const int old = have ? cfr_u(T.rl_run) : -1;
  const int run = cfr_u(row_store(T, id, src, old, have ? cfr_u(T.rl_k) : 0));
  if (run >= 0 && run != old) {
    cfr_node(T, id).row = run;
    if (cfr_u(T.rn_node) == id) T.rn_run = run;
  }
}
// The tree's base row := working row src (its root game as first created), in
// the pool and (device) in LDS.
CIT_HD void row_set_base(CfrTree& T, const uint32_t* src) {
  if (cfr_u(T.row_cap) == 0) return;
  copy_row(T, cfr_glb(T.base_hbm), src);
#if CIT_WAVE
  copy_row(T, cfr_base_w(T), src);
#endif
}
// A read-only view of node n's game: the slot itself for raw rows, else the
// row decompressed into working row `which` (device) / the tree's scratch row.
CIT_HD const CitGame& row_view(CfrTree& T, int n, int which) {
  if (cfr_u(T.row_cap) == 0) return *reinterpret_cast<const CitGame*>(row_of(T, n));
#if CIT_WAVE
  row_load(T, w_row(T, which), n);
  return cfr_w(T, which);
#else
  (void)which;
  row_load(T, T.scratch_hbm, n);
  return *reinterpret_cast<const CitGame*>(T.scratch_hbm);
#endif
}

// ------------------------------------------------------------ numpy fp64
// np.sum of a 1-D float64 run (numpy pairwise_sum); `at(i)` yields element i.
template <class At>
CIT_HD double np_leaf_sum(At at, int lo, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; i++) r += at(lo + i);
    return r;
  }
  double r[8];
  for (int j = 0; j < 8; j++) r[j] = at(lo + j);
  int i = 8;
  for (; i < n - n % 8; i += 8)
    for (int j = 0; j < 8; j++) r[j] += at(lo + i + j);
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += at(lo + i);
  return res;
}
template <int D, class At>
CIT_HD double np_sum_rec(At at, int lo, int n, uint32_t& err) {
  if (n <= 128) return np_leaf_sum(at, lo, n);
  if constexpr (D == 0) {
    err |= CIT_ERR_OVERFLOW;
    return 0.0;
  } else {
    int n2 = n / 2;
    n2 -= n2 % 8;
    return np_sum_rec<D - 1>(at, lo, n2, err) + np_sum_rec<D - 1>(at, lo + n2, n - n2, err);
  }
}
template <class At>
CIT_HD double np_sum(At at, int n, uint32_t& err) { return np_sum_rec<5>(at, 0, n, err); }

// RandomState.choice(range(n), p=p) (legacy): ValueError -> err, returns -1.
// CFR_ERR_DIAG builds (tools/diag_cfr_errors.py) also record which check
// raised: 0x200 empty, 0x400 NaN / negative, 0x800 sum != 1.
#ifdef CFR_ERR_DIAG
#define CFR_DIAG(b) (b)
#else
#define CFR_DIAG(b) 0u
#endif
#if CIT_WAVE
__device__ __forceinline__ double cfr_readlane_f64(double v, int i) {
  uint64_t b = __builtin_bit_cast(uint64_t, v);
  uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, i);
  uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), i);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
#endif
template <class P>
CIT_HD int np_choice(CitMT& rng, P p, int n, uint32_t& err) {
  if (n <= 0) { err |= CIT_ERR_VALUE | CFR_DIAG(0x200u); return -1; }
#if CIT_WAVE
  if (n <= 64) {
    // p(i) once, on lane i; the Kahan check and the cumulative sums run in
    // index order as in numpy, and the n comparisons cum_i / cdf[-1] <= u
    // (one division each) on the lanes.
    const int l = (int)__lane_id();
    const double v = l < n ? p(l) : 0.0;
    if (__ballot(l < n && (v != v || v < 0))) { err |= CIT_ERR_VALUE | CFR_DIAG(0x400u); return -1; }
    double s = cfr_readlane_f64(v, 0), c = 0.0, cum = s, mycum = s;
    for (int i = 1; i < n; i++) {
      double vi = cfr_readlane_f64(v, i);
      double y = vi - c, t = s + y;
      c = (t - s) - y;
      s = t;
      cum = cum + vi;
      mycum = l == i ? cum : mycum;
    }
    if (fabs(s - 1.0) > CFR_ATOL) { err |= CIT_ERR_VALUE | CFR_DIAG(0x800u); return -1; }
    const double tot = cum;
    double u = mt_random(rng);
    uint64_t m = __ballot(l < n && mycum / tot <= u);
    int idx = m ? 64 - __clzll((long long)m) : 0;
    return idx < n ? idx : n - 1;
  }
#endif
  double s = p(0), c = 0.0;
  for (int i = 0; i < n; i++) {
    double v = p(i);
    if (v != v || v < 0) { err |= CIT_ERR_VALUE | CFR_DIAG(0x400u); return -1; }
    if (i) {
      double y = v - c, t = s + y;
      c = (t - s) - y;
      s = t;
    }
  }
  if (fabs(s - 1.0) > CFR_ATOL) { err |= CIT_ERR_VALUE | CFR_DIAG(0x800u); return -1; }
  double tot = 0.0;
  for (int i = 0; i < n; i++) tot = i ? tot + p(i) : p(0);
  double u = mt_random(rng);
  double cum = 0.0;
  int idx = 0;
  for (int i = 0; i < n; i++) {
    cum = i ? cum + p(i) : p(0);
    if (cum / tot <= u) idx = i + 1;
  }
  return idx < n ? idx : n - 1;
}
CIT_HD int np_choice_uniform(CitMT& rng, int n, uint32_t& err) {
  double q = n > 0 ? 1.0 / n : 0.0;
  return np_choice(rng, [q](int) { return q; }, n, err);
}

// ------------------------------------------------------- option equality
// A fingerprint of a card-type sequence (Card tuples compare by type, in order).
CIT_HD uint64_t type_seq_hash(uint64_t h, int t) { return (h ^ (uint64_t)(t + 1)) * 0x100000001B3ull; }

// The form an opponent child's option is stored and compared in
// (option.__eq__, option.py:14-15): list-valued attributes become type-sequence
// fingerprints, empty_option's next_gamestate its (state, player) (GameState.__eq__).
CIT_HD CitOpt opt_key(const CitOpt& o, const CitGame& g) {
  CitOpt k = o;
  const CitPlayer& P = g.pl[o.perp];
  uint64_t h = 0xcbf29ce484222325ull;
  switch (o.name) {
    case O_EMPTY:
      k.b = o.a == 0 ? 5 : g.nx_state;
      k.c = (uint8_t)(o.a == 0 ? o.perp : g.nx_pid);
      break;
    case O_DISCARD_AND_DRAW:
    case O_CARDINAL:
      for (int i = 0; i < P.n_hand && i < CIT_HAND_MASK_MAX; i++)
        if ((o.x >> i) & 1) h = type_seq_hash(h, card_type(P.hand[i]));
      k.x = h;
      break;
    case O_SCHOLAR_PICK:
      for (int i = 0; i < g.n_seven; i++) h = type_seq_hash(h, card_type(g.seven[i]));
      k.x = h;
      break;
    case O_GIVE_BACK_CARD: {   // dict equality: order-free over (pid, type)
      uint64_t acc = 0;
      for (int i = 0; i < o.b; i++)
        acc += type_seq_hash(type_seq_hash(h, g.seer_from[i]), card_type((int)((o.x >> (8 * i)) & 0xFF)));
      k.x = acc;
      break;
    }
    default:
      break;
  }
  return k;
}
CIT_HD bool opt_eq(const CitOpt& p, const CitOpt& q) {
  if (p.name != q.name || p.perp != q.perp || p.target != q.target) return false;
  switch (p.name) {
    case O_WHICH_CARD:
      return card_type(p.a) == card_type(q.a) && (p.b == CIT_NO_CARD) == (q.b == CIT_NO_CARD) &&
             (p.b == CIT_NO_CARD || card_type(p.b) == card_type(q.b)) && p.flags == q.flags;
    case O_BUILD:
      return card_type(p.a) == card_type(q.a) && p.c == q.c;
    case O_LAB: case O_LIGHTHOUSE: case O_MUSEUM: case O_WEAPON_STORAGE: case O_WARLORD: case O_MARSHAL:
      return card_type(p.a) == card_type(q.a);
    case O_TAKE_FROM_HAND:
      return p.flags == q.flags && card_type(p.a) == card_type(q.a) && (!(p.flags & OF_BUILD) || p.c == q.c);
    case O_DIPLOMAT:
      return card_type(p.a) == card_type(q.a) && card_type(p.b) == card_type(q.b) && p.c == q.c;
    case O_EMPTY:
      return p.b == q.b && p.c == q.c;
    case O_SCHOLAR_PICK:
      return card_type(p.a) == card_type(q.a) && p.x == q.x;
    case O_DISCARD_AND_DRAW:
      return p.x == q.x;
    case O_CARDINAL:
      return card_type(p.a) == card_type(q.a) && p.x == q.x && p.c == q.c && p.flags == q.flags;
    case O_GIVE_BACK_CARD:
      return p.b == q.b && p.x == q.x;
    default:
      return p.a == q.a && p.b == q.b && p.c == q.c && p.flags == q.flags && p.x == q.x;
  }
}

// take_from_hand builds: carry_out_wizard_take_from_hand overwrites the
// option's `replica` with the count already built (option_functions.py:317);
// the stored child option keeps the overwritten value.
CIT_HD void opt_mutate(CitOpt& o, const CitGame& g) {
  if (o.name == O_TAKE_FROM_HAND && (o.flags & OF_BUILD))
    o.c = (uint8_t)count_type(g.pl[o.perp].build, g.pl[o.perp].n_build, card_type(o.a));
}

// -------------------------------------------------------------- nodes
// CFRNode(game=w, parent, depth): skip_false_choice on working row `which`,
// then a new node whose row is that game.  `skipped`: the caller already ran
// skip_false_choice (the facade's CFRNode constructor), so it is not run
// again.  Returns the node id (-1 on error).
CFR_INL3 int cfr_node(CfrTree& T_in, int which, int parent, int depth, int skipped) {
  CfrTree& T = CFR_T(T_in);
  CIT_PROF_SCOPE(7);
  which = cfr_u(which);
  parent = cfr_u(parent);
  depth = cfr_u(depth);
  CitGame& w = cfr_w(T, which);
  uint32_t e = 0;
  int n = 0;
  {
  CIT_PROF_SCOPE(21);                  // skip_false_choice
#if CIT_WAVE
  // the count and the first option come back in registers (no LDS list)
  CitOpt first = mk(O_NUM_NAMES, 0);
  if (!cfr_u(skipped)) {
    eng_prepare(T, which);
    CfrFirst c = eng_first_upto2(T, which);
    n = cfr_u(c.n);
    e |= cfr_u(c.err);
    first = cfr_uopt(c.o);
  }
  int i = 0;
  bool done = false;
  while (n == 1 && !done && !e && !w.err) {
    i++;
    int win = cfr_u(eng_carry(T, which, first));
    done = win >= 0;
    eng_prepare(T, which);
    CfrFirst c = eng_first_upto2(T, which);
    n = cfr_u(c.n);
    e |= cfr_u(c.err);
    first = cfr_uopt(c.o);
    if (i > 100) done = true;
  }
#else
  if (!cfr_u(skipped)) {
    eng_prepare(T, which);
    CfrCnt c = cfr_ucnt(eng_list_upto2(T, which));
    n = c.n;
    e |= c.err;
  }
  int i = 0;
  bool done = false;
  while (n == 1 && !done && !e && !w.err) {
    i++;
    CitOpt o = cfr_uopt(cfr_lbuf(T)[0]);
    int win = cfr_u(eng_carry(T, which, o));
    done = win >= 0;
    eng_prepare(T, which);
    CfrCnt c = cfr_ucnt(eng_list_upto2(T, which));
    n = c.n;
    e |= c.err;
    if (i > 100) done = true;
  }
#endif
  }
  T.err |= e | w.err;
  if (T.n_nodes >= T.node_cap) { T.err |= CIT_ERR_OVERFLOW | CIT_ERR_POOL_CAP; return -1; }
  int id = T.n_nodes;
  if ((id & (CFR_NB - 1)) == 0) {       // the first node of a new block
    int b = cfr_take_block(cfr_glb(T.arena), 0);
    if (b < 0) { T.err |= CIT_ERR_OVERFLOW | CIT_ERR_POOL_ARENA; return -1; }
    cfr_nbt_at(T, id >> CFR_NB_SHIFT) = b;
  }
  T.n_nodes = id + 1;
  if (id == 0) row_set_base(T, w_row(T, which));   // the root: the tree's base row
  int run;
  {
    CIT_PROF_SCOPE(22);
    run = cfr_u(row_store(T, id, w_row(T, which)));   // its row (run: diff-row pools)
  }
  CfrNode& N = cfr_node(T, id);
#if CIT_WAVE
  {   // the header's 6 words and the 12 zero words of nv, one store per lane
    uint32_t hw[6];
    hw[0] = (uint32_t)parent;
    hw[1] = (uint32_t)-1;
    hw[2] = 0;                                   // n_children, edge_cap
    hw[3] = (uint32_t)(uint16_t)depth | ((uint32_t)(uint8_t)w.gs_pid << 16) | ((uint32_t)w.gs_state << 24);
    hw[4] = (uint32_t)((w.gs_state == 0 ? NF_ROLE_PICK : 0) | (w.terminal ? NF_TERMINAL : 0)) |
            ((uint32_t)(uint8_t)w.winner << 8) | 0xffff0000u;   // sib = -1 until the parent links it
    hw[5] = (uint32_t)run;
    const int l = CFR_LANE;
    uint32_t v = 0;
    for (int k = 0; k < 6; k++) v = l == k ? hw[k] : v;
    if (l < (int)(sizeof(CfrNode) / 4)) reinterpret_cast<uint32_t*>(&N)[l] = v;
  }
#else
  N.parent = parent;
  N.first_edge = -1;
  N.n_children = 0;
  N.edge_cap = 0;
  N.depth = (int16_t)depth;
  N.player = w.gs_pid;
  N.gs_state = (int8_t)w.gs_state;
  N.flags = (uint8_t)((w.gs_state == 0 ? NF_ROLE_PICK : 0) | (w.terminal ? NF_TERMINAL : 0));
  N.winner = w.winner;
  N.sib = -1;
  N.row = run;
  for (int k = 0; k < 6; k++) N.nv[k] = 0.0;
#endif
  return id;
}

// n edge records from the run at src to the run at dst (runs are contiguous)
CIT_HD void cfr_move_edges(const CfrTree& T, int dst, int src, int n) {
  const uint32_t* s = reinterpret_cast<const uint32_t*>(cfr_edge(T, src));
  uint32_t* d = reinterpret_cast<uint32_t*>(cfr_edge(T, dst));
  const int nw = n * (int)(sizeof(CfrEdge) / 4);
#if CIT_WAVE
  {   // up to 2 dwords per lane (n <= 8: 96 dwords), both loaded before the stores
    static_assert(8 * sizeof(CfrEdge) / 4 <= 128, "a moved run fits two dwords per lane");
    const int l = CFR_LANE;
    const uint32_t a = l < nw ? s[l] : 0u, b = l + 64 < nw ? s[l + 64] : 0u;
    if (l < nw) d[l] = a;
    if (l + 64 < nw) d[l + 64] = b;
  }
#else
  for (int i = 0; i < nw; i++) d[i] = s[i];
#endif
}
CIT_HD void init_edge(CfrEdge& E, const CitOpt& o, int child) {
  E.opt = o;
  E.child = child;
  E.R = E.S = E.CS = 0.0;
}

// ------------------------------------------------------------ expansion
// The parent's player and game state for a child's expansion (the
// determinization rule of expand_for_*: deep_mccfr.py:140,158): the cached
// current node's when the child was just reached from it.
CIT_HD void cfr_parent_info(const CfrTree& T, int par, int& player, int& state) {
  if (par >= 0 && cfr_u(T.cur_node) == par) {
    player = cfr_u(T.cur_player);
    state = cfr_u(T.cur_state);
  } else if (par >= 0) {
    const CfrNode& P = cfr_node(T, par);
    player = P.player;
    state = P.gs_state;
  } else {
    player = state = -1;
  }
}

CIT_NOINLINE void cfr_expand_role_pick(CfrTree& T_in, int n, int depth) {
  CfrTree& T = CFR_T(T_in);
  CIT_PROF_SCOPE(8);            // :102-131
  n = cfr_u(n);
  depth = cfr_u(depth) + 1;
  int f = alloc_edges(T, CFR_ROLE_EDGE_SLOTS);
  if (f < 0) return;
  CfrWide* W = cfr_wide(T, f);
  for (int r = 0; r < CFR_ROLE_CHILDREN; r++)
    for (int k = 0; k < 6; k++) W[r].R[k] = W[r].S[k] = W[r].CS[k] = 0.0;
  cfr_node(T, n).first_edge = f;
  cfr_node(T, n).edge_cap = CFR_ROLE_CHILDREN;
  CitGame& h = cfr_w(T, 1);
  // the node's row once into working row 0 (free during an expansion), then
  // an LDS copy per child instead of a pool read behind the last child's stores
  row_load(T, w_row(T, 0), n);
  for (int r = 0; r < CFR_ROLE_CHILDREN && !T.err; r++) {
    copy_row(T, w_row(T, 1), w_row(T, 0));
    CitOpt last = mk(O_NUM_NAMES, 0);
    int guard = 0;
    while (h.gs_state != 1 && !T.err) {
      eng_prepare(T, 1);
#if CIT_WAVE
      const CfrRegList c = eng_list_reg(T, 1);
      const int cn = cfr_u(c.n);
      T.err |= cfr_u(c.err);
      int k = cfr_with_np(T, [&](CitMT& r_) { return np_choice_uniform(r_, cn, T.err); });
      if (T.err) break;
      last = k < 64 ? cfr_uopt(cfr_reg_opt(c, k)) : cfr_uopt(eng_pick(T, 1, k));
#else
      CfrCnt c = cfr_ucnt(eng_list_lds(T, 1));
      T.err |= c.err;
      int k = cfr_with_np(T, [&](CitMT& r_) { return np_choice_uniform(r_, c.n, T.err); });
      if (T.err) break;
      last = k < CFR_LBUF ? cfr_uopt(cfr_lbuf(T)[k]) : cfr_uopt(eng_pick(T, 1, k));
#endif
      eng_carry(T, 1, last);
      T.err |= h.err;
      if (++guard > 64) T.err |= CIT_ERR_UNSUPPORTED;
    }
    if (T.err) return;
    int c = cfr_u(cfr_node(T, 1, n, depth, 0));
    if (c < 0) return;
    init_edge((*cfr_edge(T, f + r)), last, c);
    cfr_node(T, c).sib = (int16_t)r;
    cfr_node(T, n).n_children = (int16_t)(r + 1);
  }
}

CIT_NOINLINE void cfr_expand_own(CfrTree& T_in, int n, int par, int player, int depth) {
  CfrTree& T = CFR_T(T_in);
  CIT_PROF_SCOPE(9);                   // :133-151
  n = cfr_u(n);
  par = cfr_u(par);
  player = cfr_u(player);
  depth = cfr_u(depth) + 1;
  int pp, ps;
  cfr_parent_info(T, par, pp, ps);
  const bool sample = par < 0 || player != pp;
  const bool role_sample = par >= 0 && ps != 0;
  CitGame& g = cfr_w(T, 0);
  row_load(T, w_row(T, 0), n);
  eng_prepare(T, 0);
  CfrCnt lc = cfr_ucnt(eng_list(T, 0));
  int nl = lc.n;
  T.err |= lc.err | g.err;
  if (nl > CFR_OPT_CAP) T.err |= CIT_ERR_OVERFLOW;
  row_restore(T, n, w_row(T, 0));   // get_options mutated the node's game
  if (T.err) return;
  int cnt = nl;
  int f = alloc_edges(T, cnt);
  if (f < 0) return;
  CfrNode& N = cfr_node(T, n);
  N.first_edge = f;
  N.edge_cap = (int16_t)cnt;
  const CitOpt* ob = cfr_glb(T.optbuf);
  CitGame& h = cfr_w(T, 1);
#if CIT_WAVE
  // the first 64 options in registers (lane j: option j), one round of loads:
  // a load per child would wait behind the previous child's stores (gfx9's
  // vmcnt counts both)
  uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0;
  {
    const int l = CFR_LANE;
    if (l < cnt) {
      const uint4 v = *reinterpret_cast<const uint4*>(ob + l);
      q0 = v.x;
      q1 = v.y;
      q2 = v.z;
      q3 = v.w;
    }
  }
#endif
  for (int i = 0; i < cnt && !T.err; i++) {
    CitOpt o;
#if CIT_WAVE
    if (i < 64) {
      uint32_t w4[4] = {(uint32_t)__builtin_amdgcn_readlane((int)q0, i), (uint32_t)__builtin_amdgcn_readlane((int)q1, i),
                        (uint32_t)__builtin_amdgcn_readlane((int)q2, i), (uint32_t)__builtin_amdgcn_readlane((int)q3, i)};
      __builtin_memcpy(&o, w4, 16);
    } else {
      o = ob[i];
    }
#else
    o = ob[i];
#endif
    copy_row(T, w_row(T, 1), w_row(T, 0));
    if (sample) eng_sample(T, 1, T.orig, role_sample);
    opt_mutate(o, h);
    eng_carry(T, 1, o);
    T.err |= h.err;
    if (T.err) return;
    int c = cfr_u(cfr_node(T, 1, n, depth, 0));
    if (c < 0) return;
    init_edge((*cfr_edge(T, f + i)), o, c);
    cfr_node(T, c).sib = (int16_t)i;
    cfr_node(T, n).n_children = (int16_t)(i + 1);
  }
}

CIT_NOINLINE void cfr_expand_opponent(CfrTree& T_in, int n, int par, int player, int depth, int nch, int fe,
                                      int ecap) {
  CfrTree& T = CFR_T(T_in);
  CIT_PROF_SCOPE(10);              // :153-179
  n = cfr_u(n);
  par = cfr_u(par);
  player = cfr_u(player);
  depth = cfr_u(depth) + 1;
  nch = cfr_u(nch);
  fe = cfr_u(fe);
  ecap = cfr_u(ecap);
  int pp, ps;
  cfr_parent_info(T, par, pp, ps);
  row_load(T, w_row(T, 1), n);
  CitGame& h = cfr_w(T, 1);
  if (par < 0 || player != pp) eng_sample(T, 1, T.orig, par >= 0 && ps != 0);
  eng_prepare(T, 1);
#if CIT_WAVE
  const CfrRegList lc = eng_list_reg(T, 1);
  const int ln = cfr_u(lc.n);
  T.err |= cfr_u(lc.err) | h.err;
  int k = cfr_with_np(T, [&](CitMT& r_) { return np_choice_uniform(r_, ln, T.err); });
  if (T.err) return;
  CitOpt o = k < 64 ? cfr_uopt(cfr_reg_opt(lc, k)) : cfr_uopt(eng_pick(T, 1, k));
#else
  CfrCnt lc = cfr_ucnt(eng_list_lds(T, 1));
  T.err |= lc.err | h.err;
  int k = cfr_with_np(T, [&](CitMT& r_) { return np_choice_uniform(r_, lc.n, T.err); });
  if (T.err) return;
  CitOpt o = k < CFR_LBUF ? cfr_uopt(cfr_lbuf(T)[k]) : cfr_uopt(eng_pick(T, 1, k));
#endif
  opt_mutate(o, h);
  CitOpt key = opt_key(o, h);
  eng_carry(T, 1, o);
  T.err |= h.err;
  if (T.err) return;
#if CIT_WAVE
  if (nch > 0) {   // lane j compares child j's option: one round of loads
    const int l = CFR_LANE;
    bool hit = false;
    if (l < nch) hit = opt_eq((*cfr_edge(T, fe + l)).opt, key);
    if (__ballot(hit)) return;
  }
#else
  for (int j = 0; j < nch; j++)
    if (opt_eq((*cfr_edge(T, fe + j)).opt, key)) return;
#endif
  if (fe < 0 || nch == ecap) {
    // the children's edge run grows 1 -> 2 -> 4 -> 8 -> CFR_OPP_CHILDREN
    // (most opponent nodes only ever get one child): a full run moves to a
    // new one twice as long, the old one stays unused
    const int ncap = fe < 0 ? 1 : (2 * ecap < CFR_OPP_CHILDREN ? 2 * ecap : CFR_OPP_CHILDREN);
    const int nf = cfr_u(alloc_edges(T, ncap));
    if (nf < 0) return;
    if (fe >= 0) cfr_move_edges(T, nf, fe, nch);
    CfrNode& N = cfr_node(T, n);
    N.first_edge = nf;
    N.edge_cap = (int16_t)ncap;
    fe = nf;
  }
  int c = cfr_u(cfr_node(T, 1, n, depth, 0));
  if (c < 0) return;
  init_edge((*cfr_edge(T, fe + nch)), key, c);
  cfr_node(T, c).sib = (int16_t)nch;
  cfr_node(T, n).n_children = (int16_t)(nch + 1);
}

CIT_HD void cfr_expand(CfrTree& T, int n) {                        // :93-100
  CfrNode& N = cfr_node(T, n);
  const int state = N.gs_state, nch = N.n_children, player = N.player, par = N.parent, depth = N.depth,
            ecap = N.edge_cap;
  T.rn_node = n;
  T.rn_run = N.row;
  if (state == 0 && nch == 0) {
    N.flags |= NF_ROLE_PICK;
    cfr_expand_role_pick(T, n, depth);
  } else if (player == T.orig && nch == 0) {
    cfr_expand_own(T, n, par, player, depth);
  } else if (player != T.orig && nch < CFR_OPP_CHILDREN) {
    cfr_expand_opponent(T, n, par, player, depth, nch, N.first_edge, ecap);
  }
}

// ---------------------------------------------------------- strategies
CFR_INL4 void cfr_update_strategy(CfrTree& T_in, int n) {
  CfrTree& T = CFR_T(T_in);
  CIT_PROF_SCOPE(11);               // :292-319
  n = cfr_u(n);
  CfrNode& N = cfr_node(T, n);
  const int nch = N.n_children, fe = N.first_edge, flags = N.flags;
  T.cur_node = n;
  T.cur_fe = fe;
  T.cur_nch = nch;
  T.cur_flags = flags;
  T.cur_player = N.player;
  T.cur_state = N.gs_state;
  T.rn_node = n;
  T.rn_run = N.row;
  if (nch == 0) return;
  CfrEdge* E = cfr_edge(T, fe);
#if CIT_WAVE
  static_assert(CFR_SBUF <= 128, "two edges per lane");
  if (!(flags & NF_ROLE_PICK) && nch <= CFR_SBUF && cfr_ls.sbuf_on) {
    // lanes l and l + 64 own edges l and l + 64 (their R and CS loaded in one
    // round); the numpy sums run in their serial order over LDS copies (cbuf
    // keeps the normalised CS for cfr_choose)
    double* sb = cfr_ls.sbuf;
    double* cb = cfr_ls.cbuf;
    const int l = CFR_LANE;
    const bool h0 = l < nch, h1 = l + 64 < nch;
    double r0 = 0.0, c0 = 0.0, r1 = 0.0, c1 = 0.0;
    int k0 = -1, k1 = -1;
    if (h0) {
      r0 = E[l].R;
      c0 = E[l].CS;
      k0 = E[l].child;
    }
    if (h1) {
      r1 = E[l + 64].R;
      c1 = E[l + 64].CS;
      k1 = E[l + 64].child;
    }
    if (h0) sb[l] = exp((-r0) * CFR_LN13);
    if (h1) sb[l + 64] = exp((-r1) * CFR_LN13);
    CFR_SYNC();
    double tot = np_sum([sb](int i) { return sb[i]; }, nch, T.err);
    if (h0) {
      double v = tot > 0 ? sb[l] / tot : 1.0 / nch;
      E[l].S = v;
      cb[l] = c0 + v;
    }
    if (h1) {
      double v = tot > 0 ? sb[l + 64] / tot : 1.0 / nch;
      E[l + 64].S = v;
      cb[l + 64] = c1 + v;
    }
    CFR_SYNC();
    double cs = np_sum([cb](int i) { return cb[i]; }, nch, T.err);
    CFR_SYNC();
    if (h0) {
      double v = cb[l] / cs;
      E[l].CS = v;
      cb[l] = v;
    }
    if (h1) {
      double v = cb[l + 64] / cs;
      E[l + 64].CS = v;
      cb[l + 64] = v;
    }
    // the children's ids, loaded with R and CS, kept in the spent S copies for
    // the step to the chosen child (cfr_child)
    int* kids = reinterpret_cast<int*>(sb);
    if (h0) kids[l] = k0;
    if (h1) kids[l + 64] = k1;
    CFR_SYNC();
    cfr_ls.cnode = n;
    cfr_ls.cnch = nch;
    return;
  }
  cfr_ls.cnode = -1;
#endif
  if (!(flags & NF_ROLE_PICK)) {
    for (int a = 0; a < nch; a++) E[a].S = exp((-E[a].R) * CFR_LN13);
    double tot = np_sum([E](int i) { return E[i].S; }, nch, T.err);
    for (int a = 0; a < nch; a++) E[a].S = tot > 0 ? E[a].S / tot : 1.0 / nch;
    for (int a = 0; a < nch; a++) E[a].CS += E[a].S;
    double cs = np_sum([E](int i) { return E[i].CS; }, nch, T.err);
    for (int a = 0; a < nch; a++) E[a].CS = E[a].CS / cs;
  } else {
    // role pick: [6 players, nch] arrays; totals along players (axis 0, sequential)
    CfrWide* W = cfr_wide(T, fe);
    double tots[CFR_ROLE_CHILDREN];
    bool small = false;
    for (int a = 0; a < nch; a++) {
      double tot = 0.0;
      for (int p = 0; p < 6; p++) {
        W[a].S[p] = exp((-W[a].R[p]) * CFR_LN13);
        tot = p ? tot + W[a].S[p] : W[a].S[0];
      }
      tots[a] = tot;
      small |= tot <= 1e-8;
    }
    for (int a = 0; a < nch; a++)
      for (int p = 0; p < 6; p++) {
        double v = W[a].S[p] / tots[a];
        W[a].S[p] = small ? (tots[a] > 1e-8 ? v : 1.0 / 6) : v;
      }
    for (int a = 0; a < nch; a++)
      for (int p = 0; p < 6; p++) W[a].CS[p] += W[a].S[p];
    double cs = np_sum([W](int i) { return W[i / 6].CS[i % 6]; }, nch * 6, T.err);
    for (int a = 0; a < nch; a++)
      for (int p = 0; p < 6; p++) W[a].CS[p] = W[a].CS[p] / cs;
  }
}

// action_choice(live=False) (:67-91): returns the edge index within the node
CFR_INL4 int cfr_choose(CfrTree& T_in, int n) {
  CfrTree& T = CFR_T(T_in);
  CIT_PROF_SCOPE(12);
  n = cfr_u(n);
  int nch, fe, flags;
  if (cfr_u(T.cur_node) == n) {            // cfr_update_strategy(n) read the header
    nch = cfr_u(T.cur_nch);
    fe = cfr_u(T.cur_fe);
    flags = cfr_u(T.cur_flags);
  } else {
    const CfrNode& N = cfr_node(T, n);
    nch = N.n_children;
    fe = N.first_edge;
    flags = N.flags;
  }
  const CfrEdge* E = cfr_edge(T, fe < 0 ? 0 : fe);
  if (!(flags & NF_ROLE_PICK)) {
#if CIT_WAVE
    if (cfr_ls.cnode == n && cfr_ls.cnch == nch) {   // update_strategy(n) left CS in LDS
      const double* cb = cfr_ls.cbuf;
      double tot = np_sum([cb](int i) { return cb[i]; }, nch, T.err);
      return cfr_with_np(T, [&](CitMT& r_) { return np_choice(r_, [cb, tot](int i) { return cb[i] / tot; }, nch, T.err); });
    }
#endif
    double tot = np_sum([E](int i) { return E[i].CS; }, nch, T.err);
    return cfr_with_np(T, [&](CitMT& r_) { return np_choice(r_, [E, tot](int i) { return E[i].CS / tot; }, nch, T.err); });
  }
  const CfrWide* W = cfr_wide(T, fe);
  // weighted_average_strategy (:51-65) over turn_orders_for_roles of the node's game
  const CitGame& g = row_view(T, n, 1);
  if (nch > CFR_ROLE_CHILDREN) { T.err |= CIT_ERR_OVERFLOW; return -1; }
  double w[CFR_ROLE_CHILDREN];
  int hs = 0;
  for (int i = 0; i < CIT_NP; i++) hs += g.turn[i];
  for (int a = 0; a < nch; a++) {
    double acc = 0.0;
    for (int i = 0; i < CIT_NP; i++) acc += W[a].CS[g.turn[i]] * (double)(CIT_NP - i);
    w[a] = acc / (double)hs;
  }
  double s = np_sum([&w](int i) { return w[i < CFR_ROLE_CHILDREN ? i : 0]; }, nch, T.err);
  if (s == 0.0) return cfr_with_np(T, [&](CitMT& r_) { return np_choice_uniform(r_, nch, T.err); });
  return cfr_with_np(T, [&](CitMT& r_) { return np_choice(r_, [&w, s](int i) { return w[i] / s; }, nch, T.err); });
}

// ------------------------------------------------------------- backup
// (the node's header fields come from the caller's read of its record)
CFR_INL1 void cfr_update_regrets(CfrTree& T_in, int n, int nch, int fe, int flags, int player) {
  CfrTree& T = CFR_T(T_in);
  CIT_PROF_SCOPE(13);                // :231-256
  n = cfr_u(n);
  nch = cfr_u(nch);
  fe = cfr_u(fe);
  flags = cfr_u(flags);
  player = cfr_u(player);
  CfrEdge* E = cfr_edge(T, fe);
#if CIT_WAVE
  if (nch <= 64) {
    // lane a reads child a (one round of loads for all children); the max runs
    // in the serial order over the lanes' values, so NaN / tie handling and
    // every sum are the serial loop's
    const int a = CFR_LANE;
    if (!(flags & NF_ROLE_PICK)) {
      int p = player;
      double v = 0.0;
      if (a < nch) {
        const CfrNode& C = cfr_node(T, E[a].child);
        v = cfr_wp(C.nv, cfr_nv_sum(C.nv), C.flags, p);
      }
      double mx = cfr_readlane_f64(v, 0);
      for (int k = 1; k < nch; k++) {
        double x = cfr_readlane_f64(v, k);
        if (x > mx) mx = x;
      }
      if (a < nch) E[a].R += mx - v;
    } else if (a < nch) {
      CfrWide& W = cfr_wide(T, fe)[a];
      const CfrNode& C = cfr_node(T, E[a].child);
      const double cs = cfr_nv_sum(C.nv);
      const int cf = C.flags;
      double w[6];
      for (int p = 0; p < 6; p++) w[p] = cfr_wp(C.nv, cs, cf, p);
      double mx = w[0];
      for (int p = 1; p < 6; p++) mx = (mx != mx || w[p] != w[p]) ? NAN : (w[p] > mx ? w[p] : mx);
      for (int p = 0; p < 6; p++) W.R[p] += mx - w[p];
    }
    return;
  }
#endif
  auto wp_of = [&T](int c, int p) {
    const CfrNode& C = cfr_node(T, c);
    return cfr_wp(C.nv, cfr_nv_sum(C.nv), C.flags, p);
  };
  if (!(flags & NF_ROLE_PICK)) {
    int p = player;
    double mx = wp_of(E[0].child, p);
    for (int a = 1; a < nch; a++) {
      double v = wp_of(E[a].child, p);
      if (v > mx) mx = v;
    }
    for (int a = 0; a < nch; a++) E[a].R += mx - wp_of(E[a].child, p);
  } else {
    CfrWide* W = cfr_wide(T, fe);
    for (int a = 0; a < nch; a++) {
      double wp[6];
      for (int p = 0; p < 6; p++) wp[p] = wp_of(E[a].child, p);
      double mx = wp[0];
      for (int p = 1; p < 6; p++) mx = (mx != mx || wp[p] != wp[p]) ? NAN : (wp[p] > mx ? wp[p] : mx);
      for (int p = 0; p < 6; p++) W[a].R[p] += mx - wp[p];
    }
  }
}

// reward[6] is read before the walk (it may be a node's own pred array)
CIT_NOINLINE void cfr_backprop(CfrTree& T_in, int n, double r0, double r1, double r2, double r3, double r4,
                               double r5, int model) {
  CfrTree& T = CFR_T(T_in);
  CIT_PROF_SCOPE(14);   // :276-290
  n = cfr_u(n);
  const double reward[6] = {r0, r1, r2, r3, r4, r5};
  while (n >= 0) {
    CfrNode& N = cfr_node(T, n);
    double s0 = cfr_nv_sum(N.nv);
    if (T.training || s0 == 0.0 || !model)
      for (int k = 0; k < 6; k++) N.nv[k] += reward[k];
    if (!(N.flags & NF_BACKED)) N.flags |= NF_BACKED;     // winning_probabilities = nv / nv.sum() from now on
    if (N.n_children) cfr_update_regrets(T, n, N.n_children, N.first_edge, N.flags, N.player);
    n = N.parent;
  }
}
CIT_HD void cfr_backprop_arr(CfrTree& T, int n, const double* rw, bool model) {
  cfr_backprop(T, n, rw[0], rw[1], rw[2], rw[3], rw[4], rw[5], model ? 1 : 0);
}

// ---------------------------------------------------------------- drivers
// first_edge of node n: the cached current node's without a read.
CIT_HD int cfr_first_edge(const CfrTree& T, int n) {
  return cfr_u(T.cur_node) == n ? cfr_u(T.cur_fe) : cfr_node(T, n).first_edge;
}
// Child a of node n: from the ids cfr_update_strategy(n) loaded with the
// regrets (device LDS path), else from the edge record.
CIT_HD int cfr_child(const CfrTree& T, int n, int a) {
#if CIT_WAVE
  if (cfr_u(cfr_ls.cnode) == n && cfr_u(T.cur_node) == n)
    return cfr_u(reinterpret_cast<const int*>(cfr_ls.sbuf)[a]);
#endif
  return (*cfr_edge(T, cfr_first_edge(T, n) + a)).child;
}

// cfr_train(iters) (:187-205) on the game in working row 0 (the root's game:
// skip_false_choice mutates it, as the reference mutates the game passed to
// CFRNode), as resumable slices (the tree queue of simulate_games): phase
// CP_INIT builds the root; CP_RUN resumes iteration S.it at
// node S.cur.  A slice stops at an iteration boundary, after at least one
// iteration, once its budget is spent (device: `ticks` of the 100 MHz wall
// clock since `t0`; host: `iters_left` iterations), returning 1; 0 when the
// tree is done (S.phase == CP_DONE; S.root as cfr_train returns it).  The
// tree, streams and counters come out bit-identical to one cfr_train call.
struct CfrBudget {
  uint64_t t0, ticks;
  int iters_left;
};
CIT_HD bool cfr_budget_spent(CfrBudget& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return b.ticks && wall_clock64() - b.t0 >= b.ticks;
#else
  return b.iters_left > 0 && --b.iters_left == 0;
#endif
}
CIT_HD int cfr_train_slice(CfrTree& T_in, CfrState& S_in, int iters, bool root_skipped, CfrBudget& bud) {
  CfrTree& T = CFR_T(T_in);
  CfrState& S = CFR_S(S_in);
  if (cfr_u(S.phase) == CP_DONE) return 0;
  int root, n, it;
  if (cfr_u(S.phase) == CP_INIT) {
    root = cfr_u(cfr_node(T, 0, -1, 0, root_skipped ? 1 : 0));
    S.root = root;
    S.phase = CP_DONE;
    if (root < 0 || T.err) return 0;
    if (cfr_node(T, root).flags & NF_TERMINAL) return 0;
    cfr_expand(T, root);
    S.phase = CP_RUN;
    n = root;
    it = 0;
  } else {
    root = cfr_u(S.root);
    n = cfr_u(S.cur);
    it = cfr_u(S.it);
  }
  int first = it;
  for (; it < iters && !T.err; it++) {
    if (it > first && cfr_budget_spent(bud)) {
      S.cur = n;
      S.it = it;
      return 1;
    }
    cfr_update_strategy(T, n);
    int a = cfr_u(cfr_choose(T, n));
    if (T.err) break;
    n = cfr_u(cfr_child(T, n, a));
    if (cfr_node(T, n).flags & NF_TERMINAL) {
      double rw[6] = {0, 0, 0, 0, 0, 0};
      if (cfr_node(T, n).winner >= 0) rw[cfr_node(T, n).winner] = 1.0;
      cfr_backprop_arr(T, n, rw, false);
      cfr_update_strategy(T, n);
      n = root;
    } else {
      cfr_expand(T, n);
    }
  }
  if (!T.err) cfr_update_strategy(T, root);
  S.phase = CP_DONE;
  return 0;
}

// The whole search in one call.  Returns the root id.
CIT_HD int cfr_train(CfrTree& T, int iters, bool root_skipped = false) {
  CfrState S_local;
  CfrState& S = CFR_S(S_local);
  S.phase = CP_INIT;
  CfrBudget b = {0, 0, 0};
  cfr_train_slice(T, S_local, iters, root_skipped, b);
  return cfr_u(S.root);
}

// action_choice(live=True) at the root (:67-91; game.py:312-317 for a role pick).
CIT_NOINLINE CitOpt cfr_live_choice(CfrTree& T_in, int root) {
  CfrTree& T = CFR_T(T_in);
  CIT_PROF_SCOPE(15);
  root = cfr_u(root);
  CfrNode& N = cfr_node(T, root);
  if (!(N.flags & NF_ROLE_PICK)) {
    int a = cfr_u(cfr_choose(T, root));
    if (T.err || a < 0) return mk(O_NUM_NAMES, 0);
    return (*cfr_edge(T, N.first_edge + a)).opt;
  }
  CitGame& g = cfr_w(T, 0);
  row_load(T, w_row(T, 0), root);
  eng_prepare(T, 0);
  CfrCnt lc = cfr_ucnt(eng_list(T, 0));
  int nl = lc.n;
  T.err |= lc.err;
  int pid = g.gs_pid;
  const CfrWide* W = cfr_wide(T, N.first_edge);
  const CitOpt* ob = cfr_glb(T.optbuf);
  double sum = 0.0;
  for (int j = 0; j < nl; j++) sum += W[ob[j].a].S[pid];
  int j = cfr_with_np(T, [&](CitMT& r_) { return np_choice(r_, [&](int i) { return W[ob[i].a].S[pid] / sum; }, nl, T.err); });
  row_restore(T, root, w_row(T, 0));
  if (T.err || j < 0) return mk(O_NUM_NAMES, 0);
  return ob[j];
}

// ---------------------------------------------------------- cfr_pred (model)
// Deep-MCCFR with value-net leaves (deep_mccfr.py:207-229), resumable: a tree
// runs until a node deeper than max_depth needs its first leaf evaluation,
// writes that node's encode_game row to `feat` and suspends (returns 1); the
// caller evaluates every suspended tree's row in one batched MLP launch and
// calls again with `probs`.  Only evaluations whose result the reference
// uses are requested: pred_node_value is read only at depth > max_depth, and a
// node's prediction never changes (model_inference on the same game), so it is
// computed once per node (expand_role_pick's last inference: player 5).
CIT_HD void cfr_state_load(CfrTree& T, const CfrState& S) {
  T.n_nodes = S.n_nodes;
  T.n_edges = S.n_edges;
  T.n_eblk = (S.n_edges + CFR_EB - 1) >> CFR_EB_SHIFT;
  T.err = (uint32_t)S.err;
  T.carry_outs = (uint32_t)S.carry_outs;
  T.orig = S.orig;
}
CIT_HD void cfr_state_save(const CfrTree& T, CfrState& S) {
  S.n_nodes = T.n_nodes;
  S.n_edges = T.n_edges;
  S.err = (int32_t)T.err;
  S.carry_outs = (int32_t)T.carry_outs;
}

CIT_NOINLINE void cfr_write_feat(CfrTree& T_in, int n, float* feat) {
  CfrTree& T = CFR_T(T_in);
  n = cfr_u(n);
  int pid = (cfr_node(T, n).flags & NF_ROLE_PICK) ? 5 : -1;
  CFR_SYNC();
  // the whole team (identical stores): the engine's scans are wave-wide
  if (cfr_u(T.row_cap) == 0) {
    cit_encode_game(*reinterpret_cast<const CitGame*>(row_of(T, n)), cfr_glb(feat), pid);
  } else {
    row_load(T, w_row(T, 1), n);
    cit_encode_game(cfr_w(T, 1), cfr_glb(feat), pid);
  }
  CFR_SYNC();
}

#if CIT_WAVE
// The leaf evaluation inside the search kernel (cit_cfr_pred_fused): node n's
// encode_game row (player 5 for a role-pick node, as cfr_write_feat) straight
// into LDS and the single-row forward of cit_mlp_wave.h over it.  Its scratch
// (MLPW_R_FLOATS floats) overlays the working rows w0 / w1, the list buffer
// and the strategy copies: none of them carries anything across a leaf
// evaluation (a suspended tree resumes in a fresh launch with none of them),
// except the normalised CS of node cnode, which is dropped.  The
// probabilities end at cfr_mlp_lds() + MLPW_R_PROBS.
__device__ __forceinline__ mlpw_lds_t* cfr_mlp_lds() { return (mlpw_lds_t*)(&cfr_ls.w[0][0]); }
static_assert(offsetof(CfrLds, lbuf) == offsetof(CfrLds, w) + sizeof(((CfrLds*)0)->w) &&
                  offsetof(CfrLds, sbuf) == offsetof(CfrLds, lbuf) + sizeof(((CfrLds*)0)->lbuf) &&
                  offsetof(CfrLds, cbuf) == offsetof(CfrLds, sbuf) + sizeof(((CfrLds*)0)->sbuf) &&
                  offsetof(CfrLds, cbuf) + sizeof(((CfrLds*)0)->cbuf) - offsetof(CfrLds, w) >= 4 * MLPW_R_FLOATS,
              "the leaf evaluation's LDS scratch overlays w, lbuf, sbuf and cbuf");
static_assert(4 * MLPW_R_X >= CIT_GAME_BYTES, "a diff row loaded into w0 stays clear of the encoded row");
CIT_NOINLINE void cfr_leaf_eval(CfrTree& T_in, int n, const float* wave_w) {
  CIT_PROF_SCOPE(24);
  CfrTree& T = CFR_T(T_in);
  n = cfr_u(n);
  int pid = (cfr_node(T, n).flags & NF_ROLE_PICK) ? 5 : -1;
  mlpw_lds_t* R = cfr_mlp_lds();
  CFR_SYNC();
  for (int i = CFR_LANE; i < MLPW_IN + 2; i += CFR_TEAM) R[MLPW_R_X + i] = 0.0f;
  CFR_SYNC();
  float* x = (float*)(R + MLPW_R_X);
  // the node's row into w0 first (one round of loads): the featurizer's field
  // reads are then LDS reads, not a chain of dependent HBM loads
  if (cfr_u(T.row_cap) == 0)
    copy_row(T, w_row(T, 0), row_of(T, n));
  else
    row_load(T, w_row(T, 0), n);
  CFR_SYNC();
  cit_encode_game<float, false>(cfr_w(T, 0), x, pid);
  mlpw_forward(wave_w, R);
  cfr_ls.cnode = -1;
}
#endif

// One resumption.  Working row 0 must hold the lane's game when S.phase ==
// CP_INIT.  Returns 1 when suspended for an evaluation, 2 when `bud` ran out
// at an iteration boundary (S.phase stays CP_RUN: the next resumption goes
// on from S.cur / S.it exactly where this one stopped), 0 when done (S.phase
// == CP_DONE).  With `wave_w` (device; the wave-layout weights of
// cit_mlp_pack_wave) a leaf is evaluated in place (cfr_leaf_eval) and the
// tree never suspends: the same tree as suspending, the MLP being bitwise the
// same.
CIT_NOINLINE int cfr_pred_run(CfrTree& T_in, CfrState& S_in, int iters, int max_depth, const float* probs_in,
                              float* feat, CitOpt& chosen, bool root_skipped = false, CfrBudget* bud = nullptr,
                              const float* wave_w = nullptr) {
  CfrTree& T = CFR_T(T_in);
  CfrState& S = CFR_S(S_in);
  iters = cfr_u(iters);
  max_depth = cfr_u(max_depth);
  const float* probs = cfr_glb(probs_in);
  if (S.phase == CP_DONE) return 0;
  if (S.phase == CP_INIT) {
    S.orig = T.orig;
    if (!T.arena->pred) {          // pred_node_value needs the pool's side arrays (cit_cfr_arena_reset_fmt pred=1)
      T.err |= CIT_ERR_UNSUPPORTED;
      S.root = -1;
      S.phase = CP_DONE;
      chosen = mk(O_NUM_NAMES, 0);
      return 0;
    }
    int root = cfr_u(cfr_node(T, 0, -1, 0, root_skipped ? 1 : 0));
    S.root = root;
    S.it = 0;
    if (root < 0 || T.err || (cfr_node(T, root).flags & NF_TERMINAL)) {
      if (root >= 0 && !T.err) T.err |= CIT_ERR_VALUE;   // action_choice on a childless root raises
      S.phase = CP_DONE;
      chosen = mk(O_NUM_NAMES, 0);
      return 0;
    }
    cfr_expand(T, root);
    S.cur = root;
    S.phase = CP_RUN;
  } else if (S.phase == CP_WAIT) {
    int n = S.pending;
    CfrNode& N = cfr_node(T, n);
    double* pred = cfr_pred_of(T, n);
    for (int k = 0; k < 6; k++) pred[k] = (double)(5.0f * probs[k]);   // model_reward_weights * wp (float32)
    N.flags |= NF_PRED;
    cfr_backprop_arr(T, n, pred, true);
    cfr_update_strategy(T, n);
    S.cur = S.root;
    S.it++;
    S.phase = CP_RUN;
  }
  const int first = cfr_u(S.it);
  while (S.it < iters && !T.err) {
    if (bud && S.it > first && cfr_budget_spent(*bud)) return 2;
    cfr_update_strategy(T, S.cur);
    int a = cfr_u(cfr_choose(T, S.cur));
    if (T.err) break;
    int n = cfr_u(cfr_child(T, S.cur, a));
    CfrNode& N = cfr_node(T, n);
    if (N.depth > max_depth && !(N.flags & NF_TERMINAL)) {
      cfr_expand(T, n);
      if (T.err) break;
      if (!(cfr_node(T, n).flags & NF_PRED)) {
#if CIT_WAVE
        if (wave_w) {                    // evaluate in place (cit_cfr_pred_fused)
          cfr_leaf_eval(T, n, wave_w);
          const mlpw_lds_t* pr = cfr_mlp_lds() + MLPW_R_PROBS;
          double* pred = cfr_pred_of(T, n);
          for (int k = 0; k < 6; k++) pred[k] = (double)(5.0f * pr[k]);   // as the CP_WAIT resumption
          cfr_node(T, n).flags |= NF_PRED;
#ifdef CFR_DEBUG_POISON
          {   // (see CfrLds: nothing reads the overlaid buffers after an evaluation)
            uint32_t* o = &cfr_ls.w[0][0];
            const int nw = (int)((offsetof(CfrLds, cbuf) + sizeof(cfr_ls.cbuf) - offsetof(CfrLds, w)) / 4);
            CFR_SYNC();
            for (int i = CFR_LANE; i < nw; i += CFR_TEAM) o[i] = 0xDEADBEEFu;
            CFR_SYNC();
          }
#endif
        } else
#endif
        {
          cfr_write_feat(T, n, feat);
          S.pending = n;
          S.phase = CP_WAIT;
          return 1;
        }
      }
      cfr_backprop_arr(T, n, cfr_pred_of(T, n), true);
      cfr_update_strategy(T, n);
      S.cur = S.root;
    } else if (N.flags & NF_TERMINAL) {
      double rw[6] = {0, 0, 0, 0, 0, 0};
      if (N.winner >= 0) rw[N.winner] = 1.0;
      cfr_backprop_arr(T, n, rw, true);
      cfr_update_strategy(T, n);
      S.cur = S.root;
    } else {
      cfr_expand(T, n);
      S.cur = n;
    }
    S.it++;
  }
  if (!T.err) cfr_update_strategy(T, S.root);
  chosen = mk(O_NUM_NAMES, 0);
  if (!T.err) chosen = cfr_uopt(cfr_live_choice(T, S.root));
  S.phase = CP_DONE;
  return 0;
}

// ----------------------------------------------------- training targets
// get_all_targets (deep_mccfr.py:258-274) + build_train_targets (:321-345)
// over a finished tree, pre-order.  build_train_targets is always called with
// its default threshold (get_all_targets never passes its own, :268).
#define CFR_TARGET_THRESHOLD 15.0

CIT_HD bool cfr_is_target(const CfrTree& T, int n) {
  const CfrNode& N = cfr_node(T, n);
  if (N.n_children <= 0) return false;
  double s = 0.0;
  for (int k = 0; k < 6; k++) s += N.nv[k];     // integer-valued: order-free
  return s >= CFR_TARGET_THRESHOLD;
}

// Pre-order successor within the subtree of `top` through parent links and
// sibling indices (-1 after its last node).  With `prune`, the subtree of a
// node visited fewer than CFR_TARGET_THRESHOLD times is skipped: it holds no
// target when visit counts only grow towards the root (trees searched without
// a model: every backprop adds its reward to the whole path).
CIT_HD int cfr_preorder_next(const CfrTree& T, int n, int top, bool prune = false) {
  const CfrNode& N = cfr_node(T, n);
  if (N.n_children > 0) {
    bool skip = false;
    if (prune) {
      double s = 0.0;
      for (int k = 0; k < 6; k++) s += N.nv[k];
      skip = s < CFR_TARGET_THRESHOLD;
    }
    if (!skip) return (*cfr_edge(T, N.first_edge)).child;
  }
  for (;;) {
    const CfrNode& M = cfr_node(T, n);
    int p = M.parent;
    if (n == top || p < 0) return -1;
    const CfrNode& P = cfr_node(T, p);
    int j = M.sib;
    if (j + 1 < P.n_children) return (*cfr_edge(T, P.first_edge + j + 1)).child;
    n = p;
  }
}

// The tree of lane l in a node pool (nodes | edges | rows per tree), read-only use.
CIT_HD CfrTree cfr_tree_view(uint8_t* pool, int B, long l, int node_cap, int edge_cap) {
  CfrTree T;
  cfr_tree_bind(T, pool, B, l, node_cap, edge_cap);
  return T;
}

// Target modes: CFR_TGT_TREE = get_all_targets over the tree; CFR_TGT_ROOT =
// run_utils.create_target_strategy + encode_options_from_node at the root only
// (run_utils.py:89-109; generate_test_data.py:18-26), no threshold.  Flag
// CFR_TGT_PRUNE (with TREE): the trees were searched without a model, so the
// walk skips subtrees under the visit threshold (cfr_preorder_next).
enum { CFR_TGT_TREE = 0, CFR_TGT_ROOT = 1, CFR_TGT_PRUNE = 2 };

CIT_HD bool cfr_target_sel(const CfrTree& T, int n, int mode) {
  return (mode & CFR_TGT_ROOT) ? cfr_node(T, n).n_children > 0 : cfr_is_target(T, n);
}
CIT_HD int cfr_target_next(const CfrTree& T, int n, int top, int mode) {
  return (mode & CFR_TGT_ROOT) ? -1 : cfr_preorder_next(T, n, top, (mode & CFR_TGT_PRUNE) != 0);
}

// Number of targets and of their children (option rows).
CIT_HD void cfr_count_targets(const CfrTree& T, int root, int mode, int32_t& n_targets, int32_t& n_children) {
  n_targets = n_children = 0;
  if (root < 0) return;
  for (int n = root; n >= 0; n = cfr_target_next(T, n, root, mode))
    if (cfr_target_sel(T, n, mode)) {
      n_targets++;
      n_children += cfr_node(T, n).n_children;
    }
}

// Emit the targets from offsets (t0 targets, c0 children).  Per target k:
//   meta[k] = {lane, node, player (-1: the game's own), n_children, first child row}
//   feat[k][418] = encode_game (role-pick node: player randint(0, 5) of the tree's stream)
//   value[k][6] = node_value;  regret rows dist[c0 + j] (role-pick: cumulative_regrets[i]),
//   all ones when they sum to 0;  opt_feat[c0 + j][131] = encode_option of child j.
CIT_HD void cfr_emit_targets(CfrTree& T, CitMT& py, int root, int mode, int lane, int32_t t0, int32_t c0,
                             int32_t* meta, float* feat, double* value, double* dist, float* opt_feat) {
  if (root < 0) return;
  int32_t t = t0, c = c0;
  for (int n = root; n >= 0; n = cfr_target_next(T, n, root, mode)) {
    if (!cfr_target_sel(T, n, mode)) continue;
    const CfrNode& N = cfr_node(T, n);
    const CitGame& g = row_view(T, n, 1);
    const CfrEdge* E = cfr_edge(T, N.first_edge);
    int pid = -1, row = 0;
    if (N.flags & NF_ROLE_PICK) {
      pid = (int)mt_randbelow(py, 6u);
      row = pid;
    }
    int32_t* m = meta + 5 * (long)t;
    m[0] = lane;
    m[1] = n;
    m[2] = pid;
    m[3] = N.n_children;
    m[4] = c;
    if (feat) cit_encode_game(g, feat + (long)t * CIT_FEAT, pid);
    for (int k = 0; k < 6; k++) value[(long)t * 6 + k] = N.nv[k];
    const CfrWide* W = (N.flags & NF_ROLE_PICK) ? cfr_wide(T, N.first_edge) : nullptr;
    bool zero = true;
    for (int j = 0; j < N.n_children; j++) zero = zero && (W ? W[j].R[row] : E[j].R) == 0.0;
    for (int j = 0; j < N.n_children; j++) {
      dist[c + j] = zero ? 1.0 : (W ? W[j].R[row] : E[j].R);
      cit_encode_option(E[j].opt, g, opt_feat + (long)(c + j) * CIT_OPT_FEAT);
    }
    c += N.n_children;
    t++;
  }
}
