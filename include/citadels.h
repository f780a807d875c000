/* citadels.h — C ABI of libcitadels_hip.so, the MI355X (gfx950) Citadels
 * rules engine.  Plain pointers and sizes only; every buffer argument is a
 * DEVICE pointer (hipMalloc / torch CUDA tensor storage) and every call is
 * asynchronous on `stream`.  Return value: 0, or a hipError_t / -1 (bad args).
 *
 * The reference (davpat108/CITADELS_self_play) has no FFI: its hot path is a
 * Python object API.  Each entry point below replaces one of its calls, cited
 * file:line; the Python binding a maintainer would add is in INTEGRATION.md.
 *
 * Data (see citadels_self_play_amd/csrc/cit_core.h for the exact layout):
 *   games  : B rows of cit_game_bytes() bytes, one packed game per row.  A
 *            player's hand, just-drawn cards and museum share one 88-slot card
 *            area (hand first), so none of the reference's unbounded lists
 *            overflows before a player holds more cards than a game deals.
 *   mt     : uint32 [624][B] CPython MT19937 words, structure-of-arrays.
 *   mt_idx : uint32 [B] stream positions.  Lane l reproduces the reference run
 *            after `random.seed(seeds[l])`.
 *   seer   : uint64 [B][cit_seer_scratch_words()] scratch for the Seer's
 *            RNG-drawn give-back permutations (state 8).
 *   opts   : CitOption [B][max_opts] (16 B each, layout below).
 */
#ifndef CITADELS_H
#define CITADELS_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 16-byte option descriptor.  name = option id in the order of
 * game/option.py:34-45; perp = perpetrator; target = player or -1.
 * Per name: role_pick a=rank | gold_or_card a=0 gold,1 card |
 * which_card_to_keep a,b=cards (b=255: single) | blackmail_response a=0 pay,1 not |
 * reveal_* a=0 reveal,1 not | build a=card c=replica | empty_option a=0 fresh
 * GameState(5,perp), 1 the game's next_gamestate | finish_round flags bit0
 * next_witch bit1 crown | laboratory/lighthouse/museum/weapon_storage/warlord/
 * marshal a=card | magic_school a=suit | assassination/bewitching/steal a=rank |
 * magistrate_warrant a=real b,c=fakes | blackmail a=real b=fake | spy a=suit |
 * discard_and_draw x=hand-slot mask | take_from_hand a=card flags bit0 build
 * c=replica | give_back_card b=count, x=cards (byte i) | give_crown a=0 card,1
 * gold,2 nothing | cardinal_exchange a=card b=#given c=replica flags bit0
 * factory x=hand-slot mask | abbot_gold_or_card a=#religious b=#card |
 * navigator_gold_card a=0 4gold,1 4card | scholar_card_pick a=card |
 * diplomat_exchange a=choice b=give c=money_owed. */
typedef struct CitOption {
  uint8_t name, perp;
  int8_t target;
  uint8_t a, b, c, d, flags;
  uint64_t x;
} CitOption;

int cit_abi_version(void);              /* 9: the card-area self-test moved to the test-only library (tests/testkit.py); 8: cfr_pred as one launch with in-kernel leaf evaluation (cit_cfr_pred_fused, cit_mlp_*_wave); 7: diff rows as edge-slot runs (CfrNode.row), opponent edge runs that grow; 6: per-player card areas (hand / just-drawn / museum share 88 slots); 5: packed value-MLP path */
int cit_game_bytes(void);              /* row width of `games` */
int cit_seer_scratch_words(void);      /* uint64 words of seer scratch per lane */
int cit_layout(int* out, int n);       /* struct offsets, for binding self-checks */
/* random.seed(seeds[l]) (CPython init_by_array) or, numpy_style != 0,
 * np.random.seed(seeds[l]) (init_genrand) for every lane. */
int cit_mt_seed(uint32_t* mt, uint32_t* mt_idx, int B, const uint64_t* seeds, int numpy_style,
                hipStream_t stream);
/* n raw 32-bit outputs of every lane's stream into out[B][n] (RNG parity tests). */
int cit_mt_draw(uint32_t* mt, uint32_t* mt_idx, int B, int n, uint32_t* out, hipStream_t stream);

/* random.randrange(bound) (_randbelow) from every lane's stream into out[l]. */
int cit_randbelow(uint32_t* mt, uint32_t* mt_idx, int B, int bound, int32_t* out, hipStream_t stream);

/* Game(preset) + create_game's setup_round for every lane, with the lane's
 * stream freshly seeded from seeds[l]: replaces `random.seed(s); create_game()`
 * (run_utils.py:20-27, game/game.py:17-24,420-540,144-171).  preset=0 builds
 * the random-role Game() (game.py:491-520).  seeds == NULL continues each
 * lane's current stream instead (create_game() without a reseed). */
int cit_init(void* games, uint32_t* mt, uint32_t* mt_idx, int B, const uint64_t* seeds, int preset,
             hipStream_t stream);

/* Game.get_options_from_state() for every lane (game/game.py:415-418 ->
 * game/agent.py:50-83): writes the ordered option list to opts[l][0..) and its
 * length to n_opts[l] (n_opts may exceed max_opts; the list is then cut).
 * Mutates the game and consumes its stream exactly where the reference does
 * (scholar state 9, seer state 8). */
int cit_get_options(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, CitOption* opts,
                    int max_opts, int32_t* n_opts, hipStream_t stream);
/* The same, one game per lane (the one-game-per-lane execution model of
 * cit_rollout_random's games_per_block > 0, compiled without the wave-uniform
 * list scans): a parity check of the enumeration against cit_get_options. */
int cit_get_options_lanes(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, CitOption* opts,
                          int max_opts, int32_t* n_opts, hipStream_t stream);

/* len(Game.get_options_from_state()) for every lane, counted without
 * materialising the list (the random-role cardinal / magician lists run into
 * thousands; closed-form counts).  Same mutations and stream use as
 * cit_get_options. */
int cit_count_options(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int32_t* n_opts,
                      hipStream_t stream);

/* Game.sample_private_information(players[orig_player[l]], role_sample)
 * (game/game.py:215-339; called by deep_mccfr.py:140,158): MCCFR
 * determinization of every lane's game from that player's point of view,
 * drawing from the lane's CPython stream.  An orig_player outside 0..5 sets
 * the lane's IndexError bit. */
int cit_determinize(void* games, uint32_t* mt, uint32_t* mt_idx, int B, const int32_t* orig_player, int role_sample,
                    hipStream_t stream);

/* random.choice(options) for every lane (compare_to_random.py:38,
 * run_utils.py:39; Lib/random.py:371-373): k = _randbelow(n_opts[l]) drawn
 * from the lane's stream, chosen[l] = opts[l][k], k_out[l] = k.  An empty
 * list sets the lane's IndexError bit and k_out = -1 (the reference raises). */
int cit_random_choice(void* games, uint32_t* mt, uint32_t* mt_idx, int B, const CitOption* opts, int max_opts,
                      const int32_t* n_opts, CitOption* chosen, int32_t* k_out, hipStream_t stream);

/* option.carry_out(game) for every lane (game/option.py:118-122 ->
 * game/option_functions.py): chosen[l] must come from the lane's last
 * cit_get_options.  winner[l] = index of the returned winning Agent, or -1
 * for None/False. */
int cit_carry_out(void* games, uint32_t* mt, uint32_t* mt_idx, int B, const CitOption* chosen,
                  int32_t* winner, hipStream_t stream);

/* The fused random-policy step loop of compare_to_random.py:37-39 /
 * run_utils.py:37-41 (get_options -> random.choice -> carry_out) for up to
 * max_steps steps per lane (max_steps < 0: until a winner or an error).
 * steps[l] += steps taken; winner[l] as above.  games_per_block 0 (default):
 * one game per workgroup with wave-uniform code, row and MT19937 words in LDS;
 * 1..64: that many games per wavefront, one per lane. */
int cit_rollout_random(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int max_steps,
                       int games_per_block, int32_t* steps, int32_t* winner, hipStream_t stream);
/* The same rollout as a work queue over the B games: `grid` one-wave
 * workgroups (as many as the GPU holds at once: 8 per SIMD, 8192 on MI355X)
 * take game indices from the device counter *next (reset to 0 here) until
 * all are played, so the SIMD slot of a finished game takes the next game at
 * once (cit_rollout_random's launch lasts as long as its longest game).
 * Results are those of cit_rollout_random, game by game.  Replaces the same
 * step loop (compare_to_random.py:37-39, run_utils.py:37-41) over many
 * games in flight. */
int cit_rollout_queue(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int max_steps, int grid,
                      int32_t* steps, int32_t* winner, int32_t* next, hipStream_t stream);

/* --- featurizers and the value MLP ---------------------------------------- */

/* Game.encode_game() (game/game.py:91-128) for every lane: feat[B][418] fp32.
 * pid >= 0 encodes as if gamestate.player_id == pid (deep_mccfr.py:120-123). */
int cit_encode_games(const void* games, int B, int pid, float* feat, hipStream_t stream);
/* option.encode_option() (game/option.py:52-115): out[n][131] fp32 for
 * descriptor opts[i] generated on game lane_of[i]. */
int cit_encode_options(const void* games, const CitOption* opts, const int32_t* lane_of, int n, float* out,
                       hipStream_t stream);
/* ValueOnlyNN(418, 512) eval forward + square_and_normalize
 * (algorithms/models.py:17-24, train_utils.py:143-145): probs[M][6] (and
 * logits[M][6] if non-null).  BatchNorm folded into fc1/fc2 by the caller;
 * weights transposed to [in][out] (w1t [418][512], w2t [512][256],
 * w3t [256][128], w4t [128][6]).  fp32 MFMA, each output a k-ordered fmaf
 * chain from 0, then + bias. */
int cit_mlp_forward(const float* feat, int M, const float* w1t, const float* b1, const float* w2t, const float* b2,
                    const float* w3t, const float* b3, const float* w4t, const float* b4, float* probs, float* logits,
                    hipStream_t stream);
/* The same forward, bitwise equal, as three launches that spread fc1 and
 * fc2 over one workgroup per row tile x column group (a 1,024-row leaf
 * batch fills the chip instead of 64 CUs).  The weights are first packed
 * once by cit_mlp_pack into `packed` (cit_mlp_packed_bytes() bytes of device
 * memory, the MFMA operand order plus the biases); H1 / H2 go through
 * `work`, at least cit_mlp_work_bytes(M) bytes the call owns until it
 * completes on `stream`. */
size_t cit_mlp_packed_bytes(void);
int cit_mlp_pack(const float* w1t, const float* b1, const float* w2t, const float* b2, const float* w3t,
                 const float* b3, const float* w4t, const float* b4, void* packed, hipStream_t stream);
size_t cit_mlp_work_bytes(int M);
int cit_mlp_forward_packed(const float* feat, int M, const void* packed, float* probs, float* logits, void* work,
                           size_t work_bytes, hipStream_t stream);
/* The same forward, bitwise equal, for ONE row per 64-lane wavefront: lane l
 * runs the fmaf chains of output columns l, l + 64, ... on the VALU over the
 * "row layout" of the weights (cit_mlp_pack_wave into cit_mlp_wave_bytes()
 * bytes: per layer K rows, each lane's columns of a row contiguous, then the
 * biases and a flag word), reading only the rows whose input is non-zero (a
 * zero input leaves every finite chain bit-identical; a non-finite weight
 * clears the flag and every row is read).  This is the leaf evaluation
 * cit_cfr_pred_fused runs inside its search kernel (model_inference,
 * deep_mccfr.py:364-374); cit_mlp_forward_wave runs it one row per
 * workgroup (M workgroups). */
size_t cit_mlp_wave_bytes(void);
int cit_mlp_pack_wave(const float* w1t, const float* b1, const float* w2t, const float* b2, const float* w3t,
                      const float* b3, const float* w4t, const float* b4, void* packed, hipStream_t stream);
int cit_mlp_forward_wave(const float* feat, int M, const void* packed, float* probs, float* logits,
                         hipStream_t stream);

/* --- MCCFR (algorithms/deep_mccfr.py) ------------------------------------ */

/* Node pools.  A pool of B trees = B per-tree regions (cit_cfr_pool_bytes
 * each: int32 node-block and edge-block tables for node_cap / edge_cap,
 * padded to 16 B, then the tree's base row and a scratch row) followed by one
 * arena (cit_cfr_arena_bytes_fmt(node_blocks, edge_blocks, row_cap, pred)): a
 * 64-byte header, node blocks (CFR_NB CfrNode records of 72 B: header, the
 * row run, node_value f64[6]; with pred, CFR_NB pred_node_value f64[6]; with
 * row_cap 0, CFR_NB raw row slots of CIT_GAME_BYTES, 16-byte aligned) and
 * edge blocks (CFR_EB CfrEdge slots of 48 B), after a ring of free block ids
 * per kind.  A node's game row is raw (row_cap 0) or, with row_cap > 0, a
 * diff against the tree's base row (its root game as first created) stored
 * as a run of ceil((14 + k) / 12) edge slots from CfrNode.row: 14 header
 * words (a 388-bit mask of the k differing dwords, then k) and the k dwords
 * (row_cap a multiple of 4, <= 388; a row with more than row_cap differing
 * dwords stops the tree with CIT_ERR_OVERFLOW: search it again with raw
 * rows).  A tree takes blocks as it grows (a released block first), so the
 * arena holds what the trees use, not B worst cases; a tree that reaches its
 * own caps or finds the arena exhausted stops with CIT_ERR_OVERFLOW (search it
 * again with more room).  An own node reserves its children's edges, an
 * opponent node a run that grows as it fills (1, 2, 4, 8, 10 slots: a full
 * run moves to a longer one), a role-pick node 40 slots (10 edges + their
 * [6]-wide regret / strategy columns); an edge or row run never
 * straddles an edge block.  Sizes are 64-bit; -1 on a bad capacity (either
 * table longer than out[2] of cit_cfr_block_sizes). */
int64_t cit_cfr_pool_bytes(int node_cap, int edge_cap);
int64_t cit_cfr_arena_bytes_rows(int node_blocks, int edge_blocks, int row_cap);
int64_t cit_cfr_arena_bytes_fmt(int node_blocks, int edge_blocks, int row_cap, int pred);
int64_t cit_cfr_arena_bytes(int node_blocks, int edge_blocks);     /* = ..._rows(.., 0): raw rows
                                                                     (_rows: with pred_node_value room) */
/* out[3] = {CFR_NB nodes per node block, CFR_EB edges per edge block,
 * table entries a tree may hold}. */
int cit_cfr_block_sizes(int32_t* out);
/* Before a search (cit_cfr_decide, or the first cit_cfr_pred_step): every
 * table entry -1 and the arena empty with node_blocks / edge_blocks capacity
 * and rows of format row_cap.  pool must hold B * cit_cfr_pool_bytes +
 * cit_cfr_arena_bytes_rows(...) bytes.  cit_cfr_arena_reset = row_cap 0. */
int cit_cfr_arena_reset_rows(void* pool, int B, int node_cap, int edge_cap, int node_blocks, int edge_blocks,
                             int row_cap, hipStream_t stream);
/* The same with the node-record format too: pred != 0 gives every node room
 * for pred_node_value (the pools of cfr_pred searches; cit_cfr_arena_reset /
 * _rows reserve it), pred == 0 keeps records at 72 B (cfr_train searches,
 * simulate_game's tree queue). */
int cit_cfr_arena_reset_fmt(void* pool, int B, int node_cap, int edge_cap, int node_blocks, int edge_blocks,
                            int row_cap, int pred, hipStream_t stream);
int cit_cfr_arena_reset(void* pool, int B, int node_cap, int edge_cap, int node_blocks, int edge_blocks,
                        hipStream_t stream);
int cit_cfr_opt_cap(void);             /* CitOption scratch per tree (optbuf) */
/* Error bits of a search (stats[5*l+4]) beside the engine's CIT_ERR_* bits:
 * with CIT_ERR_OVERFLOW (0x1), which node-pool capacity ran out -- 0x1000 the
 * shared arena, 0x2000 the tree's node / edge caps (rows included), 0x4000 a diff row past row_cap.
 * Only these are worth a second search (with more room / raw rows); an
 * overflow without them is an engine list capacity (a player holding more
 * than 88 cards in hand + just-drawn + museum, or more than 32 HandKnowledge
 * entries) that no retry fixes. */

/* The config-3 position harness: k = random.randint(lo, hi) drawn from the
 * lane's stream, then k random-policy steps (stops at a winner). */
int cit_advance_random(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int lo, int hi,
                       int32_t* steps, hipStream_t stream);

/* `flags` of the search entry points: CIT_CFR_ROOT_SKIPPED = the lane's game
 * already went through CFRNode.__init__'s skip_false_choice
 * (cit_skip_false_choice), so the root node is built from it as is.
 * `orig_player` [B] = CFRNode's original_player_id per lane, or NULL for the
 * game's current player before the root's skip_false_choice (run_mccfr). */
#define CIT_CFR_ROOT_SKIPPED 1
/* CIT_CFR_STRATEGY_HBM (a checking aid): update_strategy keeps no LDS copy of
 * S / CS and runs over the edge records in HBM for every node (the path the
 * kernels take for nodes with more than 96 children); the trees are bitwise
 * the same. */
#define CIT_CFR_STRATEGY_HBM 2

/* CFRNode.skip_false_choice() (algorithms/deep_mccfr.py:37-49) on every lane,
 * as the CFRNode constructor runs it on the game it is given (:19-20):
 * single-option steps are played (at most 101) until a choice or a winner.
 * carried[l] (may be NULL) = carry_outs played. */
int cit_skip_false_choice(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int32_t* carried,
                          hipStream_t stream);

/* run_mccfr(game, max_iterations=iters) without a model (run_utils.py:74-87):
 * CFRNode(game) (deep_mccfr.py:8-49) + cfr_train(iters) (:187-205) +
 * action_choice(live=True) (:67-91) for every lane, one tree per workgroup.
 * The lane's games row becomes the root's game (the root's skip_false_choice
 * mutates the game it is given, as in the reference); mt/mt_idx are the
 * games' CPython stream, np_mt/np_idx numpy's global RandomState (seed them
 * with cit_mt_seed(numpy_style=1)).  chosen[l] = the decision; stats[5*l..] =
 * {root node, nodes, edges, carry_out calls, error bits}.  The tree stays in
 * pool (reset it with cit_cfr_arena_reset first) for inspection / target
 * extraction. */
int cit_cfr_decide(void* games, uint32_t* mt, uint32_t* mt_idx, uint32_t* np_mt, uint32_t* np_idx, uint64_t* seer,
                   int B, int iters, int flags, const int32_t* orig_player, void* pool, int node_cap, int edge_cap,
                   CitOption* optbuf, CitOption* chosen, int32_t* stats, hipStream_t stream);

/* cit_cfr_decide in resumable slices (simulate_games' tree queue): each call
 * advances every unfinished tree (state[l], B x cit_cfr_state_bytes(), zero
 * before its first slice) for about slice_ticks of the 100 MHz GPU wall clock
 * (0 = to the end), stopping at an iteration boundary; *running counts the
 * trees that stopped unfinished.  A finished tree's chosen[l], stats[5*l..]
 * and root game are written as cit_cfr_decide writes them; the tree, streams
 * and counters are bit-identical to one cit_cfr_decide call.  With
 * cit_cfr_arena_release a finished tree's lane can take the next tree (reset
 * its state to zero) while the others run on. */
int cit_cfr_train_slice(void* games, uint32_t* mt, uint32_t* mt_idx, uint32_t* np_mt, uint32_t* np_idx, uint64_t* seer,
                        int B, int iters, int flags, const int32_t* orig_player, void* pool, int node_cap, int edge_cap,
                        CitOption* optbuf, void* state, int64_t slice_ticks, CitOption* chosen, int32_t* stats,
                        int32_t* running, hipStream_t stream);
/* The blocks of trees lanes[0..n_lanes) (device array) back to the arena's
 * free rings and their tables cleared; no search may run meanwhile. */
int cit_cfr_arena_release(void* pool, int B, int node_cap, int edge_cap, const int32_t* lanes, int n_lanes,
                          hipStream_t stream);

/* Deep MCCFR with value-net leaves: cfr_pred(iters, max_depth)
 * (deep_mccfr.py:207-229) as run_mccfr runs it with a model and training=False
 * (run_utils.py:78-81), resumable.  Zero `state` (B x cit_cfr_state_bytes())
 * before the first call.  Each call advances every unfinished tree until it
 * needs its next leaf evaluation (that node's encode_game row goes to
 * feat[l][418] and *waiting is incremented) or finishes (chosen[l], games[l] =
 * root game).  Between calls evaluate feat with cit_mlp_forward or cit_mlp_forward_packed into
 * probs[l][6]; stop when a call leaves *waiting == 0.  Leaves are evaluated
 * once per node (the reference recomputes the same value). */
int cit_cfr_state_bytes(void);
int cit_cfr_pred_step(void* games, uint32_t* mt, uint32_t* mt_idx, uint32_t* np_mt, uint32_t* np_idx, uint64_t* seer,
                      int B, int iters, int flags, const int32_t* orig_player, int max_depth, void* pool,
                      int node_cap, int edge_cap, CitOption* optbuf, void* state, const float* probs, float* feat,
                      CitOption* chosen, int32_t* waiting, hipStream_t stream);
/* cit_cfr_pred_step with a time slice: a tree also stops, at an iteration
 * boundary, once slice_ticks of the 100 MHz GPU wall clock have passed since
 * the launch reached it (then *running is incremented; 0 = no limit, as
 * cit_cfr_pred_step).  Call again while *waiting or *running is non-zero,
 * evaluating feat first when *waiting is; the trees, streams and counters
 * are bit-identical to cit_cfr_pred_step's rounds.  A round then ends with a
 * slice instead of with its slowest tree. */
int cit_cfr_pred_slice(void* games, uint32_t* mt, uint32_t* mt_idx, uint32_t* np_mt, uint32_t* np_idx, uint64_t* seer,
                       int B, int iters, int flags, const int32_t* orig_player, int max_depth, void* pool,
                       int node_cap, int edge_cap, CitOption* optbuf, void* state, const float* probs, float* feat,
                       CitOption* chosen, int64_t slice_ticks, int32_t* waiting, int32_t* running,
                       hipStream_t stream);
/* cfr_pred(iters, max_depth) + the live choice (run_utils.py:78-81,
 * deep_mccfr.py:207-229) as ONE launch: every tree runs to its decision
 * without suspending, evaluating each leaf's encode_game row in its own
 * kernel with the single-row forward of cit_mlp_forward_wave over
 * `wave_weights` (cit_mlp_pack_wave).  The trees, streams, chosen[l], root
 * games and pool are bit-identical to cit_cfr_pred_step's rounds with the
 * MFMA forward; stats[5*l..] as cit_cfr_decide; state (may be NULL) receives
 * each tree's final CfrState (phase done).  The pool must be reset with
 * pred != 0 (a pred-less pool stops each tree with CIT_ERR_UNSUPPORTED). */
int cit_cfr_pred_fused(void* games, uint32_t* mt, uint32_t* mt_idx, uint32_t* np_mt, uint32_t* np_idx, uint64_t* seer,
                       int B, int iters, int flags, const int32_t* orig_player, int max_depth, void* pool,
                       int node_cap, int edge_cap, CitOption* optbuf, const void* wave_weights, void* state,
                       CitOption* chosen, int32_t* stats, hipStream_t stream);

/* compare_to_random.play_games' step loop (compare_to_random.py:16-35) on
 * every lane up to its next searched decision: seats in search_mask (bit p =
 * seat p; the reference searches for seats 0 and 1) decide by search when they
 * have more than one option, the others play random.choice, with the
 * reference's exact sequence of get_options calls.  status[l] = the seat to
 * decide next, -1 game over (or max_steps random steps; <0 = no cap), -2
 * error; steps[l] += random steps taken.  The caller runs the search for the
 * stopped lanes (cit_cfr_decide / cit_cfr_pred_step), applies cit_carry_out of
 * the chosen option and calls again. */
int cit_advance_policy(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int search_mask,
                       int max_steps, int32_t* status, int32_t* steps, hipStream_t stream);

/* ---- training-data generation (train_from_scratch.py:23-36 simulate_game) ---- */

/* create_a_random_game(max_move) (run_utils.py:55-73) on every lane, whose
 * CPython stream was seeded with cit_mt_seed (random.seed): k = randint(1,
 * max_move), create_game(), a random playout to the winner, games[-k].  The
 * stream continues from the end of the playout, as in the reference.  `ring`
 * is scratch of B * max_move * cit_game_bytes() bytes (the last max_move
 * snapshots of each lane).  steps[l] = steps into the game of the position,
 * -1 on error (lane err bits set). */
int cit_random_position(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int max_move,
                        uint32_t* ring, int32_t* steps, hipStream_t stream);

/* create_a_close_to_finished_game(game) (run_utils.py:29-53) on every lane's
 * created game (cit_init: create_game, same stream): k = randint(1, 30), a
 * random playout to the winner, then games[-k], games[-(k-1)], ... (Python
 * indexing) examined with get_options until one has >= 2 options (at most
 * 100).  `store`: B * cit_close_rows() * cit_game_bytes() bytes of scratch.
 * index[l] = snapshot index of the position, -1 on error. */
int cit_close_rows(void);
int cit_close_position(void* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, uint32_t* store,
                       int32_t* index, hipStream_t stream);

/* CFRNode.action_choice(live=False) (algorithms/deep_mccfr.py:67-91) at node
 * node[l] of the finished tree of lane l (the in-search sampler: a normal node
 * draws from cumulative_strategy / sum, a role-pick node from the pick-order
 * weighted average, with np.random.choice on the lane's numpy stream).
 * edge[l] = the chosen child's index within the node, or -1 with err[l] set
 * (ValueError: no children / invalid probabilities). */
int cit_cfr_action_choice(void* pool, int B, int node_cap, int edge_cap, const int32_t* node, uint32_t* np_mt,
                          uint32_t* np_idx, int32_t* edge, int32_t* err, hipStream_t stream);

/* get_all_targets (deep_mccfr.py:258-274) / build_train_targets (:321-345)
 * over the finished trees of cit_cfr_decide (same pool, roots = stats[:,0];
 * any node id gives that node's subtree, as node.get_all_targets does).
 * Threshold: build_train_targets' default 15 (get_all_targets does not pass
 * its own).  Pass 1: counts[l] = {targets, option rows}.  Pass 2 (exclusive
 * prefix sums of counts as offsets): per target k, meta[k] = {lane, node,
 * player override (-1 none), n_children, first option row}, feat[k][418]
 * (encode_game; a role-pick node draws randint(0,5) from the lane's CPython
 * stream), value[k][6] = node_value (f64), dist[row] = regret target (f64),
 * opt_feat[row][131] = encode_option of each child, rows in child order.
 * mode 0: the whole tree (get_all_targets).  mode 1: the root only, no
 * threshold (run_utils.create_target_strategy + encode_options_from_node,
 * run_utils.py:89-109, as generate_test_data.py:18-26 uses them); feat may be
 * NULL (generate_test_data encodes the position before the search).  mode 2:
 * mode 0 for trees searched without a model (cit_cfr_decide /
 * cit_cfr_train_slice), whose visit counts only grow towards the root: the
 * walk skips subtrees under the threshold (same output, a fraction of the
 * nodes read). */
int cit_cfr_target_count(void* pool, int B, int node_cap, int edge_cap, const int32_t* roots, int mode,
                         int32_t* counts, hipStream_t stream);
int cit_cfr_targets(void* pool, int B, int node_cap, int edge_cap, const int32_t* roots, int mode, uint32_t* mt,
                    uint32_t* mt_idx, const int32_t* offsets, int32_t* meta, float* feat, double* value, double* dist,
                    float* opt_feat, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif
