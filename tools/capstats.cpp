// Measurement tool (not product code): how long do the reference's unbounded
// lists get in config-5 trees?  The engine headers are built for the host
// (product capacities, or -DCIT_AREA_CAP=... wider), every length change
// reports itself (CIT_CAP_NOTE / CIT_AREA_NOTE in cit_engine.h), and `threads` host threads
// search simulate_game trees -- random.seed(s); create_a_random_game(100);
// np.random.seed(s); cfr_train(iters) (train_from_scratch.py:get_mccfr_targets,
// the bench's config 5) -- for seeds seed0 .. seed0+n-1.
//
//   capstats <seed0> <n> <iters> <threads>  ->  one JSON line per list kind
//   (max length over all trees, the seed reaching it, a histogram of per-tree
//   maxima) and per-tree lines for trees past round 3's fixed lists.
#define CIT_CAP_STATS 1
#include "../citadels_self_play_amd/csrc/cit_host.cpp"

#include <algorithm>
#include <cstdio>
#include <mutex>

enum { K_HAND, K_BUILD, K_JD, K_MUSEUM, K_AREA, K_MUSEUM_SUM, K_DECK, K_DISCARD, K_KH, K_KHPOOL, K_N };
static const char* kNames[K_N] = {"hand", "buildings", "just_drawn", "museum", "card_area", "museum_all_players",
                                  "deck", "discard", "hand_knowledge_entries", "hand_knowledge_cards"};
// the product row's capacities (cit_core.h; hand / just_drawn / museum share the card area)
static const int kProductCap[K_N] = {88, 16, 88, 88, 88, 6 * 88, 127, 88, 32, 244};
// round 3's fixed lists (hand 32, just_drawn 40, museum 16, discard 80, kh pool 252)
static const int kOldCap[K_N] = {32, 16, 40, 16, 104, 6 * 16, 127, 80, 32, 252};

static thread_local int tl_max[K_N];

static void note(int k, int n) {
  if (n > tl_max[k]) tl_max[k] = n;
}
// a card-area list changed length (cit_engine.h area_splice)
void cit_area_note(const CitGame& g, const CitPlayer& P) {
  note(K_HAND, P.n_hand);
  note(K_JD, P.n_jd);
  note(K_MUSEUM, P.n_museum);
  note(K_AREA, P.n_hand + P.n_jd + P.n_museum);
  int tot = 0;
  for (int q = 0; q < CIT_NP; q++) tot += g.pl[q].n_museum;
  note(K_MUSEUM_SUM, tot);
}
// an append to a plain list (put_card / deck_put / kh_append)
void cit_cap_note(const CitGame& g, const void* list, int n) {
  const uint8_t* a = (const uint8_t*)list;
  int k = -1;
  for (int p = 0; p < CIT_NP && k < 0; p++)
    if (a == g.pl[p].build) k = K_BUILD;
  if (k < 0) {
    if (a == g.deck) k = K_DECK;
    else if (a == g.discard) k = K_DISCARD;
    else if (a == (const uint8_t*)g.kh) k = K_KH;
    else if (a == g.kh_pool) k = K_KHPOOL;
  }
  if (k >= 0) note(k, n);
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: capstats seed0 n iters threads\n");
    return 2;
  }
  const uint64_t seed0 = strtoull(argv[1], 0, 10);
  const int n = atoi(argv[2]), iters = atoi(argv[3]), threads = atoi(argv[4]);
  const int node_cap = iters * 7 / 2 + 512 > 1024 ? iters * 7 / 2 + 512 : 1024, edge_cap = 4 * node_cap + 4096;
  const int nb = cfr_nblocks(node_cap), eb = cfr_eblocks(edge_cap);
  const int64_t pool_bytes = cfr_pool_bytes(node_cap, edge_cap) + cfr_arena_bytes(nb, eb);
  std::atomic<int> next(0);
  std::mutex mu;
  int gmax[K_N] = {0};
  uint64_t gseed[K_N] = {0};
  std::vector<int> hist[K_N];
  for (auto& h : hist) h.assign(256, 0);
  long long errs = 0, carry = 0;
  std::vector<int> per_tree_carry(n, 0);
  auto work = [&]() {
    CitGame* g = (CitGame*)aligned_alloc(16, CIT_GAME_BYTES);
    uint8_t* pool = (uint8_t*)malloc((size_t)pool_bytes);
    std::vector<uint32_t> mt(CIT_MT_N), npmt(CIT_MT_N);
    std::vector<uint64_t> seer(CIT_SEER_MAX);
    std::vector<CitOpt> optbuf(CFR_OPT_CAP);
    std::vector<uint32_t> ring(100 * (CIT_GAME_BYTES / 4));
    for (int i; (i = next.fetch_add(1)) < n;) {
      const uint64_t seed = seed0 + (uint64_t)i;
      for (int k = 0; k < K_N; k++) tl_max[k] = 0;
      CitMT r;
      r.mt = mt.data();
      r.stride = 1;
      r.pos = 0;
      r.coop = 0;
      mt_seed_cpython(r, seed);
      int st[5] = {-1, 0, 0, 0, 1};
      uint32_t idx = 0, npidx = 0;
      if (cit_random_position(*g, r, seer.data(), ring.data(), 100) >= 0) {
        idx = r.pos;
        CitMT q;
        q.mt = npmt.data();
        q.stride = 1;
        q.pos = 0;
        q.coop = 0;
        mt_init_genrand(q, (uint32_t)seed);
        npidx = q.pos;
        cith_cfr_arena_reset(pool, 1, node_cap, edge_cap, nb, eb);
        CitOpt chosen;
        cith_cfr_decide(g, mt.data(), &idx, npmt.data(), &npidx, seer.data(), 1, iters, 0, pool, node_cap, edge_cap,
                        optbuf.data(), &chosen, st);
      }
      std::lock_guard<std::mutex> lk(mu);
      bool past = false;
      for (int k = 0; k < K_N; k++) {
        hist[k][tl_max[k] < 255 ? tl_max[k] : 255]++;
        if (tl_max[k] > gmax[k]) {
          gmax[k] = tl_max[k];
          gseed[k] = seed;
        }
        past |= tl_max[k] > kOldCap[k];
      }
      errs += st[4] != 0;
      carry += st[3];
      per_tree_carry[i] = st[3];
      if (past) {
        printf("{\"seed\": %llu, \"err\": %d, \"carry_outs\": %d", (unsigned long long)seed, st[4], st[3]);
        for (int k = 0; k < K_N; k++) printf(", \"%s\": %d", kNames[k], tl_max[k]);
        printf("}\n");
        fflush(stdout);
      }
    }
    free(pool);
    free(g);
  };
  std::vector<std::thread> ts;
  for (int t = 1; t < threads; t++) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
  for (int k = 0; k < K_N; k++) {
    printf("{\"list\": \"%s\", \"max\": %d, \"seed\": %llu, \"product_cap\": %d, \"per_tree_max_hist\": {", kNames[k],
           gmax[k], (unsigned long long)gseed[k], kProductCap[k]);
    bool first = true;
    for (int v = 0; v < 256; v++)
      if (hist[k][v]) {
        printf("%s\"%d\": %d", first ? "" : ", ", v, hist[k][v]);
        first = false;
      }
    printf("}}\n");
  }
  std::vector<int> sc = per_tree_carry;
  std::sort(sc.begin(), sc.end());
  auto pct = [&](double q) { return sc[(size_t)(q * (sc.size() - 1))]; };
  printf("{\"trees\": %d, \"iters\": %d, \"error_trees\": %lld, \"carry_outs\": %lld, \"carry_outs_per_tree\": "
         "{\"p10\": %d, \"p50\": %d, \"p90\": %d, \"p99\": %d, \"max\": %d}}\n",
         n, iters, errs, carry, pct(0.1), pct(0.5), pct(0.9), pct(0.99), sc.back());
  return 0;
}
