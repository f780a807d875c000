// Checking tool (not product code): the host build of the search under
// AddressSanitizer + UBSan, with the LDS buffer sizes of an occupancy
// experiment (e.g. -DCFR_LBUF=16 -DCFR_SBUF=32, the round-3 4-waves build),
// over the bench's configs 3 / 4 / 5 (cith_cfr_timed; config 4 with random
// value-net weights).  Build and run: tools/asan_cfr.sh.
//
//   asan_cfr <seconds per config> <config-5 iterations>
#include "../citadels_self_play_amd/csrc/cit_host.cpp"

#include <cstdio>
#include <random>

int main(int argc, char** argv) {
  const double secs = argc > 1 ? atof(argv[1]) : 20.0;
  const int it5 = argc > 2 ? atoi(argv[2]) : 2000;
  static const int dims[5] = {CIT_FEAT, 512, 256, 128, 6};
  std::vector<std::vector<float>> wv;
  std::mt19937 gen(0);
  std::normal_distribution<float> nd(0.0f, 0.05f);
  for (int layer = 0; layer < 4; layer++) {
    wv.emplace_back((size_t)dims[layer] * dims[layer + 1]);
    wv.emplace_back((size_t)dims[layer + 1]);
    for (auto& x : wv[wv.size() - 2]) x = nd(gen);
    for (auto& x : wv.back()) x = nd(gen);
  }
  const float* w[8];
  for (int i = 0; i < 8; i++) w[i] = wv[i].data();
  printf("CFR_LBUF %d CFR_SBUF %d\n", CFR_LBUF, CFR_SBUF);
  for (int config = 3; config <= 5; config++) {
    const int iters = config == 5 ? it5 : 200;
    const int nc = config == 5 ? (int)(3.5 * iters) + 512 : 4096, ec = config == 5 ? 4 * nc + 4096 : 5 * nc;
    long long dec = 0, carry = 0, errs = 0;
    double wall = 0;
    int rc = cith_cfr_timed(config, iters, 30000000ull + 1000000ull * config, secs, 1, nc, ec, w, &dec, &carry,
                            &errs, &wall);
    printf("config %d: rc %d, %lld decisions, %lld carry_outs, %lld error lanes, %.1f s\n", config, rc, dec, carry,
           errs, wall);
    fflush(stdout);
  }
  return 0;
}
