// TEST-ONLY device library (build/libcitadels_testkit.so, never loaded by the
// product path): kernels that exist to check the engine's wave paths against
// its host build, kept out of libcitadels_hip.so and include/citadels.h.
// tests/testkit.py binds it.
#include <hip/hip_runtime.h>

#include "cit_area_test.h"

namespace {

constexpr int kRowW = CIT_GAME_BYTES / 4;

// cit_area_test.h's operation sequence on each lane's game (the wave paths of
// the card-area list operations; the host build runs the scalar ones).  One
// game per 64-lane workgroup, row staged in LDS, the stream read from HBM.
__global__ __launch_bounds__(64) void k_area_test(uint32_t* games, uint32_t* mt, uint32_t* idx, int B,
                                                 const uint64_t* seeds, int n_ops, uint32_t* log) {
  __shared__ __attribute__((aligned(16))) uint32_t row[kRowW];
  const long l = blockIdx.x;
  for (int i = threadIdx.x; i < kRowW; i += blockDim.x) row[i] = games[l * kRowW + i];
  __syncthreads();
  CitGame& g = *reinterpret_cast<CitGame*>(row);
  CitMT r;
  r.mt = mt + l;
  r.stride = B;
  r.pos = idx[l];
  r.coop = 0;
  r.win = 0;
  r.win_base = -1;
  uint64_t s = seeds[l] | 1ull;
  for (int i = 0; i < n_ops && !g.err; i++) {
    uint32_t v = 0;
    area_test_op(g, r, s, &v);
    if (threadIdx.x == 0) log[l * n_ops + i] = v;
  }
  if (threadIdx.x == 0) idx[l] = r.pos;
  __syncthreads();
  for (int i = threadIdx.x; i < kRowW; i += blockDim.x) games[l * kRowW + i] = row[i];
}

// Cycle microbenchmark of random.shuffle's building blocks on one wave with
// an LDS stream (the search's determinization deck: ~60 unknown cards):
// mode 0 the n - 1 draws alone, 1 draws + serial LDS swaps (the engine's coop
// path), 2 draws + swaps in two VGPRs (CIT_SHUFFLE_REG), 3 draws first, then
// each lane traces its final position back through the swaps (round 6's
// rejected variant).  out[blk] = clock64 cycles per shuffle, averaged over
// `reps`; sink[blk] keeps the results live.
__global__ __launch_bounds__(64) void k_bench_shuffle(int mode, int n, int reps, unsigned long long* out,
                                                       uint32_t* sink) {
  __shared__ uint32_t mts[CIT_MT_N];
  __shared__ uint8_t arr[128];
  const int l = (int)threadIdx.x;
  for (int i = l; i < CIT_MT_N; i += 64) mts[i] = 0x9e3779b9u * (uint32_t)(i + 1 + 977 * blockIdx.x);
  if (l < 128) arr[l] = (uint8_t)l;
  if (l + 64 < 128) arr[l + 64] = (uint8_t)(l + 64);
  __syncthreads();
  CitMT r;
  r.mt = mts;
  r.stride = 1;
  r.pos = 0;
  r.coop = CIT_MT_WINDOW;
  r.win = 0;
  r.win_base = -1;
  uint32_t acc = 0;
  mode = __builtin_amdgcn_readfirstlane(mode);
  n = __builtin_amdgcn_readfirstlane(n);
  const unsigned long long t0 = clock64();
  for (int rep = 0; rep < reps; rep++) {
    // the search keeps a stream's position and window base in SGPRs (its
    // arguments are re-uniformised); say so here too
    r.pos = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.pos);
    r.win_base = __builtin_amdgcn_readfirstlane(r.win_base);
    if (mode == 0) {
      for (int i = n - 1; i > 0; i--) acc += mt_randbelow(r, (uint32_t)(i + 1));
#if defined(__HIP_DEVICE_COMPILE__)
    } else if (mode == 4 || mode == 5) {
      // the draws through a queue of prefetched words: the readlanes of the
      // next Q words are issued back to back (independent VALU -> SGPR moves)
      // and the rejection loop consumes them from SGPRs
      const int Q = mode == 4 ? 4 : 8;
      uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0, q4 = 0, q5 = 0, q6 = 0, q7 = 0;
      int qn = 0;
      auto pop = [&]() -> uint32_t {
        if (qn == 0) {
          uint32_t i = r.pos;
          if (i >= CIT_MT_N) {
            mt_twist_wave((cit_lds_u32*)r.mt);
            r.win_base = -1;
            i = 0;
          }
          const int b = (int)(i & ~63u);
          if (b != r.win_base) {
            const int j = b + l;
            const uint32_t wj = ((const cit_lds_u32*)r.mt)[j < CIT_MT_N ? j : 0];
            r.win = mt_temper(j < CIT_MT_N ? wj : 0u);
            r.win_base = b;
          }
          const int o = (int)(i & 63u), lim = CIT_MT_N - b < 64 ? CIT_MT_N - b : 64;
          qn = lim - o < Q ? lim - o : Q;
          q0 = (uint32_t)__builtin_amdgcn_readlane((int)r.win, o);
          q1 = (uint32_t)__builtin_amdgcn_readlane((int)r.win, (o + 1) & 63);
          q2 = (uint32_t)__builtin_amdgcn_readlane((int)r.win, (o + 2) & 63);
          q3 = (uint32_t)__builtin_amdgcn_readlane((int)r.win, (o + 3) & 63);
          if (Q == 8) {
            q4 = (uint32_t)__builtin_amdgcn_readlane((int)r.win, (o + 4) & 63);
            q5 = (uint32_t)__builtin_amdgcn_readlane((int)r.win, (o + 5) & 63);
            q6 = (uint32_t)__builtin_amdgcn_readlane((int)r.win, (o + 6) & 63);
            q7 = (uint32_t)__builtin_amdgcn_readlane((int)r.win, (o + 7) & 63);
          }
          r.pos = i + (uint32_t)qn;
        }
        const uint32_t x = q0;
        q0 = q1; q1 = q2; q2 = q3; q3 = q4; q4 = q5; q5 = q6; q6 = q7;
        qn--;
        return x;
      };
      for (int i = n - 1; i > 0; i--) {
        const uint32_t nn = (uint32_t)(i + 1);
        const int kk = bit_length(nn);
        uint32_t v = pop() >> (32 - kk);
        while (v >= nn) v = pop() >> (32 - kk);
        acc += v;
      }
#endif
#if defined(__HIP_DEVICE_COMPILE__)
    } else if (mode == 7 || mode == 8) {
      // the batched draws alone (7), or followed by serial LDS swaps (8)
      int jv0 = 0, jv1 = 0;
      fy_draws_batched(r, n, jv0, jv1);
      if (mode == 7) {
        acc += (uint32_t)jv0 + (uint32_t)jv1;
      } else {
        for (int t = 0; t < n - 1; t++) {
          const int i = n - 1 - t;
          const int j = t < 64 ? __builtin_amdgcn_readlane(jv0, t) : __builtin_amdgcn_readlane(jv1, t - 64);
          const uint8_t x = arr[i];
          arr[i] = arr[j];
          arr[j] = x;
        }
      }
#endif
    } else if (mode == 6) {
      shuffle_arr(r, arr, n);   // the engine's coop path (CIT_SHUFFLE_BATCH: batched draws + traced swaps)
    } else if (mode == 1) {
      for (int i = n - 1; i > 0; i--) {
        const int j = (int)mt_randbelow(r, (uint32_t)(i + 1));
        const uint8_t t = arr[i];
        arr[i] = arr[j];
        arr[j] = t;
      }
    } else if (mode == 2) {
      int v0 = l < n ? arr[l] : 0, v1 = l + 64 < n ? arr[l + 64] : 0;
      for (int i = n - 1; i > 0; i--) {
        const int j = __builtin_amdgcn_readfirstlane((int)mt_randbelow(r, (uint32_t)(i + 1)));
        const int x = i < 64 ? __builtin_amdgcn_readlane(v0, i) : __builtin_amdgcn_readlane(v1, i - 64);
        const int y = j < 64 ? __builtin_amdgcn_readlane(v0, j) : __builtin_amdgcn_readlane(v1, j - 64);
        v0 = l == i ? y : (l == j ? x : v0);
        v1 = l + 64 == i ? y : (l + 64 == j ? x : v1);
      }
      if (l < n) arr[l] = (uint8_t)v0;
      if (l + 64 < n) arr[l + 64] = (uint8_t)v1;
    } else {
      int jv0 = 0, jv1 = 0;
      for (int t = 0; t < n - 1; t++) {
        const int j = __builtin_amdgcn_readfirstlane((int)mt_randbelow(r, (uint32_t)(n - t)));
        jv0 = l == t ? j : jv0;
        jv1 = l + 64 == t ? j : jv1;
      }
      int p0 = 0, p1 = 0;
      for (int u = n - 2; u >= 0; u--) {
        const int j = u < 64 ? __builtin_amdgcn_readlane(jv0, u) : __builtin_amdgcn_readlane(jv1, u - 64);
        const int i = n - 1 - u;
        const int s0 = p0 == i ? j : (p0 == j ? i : p0);
        p0 = l < i ? s0 : (l == i ? j : p0);
        const int s1 = p1 == i ? j : (p1 == j ? i : p1);
        p1 = l + 64 < i ? s1 : (l + 64 == i ? j : p1);
      }
      const int x0 = l < n ? arr[p0] : 0, x1 = l + 64 < n ? arr[p1] : 0;
      if (l < n) arr[l] = (uint8_t)x0;
      if (l + 64 < n) arr[l + 64] = (uint8_t)x1;
    }
  }
  const unsigned long long t1 = clock64();
  __syncthreads();
  if (l == 0) {
    out[blockIdx.x] = (t1 - t0) / (unsigned long long)(reps > 0 ? reps : 1);
    uint32_t h = acc;
    for (int i = 0; i < n; i++) h = h * 31u + arr[i];
    sink[blockIdx.x] = h;
  }
}

// The batched shuffle (shuffle_seq under CIT_SHUFFLE_BATCH) against the
// serial draws + swaps, from the same stream: block b copies words[b] (624
// untempered MT words) into LDS, starts at pos0[b] and shuffles an identity
// sequence of n `reps` times (crossing twists), recording each result
// (out[batched][b][rep][n]) and, after the last, the stream position and
// three further draws (tail[batched][b][4]).
__global__ __launch_bounds__(64) void k_shuffle_check(int n, int reps, const uint32_t* words, const int* pos0,
                                                     uint8_t* out, uint32_t* tail) {
  __shared__ uint32_t mts[CIT_MT_N];
  __shared__ uint8_t arr[128];
  const int l = (int)threadIdx.x, b = (int)blockIdx.x, B = (int)gridDim.x;
  for (int batched = 0; batched < 2; batched++) {
    for (int i = l; i < CIT_MT_N; i += 64) mts[i] = words[(long)b * CIT_MT_N + i];
    arr[l] = (uint8_t)l;
    arr[l + 64] = (uint8_t)(l + 64);
    __syncthreads();
    CitMT r;
    r.mt = mts;
    r.stride = 1;
    r.pos = (uint32_t)__builtin_amdgcn_readfirstlane(pos0[b]);
    r.coop = CIT_MT_WINDOW;
    r.win = 0;
    r.win_base = -1;
    const int nn = __builtin_amdgcn_readfirstlane(n);
    for (int rep = 0; rep < reps; rep++) {
      if (batched) {
        shuffle_arr(r, arr, nn);
      } else {
        for (int i = nn - 1; i > 0; i--) {
          const int j = (int)mt_randbelow(r, (uint32_t)(i + 1));
          const uint8_t t = arr[i];
          arr[i] = arr[j];
          arr[j] = t;
        }
      }
      __syncthreads();
      uint8_t* o = out + (((long)batched * B + b) * reps + rep) * nn;
      if (l < nn) o[l] = arr[l];
      if (l + 64 < nn) o[l + 64] = arr[l + 64];
      __syncthreads();
    }
    uint32_t* tl = tail + ((long)batched * B + b) * 4;
    const uint32_t p = r.pos;
    const uint32_t d0 = mt_randbelow(r, 1000u), d1 = mt_randbelow(r, 37u), d2 = mt_next(r);
    if (l == 0) {
      tl[0] = p;
      tl[1] = d0;
      tl[2] = d1;
      tl[3] = d2;
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" {

// k_shuffle_check over `blocks` one-wave workgroups
int citk_shuffle_check(int n, int reps, int blocks, const uint32_t* words, const int* pos0, uint8_t* out,
                       uint32_t* tail, hipStream_t stream) {
  if (n < 2 || n > 128 || reps < 1 || blocks < 1 || !words || !pos0 || !out || !tail) return -1;
  hipLaunchKernelGGL(k_shuffle_check, dim3(blocks), dim3(64), 0, stream, n, reps, words, pos0, out, tail);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// k_bench_shuffle over `blocks` one-wave workgroups (out / sink: [blocks])
int citk_bench_shuffle(int mode, int n, int reps, int blocks, unsigned long long* out, uint32_t* sink,
                       hipStream_t stream) {
  if (n < 2 || n > 128 || reps < 1 || blocks < 1 || !out || !sink) return -1;
  hipLaunchKernelGGL(k_bench_shuffle, dim3(blocks), dim3(64), 0, stream, mode, n, reps, out, sink);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// lane l runs a pseudo-random sequence of n_ops list operations (seeds[l]) on
// its game row (zeroed by the caller); log[l][i] records op i
int citk_area_test(void* games, uint32_t* mt, uint32_t* mt_idx, int B, const uint64_t* seeds, int n_ops,
                   uint32_t* log, hipStream_t stream) {
  if (B <= 0 || n_ops < 0 || !games || !mt || !mt_idx || !seeds || (n_ops && !log)) return -1;
  hipLaunchKernelGGL(k_area_test, dim3(B), dim3(64), 0, stream, (uint32_t*)games, mt, mt_idx, B, seeds, n_ops, log);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // extern "C"
