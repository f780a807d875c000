// TEST-ONLY device library (build/libcitadels_testkit.so, never loaded by the
// product path): kernels that exist to check the engine's wave paths against
// its host build, kept out of libcitadels_hip.so and include/citadels.h.
// tests/testkit.py binds it.
#include <hip/hip_runtime.h>

#define CIT_SHUFFLE_REG 1      // as the rollout unit (cit_hip.hip) builds the engine
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

}  // namespace

extern "C" {

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
