// Value-MLP leaf evaluation (algorithms/models.py ValueOnlyNN, eval mode, BN
// folded into fc1/fc2) on fp32 MFMA, plus the encode_game featurizer kernel.
//
//   wp = square_and_normalize(fc4(relu(fc3(relu(fc2'(relu(fc1'(x))))))))
//        (models.py:17-24, train_utils.py:143-145, deep_mccfr.py:364-374)
//
// One workgroup = 4 waves = a 32-row batch tile; every layer is a chain of
// v_mfma_f32_32x32x2_f32 (exact f32: a k-ordered fmaf chain per output,
// starting from 0, then + bias, then ReLU), activations staged in LDS,
// weights pre-transposed to [k][n] so a half-wave reads 128 contiguous bytes.
// fc4 (6 outputs) runs as one padded 32-column tile.
// One row per lane (the featurizer kernels): no wave-uniform engine scans.
#define CIT_NO_WAVE 1
#include <hip/hip_runtime.h>

#include "../../include/citadels.h"
#include "cit_engine.h"

#define MLP_IN 418
#define MLP_H1 512
#define MLP_H2 256
#define MLP_H3 128
#define MLP_OUT 6
#define MLP_ROWS 32
#define MLP_XS (MLP_IN + 3)      // odd LDS row strides: the 32 rows of a column read hit 32 banks
#define MLP_H1S (MLP_H1 + 1)
#define MLP_H2S (MLP_H2 + 1)
#define MLP_H3S (MLP_H3 + 1)

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

// out[r][n0 + j] for the wave's 32x32 tile: sum_k in[r][k] * WT[k][n], k in order
template <int K, int N>
__device__ __forceinline__ void tile_layer(const float* in, int in_s, const float* __restrict__ WT,
                                           const float* __restrict__ bias, float* out, int out_s, int n0, bool relu,
                                           int nvalid) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  f32x16 acc;
  for (int i = 0; i < 16; i++) acc[i] = 0.0f;
  const int col = n0 + r;
  const bool cv = col < nvalid;
#pragma unroll 4
  for (int kk = 0; kk < K / 2; kk++) {
    int k = 2 * kk + h;
    float a = in[r * in_s + k];
    float b = cv ? WT[(long)k * N + col] : 0.0f;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
  if (!cv) return;
  float bb = bias[col];
  for (int i = 0; i < 16; i++) {
    int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    float v = acc[i] + bb;
    out[row * out_s + col] = relu ? (v > 0.0f ? v : 0.0f) : v;
  }
}

__global__ __launch_bounds__(256) void k_mlp(const float* __restrict__ feat, int M, const float* __restrict__ w1t,
                                            const float* __restrict__ b1, const float* __restrict__ w2t,
                                            const float* __restrict__ b2, const float* __restrict__ w3t,
                                            const float* __restrict__ b3, const float* __restrict__ w4t,
                                            const float* __restrict__ b4, float* __restrict__ probs,
                                            float* __restrict__ logits) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* X = sm;                                   // [32][MLP_XS]   (later reused for H2)
  float* H1 = sm + MLP_ROWS * MLP_XS;              // [32][MLP_H1S]  (later reused for H3 / logits)
  float* H2 = X;
  float* H3 = H1;
  const int m0 = blockIdx.x * MLP_ROWS;
  const int nrows = min(MLP_ROWS, M - m0);
  const int wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < MLP_ROWS * MLP_IN; i += blockDim.x) {
    int r = i / MLP_IN, k = i - r * MLP_IN;
    X[r * MLP_XS + k] = r < nrows ? feat[(long)(m0 + r) * MLP_IN + k] : 0.0f;
  }
  __syncthreads();
  for (int t = wave; t < MLP_H1 / 32; t += 4) tile_layer<MLP_IN, MLP_H1>(X, MLP_XS, w1t, b1, H1, MLP_H1S, t * 32, true, MLP_H1);
  __syncthreads();
  for (int t = wave; t < MLP_H2 / 32; t += 4) tile_layer<MLP_H1, MLP_H2>(H1, MLP_H1S, w2t, b2, H2, MLP_H2S, t * 32, true, MLP_H2);
  __syncthreads();
  for (int t = wave; t < MLP_H3 / 32; t += 4) tile_layer<MLP_H2, MLP_H3>(H2, MLP_H2S, w3t, b3, H3, MLP_H3S, t * 32, true, MLP_H3);
  __syncthreads();
  float* L = X;                                    // [32][8] logits
  if (wave == 0) tile_layer<MLP_H3, MLP_OUT>(H3, MLP_H3S, w4t, b4, L, 8, 0, false, MLP_OUT);
  __syncthreads();
  if (threadIdx.x < nrows) {
    int r = threadIdx.x;
    float sq[MLP_OUT], s = 0.0f;
    for (int j = 0; j < MLP_OUT; j++) {
      float v = L[r * 8 + j];
      sq[j] = v * v;
      s += sq[j];
      if (logits) logits[(long)(m0 + r) * MLP_OUT + j] = v;
    }
    for (int j = 0; j < MLP_OUT; j++) probs[(long)(m0 + r) * MLP_OUT + j] = sq[j] / s;
  }
}

__global__ void k_encode(const uint32_t* __restrict__ games, int B, int pid, float* __restrict__ feat) {
  long l = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= B) return;
  const CitGame& g = *reinterpret_cast<const CitGame*>(games + l * (CIT_GAME_BYTES / 4));
  cit_encode_game(g, feat + l * CIT_FEAT, pid);
}

__global__ void k_encode_options(const uint32_t* __restrict__ games, const CitOpt* __restrict__ opts,
                                 const int32_t* __restrict__ lane_of, int n, float* __restrict__ out) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const CitGame& g = *reinterpret_cast<const CitGame*>(games + (long)lane_of[i] * (CIT_GAME_BYTES / 4));
  cit_encode_option(opts[i], g, out + i * CIT_OPT_FEAT);
}

size_t mlp_lds() { return (size_t)MLP_ROWS * (MLP_XS + MLP_H1S) * sizeof(float); }
bool g_mlp_attr = false;

}  // namespace

#define CHECK_LAUNCH()                       \
  do {                                       \
    hipError_t _e = hipGetLastError();       \
    return _e == hipSuccess ? 0 : (int)_e;   \
  } while (0)

extern "C" {

int cit_encode_games(const void* games, int B, int pid, float* feat, hipStream_t stream) {
  if (B <= 0 || !games || !feat || pid < -1 || pid > 5) return -1;
  hipLaunchKernelGGL(k_encode, dim3((B + 63) / 64), dim3(64), 0, stream, (const uint32_t*)games, B, pid, feat);
  CHECK_LAUNCH();
}

int cit_encode_options(const void* games, const CitOption* opts, const int32_t* lane_of, int n, float* out,
                       hipStream_t stream) {
  if (n < 0 || (n && (!games || !opts || !lane_of || !out))) return -1;
  if (!n) return 0;
  hipLaunchKernelGGL(k_encode_options, dim3((n + 63) / 64), dim3(64), 0, stream, (const uint32_t*)games,
                     (const CitOpt*)opts, lane_of, n, out);
  CHECK_LAUNCH();
}

int cit_mlp_forward(const float* feat, int M, const float* w1t, const float* b1, const float* w2t, const float* b2,
                    const float* w3t, const float* b3, const float* w4t, const float* b4, float* probs, float* logits,
                    hipStream_t stream) {
  if (M < 0 || (M && (!feat || !w1t || !b1 || !w2t || !b2 || !w3t || !b3 || !w4t || !b4 || !probs))) return -1;
  if (!M) return 0;
  if (!g_mlp_attr) {
    hipError_t e = hipFuncSetAttribute((const void*)k_mlp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlp_lds());
    if (e != hipSuccess) return (int)e;
    g_mlp_attr = true;
  }
  hipLaunchKernelGGL(k_mlp, dim3((M + MLP_ROWS - 1) / MLP_ROWS), dim3(256), mlp_lds(), stream, feat, M, w1t, b1, w2t,
                     b2, w3t, b3, w4t, b4, probs, logits);
  CHECK_LAUNCH();
}

}  // extern "C"
