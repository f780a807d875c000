// Value-MLP leaf evaluation (algorithms/models.py ValueOnlyNN, eval mode, BN
// folded into fc1/fc2) on fp32 MFMA, plus the encode_game featurizer kernel.
//
//   wp = square_and_normalize(fc4(relu(fc3(relu(fc2'(relu(fc1'(x))))))))
//        (models.py:17-24, train_utils.py:143-145, deep_mccfr.py:364-374)
//
// One workgroup = 16 waves = a 16-row batch tile; every layer is a chain of
// v_mfma_f32_16x16x4_f32 (exact f32: a k-ordered fmaf chain per output,
// starting from 0, then + bias, then ReLU), activations staged in LDS,
// weights pre-transposed to [k][n] so a quarter-wave reads 64 contiguous bytes.
// fc4 (6 outputs) runs as one padded 16-column tile.
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
#define MLP_ROWS 16
#define MLP_XS (MLP_IN + 3)      // odd LDS row strides: the 16 rows of a column read hit 16 banks
#define MLP_H1S (MLP_H1 + 1)
#define MLP_H2S (MLP_H2 + 1)
#define MLP_H3S (MLP_H3 + 1)


namespace {

// NT 16x16 output tiles of one wave, columns n0 + 16 t + (0..15):
// out[r][c] = sum_k in[r][k] * WT[k][c], k in order: one
// v_mfma_f32_16x16x4_f32 per 4 k (lane l holds A[l % 16][4 kk + l / 16] and
// B[4 kk + l / 16][l % 16]; the f32 MFMA accumulates its k in order, exactly
// an fmaf chain).  K is padded to a multiple of 4 with zeros (a zero product
// leaves the accumulator bit-identical: it is never -0).  The NT tiles'
// chains interleave, and each weight column is read MLP_PF steps ahead (a
// register ring) so the per-lane 4-byte L2 loads overlap the MFMAs.
#define MLP_PF 6
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int K, int N, int NT>
__device__ __forceinline__ void tile16_layer(const float* in, int in_s, const float* __restrict__ WT,
                                             const float* __restrict__ bias, float* out, int out_s, int n0,
                                             bool relu, int nvalid) {
  constexpr int KK = (K + 3) / 4;
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  f32x4 acc[NT];
  int col[NT];
  bool cv[NT];
#pragma unroll
  for (int t = 0; t < NT; t++) {
    for (int i = 0; i < 4; i++) acc[t][i] = 0.0f;
    col[t] = n0 + 16 * t + r;
    cv[t] = col[t] < nvalid;
  }
  auto wgt = [&](int t, int kk) -> float {
    int k = 4 * kk + q;
    return (k < K && cv[t]) ? WT[(long)k * N + col[t]] : 0.0f;
  };
  const float* ip = in + r * in_s + q;
  float b[MLP_PF][NT];
#pragma unroll
  for (int i = 0; i < MLP_PF; i++)
#pragma unroll
    for (int t = 0; t < NT; t++) b[i][t] = i < KK ? wgt(t, i) : 0.0f;
  for (int k0 = 0; k0 < KK; k0 += MLP_PF) {
#pragma unroll
    for (int i = 0; i < MLP_PF; i++) {
      const int kk = k0 + i;
      if (kk < KK) {
        float a = 4 * kk + q < K ? ip[4 * kk] : 0.0f;
#pragma unroll
        for (int t = 0; t < NT; t++) {
          float bn = kk + MLP_PF < KK ? wgt(t, kk + MLP_PF) : 0.0f;
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[i][t], acc[t], 0, 0, 0);
          b[i][t] = bn;
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; t++) {
    if (!cv[t]) continue;
    float bb = bias[col[t]];
    for (int i = 0; i < 4; i++) {
      int row = 4 * q + i;
      float v = acc[t][i] + bb;
      out[row * out_s + col[t]] = relu ? (v > 0.0f ? v : 0.0f) : v;
    }
  }
}

// One workgroup = 16 waves on a 16-row batch tile (a 4096-row call is 256
// workgroups: every CU): layer 1's 32 column tiles two per wave, then one
// per wave for layers 2-3 (16 / 8 tiles) and wave 0 for the 6 logits.
#define MLP_WAVES 16
__global__ __launch_bounds__(64 * MLP_WAVES) void k_mlp(const float* __restrict__ feat, int M,
                                                       const float* __restrict__ w1t, const float* __restrict__ b1,
                                                       const float* __restrict__ w2t, const float* __restrict__ b2,
                                                       const float* __restrict__ w3t, const float* __restrict__ b3,
                                                       const float* __restrict__ w4t, const float* __restrict__ b4,
                                                       float* __restrict__ probs, float* __restrict__ logits) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* X = sm;                                   // [16][MLP_XS]   (later reused for H2)
  float* H1 = sm + MLP_ROWS * MLP_XS;              // [16][MLP_H1S]  (later reused for H3 / logits)
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
  tile16_layer<MLP_IN, MLP_H1, 2>(X, MLP_XS, w1t, b1, H1, MLP_H1S, wave * 32, true, MLP_H1);
  __syncthreads();
  tile16_layer<MLP_H1, MLP_H2, 1>(H1, MLP_H1S, w2t, b2, H2, MLP_H2S, wave * 16, true, MLP_H2);
  __syncthreads();
  if (wave < MLP_H3 / 16) tile16_layer<MLP_H2, MLP_H3, 1>(H2, MLP_H2S, w3t, b3, H3, MLP_H3S, wave * 16, true, MLP_H3);
  __syncthreads();
  float* L = X;                                    // [16][8] logits
  if (wave == 0) tile16_layer<MLP_H3, MLP_OUT, 1>(H3, MLP_H3S, w4t, b4, L, 8, 0, false, MLP_OUT);
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
  hipLaunchKernelGGL(k_mlp, dim3((M + MLP_ROWS - 1) / MLP_ROWS), dim3(64 * MLP_WAVES), mlp_lds(), stream, feat, M, w1t, b1, w2t,
                     b2, w3t, b3, w4t, b4, probs, logits);
  CHECK_LAUNCH();
}

}  // extern "C"
