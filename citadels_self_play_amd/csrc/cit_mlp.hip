// Value-MLP leaf evaluation (algorithms/models.py ValueOnlyNN, eval mode, BN
// folded into fc1/fc2) on fp32 MFMA, plus the encode_game featurizer kernel.
//
//   wp = square_and_normalize(fc4(relu(fc3(relu(fc2'(relu(fc1'(x))))))))
//        (models.py:17-24, train_utils.py:143-145, deep_mccfr.py:364-374)
//
// Every layer is a chain of v_mfma_f32_16x16x4_f32 per 16x16 output tile
// (exact f32: a k-ordered fmaf chain per output, starting from 0, then + bias,
// then ReLU), inputs staged in LDS, weights pre-transposed to [k][n] so a
// quarter-wave reads 64 contiguous bytes.  fc4 (6 outputs) runs as one padded
// 16-column tile.  Two schedules of the same chains (bitwise equal outputs):
//  * k_mlp: one workgroup = 16 waves = a 16-row batch tile through all four
//    layers (no workspace; one CU per 16 rows, so a call under 4,096 rows
//    leaves CUs idle and costs one CU's four-layer latency, ~42 us);
//  * k_mlp_layer x2 + k_mlp_head (cit_mlp_forward_packed): fc1 and fc2
//    spread their 16x16 tiles over 4-wave workgroups (one tile per wave,
//    rows x column groups), H1 / H2 through a caller workspace, then fc3 +
//    fc4 + square_and_normalize per 16-row tile; weights MFMA-packed once by
//    cit_mlp_pack (one 16-byte load per lane per four MFMAs).
// One row per lane (the featurizer kernels): no wave-uniform engine scans.
#define CIT_NO_WAVE 1
#include <hip/hip_runtime.h>

#include "../../include/citadels.h"
#include "cit_engine.h"
#include "cit_mlp_wave.h"

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
template <int K, int N, int NT, int PF = MLP_PF>
__device__ __forceinline__ void tile16_layer(const float* in, int in_s, const float* __restrict__ WT,
                                             const float* __restrict__ bias, float* out, int out_s, int n0,
                                             bool relu, int nvalid, int nrows = 16) {
  constexpr int KK = (K + 3) / 4;
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  f32x4 acc[NT];
  int col[NT], colc[NT];
  bool cv[NT];
#pragma unroll
  for (int t = 0; t < NT; t++) {
    for (int i = 0; i < 4; i++) acc[t][i] = 0.0f;
    col[t] = n0 + 16 * t + r;
    cv[t] = col[t] < nvalid;
    colc[t] = cv[t] ? col[t] : nvalid - 1;
  }
  // both operands run PF steps ahead in register rings (the LDS activation
  // read as well as the L2 weight read), so an MFMA never waits on a load
  // issued in its own step.  Operands past K (or past the valid columns)
  // read a clamped in-bounds address and are zeroed when consumed, not when
  // loaded (a select at load time would wait for the load).
  auto wgt = [&](int t, int kk) -> float {
    const int k = 4 * kk + q;
    return WT[(long)(k < K ? k : K - 1) * N + colc[t]];
  };
  const float* ip = in + r * in_s + q;
  auto act = [&](int kk) -> float { return ip[4 * (4 * kk + q < K ? kk : 0)]; };
  float b[PF][NT], av[PF];
#pragma unroll
  for (int i = 0; i < PF; i++) {
    av[i] = act(i);
#pragma unroll
    for (int t = 0; t < NT; t++) b[i][t] = wgt(t, i);
  }
  for (int k0 = 0; k0 < KK; k0 += PF) {
#pragma unroll
    for (int i = 0; i < PF; i++) {
      const int kk = k0 + i;
      if (kk < KK) {
        const bool kv = 4 * kk + q < K;
        const float a = kv ? av[i] : 0.0f;
        av[i] = act(kk + PF);
#pragma unroll
        for (int t = 0; t < NT; t++) {
          const float w = kv && cv[t] ? b[i][t] : 0.0f;
          b[i][t] = wgt(t, kk + PF);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w, acc[t], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);   // keep each step's prefetches in that step
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; t++) {
    if (!cv[t]) continue;
    float bb = bias[col[t]];
    for (int i = 0; i < 4; i++) {
      int row = 4 * q + i;
      if (row >= nrows) continue;
      float v = acc[t][i] + bb;
      out[row * out_s + col[t]] = relu ? (v > 0.0f ? v : 0.0f) : v;
    }
  }
}

// Rows m0.. of a [M][K] matrix into LDS: element (r, k < KP) of the tile
// goes to X[dst(r, k)] (zero past K or past the valid rows).  Every thread's
// loads are issued before any is waited on (clamped in-bounds addresses,
// then a select): a load-wait-store loop would pay one L2/HBM latency per
// element.
template <int K, int KP, int NTH, class Dst>
__device__ __forceinline__ void mlp_stage(const float* __restrict__ in, int m0, int nrows, float* X, Dst dst) {
  constexpr int TOT = MLP_ROWS * KP, IT = (TOT + NTH - 1) / NTH;
  float v[IT];
#pragma unroll
  for (int it = 0; it < IT; it++) {
    const int i = threadIdx.x + it * NTH;
    const int r = i / KP, k = i - r * KP;
    const int rc = r < nrows ? r : nrows - 1, kc = k < K ? k : K - 1;
    const float x = in[(long)(m0 + rc) * K + kc];
    v[it] = (i < TOT && r < nrows && k < K) ? x : 0.0f;
  }
#pragma unroll
  for (int it = 0; it < IT; it++) {
    const int i = threadIdx.x + it * NTH;
    const int r = i / KP, k = i - r * KP;
    if (i < TOT) X[dst(r, k)] = v[it];
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
  mlp_stage<MLP_IN, MLP_IN, 64 * MLP_WAVES>(feat, m0, nrows, X, [](int r, int k) { return r * MLP_XS + k; });
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

// ---------------------------------------------------------------- packed path
// The layer-split schedule reads MFMA-packed weights (cit_mlp_pack): for a
// layer (K, N), 16-column tile nt and k-group g (4 MFMA steps = 16 k), lane
// l = 16 q + r holds the float4 {W[16 g + 4 j + q][16 nt + r], j = 0..3}
// (zero past K or N), so one 16-byte load per lane feeds four chained MFMAs
// and a wave's load is 1 KB contiguous.  The 16 input rows sit in LDS in the
// matching order (row r: group g, quarter q, step j at (4 g + q) * 4 + j), so
// the activation operand is one ds_read_b128 per group as well.  The k order
// of every chain is unchanged (k ascending, zero padding only past K): the
// outputs are bitwise those of k_mlp / the fmaf oracle.
__host__ __device__ constexpr int mlp_kg(int K) { return ((K + 3) / 4 + 3) / 4; }
__host__ __device__ constexpr int mlp_ps(int K) { return mlp_kg(K) * 16 + 4; }   // LDS row stride (floats)
#define MLP_P1 0
#define MLP_P2 (MLP_P1 + (MLP_H1 / 16) * mlp_kg(MLP_IN) * 256)
#define MLP_P3 (MLP_P2 + (MLP_H2 / 16) * mlp_kg(MLP_H1) * 256)
#define MLP_P4 (MLP_P3 + (MLP_H3 / 16) * mlp_kg(MLP_H2) * 256)
#define MLP_PB1 (MLP_P4 + mlp_kg(MLP_H3) * 256)
#define MLP_PB2 (MLP_PB1 + MLP_H1)
#define MLP_PB3 (MLP_PB2 + MLP_H2)
#define MLP_PB4 (MLP_PB3 + MLP_H3)
#define MLP_PTOTAL (MLP_PB4 + 16)

__device__ __forceinline__ float mlp_pack_w(const float* W, int K, int N, long e) {
  const int j = (int)(e & 3), l = (int)((e >> 2) & 63);
  const long rest = e >> 8;
  const int kg = mlp_kg(K);
  const int g = (int)(rest % kg), nt = (int)(rest / kg);
  const int k = 16 * g + 4 * j + (l >> 4), c = 16 * nt + (l & 15);
  return (k < K && c < N) ? W[(long)k * N + c] : 0.0f;
}

__global__ void k_mlp_pack(const float* __restrict__ w1t, const float* __restrict__ b1, const float* __restrict__ w2t,
                           const float* __restrict__ b2, const float* __restrict__ w3t, const float* __restrict__ b3,
                           const float* __restrict__ w4t, const float* __restrict__ b4, float* __restrict__ P) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= MLP_PTOTAL) return;
  float v;
  if (i < MLP_P2) v = mlp_pack_w(w1t, MLP_IN, MLP_H1, i - MLP_P1);
  else if (i < MLP_P3) v = mlp_pack_w(w2t, MLP_H1, MLP_H2, i - MLP_P2);
  else if (i < MLP_P4) v = mlp_pack_w(w3t, MLP_H2, MLP_H3, i - MLP_P3);
  else if (i < MLP_PB1) v = mlp_pack_w(w4t, MLP_H3, MLP_OUT, i - MLP_P4);
  else if (i < MLP_PB2) v = b1[i - MLP_PB1];
  else if (i < MLP_PB3) v = b2[i - MLP_PB2];
  else if (i < MLP_PB4) v = b3[i - MLP_PB3];
  else v = i - MLP_PB4 < MLP_OUT ? b4[i - MLP_PB4] : 0.0f;
  P[i] = v;
}

// Rows m0.. into LDS in the packed activation order (row r: group g,
// quarter q, step j at (4 g + q) * 4 + j).
template <int K, int NTH>
__device__ __forceinline__ void mlp_stage_packed(const float* __restrict__ in, int m0, int nrows, float* X) {
  constexpr int S = mlp_ps(K);
  mlp_stage<K, mlp_kg(K) * 16, NTH>(in, m0, nrows, X, [](int r, int k) {
    return r * S + ((k >> 4) * 4 + (k & 3)) * 4 + ((k >> 2) & 3);
  });
}

// One 16x16 output tile (column tile nt of a (K, N) layer) as a chain of
// 4 * mlp_kg(K) MFMAs; both operands run PFG groups ahead in register rings.
template <int K, int PFG>
__device__ __forceinline__ f32x4 mlp_tile_packed(const float* X, const float* __restrict__ Wl, int nt) {
  constexpr int KG = mlp_kg(K), S = mlp_ps(K);
  const int lane = threadIdx.x & 63;
  const f32x4* xa = reinterpret_cast<const f32x4*>(X + (lane & 15) * S + (lane >> 4) * 4);   // + 4 g (float4 units)
  const f32x4* wb = reinterpret_cast<const f32x4*>(Wl) + (long)nt * KG * 64 + lane;          // + 64 g
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  f32x4 a[PFG], w[PFG];
#pragma unroll
  for (int i = 0; i < PFG; i++) {
    const int g = i < KG ? i : KG - 1;
    a[i] = xa[4 * g];
    w[i] = wb[64 * g];
  }
  for (int g0 = 0; g0 < KG; g0 += PFG) {
#pragma unroll
    for (int i = 0; i < PFG; i++) {
      const int g = g0 + i;
      if (g < KG) {
        const f32x4 ac = a[i], wc = w[i];
        const int gn = g + PFG < KG ? g + PFG : KG - 1;
        a[i] = xa[4 * gn];
        w[i] = wb[64 * gn];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ac.x, wc.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ac.y, wc.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ac.z, wc.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ac.w, wc.w, acc, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);   // keep each group's prefetches in that group
      }
    }
  }
  return acc;
}

// fc1 / fc2 as their own launches: blockIdx.x = 16-row tile, blockIdx.y = a
// group of four 16-column tiles, one per wave (a 1,024-row call is 512
// workgroups for fc1, 256 for fc2); output rows [M][N] (+ bias, ReLU).
#define MLP_LAYER_WAVES 4
#define MLP_PFG 8
template <int K, int N>
__global__ __launch_bounds__(64 * MLP_LAYER_WAVES) void k_mlp_layer(const float* __restrict__ in, int M,
                                                                   const float* __restrict__ Wl,
                                                                   const float* __restrict__ bias,
                                                                   float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float X[MLP_ROWS * mlp_ps(K)];
  const int m0 = blockIdx.x * MLP_ROWS;
  const int nrows = min(MLP_ROWS, M - m0);
  mlp_stage_packed<K, 64 * MLP_LAYER_WAVES>(in, m0, nrows, X);
  __syncthreads();
  const int nt = blockIdx.y * MLP_LAYER_WAVES + (threadIdx.x >> 6);
  if (nt * 16 >= N) return;
  const f32x4 acc = mlp_tile_packed<K, MLP_PFG>(X, Wl, nt);
  const int lane = threadIdx.x & 63, col = nt * 16 + (lane & 15), q = lane >> 4;
  const float bb = bias[col];
  for (int i = 0; i < 4; i++) {
    const int row = 4 * q + i;
    if (row < nrows) {
      const float v = acc[i] + bb;
      out[(long)(m0 + row) * N + col] = v > 0.0f ? v : 0.0f;
    }
  }
}

// fc3 (8 column tiles, one per wave; H3 written to LDS in the packed order)
// + fc4 (wave 0) + square_and_normalize for one 16-row tile of H2.
#define MLP_HEAD_WAVES (MLP_H3 / 16)
__global__ __launch_bounds__(64 * MLP_HEAD_WAVES) void k_mlp_head(const float* __restrict__ h2, int M,
                                                                 const float* __restrict__ P,
                                                                 float* __restrict__ probs,
                                                                 float* __restrict__ logits) {
  __shared__ __attribute__((aligned(16))) float X2[MLP_ROWS * mlp_ps(MLP_H2)];
  __shared__ __attribute__((aligned(16))) float X3[MLP_ROWS * mlp_ps(MLP_H3)];
  __shared__ float L[MLP_ROWS * 8];
  const int m0 = blockIdx.x * MLP_ROWS;
  const int nrows = min(MLP_ROWS, M - m0);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  mlp_stage_packed<MLP_H2, 64 * MLP_HEAD_WAVES>(h2, m0, nrows, X2);
  __syncthreads();
  {
    const f32x4 acc = mlp_tile_packed<MLP_H2, MLP_PFG>(X2, P + MLP_P3, wave);
    const int c = wave * 16 + r;
    const float bb = P[MLP_PB3 + c];
    for (int i = 0; i < 4; i++) {
      const float v = acc[i] + bb;
      X3[(4 * q + i) * mlp_ps(MLP_H3) + ((c >> 4) * 4 + (c & 3)) * 4 + ((c >> 2) & 3)] = v > 0.0f ? v : 0.0f;
    }
  }
  __syncthreads();
  if (wave == 0) {
    const f32x4 acc = mlp_tile_packed<MLP_H3, MLP_PFG>(X3, P + MLP_P4, 0);
    if (r < MLP_OUT) {
      const float bb = P[MLP_PB4 + r];
      for (int i = 0; i < 4; i++) L[(4 * q + i) * 8 + r] = acc[i] + bb;
    }
  }
  __syncthreads();
  if (threadIdx.x < nrows) {
    const int rr = threadIdx.x;
    float sq[MLP_OUT], s = 0.0f;
    for (int j = 0; j < MLP_OUT; j++) {
      const float v = L[rr * 8 + j];
      sq[j] = v * v;
      s += sq[j];
      if (logits) logits[(long)(m0 + rr) * MLP_OUT + j] = v;
    }
    for (int j = 0; j < MLP_OUT; j++) probs[(long)(m0 + rr) * MLP_OUT + j] = sq[j] / s;
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

// ------------------------------------------------------- one row per wave
// The wave layout (cit_mlp_wave.h) of the folded weights, and the single-row
// forward the search runs inside its kernel (cit_cfr_pred_fused), here one
// row per 64-lane workgroup so it can be checked against the oracle alone.
__global__ void k_mlp_pack_wave(const float* __restrict__ w1t, const float* __restrict__ b1,
                                const float* __restrict__ w2t, const float* __restrict__ b2,
                                const float* __restrict__ w3t, const float* __restrict__ b3,
                                const float* __restrict__ w4t, const float* __restrict__ b4, float* __restrict__ Q) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= MLPW_TOTAL) return;
  float v;
  if (i < MLPW_L2) v = mlpw_pack_elem(w1t, MLPW_IN, MLPW_H1, i - MLPW_L1);
  else if (i < MLPW_L3) v = mlpw_pack_elem(w2t, MLPW_H1, MLPW_H2, i - MLPW_L2);
  else if (i < MLPW_L4) v = mlpw_pack_elem(w3t, MLPW_H2, MLPW_H3, i - MLPW_L3);
  else if (i < MLPW_B1) v = mlpw_pack_elem(w4t, MLPW_H3, MLPW_OUT, i - MLPW_L4);
  else if (i < MLPW_B2) v = b1[i - MLPW_B1];
  else if (i < MLPW_B3) v = b2[i - MLPW_B2];
  else if (i < MLPW_B4) v = b3[i - MLPW_B3];
  else if (i < MLPW_FLAG) v = i - MLPW_B4 < MLPW_OUT ? b4[i - MLPW_B4] : 0.0f;
  else return;                                         // the flag word (k_mlp_wave_flag)
  Q[i] = v;
  // a non-finite weight: every input row must be read (0 * inf is NaN, not a no-op)
  if (i < MLPW_B1 && !__builtin_isfinite(v)) atomicAnd(reinterpret_cast<uint32_t*>(Q + MLPW_FLAG), 0u);
}
__global__ void k_mlp_wave_flag(float* __restrict__ Q) { *reinterpret_cast<uint32_t*>(Q + MLPW_FLAG) = 1u; }

__global__ __launch_bounds__(64) void k_mlp_wave(const float* __restrict__ feat, int M, const float* __restrict__ Q,
                                                 float* __restrict__ probs, float* __restrict__ logits) {
  __shared__ __attribute__((aligned(16))) float R[MLPW_R_FLOATS];
  const long m = blockIdx.x;
  if (m >= M) return;
  for (int i = threadIdx.x; i < MLPW_IN + 2; i += 64) R[MLPW_R_X + i] = i < MLPW_IN ? feat[m * MLPW_IN + i] : 0.0f;
  mlpw_forward(Q, (mlpw_lds_t*)R);
  if (threadIdx.x < MLPW_OUT) {
    probs[m * MLPW_OUT + threadIdx.x] = R[MLPW_R_PROBS + threadIdx.x];
    if (logits) logits[m * MLPW_OUT + threadIdx.x] = R[MLPW_R_LOGITS + threadIdx.x];
  }
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

size_t cit_mlp_packed_bytes(void) { return (size_t)MLP_PTOTAL * sizeof(float); }

int cit_mlp_pack(const float* w1t, const float* b1, const float* w2t, const float* b2, const float* w3t,
                 const float* b3, const float* w4t, const float* b4, void* packed, hipStream_t stream) {
  if (!w1t || !b1 || !w2t || !b2 || !w3t || !b3 || !w4t || !b4 || !packed) return -1;
  hipLaunchKernelGGL(k_mlp_pack, dim3((MLP_PTOTAL + 255) / 256), dim3(256), 0, stream, w1t, b1, w2t, b2, w3t, b3, w4t,
                     b4, (float*)packed);
  CHECK_LAUNCH();
}

size_t cit_mlp_work_bytes(int M) { return M > 0 ? (size_t)M * (MLP_H1 + MLP_H2) * sizeof(float) : 0; }

int cit_mlp_forward_packed(const float* feat, int M, const void* packed, float* probs, float* logits, void* work,
                           size_t work_bytes, hipStream_t stream) {
  if (M < 0 || (M && (!feat || !packed || !probs))) return -1;
  if (!M) return 0;
  if (!work || work_bytes < cit_mlp_work_bytes(M)) return -1;
  const float* P = (const float*)packed;
  float* h1 = (float*)work;
  float* h2 = h1 + (size_t)M * MLP_H1;
  const int tiles = (M + MLP_ROWS - 1) / MLP_ROWS;
  hipLaunchKernelGGL((k_mlp_layer<MLP_IN, MLP_H1>), dim3(tiles, MLP_H1 / (16 * MLP_LAYER_WAVES)),
                     dim3(64 * MLP_LAYER_WAVES), 0, stream, feat, M, P + MLP_P1, P + MLP_PB1, h1);
  hipLaunchKernelGGL((k_mlp_layer<MLP_H1, MLP_H2>), dim3(tiles, MLP_H2 / (16 * MLP_LAYER_WAVES)),
                     dim3(64 * MLP_LAYER_WAVES), 0, stream, h1, M, P + MLP_P2, P + MLP_PB2, h2);
  hipLaunchKernelGGL(k_mlp_head, dim3(tiles), dim3(64 * MLP_HEAD_WAVES), 0, stream, h2, M, P, probs, logits);
  CHECK_LAUNCH();
}

size_t cit_mlp_wave_bytes(void) { return (size_t)MLPW_TOTAL * sizeof(float); }

int cit_mlp_pack_wave(const float* w1t, const float* b1, const float* w2t, const float* b2, const float* w3t,
                      const float* b3, const float* w4t, const float* b4, void* packed, hipStream_t stream) {
  if (!w1t || !b1 || !w2t || !b2 || !w3t || !b3 || !w4t || !b4 || !packed) return -1;
  hipLaunchKernelGGL(k_mlp_wave_flag, dim3(1), dim3(1), 0, stream, (float*)packed);
  hipLaunchKernelGGL(k_mlp_pack_wave, dim3((unsigned)((MLPW_TOTAL + 255) / 256)), dim3(256), 0, stream, w1t, b1, w2t,
                     b2, w3t, b3, w4t, b4, (float*)packed);
  CHECK_LAUNCH();
}

int cit_mlp_forward_wave(const float* feat, int M, const void* packed, float* probs, float* logits,
                         hipStream_t stream) {
  if (M < 0 || (M && (!feat || !packed || !probs))) return -1;
  if (!M) return 0;
  hipLaunchKernelGGL(k_mlp_wave, dim3(M), dim3(64), 0, stream, feat, M, (const float*)packed, probs, logits);
  CHECK_LAUNCH();
}

}  // extern "C"
