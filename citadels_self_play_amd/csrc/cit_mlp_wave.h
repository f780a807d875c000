// Value-MLP forward of ONE row by ONE wavefront: the search's in-kernel leaf
// evaluation (cfr_pred without suspending the tree, cit_cfr_pred_fused) and
// its test entry (cit_mlp_forward_wave).
//
//   wp = square_and_normalize(fc4(relu(fc3(relu(fc2'(relu(fc1'(x))))))))
//        (algorithms/models.py:17-24, algorithms/train_utils.py:143-145,
//         algorithms/deep_mccfr.py:364-374)
//
// Lane l owns output columns l, l + 64, ... of every layer and runs each
// column's k-ordered fmaf chain from 0, then + bias, then ReLU: the arithmetic
// of oracle/mlp_fma.c and of the MFMA kernels (cit_mlp.hip), so the outputs
// are bitwise theirs.  One row cannot fill a matrix core, and what bounds a
// single-row forward is the weight stream, so the chains run on the VALU
// (v_pk_fma_f32: two columns per instruction) with the weight rows loaded
// PF rows ahead, and only the rows whose input is non-zero are read:
//
// Zero inputs are skipped.  encode_game rows are mostly zero (one-hots and
// counts: ~60-90 of 418 non-zero) and a ReLU output is exactly +0 for about
// half the units, and fmaf(0, w, acc) == acc bit for bit whenever w is finite
// and acc is not -0; a chain's accumulator starts at +0, stays +0 until its
// first non-zero product and is never -0 afterwards except by underflow of a
// product smaller than half the least denormal -- and then only its sign of
// zero could differ, which the bias add (+0 + b == -0 + b for b != 0) and the
// ReLU / squaring that follow erase.  So the skipped chains equal the full
// ones; with a non-finite weight (0 * inf = NaN) the pack clears the flag
// word and every row is read.
//
// Weights in the "row layout" (cit_mlp_pack_wave): layer (K, N) as K rows; for
// N a multiple of 64 row k holds lane l's S = N / 64 columns contiguously
// ({W[k][64 s + l]}_s at float k * N + l * S: one 16- or 32-byte load per lane,
// a wave's load is the whole 2 KB / 1 KB / 512 B row); fc4 (N = 6): row k =
// {W[k][0..5], 0, 0} (8 floats, lanes below 6 read one float each).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MLPW_HD __host__ __device__
#else
#define MLPW_HD
#endif

#define MLPW_IN 418
#define MLPW_H1 512
#define MLPW_H2 256
#define MLPW_H3 128
#define MLPW_OUT 6

MLPW_HD constexpr int mlpw_rs(int N) { return N >= 64 ? N : 8; }              // row stride (floats)
MLPW_HD constexpr long mlpw_floats(int K, int N) { return (long)K * mlpw_rs(N); }
#define MLPW_L1 0L
#define MLPW_L2 (MLPW_L1 + mlpw_floats(MLPW_IN, MLPW_H1))
#define MLPW_L3 (MLPW_L2 + mlpw_floats(MLPW_H1, MLPW_H2))
#define MLPW_L4 (MLPW_L3 + mlpw_floats(MLPW_H2, MLPW_H3))
#define MLPW_B1 (MLPW_L4 + mlpw_floats(MLPW_H3, MLPW_OUT))
#define MLPW_B2 (MLPW_B1 + MLPW_H1)
#define MLPW_B3 (MLPW_B2 + MLPW_H2)
#define MLPW_B4 (MLPW_B3 + MLPW_H3)
#define MLPW_FLAG (MLPW_B4 + 8)              // uint32: 1 = every weight finite (zero inputs may be skipped)
#define MLPW_TOTAL (MLPW_FLAG + 4)

// The forward's LDS scratch (floats): h1 [0, 512) | x [512, 932) (418 + two
// zero pads) -- layer 1 reads x and writes h1 --, then h2 over x, h3 over h1,
// and the logits / probabilities at [768, 780).
#define MLPW_R_H1 0
#define MLPW_R_X 512
#define MLPW_R_H2 512
#define MLPW_R_H3 0
#define MLPW_R_LOGITS 768
#define MLPW_R_PROBS 776
// the layer's non-zero inputs as a u16 list (<= 512 entries + the ring's
// look-ahead pad), after x: 544 u16 = 272 floats
#define MLPW_R_LIST 932
#define MLPW_LIST_CAP 544
#define MLPW_R_FLOATS (MLPW_R_LIST + MLPW_LIST_CAP / 2)

// Element e of the row layout of W [K][N] (row-major, k major).
MLPW_HD inline float mlpw_pack_elem(const float* W, int K, int N, long e) {
  const int rs = mlpw_rs(N);
  const int k = (int)(e / rs), i = (int)(e % rs);
  int c = i;
  if (N >= 64) {
    const int S = N / 64, l = i / S, s = i % S;
    c = 64 * s + l;
  }
  return (k < K && c < N) ? W[(long)k * N + c] : 0.0f;
}

#if defined(__HIPCC__)
typedef __attribute__((address_space(3))) float mlpw_lds_t;
typedef float mlpw_f4 __attribute__((ext_vector_type(4)));
typedef float mlpw_f2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) float mlpw_gf_t;

// a wave-uniform global pointer (scalar base, global_* instructions)
__device__ __forceinline__ mlpw_gf_t* mlpw_glb(const float* p) {
  uint64_t a = (uint64_t)(uintptr_t)p;
  uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  return (mlpw_gf_t*)(((uint64_t)hi << 32) | lo);
}

// The non-zero inputs of a layer as 64-bit masks, one per 64 inputs (every
// input when !skip), held in two VGPRs (lane i: chunk i's mask) so a scalar
// cursor walks the set bits in ascending order with readlane / ctz -- no LDS
// list, so the next row's address is a few scalar instructions away.
struct MlpwMask {
  uint32_t lo, hi;      // lane i: bits of chunk i (per lane: a VGPR)
  int nnz;              // set bits in all (wave-uniform)
};
template <int K>
__device__ __forceinline__ MlpwMask mlpw_mask(const mlpw_lds_t* x, bool skip) {
  const int lane = __lane_id();
  MlpwMask M{0u, 0u, 0};
#pragma unroll
  for (int i = 0; i < K; i += 64) {
    const int k = i + lane;
    const bool nz = k < K && (!skip || x[k < K ? k : 0] != 0.0f);
    const uint64_t m = __ballot(nz);
    if (lane == i / 64) {
      M.lo = (uint32_t)m;
      M.hi = (uint32_t)(m >> 32);
    }
    M.nnz += __popcll(m);
  }
  M.nnz = __builtin_amdgcn_readfirstlane(M.nnz);
  return M;
}
// A cursor over the set bits of a MlpwMask (scalar state).
struct MlpwCursor {
  int ci;               // current chunk
  uint64_t cm;          // its bits not yet taken
};
__device__ __forceinline__ uint64_t mlpw_chunk(const MlpwMask& M, int ci) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)M.hi, ci) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)M.lo, ci);
}
// The next set input index (0 past the end: a dummy row, never consumed).
template <int K>
__device__ __forceinline__ int mlpw_next(const MlpwMask& M, MlpwCursor& c) {
  constexpr int NCH = (K + 63) / 64;
  while (c.cm == 0 && c.ci < NCH - 1) {
    c.ci++;
    c.cm = mlpw_chunk(M, c.ci);
  }
  if (c.cm == 0) return 0;
  const int b = __builtin_ctzll(c.cm);
  c.cm &= c.cm - 1;
  return 64 * c.ci + b;
}

// S floats of weight row k for this lane (S = 8, 4, 2 or 1).
template <int S>
struct mlpw_row {
  float v[S];
};
template <int N>
__device__ __forceinline__ mlpw_row<(N >= 64 ? N / 64 : 1)> mlpw_ld(const __attribute__((address_space(1))) char* W,
                                                                     int k, uint32_t voff) {
  constexpr int S = N >= 64 ? N / 64 : 1;
  const __attribute__((address_space(1))) char* rb = W + (long)k * (mlpw_rs(N) * 4);     // uniform
  mlpw_row<S> r;
  if constexpr (S >= 4) {
#pragma unroll
    for (int j = 0; j < S / 4; j++) {
      const mlpw_f4 q = *(const __attribute__((address_space(1))) mlpw_f4*)(rb + voff + 16 * j);
      r.v[4 * j] = q.x;
      r.v[4 * j + 1] = q.y;
      r.v[4 * j + 2] = q.z;
      r.v[4 * j + 3] = q.w;
    }
  } else if constexpr (S == 2) {
    const mlpw_f2 q = *(const __attribute__((address_space(1))) mlpw_f2*)(rb + voff);
    r.v[0] = q.x;
    r.v[1] = q.y;
  } else {
    r.v[0] = *(const __attribute__((address_space(1))) float*)(rb + voff);
  }
  return r;
}

// One layer over the non-zero inputs: y[c] = act(fmaf chain over the set k,
// ascending, of x[k] * W[k][c], from 0, + b[c]) for this lane's columns; the
// rows (and their x[k]) run PF set bits ahead in a register ring.
template <int K, int N, int PF, bool RELU>
__device__ __forceinline__ void mlpw_layer(const float* Wl, const float* bias, const mlpw_lds_t* x,
                                           const MlpwMask& M, mlpw_lds_t* y) {
  constexpr int S = N >= 64 ? N / 64 : 1;
  const int lane = __lane_id();
  const __attribute__((address_space(1))) char* wb = (const __attribute__((address_space(1))) char*)mlpw_glb(Wl);
  const uint32_t voff = (uint32_t)(N >= 64 ? lane * S : (lane < N ? lane : N - 1)) * 4u;
  const int nnz = M.nnz;
  MlpwCursor cur{0, mlpw_chunk(M, 0)};
  float acc[S];
#pragma unroll
  for (int s = 0; s < S; s++) acc[s] = 0.0f;
  mlpw_row<S> w[PF];
  float xr[PF];
#pragma unroll
  for (int i = 0; i < PF; i++) {
    const int k = mlpw_next<K>(M, cur);
    w[i] = mlpw_ld<N>(wb, k, voff);
    xr[i] = x[k];
    __builtin_amdgcn_sched_barrier(0);     // issue the ring in input order (the oldest rows are consumed first)
  }
  auto step = [&](int i) {
    const float xv = xr[i];
    if constexpr (S == 1) {
      acc[0] = __builtin_fmaf(xv, w[i].v[0], acc[0]);
    } else {
      const mlpw_f2 xx = mlpw_f2{xv, xv};
#pragma unroll
      for (int s = 0; s < S; s += 2) {
        const mlpw_f2 r = __builtin_elementwise_fma(xx, mlpw_f2{w[i].v[s], w[i].v[s + 1]},
                                                    mlpw_f2{acc[s], acc[s + 1]});
        acc[s] = r.x;
        acc[s + 1] = r.y;
      }
    }
    const int k = mlpw_next<K>(M, cur);     // refill the slot PF inputs ahead
    w[i] = mlpw_ld<N>(wb, k, voff);
    xr[i] = x[k];
    __builtin_amdgcn_sched_barrier(0);
  };
  // whole rings without per-step guards (a guard would make the load-count
  // waits conservative: every step would wait for nearly all loads in flight)
  const int full = nnz - nnz % PF;
#pragma nounroll
  for (int t0 = 0; t0 < full; t0 += PF) {
#pragma unroll
    for (int i = 0; i < PF; i++) step(i);
  }
#pragma unroll
  for (int i = 0; i < PF - 1; i++)
    if (i < nnz - full) step(i);
  mlpw_gf_t* bp = mlpw_glb(bias);
#pragma unroll
  for (int s = 0; s < S; s++) {
    const int c = N >= 64 ? 64 * s + lane : lane;
    if (c < N) {
      const float v = acc[s] + bp[c];
      y[c] = RELU ? (v > 0.0f ? v : 0.0f) : v;
    }
  }
}

#ifndef MLPW_LIST
#define MLPW_LIST 1
#endif
// rows in flight per layer (multiples of 4; a layer-1 row is 8 VGPRs a lane)
#ifndef MLPW_PF1
#define MLPW_PF1 8
#endif
#ifndef MLPW_PF2
#define MLPW_PF2 12
#endif
#ifndef MLPW_PF3
#define MLPW_PF3 16
#endif
#ifndef MLPW_PF4
#define MLPW_PF4 16
#endif
typedef __attribute__((address_space(3))) uint16_t mlpw_lds_u16;
typedef unsigned mlpw_u2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) mlpw_u2 mlpw_lds_u2;
// The same layer driven by a list instead of the mask cursor: the non-zero
// inputs, ascending, are compacted once into a u16 list in LDS (one ballot
// per 64 inputs), and the ring reads the list four entries at a time, four
// steps ahead of the rows it issues -- a step is then a row address, two
// loads and the FMAs (the cursor's ~30 scalar instructions per row gone).
// The list is padded with row 0 past its end, so the look-ahead never
// issues a load outside the layer.  Same inputs in the same order: the
// chains are the cursor's, bit for bit.
template <int K, int N, int PF, bool RELU>
__device__ __forceinline__ void mlpw_layer_list(const float* Wl, const float* bias, const mlpw_lds_t* x, bool skip,
                                                mlpw_lds_u16* list, mlpw_lds_t* y) {
  static_assert(PF % 4 == 0 && K + PF + 8 <= MLPW_LIST_CAP, "list look-ahead");
  constexpr int S = N >= 64 ? N / 64 : 1;
  const int lane = __lane_id();
  const uint64_t below = (1ull << lane) - 1;
  int nnz = 0;
#pragma unroll
  for (int i = 0; i < K; i += 64) {
    const int k = i + lane;
    const float xv = x[k < K ? k : 0];
    const bool nz = k < K && (!skip || xv != 0.0f);
    const uint64_t m = __ballot(nz);
    if (nz) list[nnz + __popcll(m & below)] = (uint16_t)k;
    nnz += __popcll(m);
  }
  nnz = __builtin_amdgcn_readfirstlane(nnz);
  if (lane < PF + 8) list[nnz + lane] = 0;
  const __attribute__((address_space(1))) char* wb = (const __attribute__((address_space(1))) char*)mlpw_glb(Wl);
  const uint32_t voff = (uint32_t)(N >= 64 ? lane * S : (lane < N ? lane : N - 1)) * 4u;
  const mlpw_lds_u2* l4 = (const mlpw_lds_u2*)list;          // four entries per 8-byte read
  float acc[S];
#pragma unroll
  for (int s = 0; s < S; s++) acc[s] = 0.0f;
  mlpw_row<S> w[PF];
  float xr[PF];
  auto entry = [](mlpw_u2 q, int j) {
    const uint32_t v = (uint32_t)__builtin_amdgcn_readfirstlane((int)(j < 2 ? q.x : q.y));
    return (int)((j & 1) ? (v >> 16) : (v & 0xffffu));
  };
#pragma unroll
  for (int i = 0; i < PF; i += 4) {
    const mlpw_u2 q = l4[i / 4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int k = entry(q, j);
      w[i + j] = mlpw_ld<N>(wb, k, voff);
      xr[i + j] = x[k];
    }
  }
  mlpw_u2 q0 = l4[PF / 4], q1 = l4[PF / 4 + 1];   // the next eight entries to issue (read 4 steps ahead)
  auto step = [&](int i, int t) {        // t: the step's list position (t % 4 == i % 4)
    const float xv = xr[i];
    if constexpr (S == 1) {
      acc[0] = __builtin_fmaf(xv, w[i].v[0], acc[0]);
    } else {
      const mlpw_f2 xx = mlpw_f2{xv, xv};
#pragma unroll
      for (int s = 0; s < S; s += 2) {
        const mlpw_f2 r = __builtin_elementwise_fma(xx, mlpw_f2{w[i].v[s], w[i].v[s + 1]},
                                                    mlpw_f2{acc[s], acc[s + 1]});
        acc[s] = r.x;
        acc[s + 1] = r.y;
      }
    }
    const int k = entry(q0, i & 3);      // refill the slot with entry t + PF
    w[i] = mlpw_ld<N>(wb, k, voff);
    xr[i] = x[k];
    if ((i & 3) == 3) {                  // entries t + PF + 5 .. t + PF + 8, used four steps on
      q0 = q1;
      q1 = l4[(t + PF + 5) / 4];
    }
  };
  const int full = nnz - nnz % PF;
#pragma nounroll
  for (int t0 = 0; t0 < full; t0 += PF) {
#pragma unroll
    for (int i = 0; i < PF; i++) step(i, t0 + i);
  }
#pragma unroll
  for (int i = 0; i < PF - 1; i++)
    if (i < nnz - full) step(i, full + i);
  mlpw_gf_t* bp = mlpw_glb(bias);
#pragma unroll
  for (int s = 0; s < S; s++) {
    const int c = N >= 64 ? 64 * s + lane : lane;
    if (c < N) {
      const float v = acc[s] + bp[c];
      y[c] = RELU ? (v > 0.0f ? v : 0.0f) : v;
    }
  }
}

// The forward over the row at R + MLPW_R_X (MLPW_IN floats) with the
// row-layout weights Q: logits to R + MLPW_R_LOGITS, probabilities
// (square_and_normalize, the sum in index order) to R + MLPW_R_PROBS.  The
// caller's workgroup is this one wavefront; the barriers order the lanes'
// LDS writes before other lanes read them.
__device__ __forceinline__ void mlpw_forward(const float* Q, mlpw_lds_t* R) {
  const bool skip = *(const __attribute__((address_space(1))) uint32_t*)(mlpw_glb(Q) + MLPW_FLAG) != 0u;
  __syncthreads();
#if MLPW_LIST
  mlpw_lds_u16* list = (mlpw_lds_u16*)(R + MLPW_R_LIST);
  mlpw_layer_list<MLPW_IN, MLPW_H1, MLPW_PF1, true>(Q + MLPW_L1, Q + MLPW_B1, R + MLPW_R_X, skip, list, R + MLPW_R_H1);
  __syncthreads();
  mlpw_layer_list<MLPW_H1, MLPW_H2, MLPW_PF2, true>(Q + MLPW_L2, Q + MLPW_B2, R + MLPW_R_H1, skip, list, R + MLPW_R_H2);
  __syncthreads();
  mlpw_layer_list<MLPW_H2, MLPW_H3, MLPW_PF3, true>(Q + MLPW_L3, Q + MLPW_B3, R + MLPW_R_H2, skip, list, R + MLPW_R_H3);
  __syncthreads();
  mlpw_layer_list<MLPW_H3, MLPW_OUT, MLPW_PF4, false>(Q + MLPW_L4, Q + MLPW_B4, R + MLPW_R_H3, skip, list, R + MLPW_R_LOGITS);
  __syncthreads();
#else
  MlpwMask M = mlpw_mask<MLPW_IN>(R + MLPW_R_X, skip);
  mlpw_layer<MLPW_IN, MLPW_H1, 8, true>(Q + MLPW_L1, Q + MLPW_B1, R + MLPW_R_X, M, R + MLPW_R_H1);
  __syncthreads();
  M = mlpw_mask<MLPW_H1>(R + MLPW_R_H1, skip);
  mlpw_layer<MLPW_H1, MLPW_H2, 12, true>(Q + MLPW_L2, Q + MLPW_B2, R + MLPW_R_H1, M, R + MLPW_R_H2);
  __syncthreads();
  M = mlpw_mask<MLPW_H2>(R + MLPW_R_H2, skip);
  mlpw_layer<MLPW_H2, MLPW_H3, 16, true>(Q + MLPW_L3, Q + MLPW_B3, R + MLPW_R_H2, M, R + MLPW_R_H3);
  __syncthreads();
  M = mlpw_mask<MLPW_H3>(R + MLPW_R_H3, skip);
  mlpw_layer<MLPW_H3, MLPW_OUT, 16, false>(Q + MLPW_L4, Q + MLPW_B4, R + MLPW_R_H3, M, R + MLPW_R_LOGITS);
  __syncthreads();
#endif
  float sq[MLPW_OUT], s = 0.0f;
#pragma unroll
  for (int j = 0; j < MLPW_OUT; j++) {
    const float v = R[MLPW_R_LOGITS + j];
    sq[j] = v * v;
    s += sq[j];
  }
  if (__lane_id() < MLPW_OUT) {
    const int j = __lane_id();
    float q = sq[0];
#pragma unroll
    for (int i = 1; i < MLPW_OUT; i++) q = j == i ? sq[i] : q;
    R[MLPW_R_PROBS + j] = q / s;
  }
  __syncthreads();
}
#endif
