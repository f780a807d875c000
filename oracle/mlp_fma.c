/* CPU ORACLE (test infrastructure only): the value MLP
 * (algorithms/models.py ValueOnlyNN(418, 512), eval, BatchNorm folded) +
 * square_and_normalize (algorithms/train_utils.py:143-145), restated as
 * k-ordered fmaf chains from 0, then + bias, then ReLU: the exact arithmetic of
 * v_mfma_f32_32x32x2_f32 that the device kernel (cit_mlp.hip) performs.
 * Compared with torch's fp32 forward of the reference class it agrees within
 * the tolerance stated in tests/test_mlp_host.py.  Built by
 * __graft_entry__.build() into oracle/_ref/libmlp_fma.so. */
#include <math.h>

static void layer(const float* x, int K, const float* wt, int N, const float* b, int relu, float* y) {
  for (int n = 0; n < N; n++) {
    float acc = 0.0f;
    for (int k = 0; k < K; k++) acc = fmaf(x[k], wt[(long)k * N + n], acc);
    float v = acc + b[n];
    y[n] = relu ? (v > 0.0f ? v : 0.0f) : v;
  }
}

void mlp_forward(const float* feat, int M, const float* w1t, const float* b1, const float* w2t, const float* b2,
                 const float* w3t, const float* b3, const float* w4t, const float* b4, float* probs, float* logits) {
  float h1[512], h2[256], h3[128], o[6];
  for (int m = 0; m < M; m++) {
    layer(feat + (long)m * 418, 418, w1t, 512, b1, 1, h1);
    layer(h1, 512, w2t, 256, b2, 1, h2);
    layer(h2, 256, w3t, 128, b3, 1, h3);
    layer(h3, 128, w4t, 6, b4, 0, o);
    float sq[6], s = 0.0f;
    for (int j = 0; j < 6; j++) {
      sq[j] = o[j] * o[j];
      s += sq[j];
      if (logits) logits[(long)m * 6 + j] = o[j];
    }
    for (int j = 0; j < 6; j++) probs[(long)m * 6 + j] = sq[j] / s;
  }
}
