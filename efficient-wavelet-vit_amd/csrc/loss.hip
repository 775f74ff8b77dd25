// combined_loss of the reference's training step (train.py:55-91) in one launch, with its
// gradients: BCEWithLogits(pos_weight, mean) on the logits + w * orthogonal_loss(space, freq)
// (F.normalize rows, cov = s^T f, off-diagonal Frobenius norm^2 / (D (D - 1))).
//
// On torch this is ~15 forward and ~25 backward launches of [B, D] = [8, 128] elementwise /
// reduction kernels between the end of the forward and the start of the backward — the
// critical path of the step.  The whole problem is a few hundred KFLOP, so one workgroup
// computes the loss and every input gradient at once; the backward of the autograd op only
// scales them by the incoming gradient.
#include "common.h"

namespace ewvit {

// LDS: u, v [B][D] normalised rows, gu, gv [B][D] their gradients, inv norms, reductions.
// BT >= B: a thread keeps its cov row's (column's) B operands and gradients in registers.
template <int BT>
__global__ __launch_bounds__(256) void combined_loss_kernel(const float *__restrict__ logits,
                                                            const float *__restrict__ labels,
                                                            const float *__restrict__ X, const float *__restrict__ Y,
                                                            int B, int D, const float *__restrict__ pos_w,
                                                            const float *__restrict__ wdev, float lam,
                                                            float *__restrict__ out, float *__restrict__ dlog,
                                                            float *__restrict__ dX, float *__restrict__ dY) {
  extern __shared__ float sm[];
  float *u = sm, *v = u + B * D, *gu = v + B * D, *gv = gu + B * D;
  float *nx = gv + B * D, *ny = nx + B;           // clamped norms
  float *red = ny + B;                            // [8]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
  const float eps = 1e-12f;
  // row norms (F.normalize: x / max(||x||_2, eps)), a wave per row
  for (int r = wv; r < 2 * B; r += nw) {
    const float *src = r < B ? X + (int64_t)r * D : Y + (int64_t)(r - B) * D;
    float ss = 0.f;
    for (int i = lane; i < D; i += 64) ss += src[i] * src[i];
    ss = wave_sum(ss);
    if (lane == 0) (r < B ? nx[r] : ny[r - B]) = fmaxf(sqrtf(ss), eps);
  }
  __syncthreads();
  for (int e = tid; e < B * D; e += blockDim.x) {
    const int b = e / D;
    u[e] = X[e] / nx[b];
    v[e] = Y[e] / ny[b];
  }
  __syncthreads();
  // d(orth)/d(cov[i][j]) = k * cov[i][j] off the diagonal, k = 2 / (D (D - 1))
  const float k = 2.0f / ((float)D * (float)(D - 1));
  float sq = 0.f;
  for (int i = tid; i < D; i += blockDim.x) {       // rows of cov: gu[:, i] = sum_j k c_ij v[:, j]
    float a[BT], g[BT];
#pragma unroll
    for (int b = 0; b < BT; ++b) { a[b] = b < B ? u[b * D + i] : 0.f; g[b] = 0.f; }
    for (int j = 0; j < D; ++j) {
      if (j == i) continue;
      float c = 0.f;
#pragma unroll
      for (int b = 0; b < BT; ++b) c += a[b] * (b < B ? v[b * D + j] : 0.f);
      sq += c * c;
#pragma unroll
      for (int b = 0; b < BT; ++b) g[b] += k * c * (b < B ? v[b * D + j] : 0.f);
    }
#pragma unroll
    for (int b = 0; b < BT; ++b)
      if (b < B) gu[b * D + i] = g[b];
  }
  for (int j = tid; j < D; j += blockDim.x) {       // columns: gv[:, j] = sum_i k c_ij u[:, i]
    float a[BT], g[BT];
#pragma unroll
    for (int b = 0; b < BT; ++b) { a[b] = b < B ? v[b * D + j] : 0.f; g[b] = 0.f; }
    for (int i = 0; i < D; ++i) {
      if (i == j) continue;
      float c = 0.f;
#pragma unroll
      for (int b = 0; b < BT; ++b) c += (b < B ? u[b * D + i] : 0.f) * a[b];
#pragma unroll
      for (int b = 0; b < BT; ++b) g[b] += k * c * (b < B ? u[b * D + i] : 0.f);
    }
#pragma unroll
    for (int b = 0; b < BT; ++b)
      if (b < B) gv[b * D + j] = g[b];
  }
  sq = wave_sum(sq);
  if (lane == 0) red[wv] = sq;
  __syncthreads();
  float tot_sq = 0.f;
  for (int w = 0; w < nw; ++w) tot_sq += red[w];
  const float orth = tot_sq / ((float)D * (float)(D - 1));
  const float wgt = wdev ? *wdev : lam;
  // normalize backward, a wave per row: dx = (g - u (u . g)) / n when ||x|| > eps, else g / eps
  for (int r = wv; r < 2 * B; r += nw) {
    const int b = r < B ? r : r - B;
    const float *uu = (r < B ? u : v) + b * D, *gg = (r < B ? gu : gv) + b * D;
    const float *src = r < B ? X + (int64_t)b * D : Y + (int64_t)b * D;
    float *dst = r < B ? dX + (int64_t)b * D : dY + (int64_t)b * D;
    const float n = r < B ? nx[b] : ny[b];
    float ss = 0.f, dot = 0.f;
    for (int i = lane; i < D; i += 64) { ss += src[i] * src[i]; dot += uu[i] * gg[i]; }
    ss = wave_sum(ss);
    dot = wave_sum(dot);
    const bool live = sqrtf(ss) > eps;
    for (int i = lane; i < D; i += 64) dst[i] = wgt * (live ? (gg[i] - uu[i] * dot) / n : gg[i] / n);
  }
  // BCEWithLogits(pos_weight p), mean: l = (1 - y) x + (1 + (p - 1) y) softplus(-x),
  // dl/dx = (1 + (p - 1) y) sigmoid(x) - p y
  if (wv == 0) {
    const float p = pos_w ? *pos_w : 1.0f;
    float l = 0.f;
    for (int b = lane; b < B; b += 64) {
      const float x = logits[b], y = labels[b];
      const float L = 1.0f + (p - 1.0f) * y;
      l += (1.0f - y) * x + L * (log1pf(expf(-fabsf(x))) + fmaxf(-x, 0.0f));
      dlog[b] = (L / (1.0f + expf(-x)) - p * y) / (float)B;
    }
    l = wave_sum(l) / (float)B;
    if (lane == 0) {
      out[0] = l + wgt * orth;
      out[1] = l;
      out[2] = orth;
    }
  }
}

}  // namespace ewvit

using namespace ewvit;

extern "C" int ewvit_combined_loss(const float *logits, const float *labels, const float *space, const float *freq,
                                   int64_t B, int64_t D, const float *pos_weight, const float *weight, float lam,
                                   float *out, float *d_logits, float *d_space, float *d_freq, void *stream) {
  EWVIT_CHECK_ARG(logits && labels && space && freq && out && d_logits && d_space && d_freq,
                  "combined_loss: null pointer");
  EWVIT_CHECK_ARG(B >= 1 && B <= 64 && D >= 2 && D <= 512, "combined_loss: B %lld (1..64) / D %lld (2..512)",
                  (long long)B, (long long)D);
  const size_t lds = (size_t)(4 * B * D + 2 * B + 8) * sizeof(float);
  EWVIT_CHECK_ARG(lds <= 64 * 1024, "combined_loss: B * D = %lld too large for one workgroup", (long long)(B * D));
#define EWVIT_LOSS(BT_)                                                                                        \
  hipLaunchKernelGGL(combined_loss_kernel<BT_>, dim3(1), dim3(256), lds, as_stream(stream), logits, labels, space, freq, \
                     (int)B, (int)D, pos_weight, weight, lam, out, d_logits, d_space, d_freq)
  if (B <= 8) EWVIT_LOSS(8);
  else if (B <= 16) EWVIT_LOSS(16);
  else if (B <= 32) EWVIT_LOSS(32);
  else EWVIT_LOSS(64);
#undef EWVIT_LOSS
  return launch_status("combined_loss");
}
