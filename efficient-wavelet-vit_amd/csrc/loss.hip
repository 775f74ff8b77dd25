// combined_loss of the reference's training step (train.py:55-91) in one launch, with its
// gradients: BCEWithLogits(pos_weight, mean) on the logits + w * orthogonal_loss(space, freq)
// (F.normalize rows, cov = s^T f, off-diagonal Frobenius norm^2 / (D (D - 1))).
//
// On torch this is ~15 forward and ~25 backward launches of [B, D] = [8, 128] elementwise /
// reduction kernels between the end of the forward and the start of the backward — the
// critical path of the step.  The whole problem is a few hundred KFLOP, so one workgroup
// computes the loss and every input gradient at once; the backward of the autograd op only
// scales them by the incoming gradient.
#include <algorithm>

#include "common.h"

namespace ewvit {

// LDS: u, v [B][D] normalised rows, gu, gv [B][D] their gradients, norms, reductions, and
// P - 1 ... P partial-gradient slabs [P][B][D] when the other index of cov is split P ways.
// A thread owns one cov row (column) i and every P-th j of it: its B operands and
// gradients stay in registers (BT >= B) and 1024 threads keep 16 waves in flight — one
// thread per row walked all D j's serially and the loss took ~100 us at [8, 128].
template <int BT>
__global__ __launch_bounds__(BT > 16 ? 256 : 1024) void combined_loss_kernel(const float *__restrict__ logits,
                                                             const float *__restrict__ labels,
                                                             const float *__restrict__ X, const float *__restrict__ Y,
                                                             int B, int D, int P, const float *__restrict__ pos_w,
                                                             const float *__restrict__ wdev, float lam,
                                                             float *__restrict__ out, float *__restrict__ dlog,
                                                             float *__restrict__ dX, float *__restrict__ dY) {
  extern __shared__ float sm[];
  const int BD = B * D;
  float *u = sm, *v = u + BD, *gu = v + BD, *gv = gu + BD;
  float *nx = gv + BD, *ny = nx + B;              // clamped norms
  float *red = ny + B;                            // [16]
  float *part = red + 16;                         // [P][B][D] when P > 1
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
  const float eps = 1e-12f;
  // the loads the last phase needs, issued first so their latency overlaps the rest
  const float wgt = wdev ? *wdev : lam;
  const float pw = pos_w ? *pos_w : 1.0f;
  const float xl = tid < B ? logits[tid] : 0.f, yl = tid < B ? labels[tid] : 0.f;
  for (int e = tid; e < BD; e += blockDim.x) { u[e] = X[e]; v[e] = Y[e]; }
  __syncthreads();
  // row norms (F.normalize: x / max(||x||_2, eps)), a wave per row
  for (int r = wv; r < 2 * B; r += nw) {
    const float *src = r < B ? u + r * D : v + (r - B) * D;
    float ss = 0.f;
    for (int i = lane; i < D; i += 64) ss += src[i] * src[i];
    ss = wave_sum(ss);
    if (lane == 0) (r < B ? nx[r] : ny[r - B]) = fmaxf(sqrtf(ss), eps);
  }
  __syncthreads();
  for (int e = tid; e < BD; e += blockDim.x) {
    const int b = e / D;
    u[e] = u[e] / nx[b];
    v[e] = v[e] / ny[b];
  }
  __syncthreads();
  // d(orth)/d(cov[i][j]) = k * cov[i][j] off the diagonal, k = 2 / (D (D - 1))
  const float k = 2.0f / ((float)D * (float)(D - 1));
  float sq = 0.f;
  for (int pass = 0; pass < 2; ++pass) {          // 0: rows, gu[:, i] = sum_j k c_ij v[:, j]; 1: columns
    const float *mine = pass ? v : u, *other = pass ? u : v;
    float *dst = P > 1 ? part : (pass ? gv : gu);
    for (int t = tid; t < P * D; t += blockDim.x) {
      const int own = t % D, p = t / D;           // the cov row (column) and its share of the other index
      float a[BT], g[BT];
#pragma unroll
      for (int b = 0; b < BT; ++b) { a[b] = b < B ? mine[b * D + own] : 0.f; g[b] = 0.f; }
      // rows b >= B read row B - 1 (finite) against a[b] = 0: unconditional LDS loads — a
      // guarded load per b was a branch and a wait each, 16 serial LDS round trips a j
      for (int j = p; j < D; j += P) {
        if (j == own) continue;
        float o[BT];
#pragma unroll
        for (int b = 0; b < BT; ++b) o[b] = other[(b < B ? b : B - 1) * D + j];
        float c = 0.f;
#pragma unroll
        for (int b = 0; b < BT; ++b) c += a[b] * o[b];
        if (pass == 0) sq += c * c;
#pragma unroll
        for (int b = 0; b < BT; ++b) g[b] += k * c * o[b];
      }
#pragma unroll
      for (int b = 0; b < BT; ++b)
        if (b < B) dst[(p * B + b) * D + own] = g[b];
    }
    if (P > 1) {
      __syncthreads();
      float *g = pass ? gv : gu;
      for (int e = tid; e < BD; e += blockDim.x) {
        float t = 0.f;
        for (int q = 0; q < P; ++q) t += part[q * BD + e];
        g[e] = t;
      }
      __syncthreads();                            // the slabs are rewritten by the next pass
    }
  }
  sq = wave_sum(sq);
  if (lane == 0) red[wv] = sq;
  __syncthreads();
  float tot_sq = 0.f;
  for (int w = 0; w < nw; ++w) tot_sq += red[w];
  const float orth = tot_sq / ((float)D * (float)(D - 1));
  // normalize backward, a wave per row: dx = (g - u (u . g)) / n when ||x|| > eps, else g / eps
  for (int r = wv; r < 2 * B; r += nw) {
    const int b = r < B ? r : r - B;
    const float *uu = (r < B ? u : v) + b * D, *gg = (r < B ? gu : gv) + b * D;
    float *dst = r < B ? dX + (int64_t)b * D : dY + (int64_t)b * D;
    const float n = r < B ? nx[b] : ny[b];
    float dot = 0.f;
    for (int i = lane; i < D; i += 64) dot += uu[i] * gg[i];
    dot = wave_sum(dot);
    const bool live = n > eps;                    // n = max(||x||, eps)
    for (int i = lane; i < D; i += 64) dst[i] = wgt * (live ? (gg[i] - uu[i] * dot) / n : gg[i] / n);
  }
  // BCEWithLogits(pos_weight p), mean: l = (1 - y) x + (1 + (p - 1) y) softplus(-x),
  // dl/dx = (1 + (p - 1) y) sigmoid(x) - p y
  if (wv == 0) {                                  // B <= 64: a lane per logit
    float l = 0.f;
    if (lane < B) {
      const float x = xl, y = yl;
      const float L = 1.0f + (pw - 1.0f) * y;
      l = (1.0f - y) * x + L * (log1pf(expf(-fabsf(x))) + fmaxf(-x, 0.0f));
      dlog[lane] = (L / (1.0f + expf(-x)) - pw * y) / (float)B;
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
  // the row / column split: P threads per cov row, partial slabs in the LDS left over
  const int64_t base = 4 * B * D + 2 * B + 16;
  EWVIT_CHECK_ARG(base <= 16384, "combined_loss: B * D = %lld too large for one workgroup", (long long)(B * D));
  const int nt = B > 16 ? 256 : 1024;              // B > 16: 64+ operand / gradient registers a thread
  int64_t P = std::min<int64_t>(nt / D, (16384 - base) / (B * D));
  if (P < 2) P = 1;
  const size_t lds = (size_t)(base + (P > 1 ? P * B * D : 0)) * sizeof(float);
#define EWVIT_LOSS(BT_)                                                                                         \
  hipLaunchKernelGGL(combined_loss_kernel<BT_>, dim3(1), dim3(nt), lds, as_stream(stream), logits, labels, space, \
                     freq, (int)B, (int)D, (int)P, pos_weight, weight, lam, out, d_logits, d_space, d_freq)
  if (B <= 8) EWVIT_LOSS(8);
  else if (B <= 16) EWVIT_LOSS(16);
  else if (B <= 32) EWVIT_LOSS(32);
  else EWVIT_LOSS(64);
#undef EWVIT_LOSS
  return launch_status("combined_loss");
}
