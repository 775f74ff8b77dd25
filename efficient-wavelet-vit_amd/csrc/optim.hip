// Multi-tensor Adam (torch.optim.Adam semantics: L2 weight decay folded into the
// gradient, bias-corrected moments, no amsgrad) for the training step of
// train.py:93-115 (the reference's optimizer, train.py:273-275: Adam lr 1e-4, wd 1e-4).
//
// One launch updates up to EWVIT_ADAM_MAX tensors, their pointers and sizes passed by
// value in the kernel arguments (so the update is graph-capturable even though the
// autograd gradients are fresh allocations every eager step).  A workgroup takes one
// 4096-element chunk of one tensor (16-B loads, 4 per thread in flight per operand);
// each tensor's step counter is a device float read by its workgroups (advanced by the
// caller before the launch), so a replayed graph keeps the bias corrections exact.
// Traffic per element: read p, g, m, v (16 B) + write p, m, v (12 B).
#include "common.h"

namespace ewvit {

constexpr int ADAM_CHUNK = 4096;   // elements per workgroup

struct AdamArgs {
  int n;                               // tensors in this launch
  int chunk0[EWVIT_ADAM_MAX + 1];      // prefix sums of chunks per tensor
  int64_t numel[EWVIT_ADAM_MAX];
  float *p[EWVIT_ADAM_MAX];
  const float *g[EWVIT_ADAM_MAX];
  float *m[EWVIT_ADAM_MAX];
  float *v[EWVIT_ADAM_MAX];
  const float *step[EWVIT_ADAM_MAX];   // per-tensor step counters (device f32)
};

// Same operation order as torch.optim.Adam's foreach path (adam.py _multi_tensor_adam):
// g += wd*p; m = lerp(m, g, 1-b1); v = v*b2 + (1-b2)*g*g; p += -step_size * m/(sqrt(v)/bc2s + eps).
__device__ __forceinline__ void adam_elem(float &p, float g, float &m, float &v, float omb1, float b2, float omb2,
                                          float wd, float neg_step_size, float bc2s, float eps) {
  g = fmaf(wd, p, g);
  m = m + omb1 * (g - m);
  v = v * b2;
  v = v + omb2 * g * g;
  const float denom = sqrtf(v) / bc2s + eps;
  p = p + neg_step_size * (m / denom);
}

// one 4096-element chunk of one tensor (both launch forms)
__device__ __forceinline__ void adam_chunk(float *__restrict__ P, const float *__restrict__ G, float *__restrict__ M,
                                          float *__restrict__ V, int64_t n, int64_t base, const float *step_ptr,
                                          double lr_host, const double *lr_dev, double b1, double b2, float eps,
                                          float wd) {
  // bias corrections in double, as torch computes them on the host (1 - 0.999^t cancels
  // badly in f32), then rounded once to the f32 scalars the element update uses
  const double st = (double)*step_ptr;
  // the learning rate from device memory when given (a replayed graph follows the caller's
  // LR schedule, train.py:274,300), else the launch-time constant
  const double lr = lr_dev ? *lr_dev : lr_host;
  const float neg_step_size = (float)(-(lr / (1.0 - pow(b1, st))));
  const float bc2s = (float)sqrt(1.0 - pow(b2, st));
  const float omb1 = (float)(1.0 - b1), omb2 = (float)(1.0 - b2), fb2 = (float)b2;
  const bool vec = ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(G) |
                     reinterpret_cast<uintptr_t>(M) | reinterpret_cast<uintptr_t>(V)) & 15) == 0;
  const int64_t end = base + ADAM_CHUNK < n ? base + ADAM_CHUNK : n;
  if (vec && end - base == ADAM_CHUNK) {
    // 4 float4 per thread and operand, loads of all four issued before any math
    float4 pv[4], gv[4], mv[4], vv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = base + (int64_t)(u * 256 + threadIdx.x) * 4;
      pv[u] = *reinterpret_cast<const float4 *>(P + i);
      gv[u] = *reinterpret_cast<const float4 *>(G + i);
      mv[u] = *reinterpret_cast<const float4 *>(M + i);
      vv[u] = *reinterpret_cast<const float4 *>(V + i);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      adam_elem(pv[u].x, gv[u].x, mv[u].x, vv[u].x, omb1, fb2, omb2, wd, neg_step_size, bc2s, eps);
      adam_elem(pv[u].y, gv[u].y, mv[u].y, vv[u].y, omb1, fb2, omb2, wd, neg_step_size, bc2s, eps);
      adam_elem(pv[u].z, gv[u].z, mv[u].z, vv[u].z, omb1, fb2, omb2, wd, neg_step_size, bc2s, eps);
      adam_elem(pv[u].w, gv[u].w, mv[u].w, vv[u].w, omb1, fb2, omb2, wd, neg_step_size, bc2s, eps);
      const int64_t i = base + (int64_t)(u * 256 + threadIdx.x) * 4;
      *reinterpret_cast<float4 *>(P + i) = pv[u];
      *reinterpret_cast<float4 *>(M + i) = mv[u];
      *reinterpret_cast<float4 *>(V + i) = vv[u];
    }
    return;
  }
  for (int64_t i = base + threadIdx.x; i < end; i += 256) {
    float p = P[i], m = M[i], v = V[i];
    adam_elem(p, G[i], m, v, omb1, fb2, omb2, wd, neg_step_size, bc2s, eps);
    P[i] = p; M[i] = m; V[i] = v;
  }
}


__global__ __launch_bounds__(256) void adam_multi_kernel(AdamArgs a, double lr_host, const double *lr_dev, double b1,
                                                         double b2, float eps, float wd) {
  // tensor of this workgroup: scalar search over the prefix sums (uniform)
  const int blk = blockIdx.x;
  int t = 0;
  while (t + 1 < a.n && a.chunk0[t + 1] <= blk) ++t;
  adam_chunk(a.p[t], a.g[t], a.m[t], a.v[t], a.numel[t], (int64_t)(blk - a.chunk0[t]) * ADAM_CHUNK, a.step[t],
             lr_host, lr_dev, b1, b2, eps, wd);
}

// every tensor of a parameter group in ONE launch: a device table of entries {p, g, m, v,
// step, numel, first chunk} (int64 words, EWVIT_ADAM_ENTRY of them per tensor); a workgroup
// finds its tensor by binary search over the first-chunk column (read-only table)
__global__ __launch_bounds__(256) void adam_table_kernel(const int64_t *__restrict__ tab, int n, double lr_host,
                                                         const double *lr_dev, double b1, double b2, float eps,
                                                         float wd) {
  const int64_t blk = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[(int64_t)mid * EWVIT_ADAM_ENTRY + 6] <= blk) lo = mid; else hi = mid - 1;
  }
  const int64_t *e = tab + (int64_t)lo * EWVIT_ADAM_ENTRY;
  adam_chunk(reinterpret_cast<float *>(e[0]), reinterpret_cast<const float *>(e[1]), reinterpret_cast<float *>(e[2]),
             reinterpret_cast<float *>(e[3]), e[5], (blk - e[6]) * ADAM_CHUNK, reinterpret_cast<const float *>(e[4]),
             lr_host, lr_dev, b1, b2, eps, wd);
}

}  // namespace ewvit

using namespace ewvit;

extern "C" int ewvit_adam_step(int n, float *const *params, const float *const *grads, float *const *exp_avg,
                               float *const *exp_avg_sq, const int64_t *numel, const float *const *steps, double lr,
                               const double *lr_dev, double beta1, double beta2, float eps, float weight_decay, void *stream) {
  EWVIT_CHECK_ARG(n >= 0 && n <= EWVIT_ADAM_MAX, "adam_step: %d tensors (max %d per launch)", n, EWVIT_ADAM_MAX);
  if (n == 0) return 0;
  AdamArgs a;
  a.n = n;
  int64_t chunks = 0;
  for (int i = 0; i < n; ++i) {
    EWVIT_CHECK_ARG(params[i] && grads[i] && exp_avg[i] && exp_avg_sq[i] && steps[i] && numel[i] > 0,
                    "adam_step: tensor %d", i);
    a.chunk0[i] = (int)chunks;
    chunks += (numel[i] + ADAM_CHUNK - 1) / ADAM_CHUNK;
    EWVIT_CHECK_ARG(chunks < ((int64_t)1 << 30), "adam_step: too many elements");
    a.numel[i] = numel[i];
    a.p[i] = params[i];
    a.g[i] = grads[i];
    a.m[i] = exp_avg[i];
    a.v[i] = exp_avg_sq[i];
    a.step[i] = steps[i];
  }
  a.chunk0[n] = (int)chunks;
  hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)chunks), dim3(256), 0, as_stream(stream), a, lr, lr_dev, beta1, beta2, eps,
                     weight_decay);
  return launch_status("adam_step");
}

extern "C" int64_t ewvit_adam_chunks(int64_t numel) { return (numel + ADAM_CHUNK - 1) / ADAM_CHUNK; }

extern "C" int ewvit_adam_step_table(const int64_t *table, int n, int64_t nchunks, double lr, const double *lr_dev,
                                     double beta1, double beta2, float eps, float weight_decay, void *stream) {
  EWVIT_CHECK_ARG(table && n > 0 && nchunks > 0 && nchunks < ((int64_t)1 << 31), "adam_step_table: bad table");
  hipLaunchKernelGGL(adam_table_kernel, dim3((unsigned)nchunks), dim3(256), 0, as_stream(stream), table, n, lr, lr_dev,
                     beta1, beta2, eps, weight_decay);
  return launch_status("adam_step_table");
}
