// Short-sequence multi-head attention forward/backward (gfx950).
//
// The hot path's attentions are degenerate: the ViT runs over n = 2 tokens
// (CLS + one 7x7 patch; network/sfe.py:59-70) and the cross-attention over
// 1 query x 2 keys (x and its context, kv_include_self; network/dama.py:33-53).
// QK^T and AV are therefore 2x2 / 1x2 products per (frame, head): no MFMA
// shape fits them, and the work is a few hundred FLOPs per head.  One 64-lane
// wave owns one (batch, head): lane = head-dim element (two elements when
// d > 64), dot products reduce across the wave with DPP/shuffles, softmax in
// registers.  The projection GEMMs around it are on MFMA (gemm.hip).
#include "common.h"

namespace ewvit {

constexpr int AT_MAXN = 8;

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

struct AttnPtrs {
  const bf16_t *q, *k, *v;
  int64_t sq_b, sq_n, sk_b, sk_n, sv_b, sv_n;
};

__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnPtrs a, bf16_t *o, int64_t so_b,
                                                       int64_t so_n, float *p, int64_t B, int H,
                                                       int nq, int nk, int d, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t bh = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (bh >= B * H) return;
  const int64_t b = bh / H;
  const int h = (int)(bh % H);
  float kk[AT_MAXN][2], vv[AT_MAXN][2];
#pragma unroll
  for (int j = 0; j < AT_MAXN; ++j)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int c = lane + 64 * e;
      const bool ok = j < nk && c < d;
      kk[j][e] = ok ? bf2f(a.k[b * a.sk_b + j * a.sk_n + h * d + c]) : 0.f;
      vv[j][e] = ok ? bf2f(a.v[b * a.sv_b + j * a.sv_n + h * d + c]) : 0.f;
    }
  for (int i = 0; i < nq; ++i) {
    float qq[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int c = lane + 64 * e;
      qq[e] = c < d ? bf2f(a.q[b * a.sq_b + i * a.sq_n + h * d + c]) : 0.f;
    }
    float s[AT_MAXN];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < AT_MAXN; ++j) {
      if (j < nk) {
        s[j] = wsum(qq[0] * kk[j][0] + qq[1] * kk[j][1]) * scale;
        mx = fmaxf(mx, s[j]);
      }
    }
    float den = 0.f;
#pragma unroll
    for (int j = 0; j < AT_MAXN; ++j)
      if (j < nk) { s[j] = __expf(s[j] - mx); den += s[j]; }
    const float inv = 1.0f / den;
    float out[2] = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < AT_MAXN; ++j)
      if (j < nk) {
        const float pj = s[j] * inv;
        out[0] += pj * vv[j][0];
        out[1] += pj * vv[j][1];
        if (lane == 0 && p) p[(bh * nq + i) * nk + j] = pj;
      }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int c = lane + 64 * e;
      if (c < d) o[b * so_b + i * so_n + h * d + c] = f2bf(out[e]);
    }
  }
}

__global__ __launch_bounds__(256) void attn_bwd_kernel(AttnPtrs a, const bf16_t *dout, int64_t sdo_b,
                                                       int64_t sdo_n, const float *p, bf16_t *dq,
                                                       bf16_t *dk, bf16_t *dv, int64_t B, int H, int nq,
                                                       int nk, int d, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t bh = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (bh >= B * H) return;
  const int64_t b = bh / H;
  const int h = (int)(bh % H);
  float kk[AT_MAXN][2], vv[AT_MAXN][2], gk[AT_MAXN][2], gv[AT_MAXN][2];
#pragma unroll
  for (int j = 0; j < AT_MAXN; ++j)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int c = lane + 64 * e;
      const bool ok = j < nk && c < d;
      kk[j][e] = ok ? bf2f(a.k[b * a.sk_b + j * a.sk_n + h * d + c]) : 0.f;
      vv[j][e] = ok ? bf2f(a.v[b * a.sv_b + j * a.sv_n + h * d + c]) : 0.f;
      gk[j][e] = 0.f;
      gv[j][e] = 0.f;
    }
  for (int i = 0; i < nq; ++i) {
    float qq[2], go[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int c = lane + 64 * e;
      qq[e] = c < d ? bf2f(a.q[b * a.sq_b + i * a.sq_n + h * d + c]) : 0.f;
      go[e] = c < d ? bf2f(dout[b * sdo_b + i * sdo_n + h * d + c]) : 0.f;
    }
    float pj[AT_MAXN], dp[AT_MAXN];
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < AT_MAXN; ++j)
      if (j < nk) {
        pj[j] = p[(bh * nq + i) * nk + j];
        dp[j] = wsum(go[0] * vv[j][0] + go[1] * vv[j][1]);
        dot += pj[j] * dp[j];
      }
    float gq[2] = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < AT_MAXN; ++j)
      if (j < nk) {
        const float ds = pj[j] * (dp[j] - dot) * scale;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          gq[e] += ds * kk[j][e];
          gk[j][e] += ds * qq[e];
          gv[j][e] += pj[j] * go[e];
        }
      }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int c = lane + 64 * e;
      if (c < d) dq[b * a.sq_b + i * a.sq_n + h * d + c] = f2bf(gq[e]);
    }
  }
#pragma unroll
  for (int j = 0; j < AT_MAXN; ++j)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int c = lane + 64 * e;
      if (j < nk && c < d) {
        dk[b * a.sk_b + j * a.sk_n + h * d + c] = f2bf(gk[j][e]);
        dv[b * a.sv_b + j * a.sv_n + h * d + c] = f2bf(gv[j][e]);
      }
    }
}

}  // namespace ewvit

using namespace ewvit;

#define ATTN_CHECK(nm)                                                                        \
  EWVIT_CHECK_ARG(B >= 0 && H > 0, nm ": bad B/H");                                          \
  EWVIT_CHECK_ARG(nq >= 1 && nq <= AT_MAXN && nk >= 1 && nk <= AT_MAXN,                      \
                  nm ": nq=%d nk=%d outside [1,%d]", nq, nk, AT_MAXN);                       \
  EWVIT_CHECK_ARG(d >= 1 && d <= 128, nm ": head dim %d outside [1,128]", d)

extern "C" int ewvit_attn_fwd(const void *q, int64_t sq_b, int64_t sq_n, const void *k, int64_t sk_b,
                              int64_t sk_n, const void *v, int64_t sv_b, int64_t sv_n, void *o,
                              int64_t so_b, int64_t so_n, float *p, int64_t B, int64_t H, int nq,
                              int nk, int d, float scale, void *stream) {
  EWVIT_CHECK_ARG(q && k && v && o, "attn_fwd: null pointer");
  ATTN_CHECK("attn_fwd");
  if (B == 0) return 0;
  AttnPtrs a{(const bf16_t *)q, (const bf16_t *)k, (const bf16_t *)v, sq_b, sq_n, sk_b, sk_n, sv_b, sv_n};
  hipLaunchKernelGGL(attn_fwd_kernel, dim3((unsigned)((B * H + 3) / 4)), dim3(256), 0,
                     as_stream(stream), a, (bf16_t *)o, so_b, so_n, p, B, (int)H, nq, nk, d, scale);
  return launch_status("attn_fwd");
}

extern "C" int ewvit_attn_bwd(const void *dout, int64_t sdo_b, int64_t sdo_n, const void *q,
                              int64_t sq_b, int64_t sq_n, const void *k, int64_t sk_b, int64_t sk_n,
                              const void *v, int64_t sv_b, int64_t sv_n, const float *p, void *dq,
                              void *dk, void *dv, int64_t B, int64_t H, int nq, int nk, int d,
                              float scale, void *stream) {
  EWVIT_CHECK_ARG(dout && q && k && v && p && dq && dk && dv, "attn_bwd: null pointer");
  ATTN_CHECK("attn_bwd");
  if (B == 0) return 0;
  AttnPtrs a{(const bf16_t *)q, (const bf16_t *)k, (const bf16_t *)v, sq_b, sq_n, sk_b, sk_n, sv_b, sv_n};
  hipLaunchKernelGGL(attn_bwd_kernel, dim3((unsigned)((B * H + 3) / 4)), dim3(256), 0,
                     as_stream(stream), a, (const bf16_t *)dout, sdo_b, sdo_n, p, (bf16_t *)dq,
                     (bf16_t *)dk, (bf16_t *)dv, B, (int)H, nq, nk, d, scale);
  return launch_status("attn_bwd");
}
