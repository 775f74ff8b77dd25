// LayerNorm forward/backward (gfx950): one 64-lane wave per row.
// Replaces nn.LayerNorm of network/sfe.py:23 (PreNorm, D=512) and
// network/dama.py:62,64 (cross-attention pre-norms, D=128).  Statistics in f32
// (two-pass mean / centred variance in registers), biased variance, eps inside
// the rsqrt — torch's formula.
#include "common.h"

namespace ewvit {

constexpr int LN_MAXV = 16;  // up to D = 1024 per wave

__global__ __launch_bounds__(256) void ln_fwd_kernel(const void *x, int xdt, int64_t ldx,
                                                     const float *gamma, const float *beta, void *y,
                                                     int ydt, float *mean, float *rstd, int64_t M,
                                                     int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    v[i] = (c < D) ? load_dt(x, row * ldx + c, xdt) : 0.f;
    s += v[i];
  }
  const float mu = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    const float d = (c < D) ? v[i] - mu : 0.f;
    q += d * d;
  }
  const float rs = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < D) store_dt(y, row * D + c, (v[i] - mu) * rs * gamma[c] + beta[c], ydt);
  }
  if (lane == 0) {
    if (mean) mean[row] = mu;
    if (rstd) rstd[row] = rs;
  }
}

// dx = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat)); dgamma = sum dy*xhat; dbeta = sum dy.
// Each block leaves its dgamma / dbeta partial sums in part[block][2][D]; ln_bwd_fold_kernel
// adds them in block order (deterministic, no zero-filled accumulator, no float atomics).
__global__ __launch_bounds__(256) void ln_bwd_kernel(const void *dy, int dydt, const void *x, int xdt,
                                                     int64_t ldx, const float *gamma, const float *mean,
                                                     const float *rstd, float *dx, int acc_dx,
                                                     float *part, int64_t M, int D,
                                                     int rows_per_block) {
  __shared__ float sg[4][1024];
  __shared__ float sb[4][1024];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float pg[LN_MAXV], pb[LN_MAXV];
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) { pg[i] = 0.f; pb[i] = 0.f; }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  for (int64_t row = r0 + w; row < r0 + rows_per_block && row < M; row += 4) {
    const float mu = mean[row], rs = rstd[row];
    float xh[LN_MAXV], g[LN_MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      const int c = lane + 64 * i;
      if (c < D) {
        const float d = load_dt(dy, row * D + c, dydt);
        xh[i] = (load_dt(x, row * ldx + c, xdt) - mu) * rs;
        g[i] = d * gamma[c];
        s1 += g[i];
        s2 += g[i] * xh[i];
        pg[i] += d * xh[i];
        pb[i] += d;
      } else {
        xh[i] = 0.f; g[i] = 0.f;
      }
    }
    const float m1 = wave_sum(s1) / (float)D, m2 = wave_sum(s2) / (float)D;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      const int c = lane + 64 * i;
      if (c < D) {
        const float v = rs * (g[i] - m1 - xh[i] * m2);
        const int64_t o = row * D + c;
        dx[o] = acc_dx ? dx[o] + v : v;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < D) { sg[w][c] = pg[i]; sb[w][c] = pb[i]; }
  }
  __syncthreads();
  float *pp = part + (int64_t)blockIdx.x * 2 * D;
  for (int c = threadIdx.x; c < D; c += 256) {
    pp[c] = (sg[0][c] + sg[1][c]) + (sg[2][c] + sg[3][c]);
    pp[D + c] = (sb[0][c] + sb[1][c]) + (sb[2][c] + sb[3][c]);
  }
}

// dgamma / dbeta from the per-block partials: thread per column, blocks in order
__global__ __launch_bounds__(256) void ln_bwd_fold_kernel(const float *part, int nblk, int D, float *dgamma,
                                                          float *dbeta) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= 2 * D) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += part[(int64_t)b * 2 * D + c];
  if (c < D) { if (dgamma) dgamma[c] = s; }
  else if (dbeta) dbeta[c - D] = s;
}

}  // namespace ewvit

using namespace ewvit;

extern "C" int ewvit_layernorm_fwd(const void *x, int x_dtype, int64_t ldx, const float *gamma,
                                   const float *beta, void *y, int y_dtype, float *mean, float *rstd,
                                   int64_t M, int64_t D, float eps, void *stream) {
  EWVIT_CHECK_ARG(x && gamma && beta && y, "layernorm_fwd: null pointer");
  EWVIT_CHECK_ARG(dtype_ok(x_dtype) && dtype_ok(y_dtype), "layernorm_fwd: bad dtype");
  EWVIT_CHECK_ARG(D > 0 && D <= 64 * LN_MAXV, "layernorm_fwd: D=%lld not in (0,1024]", (long long)D);
  if (M == 0) return 0;
  hipLaunchKernelGGL(ln_fwd_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, as_stream(stream), x,
                     x_dtype, ldx, gamma, beta, y, y_dtype, mean, rstd, M, (int)D, eps);
  return launch_status("layernorm_fwd");
}

static int ln_bwd_rpb(int64_t M) { return M >= 16384 ? 16 : 4; }

extern "C" int64_t ewvit_layernorm_bwd_workspace(int64_t M, int64_t D) {
  return (M + ln_bwd_rpb(M) - 1) / ln_bwd_rpb(M) * 2 * D * (int64_t)sizeof(float);
}

extern "C" int ewvit_layernorm_bwd(const void *dy, int dy_dtype, const void *x, int x_dtype,
                                   int64_t ldx, const float *gamma, const float *mean,
                                   const float *rstd, float *dx, int accumulate_dx, float *dgamma,
                                   float *dbeta, float *workspace, int64_t M, int64_t D, void *stream) {
  EWVIT_CHECK_ARG(dy && x && gamma && mean && rstd && dx && workspace, "layernorm_bwd: null pointer");
  EWVIT_CHECK_ARG(dtype_ok(dy_dtype) && dtype_ok(x_dtype), "layernorm_bwd: bad dtype");
  EWVIT_CHECK_ARG(D > 0 && D <= 64 * LN_MAXV, "layernorm_bwd: D=%lld not in (0,1024]", (long long)D);
  if (M == 0) return 0;
  // one row per wave: the token counts here are small (M = 128..512), so the grid,
  // not per-block atomics, sets the time
  const int rpb = ln_bwd_rpb(M);
  const int nblk = (int)((M + rpb - 1) / rpb);
  hipLaunchKernelGGL(ln_bwd_kernel, dim3((unsigned)nblk), dim3(256), 0,
                     as_stream(stream), dy, dy_dtype, x, x_dtype, ldx, gamma, mean, rstd, dx,
                     accumulate_dx, workspace, M, (int)D, rpb);
  if (int rc = launch_status("layernorm_bwd")) return rc;
  if (!dgamma && !dbeta) return 0;
  hipLaunchKernelGGL(ln_bwd_fold_kernel, dim3((unsigned)((2 * D + 255) / 256)), dim3(256), 0, as_stream(stream),
                     workspace, nblk, (int)D, dgamma, dbeta);
  return launch_status("layernorm_bwd fold");
}
