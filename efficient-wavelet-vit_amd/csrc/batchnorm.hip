// BatchNorm2d (train / eval) fused with its activation, channels-last (gfx950).
//
// Every conv of the hot path is followed by BatchNorm2d + activation: ReLU in the
// MWT stack (network/mwt.py:23-72), SiLU / none in the EfficientNetV2-S backbone
// (torchvision Conv2dNormActivation, reached from network/sfe.py:111-113).  On
// MIOpen that was 3 BN kernels + a separate activation kernel each way, per layer.
// Here: forward = statistics pass + finalize + one apply pass writing act(bn(x));
// backward = one reduction pass (sum g, sum g*xhat with g = dy * act'(z)) +
// finalize + one dx pass.  x is the only saved activation (the pre-activation z
// is recomputed from it).  Layout [M = N*H*W][C], bf16 or f32; 8 channels
// (16 B for bf16) per thread.
//
// Statistics are numerically stable: each thread accumulates sums shifted by its
// first sample, converts them to (mean, M2), and (count, mean, M2) triples are
// merged with Chan's parallel formula across lanes, waves and blocks.
// Running stats follow torch: running = (1-m)*running + m*stat, with the unbiased
// batch variance for running_var and the biased one for normalisation.
#include "common.h"

namespace ewvit {

template <int DT>
__device__ __forceinline__ void ld8(const void *p, int64_t i, float (&v)[8]) {
  if (DT == EWVIT_BF16) {
    const uint4 q = *reinterpret_cast<const uint4 *>(reinterpret_cast<const bf16_t *>(p) + i);
    const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(w[j] << 16);
      v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
    }
  } else {
    const float4 *q = reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(p) + i);
    const float4 a = q[0], b = q[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}
template <int DT>
__device__ __forceinline__ void st8(void *p, int64_t i, const float (&v)[8]) {
  if (DT == EWVIT_BF16) {
    unsigned w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = (unsigned)f2bf(v[2 * j]) | ((unsigned)f2bf(v[2 * j + 1]) << 16);
    *reinterpret_cast<uint4 *>(reinterpret_cast<bf16_t *>(p) + i) = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    float4 *q = reinterpret_cast<float4 *>(reinterpret_cast<float *>(p) + i);
    q[0] = make_float4(v[0], v[1], v[2], v[3]);
    q[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
}

__device__ __forceinline__ float act_fwd(float z, int act) {
  if (act == 1) return z > 0.f ? z : 0.f;
  if (act == 2) return z / (1.f + __expf(-z));
  return z;
}
__device__ __forceinline__ float act_grad(float z, int act) {
  if (act == 1) return z > 0.f ? 1.f : 0.f;
  if (act == 2) {
    const float s = 1.f / (1.f + __expf(-z));
    return s * (1.f + z * (1.f - s));
  }
  return 1.f;
}

// Chan: merge (nb, mb, M2b) into (na, ma, M2a)
__device__ __forceinline__ void chan(float &na, float &ma, float &qa, float nb, float mb, float qb) {
  const float n = na + nb;
  if (n == 0.f) return;
  const float d = mb - ma;
  const float f = nb / n;
  ma += d * f;
  qa += qb + d * d * na * f;
  na = n;
}

struct BnPlan {
  int C8, R, nblocks;
  int64_t rows_per_block;
};

static BnPlan bn_plan(int64_t M, int64_t C) {
  BnPlan p;
  p.C8 = (int)(C / 8);
  p.R = p.C8 >= 256 ? 1 : 256 / p.C8;
  // rows per thread: aim at ~1024 blocks (4 per CU) so the small late-stage maps
  // (e.g. 64x7x7 rows x 1536 ch) still fill the chip; 1..64 rows per thread
  int64_t rpt = (M + (int64_t)p.R * 1024 - 1) / ((int64_t)p.R * 1024);
  rpt = rpt < 1 ? 1 : (rpt > 64 ? 64 : rpt);
  p.rows_per_block = (int64_t)p.R * rpt;
  int64_t nb = (M + p.rows_per_block - 1) / p.rows_per_block;
  if (nb < 1) nb = 1;
  p.nblocks = (int)nb;
  return p;
}

// ---- pass 1 (forward): per-block (mean, M2) per channel; count is rows in block
template <int DT>
__global__ __launch_bounds__(256) void bn_stats_kernel(const void *__restrict__ x, int64_t M, int C, int R,
                                                       int64_t rpb, float *__restrict__ part) {
  __shared__ float sm[256 * 8 * 3];
  // blockIdx.y = statistics group (consecutive blocks of M rows, own batch stats)
  x = reinterpret_cast<const char *>(x) + (int64_t)blockIdx.y * M * C * (DT == EWVIT_BF16 ? 2 : 4);
  part += (int64_t)blockIdx.y * gridDim.x * (2 * C + 1);
  const int C8 = C >> 3;
  const int tid = threadIdx.x;
  const int rg = tid / C8, c8 = tid % C8;
  const bool active = rg < R && c8 < C8;
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = r0 + rpb < M ? r0 + rpb : M;
  float n = 0.f, K[8], S[8], SS[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { K[j] = 0.f; S[j] = 0.f; SS[j] = 0.f; }
  if (active) {
    bool first = true;
    for (int64_t r = r0 + rg; r < r1; r += R) {
      float v[8];
      ld8<DT>(x, r * C + c8 * 8, v);
      if (first) {
#pragma unroll
        for (int j = 0; j < 8; ++j) K[j] = v[j];
        first = false;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[j] - K[j];
        S[j] += d;
        SS[j] = fmaf(d, d, SS[j]);
      }
      n += 1.f;
    }
  }
  // per-thread (n, mean, M2)
  float mean[8], m2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float mu = n > 0.f ? S[j] / n : 0.f;
    mean[j] = K[j] + mu;
    m2[j] = n > 0.f ? SS[j] - S[j] * mu : 0.f;
  }
  // merge the R row groups of each channel group through LDS (sequential, fixed order)
  float *sn = sm, *smu = sm + 256, *sq = sm + 256 + 256 * 8;
  if (active) {
    sn[tid] = n;
#pragma unroll
    for (int j = 0; j < 8; ++j) { smu[tid * 8 + j] = mean[j]; sq[tid * 8 + j] = m2[j]; }
  }
  __syncthreads();
  if (tid < C8) {
    float na = sn[tid];
    float ma[8], qa[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { ma[j] = smu[tid * 8 + j]; qa[j] = sq[tid * 8 + j]; }
    for (int g = 1; g < R; ++g) {
      const int t = g * C8 + tid;
      const float nb = sn[t];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float nn = na;
        chan(nn, ma[j], qa[j], nb, smu[t * 8 + j], sq[t * 8 + j]);
      }
      na += nb;
    }
    float *pb = part + (int64_t)blockIdx.x * (2 * C + 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      pb[tid * 8 + j] = ma[j];
      pb[C + tid * 8 + j] = qa[j];
    }
    if (tid == 0) pb[2 * C] = na;
  }
}

// ---- finalize (forward): merge blocks; save mean / invstd; update running stats;
// scale = gamma*invstd, shift = beta - mean*scale into ss[2][C]
__global__ __launch_bounds__(256) void bn_finalize_fwd_kernel(const float *__restrict__ part, int nblocks, int groups,
                                                              int C, const float *__restrict__ gamma,
                                                              const float *__restrict__ beta, float *running_mean,
                                                              float *running_var, float momentum, float eps,
                                                              float *save_mean, float *save_invstd,
                                                              float *__restrict__ ss) {
  // one block per channel: 256 threads merge strided partials, then an LDS tree;
  // statistics groups are finalised in order, so the running stats see the
  // groups' updates in sequence (the reference calls the module once per group)
  __shared__ float tn[256], tm[256], tq[256];
  const int c = blockIdx.x, t = threadIdx.x;
  for (int grp = 0; grp < groups; ++grp) {
    const float *pg = part + (int64_t)grp * nblocks * (2 * C + 1);
    float n = 0.f, mu = 0.f, q = 0.f;
    for (int b = t; b < nblocks; b += 256) {
      const float *pb = pg + (int64_t)b * (2 * C + 1);
      chan(n, mu, q, pb[2 * C], pb[c], pb[C + c]);
    }
    tn[t] = n; tm[t] = mu; tq[t] = q;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
      if (t < h) {
        float na = tn[t], ma = tm[t], qa = tq[t];
        chan(na, ma, qa, tn[t + h], tm[t + h], tq[t + h]);
        tn[t] = na; tm[t] = ma; tq[t] = qa;
      }
      __syncthreads();
    }
    if (t == 0) {
      n = tn[0]; mu = tm[0]; q = tq[0];
      const float var = n > 0.f ? q / n : 0.f;
      const float inv = rsqrtf(var + eps);
      if (save_mean) save_mean[grp * C + c] = mu;
      if (save_invstd) save_invstd[grp * C + c] = inv;
      if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mu;
      if (running_var) {
        const float unb = n > 1.f ? q / (n - 1.f) : var;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
      }
      const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
      ss[grp * 2 * C + c] = g * inv;
      ss[grp * 2 * C + C + c] = b - mu * g * inv;
    }
    __syncthreads();
  }
}

// eval: scale/shift from running stats
__global__ __launch_bounds__(256) void bn_eval_coeff_kernel(const float *__restrict__ rm, const float *__restrict__ rv,
                                                            const float *__restrict__ gamma,
                                                            const float *__restrict__ beta, float eps, int C,
                                                            float *__restrict__ ss) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = rsqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  ss[c] = g * inv;
  ss[C + c] = b - rm[c] * g * inv;
}

// ---- apply: y = act(x * scale + shift)
template <int DT>
__global__ __launch_bounds__(256) void bn_apply_kernel(const void *__restrict__ x, void *__restrict__ y,
                                                       const float *__restrict__ ss, int64_t Mg, int C, int R,
                                                       int64_t rpb, int act) {
  // grid (blocks per group, groups); thread (row group rg, channel vector c8) walks
  // rows rg, rg+R, ... of its block with its 16 coefficients held in registers
  const int C8 = C >> 3;
  const int rg = threadIdx.x / C8, c8 = threadIdx.x % C8;
  if (rg >= R) return;
  const int64_t goff = (int64_t)blockIdx.y * Mg * C;
  ss += blockIdx.y * 2 * C;
  const int c = c8 * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = ss[c + j]; sh[j] = ss[C + c + j]; }
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = r0 + rpb < Mg ? r0 + rpb : Mg;
  for (int64_t r = r0 + rg; r < r1; r += R) {
    const int64_t i = goff + r * C + c;
    float v[8];
    ld8<DT>(x, i, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = act_fwd(fmaf(v[j], sc[j], sh[j]), act);
    st8<DT>(y, i, v);
  }
}

// ---- backward pass 1: per-block sums of g and g*xhat, g = dy * act'(z)
template <int DT>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const void *__restrict__ dy, const void *__restrict__ x,
                                                            const float *__restrict__ mean,
                                                            const float *__restrict__ invstd,
                                                            const float *__restrict__ gamma,
                                                            const float *__restrict__ beta, int64_t M, int C, int R,
                                                            int64_t rpb, int act, float *__restrict__ part) {
  __shared__ float sm[256 * 8 * 2];
  // blockIdx.y = statistics group: its rows, saved stats and partial slab
  {
    const int64_t off = (int64_t)blockIdx.y * M * C * (DT == EWVIT_BF16 ? 2 : 4);
    x = reinterpret_cast<const char *>(x) + off;
    dy = reinterpret_cast<const char *>(dy) + off;
    mean += blockIdx.y * C;
    invstd += blockIdx.y * C;
    part += (int64_t)blockIdx.y * gridDim.x * 2 * C;
  }
  const int C8 = C >> 3;
  const int tid = threadIdx.x;
  const int rg = tid / C8, c8 = tid % C8;
  const bool active = rg < R && c8 < C8;
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = r0 + rpb < M ? r0 + rpb : M;
  float sg[8], sgx[8], mu[8], iv[8], ga[8], be[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sg[j] = 0.f; sgx[j] = 0.f;
    const int c = active ? c8 * 8 + j : 0;
    mu[j] = mean[c]; iv[j] = invstd[c];
    ga[j] = gamma ? gamma[c] : 1.f; be[j] = beta ? beta[c] : 0.f;
  }
  if (active) {
    for (int64_t r = r0 + rg; r < r1; r += R) {
      float vx[8], vd[8];
      ld8<DT>(x, r * C + c8 * 8, vx);
      ld8<DT>(dy, r * C + c8 * 8, vd);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (vx[j] - mu[j]) * iv[j];
        const float g = act ? vd[j] * act_grad(fmaf(xh, ga[j], be[j]), act) : vd[j];
        sg[j] += g;
        sgx[j] = fmaf(g, xh, sgx[j]);
      }
    }
  }
  float *s1 = sm, *s2 = sm + 256 * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[tid * 8 + j] = sg[j]; s2[tid * 8 + j] = sgx[j]; }
  __syncthreads();
  if (tid < C8) {
    float a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = s1[tid * 8 + j]; b[j] = s2[tid * 8 + j]; }
    for (int g = 1; g < R; ++g) {
      const int t = g * C8 + tid;
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[j] += s1[t * 8 + j]; b[j] += s2[t * 8 + j]; }
    }
    float *pb = part + (int64_t)blockIdx.x * 2 * C;
#pragma unroll
    for (int j = 0; j < 8; ++j) { pb[tid * 8 + j] = a[j]; pb[C + tid * 8 + j] = b[j]; }
  }
}

// finalize (backward): dgamma = sum g*xhat, dbeta = sum g; coefficients for dx
__global__ __launch_bounds__(256) void bn_finalize_bwd_kernel(const float *__restrict__ part, int nblocks, int groups,
                                                              int C, int64_t Mg, float *dgamma, float *dbeta,
                                                              int accumulate, float *__restrict__ coef) {
  __shared__ float ta[256], tb[256];
  const int c = blockIdx.x, t = threadIdx.x;
  float ga = 0.f, gb = 0.f;  // sums over all groups (the parameters are shared)
  for (int grp = 0; grp < groups; ++grp) {
    const float *pg = part + (int64_t)grp * nblocks * 2 * C;
    float a = 0.f, b = 0.f;
    for (int k = t; k < nblocks; k += 256) {
      a += pg[(int64_t)k * 2 * C + c];
      b += pg[(int64_t)k * 2 * C + C + c];
    }
    ta[t] = a; tb[t] = b;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
      if (t < h) { ta[t] += ta[t + h]; tb[t] += tb[t + h]; }
      __syncthreads();
    }
    if (t == 0) {
      coef[grp * 2 * C + c] = ta[0] / (float)Mg;
      coef[grp * 2 * C + C + c] = tb[0] / (float)Mg;
      ga += ta[0];
      gb += tb[0];
    }
    __syncthreads();
  }
  if (t != 0) return;
  if (dbeta) dbeta[c] = accumulate ? dbeta[c] + ga : ga;
  if (dgamma) dgamma[c] = accumulate ? dgamma[c] + gb : gb;
}

// dx = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat))
template <int DT>
__global__ __launch_bounds__(256) void bn_bwd_dx_kernel(const void *__restrict__ dy, const void *__restrict__ x,
                                                        const float *__restrict__ mean,
                                                        const float *__restrict__ invstd,
                                                        const float *__restrict__ gamma,
                                                        const float *__restrict__ beta,
                                                        const float *__restrict__ coef, void *__restrict__ dx,
                                                        int64_t Mg, int C, int R, int64_t rpb, int act) {
  // same (row group, channel vector) walk as bn_apply_kernel; per-channel
  // constants in registers: k = gamma*invstd, mean, invstd, gamma, beta, 2 coefs
  const int C8 = C >> 3;
  const int rg = threadIdx.x / C8, c8 = threadIdx.x % C8;
  if (rg >= R) return;
  const int64_t goff = (int64_t)blockIdx.y * Mg * C;
  mean += blockIdx.y * C;
  invstd += blockIdx.y * C;
  coef += blockIdx.y * 2 * C;
  const int c = c8 * 8;
  float mu[8], iv[8], ga[8], be[8], c0[8], c1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = mean[c + j]; iv[j] = invstd[c + j];
    ga[j] = gamma ? gamma[c + j] : 1.f; be[j] = beta ? beta[c + j] : 0.f;
    c0[j] = coef[c + j]; c1[j] = coef[C + c + j];
  }
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = r0 + rpb < Mg ? r0 + rpb : Mg;
  for (int64_t r = r0 + rg; r < r1; r += R) {
    const int64_t i = goff + r * C + c;
    float vx[8], vd[8], o[8];
    ld8<DT>(x, i, vx);
    ld8<DT>(dy, i, vd);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xh = (vx[j] - mu[j]) * iv[j];
      const float g = act ? vd[j] * act_grad(fmaf(xh, ga[j], be[j]), act) : vd[j];
      o[j] = ga[j] * iv[j] * (g - c0[j] - xh * c1[j]);
    }
    st8<DT>(dx, i, o);
  }
}

}  // namespace ewvit

using namespace ewvit;

extern "C" int64_t ewvit_bn_workspace(int64_t M, int64_t C, int groups) {
  if (groups < 1) groups = 1;
  const BnPlan p = bn_plan(M / groups, C);
  return ((int64_t)groups * ((int64_t)p.nblocks * (2 * C + 1) + 2 * C)) * (int64_t)sizeof(float);
}

extern "C" int ewvit_bn_fwd(const void *x, void *y, int dtype, int64_t M, int64_t C, const float *gamma,
                            const float *beta, float *running_mean, float *running_var, int training,
                            float momentum, float eps, int act, float *save_mean, float *save_invstd,
                            int groups, float *workspace, void *stream) {
  EWVIT_CHECK_ARG(x && y && workspace && dtype_ok(dtype), "bn_fwd: bad args");
  EWVIT_CHECK_ARG(C > 0 && C % 8 == 0 && C <= 2048, "bn_fwd: C=%lld must be a multiple of 8, <= 2048", (long long)C);
  EWVIT_CHECK_ARG(act >= 0 && act <= 2, "bn_fwd: act=%d", act);
  EWVIT_CHECK_ARG(training || (running_mean && running_var), "bn_fwd: eval needs running stats");
  EWVIT_CHECK_ARG(groups >= 1 && groups <= 65535 && M % groups == 0, "bn_fwd: M=%lld not divisible into %d groups",
                  (long long)M, groups);
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  const int64_t Mg = M / groups;
  const BnPlan p = bn_plan(Mg, C);
  float *ss = workspace + (int64_t)groups * p.nblocks * (2 * C + 1);
  if (training) {
    dim3 grid(p.nblocks, groups);
    if (dtype == EWVIT_BF16)
      hipLaunchKernelGGL(bn_stats_kernel<EWVIT_BF16>, grid, dim3(256), 0, s, x, Mg, (int)C, p.R,
                         p.rows_per_block, workspace);
    else
      hipLaunchKernelGGL(bn_stats_kernel<EWVIT_F32>, grid, dim3(256), 0, s, x, Mg, (int)C, p.R,
                         p.rows_per_block, workspace);
    hipLaunchKernelGGL(bn_finalize_fwd_kernel, dim3((unsigned)C), dim3(256), 0, s, workspace, p.nblocks, groups,
                       (int)C, gamma, beta, running_mean, running_var, momentum, eps, save_mean, save_invstd, ss);
  } else {
    EWVIT_CHECK_ARG(groups == 1, "bn_fwd: eval mode takes one group");
    hipLaunchKernelGGL(bn_eval_coeff_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, running_mean,
                       running_var, gamma, beta, eps, (int)C, ss);
  }
  dim3 agrid(p.nblocks, training ? groups : 1);
  const int64_t aMg = training ? Mg : M;
  const BnPlan ap = training ? p : bn_plan(M, C);
  agrid.x = ap.nblocks;
  if (dtype == EWVIT_BF16)
    hipLaunchKernelGGL(bn_apply_kernel<EWVIT_BF16>, agrid, dim3(256), 0, s, x, y, ss, aMg, (int)C, ap.R,
                       ap.rows_per_block, act);
  else
    hipLaunchKernelGGL(bn_apply_kernel<EWVIT_F32>, agrid, dim3(256), 0, s, x, y, ss, aMg, (int)C, ap.R,
                       ap.rows_per_block, act);
  return launch_status("bn_fwd");
}

extern "C" int ewvit_bn_bwd(const void *dy, const void *x, void *dx, int dtype, int64_t M, int64_t C,
                            const float *gamma, const float *beta, const float *save_mean,
                            const float *save_invstd, int act, float *dgamma, float *dbeta, int accumulate,
                            int groups, float *workspace, void *stream) {
  EWVIT_CHECK_ARG(dy && x && dx && save_mean && save_invstd && workspace && dtype_ok(dtype), "bn_bwd: bad args");
  EWVIT_CHECK_ARG(C > 0 && C % 8 == 0 && C <= 2048, "bn_bwd: C=%lld must be a multiple of 8, <= 2048", (long long)C);
  EWVIT_CHECK_ARG(act >= 0 && act <= 2, "bn_bwd: act=%d", act);
  EWVIT_CHECK_ARG(groups >= 1 && groups <= 65535 && M % groups == 0, "bn_bwd: M=%lld not divisible into %d groups",
                  (long long)M, groups);
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  const int64_t Mg = M / groups;
  const BnPlan p = bn_plan(Mg, C);
  float *coef = workspace + (int64_t)groups * p.nblocks * (2 * C + 1);
  dim3 grid(p.nblocks, groups);
  if (dtype == EWVIT_BF16)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<EWVIT_BF16>, grid, dim3(256), 0, s, dy, x, save_mean,
                       save_invstd, gamma, beta, Mg, (int)C, p.R, p.rows_per_block, act, workspace);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<EWVIT_F32>, grid, dim3(256), 0, s, dy, x, save_mean,
                       save_invstd, gamma, beta, Mg, (int)C, p.R, p.rows_per_block, act, workspace);
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3((unsigned)C), dim3(256), 0, s, workspace, p.nblocks, groups,
                     (int)C, Mg, dgamma, dbeta, accumulate, coef);
  if (dtype == EWVIT_BF16)
    hipLaunchKernelGGL(bn_bwd_dx_kernel<EWVIT_BF16>, grid, dim3(256), 0, s, dy, x, save_mean, save_invstd, gamma,
                       beta, coef, dx, Mg, (int)C, p.R, p.rows_per_block, act);
  else
    hipLaunchKernelGGL(bn_bwd_dx_kernel<EWVIT_F32>, grid, dim3(256), 0, s, dy, x, save_mean, save_invstd, gamma,
                       beta, coef, dx, Mg, (int)C, p.R, p.rows_per_block, act);
  return launch_status("bn_bwd");
}
