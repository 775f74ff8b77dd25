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
// Statistics are numerically stable and deterministic: every block accumulates
// sums shifted by one sample per channel (row 0 of its statistics group, the
// same shift for all blocks), so partials add exactly like plain sums while the
// cancellation in E[(x-K)^2] - E[x-K]^2 stays at the scale of the variance even
// for |mean| >> std.  Partial slabs are reduced in a fixed order.
// Running stats follow torch: running = (1-m)*running + m*stat, with the unbiased
// batch variance for running_var and the biased one for normalisation.
#include "common.h"

namespace ewvit {

// raw 8-element vector of dtype DT (16 B bf16 / 32 B f32), loaded in one phase and
// unpacked in the next so a batch of rows has its loads in flight together
template <int DT> struct Raw8;
template <> struct Raw8<EWVIT_BF16> { uint4 q; };
template <> struct Raw8<EWVIT_F32> { float4 a, b; };

template <int DT>
__device__ __forceinline__ Raw8<DT> ldraw(const void *p, int64_t i) {
  Raw8<DT> r;
  if constexpr (DT == EWVIT_BF16) {
    r.q = *reinterpret_cast<const uint4 *>(reinterpret_cast<const bf16_t *>(p) + i);
  } else {
    const float4 *q = reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(p) + i);
    r.a = q[0]; r.b = q[1];
  }
  return r;
}
template <int DT>
__device__ __forceinline__ void unpack(const Raw8<DT> &r, float (&v)[8]) {
  if constexpr (DT == EWVIT_BF16) {
    const unsigned w[4] = {r.q.x, r.q.y, r.q.z, r.q.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(w[j] << 16);
      v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
    }
  } else {
    v[0] = r.a.x; v[1] = r.a.y; v[2] = r.a.z; v[3] = r.a.w; v[4] = r.b.x; v[5] = r.b.y; v[6] = r.b.z; v[7] = r.b.w;
  }
}

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

template <int ACT>
__device__ __forceinline__ float act_fwd(float z) {
  if (ACT == 1) return z > 0.f ? z : 0.f;
  if (ACT == 2) return z * __builtin_amdgcn_rcpf(1.f + __expf(-z));   // v_rcp_f32 (1 ulp), not IEEE div
  return z;
}
template <int ACT>
__device__ __forceinline__ float act_grad(float z) {
  if (ACT == 1) return z > 0.f ? 1.f : 0.f;
  if (ACT == 2) {
    const float s = __builtin_amdgcn_rcpf(1.f + __expf(-z));
    return s * (1.f + z * (1.f - s));
  }
  return 1.f;
}

struct BnPlan {
  int C8, R, threads, nblocks;
  int64_t rows_per_block;
};

// R row groups of C8 channel-vector threads per block; the block is R*C8 threads
// rounded up to whole waves (no idle quarter-blocks when C8 does not divide 256)
static void bn_shape(BnPlan &p, int64_t C) {
  p.C8 = (int)(C / 8);
  p.R = p.C8 >= 256 ? 1 : 256 / p.C8;
  p.threads = (p.R * p.C8 + 63) / 64 * 64;
}

// elementwise passes (apply, dx): ~1024 blocks (4 per CU) for the large maps, but at
// least 8 rows per thread, so the per-channel constants a thread loads are amortised
// over its rows on the small late-stage maps (e.g. 64x7x7 rows x 1536 ch); <= 64 rows
static BnPlan bn_plan(int64_t M, int64_t C) {
  BnPlan p;
  bn_shape(p, C);
  int64_t rpt = (M + (int64_t)p.R * 1024 - 1) / ((int64_t)p.R * 1024);
  rpt = rpt < 8 ? 8 : (rpt > 64 ? 64 : rpt);
  p.rows_per_block = (int64_t)p.R * rpt;
  int64_t nb = (M + p.rows_per_block - 1) / p.rows_per_block;
  if (nb < 1) nb = 1;
  p.nblocks = (int)nb;
  return p;
}

// reduction passes (stats, bwd sums): <= 256 blocks per group (the finalize sums a
// group's partial rows in one batch of loads), ~512 over all groups, >= 16 rows per
// thread, so the partial slabs stay small next to the tensor they summarise
static BnPlan bn_red_plan(int64_t M, int64_t C, int groups) {
  BnPlan p;
  bn_shape(p, C);
  int64_t nb = (512 + groups - 1) / groups;
  if (nb > 256) nb = 256;
  const int64_t maxnb = M / ((int64_t)p.R * 16);
  if (nb > maxnb) nb = maxnb;
  if (nb < 1) nb = 1;
  int64_t rpb = (M + nb - 1) / nb;
  rpb = (rpb + p.R - 1) / p.R * p.R;
  p.rows_per_block = rpb;
  p.nblocks = (int)((M + rpb - 1) / rpb);
  if (p.nblocks < 1) p.nblocks = 1;
  return p;
}

// workspace layout (floats): [groups][nred][2C] partials | [groups][C] shifts | [groups][2C] coefficients
static int64_t ws_part(const BnPlan &rp, int64_t C, int groups) { return (int64_t)groups * rp.nblocks * 2 * C; }

// the batched walk of a (row group, channel vector) thread over rows r0+rg,
// r0+rg+R, ... < r1: NB rows are loaded (`load(r)` -> raw registers) before any
// is used (`use(r, raw)`), so NB rows' loads are in flight together
template <int NB, typename L, typename U>
__device__ __forceinline__ void row_walk(int64_t r0, int64_t r1, int rg, int R, L &&load, U &&use) {
  using T = decltype(load(int64_t(0)));
  int64_t r = r0 + rg;
  for (; r + (NB - 1) * (int64_t)R < r1; r += NB * (int64_t)R) {
    T t[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) t[q] = load(r + q * (int64_t)R);
    __builtin_amdgcn_sched_barrier(0);   // keep the batch's loads ahead of their uses
#pragma unroll
    for (int q = 0; q < NB; ++q) use(r + q * (int64_t)R, t[q]);
  }
  for (; r < r1; r += R) use(r, load(r));
}

template <int DT> struct Raw8x2 { Raw8<DT> x, d; };

// ---- pass 1 (forward): per-block sums of (x - K) and (x - K)^2 per channel
template <int DT>
__global__ __launch_bounds__(256) void bn_stats_kernel(const void *__restrict__ x, int64_t M, int C, int R,
                                                       int64_t rpb, float *__restrict__ part,
                                                       float *__restrict__ shifts) {
  __shared__ float sm[256 * 8 * 2];
  // blockIdx.y = statistics group (consecutive blocks of M rows, own batch stats)
  x = reinterpret_cast<const char *>(x) + (int64_t)blockIdx.y * M * C * (DT == EWVIT_BF16 ? 2 : 4);
  part += (int64_t)blockIdx.y * gridDim.x * 2 * C;
  const int C8 = C >> 3;
  const int tid = threadIdx.x;
  const int rg = tid / C8, c8 = tid % C8;
  const bool active = rg < R && c8 < C8;
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = r0 + rpb < M ? r0 + rpb : M;
  float K[8], S[8], SS[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { K[j] = 0.f; S[j] = 0.f; SS[j] = 0.f; }
  if (active) {
    ld8<DT>(x, (int64_t)c8 * 8, K);   // the group's shift: its row 0
    if (blockIdx.x == 0 && rg == 0)
#pragma unroll
      for (int j = 0; j < 8; ++j) shifts[blockIdx.y * C + c8 * 8 + j] = K[j];
    row_walk<8>(r0, r1, rg, R, [&](int64_t rr) { return ldraw<DT>(x, rr * C + c8 * 8); },
                [&](int64_t, const Raw8<DT> &raw) {
      float v[8];
      unpack<DT>(raw, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[j] - K[j];
        S[j] += d;
        SS[j] = fmaf(d, d, SS[j]);
      }
    });
  }
  // sum the R row groups of each channel vector through LDS (fixed order)
  float *s1 = sm, *s2 = sm + 256 * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[tid * 8 + j] = S[j]; s2[tid * 8 + j] = SS[j]; }
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

// Sum the partial slab column c over nblocks rows: a block is 8 channels x 32 lanes;
// lane l loads rows l, l+32, ... (up to 256 rows in one batch of loads in flight —
// the slab was just written by other XCDs, so each dependent round trip is costly),
// then the 32 lanes combine in a fixed shuffle tree.  Every lane returns the sums.
__device__ __forceinline__ void slab_sum(const float *__restrict__ pg, int nblocks, int C, int c, bool ok,
                                         float &a, float &b) {
  const int l = threadIdx.x & 31;
  a = 0.f; b = 0.f;
  if (ok) {
    for (int k0 = 0; k0 < nblocks; k0 += 256) {
      float va[8], vb[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = k0 + l + 32 * q;
        va[q] = k < nblocks ? pg[(int64_t)k * 2 * C + c] : 0.f;
        vb[q] = k < nblocks ? pg[(int64_t)k * 2 * C + C + c] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) { a += va[q]; b += vb[q]; }
    }
  }
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
}

// ---- finalize (forward): mean / invstd per group; running stats updated group by
// group in order (the reference calls the module once per group);
// scale = gamma*invstd, shift = beta - mean*scale into ss[groups][2][C]
__global__ __launch_bounds__(256) void bn_finalize_fwd_kernel(const float *__restrict__ part, int nblocks, int groups,
                                                              int C, int64_t Mg, const float *__restrict__ shifts,
                                                              const float *__restrict__ gamma,
                                                              const float *__restrict__ beta, float *running_mean,
                                                              float *running_var, float momentum, float eps,
                                                              float *save_mean, float *save_invstd,
                                                              int64_t *counter, float *__restrict__ ss) {
  if (counter && blockIdx.x == 0 && threadIdx.x == 0) *counter += groups;
  const int c = blockIdx.x * 8 + (threadIdx.x >> 5);
  const bool ok = c < C;
  const float n = (float)Mg;
  for (int grp = 0; grp < groups; ++grp) {
    float S, SS;
    slab_sum(part + (int64_t)grp * nblocks * 2 * C, nblocks, C, c, ok, S, SS);
    if ((threadIdx.x & 31) == 0 && ok) {
      const float d = S / n;
      const float mu = shifts[grp * C + c] + d;
      const float var = fmaxf(SS / n - d * d, 0.f);
      const float inv = rsqrtf(var + eps);
      if (save_mean) save_mean[grp * C + c] = mu;
      if (save_invstd) save_invstd[grp * C + c] = inv;
      if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mu;
      if (running_var) {
        const float unb = Mg > 1 ? var * (n / (n - 1.f)) : var;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
      }
      const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
      ss[grp * 2 * C + c] = g * inv;
      ss[grp * 2 * C + C + c] = b - mu * g * inv;
    }
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
template <int DT, int ACT>
__global__ __launch_bounds__(256) void bn_apply_kernel(const void *__restrict__ x, void *__restrict__ y,
                                                       const float *__restrict__ ss, int64_t Mg, int C, int R,
                                                       int64_t rpb) {
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
  row_walk<8>(r0, r1, rg, R, [&](int64_t rr) { return ldraw<DT>(x, goff + rr * C + c); },
              [&](int64_t rr, const Raw8<DT> &raw) {
    float v[8];
    unpack<DT>(raw, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = act_fwd<ACT>(fmaf(v[j], sc[j], sh[j]));
    st8<DT>(y, goff + rr * C + c, v);
  });
}

// ---- backward pass 1: per-block sums of g and g*xhat, g = dy * act'(z)
template <int DT, int ACT>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const void *__restrict__ dy, const void *__restrict__ x,
                                                            const float *__restrict__ mean,
                                                            const float *__restrict__ invstd,
                                                            const float *__restrict__ gamma,
                                                            const float *__restrict__ beta, int64_t M, int C, int R,
                                                            int64_t rpb, float *__restrict__ part) {
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
    row_walk<8>(r0, r1, rg, R,
                [&](int64_t rr) { return Raw8x2<DT>{ldraw<DT>(x, rr * C + c8 * 8), ldraw<DT>(dy, rr * C + c8 * 8)}; },
                [&](int64_t, const Raw8x2<DT> &raw) {
      float vx[8], vd[8];
      unpack<DT>(raw.x, vx);
      unpack<DT>(raw.d, vd);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (vx[j] - mu[j]) * iv[j];
        const float g = ACT ? vd[j] * act_grad<ACT>(fmaf(xh, ga[j], be[j])) : vd[j];
        sg[j] += g;
        sgx[j] = fmaf(g, xh, sgx[j]);
      }
    });
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
  const int c = blockIdx.x * 8 + (threadIdx.x >> 5);
  const bool ok = c < C;
  float ga = 0.f, gb = 0.f;  // sums over all groups (the parameters are shared)
  for (int grp = 0; grp < groups; ++grp) {
    float a, b;
    slab_sum(part + (int64_t)grp * nblocks * 2 * C, nblocks, C, c, ok, a, b);
    if ((threadIdx.x & 31) == 0 && ok) {
      coef[grp * 2 * C + c] = a / (float)Mg;
      coef[grp * 2 * C + C + c] = b / (float)Mg;
      ga += a;
      gb += b;
    }
  }
  if ((threadIdx.x & 31) != 0 || !ok) return;
  if (dbeta) dbeta[c] = accumulate ? dbeta[c] + ga : ga;
  if (dgamma) dgamma[c] = accumulate ? dgamma[c] + gb : gb;
}

// dx = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat))
template <int DT, int ACT>
__global__ __launch_bounds__(256) void bn_bwd_dx_kernel(const void *__restrict__ dy, const void *__restrict__ x,
                                                        const float *__restrict__ mean,
                                                        const float *__restrict__ invstd,
                                                        const float *__restrict__ gamma,
                                                        const float *__restrict__ beta,
                                                        const float *__restrict__ coef, void *__restrict__ dx,
                                                        int64_t Mg, int C, int R, int64_t rpb) {
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
  row_walk<8>(r0, r1, rg, R,
              [&](int64_t rr) { return Raw8x2<DT>{ldraw<DT>(x, goff + rr * C + c), ldraw<DT>(dy, goff + rr * C + c)}; },
              [&](int64_t rr, const Raw8x2<DT> &raw) {
    const int64_t i = goff + rr * C + c;
    float vx[8], vd[8], o[8];
    unpack<DT>(raw.x, vx);
    unpack<DT>(raw.d, vd);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xh = (vx[j] - mu[j]) * iv[j];
      const float g = ACT ? vd[j] * act_grad<ACT>(fmaf(xh, ga[j], be[j])) : vd[j];
      o[j] = ga[j] * iv[j] * (g - c0[j] - xh * c1[j]);
    }
    st8<DT>(dx, i, o);
  });
}

}  // namespace ewvit

using namespace ewvit;

// instantiate launch L(dtype, act) for the runtime (dtype, act) pair
#define BN_DISPATCH(L)                                  \
  do {                                                  \
    if (dtype == EWVIT_BF16) {                          \
      if (act == 0) L(EWVIT_BF16, 0);                   \
      else if (act == 1) L(EWVIT_BF16, 1);              \
      else L(EWVIT_BF16, 2);                            \
    } else {                                            \
      if (act == 0) L(EWVIT_F32, 0);                    \
      else if (act == 1) L(EWVIT_F32, 1);               \
      else L(EWVIT_F32, 2);                             \
    }                                                   \
  } while (0)

extern "C" int64_t ewvit_bn_workspace(int64_t M, int64_t C, int groups) {
  if (groups < 1) groups = 1;
  const BnPlan rp = bn_red_plan(M / groups, C, groups);
  return (ws_part(rp, C, groups) + (int64_t)groups * 3 * C) * (int64_t)sizeof(float);
}

extern "C" int ewvit_bn_fwd(const void *x, void *y, int dtype, int64_t M, int64_t C, const float *gamma,
                            const float *beta, float *running_mean, float *running_var, int training,
                            float momentum, float eps, int act, float *save_mean, float *save_invstd,
                            int groups, int64_t *num_batches_tracked, float *workspace, void *stream) {
  EWVIT_CHECK_ARG(x && y && workspace && dtype_ok(dtype), "bn_fwd: bad args");
  EWVIT_CHECK_ARG(C > 0 && C % 8 == 0 && C <= 2048, "bn_fwd: C=%lld must be a multiple of 8, <= 2048", (long long)C);
  EWVIT_CHECK_ARG(act >= 0 && act <= 2, "bn_fwd: act=%d", act);
  EWVIT_CHECK_ARG(training || (running_mean && running_var), "bn_fwd: eval needs running stats");
  EWVIT_CHECK_ARG(groups >= 1 && groups <= 65535 && M % groups == 0, "bn_fwd: M=%lld not divisible into %d groups",
                  (long long)M, groups);
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  const int64_t Mg = M / groups;
  const BnPlan rp = bn_red_plan(Mg, C, groups);
  float *shifts = workspace + ws_part(rp, C, groups);
  float *ss = shifts + (int64_t)groups * C;
  const unsigned cblocks = (unsigned)((C + 7) / 8);
  if (training) {
    dim3 grid(rp.nblocks, groups);
    if (dtype == EWVIT_BF16)
      hipLaunchKernelGGL(bn_stats_kernel<EWVIT_BF16>, grid, dim3(rp.threads), 0, s, x, Mg, (int)C, rp.R,
                         rp.rows_per_block, workspace, shifts);
    else
      hipLaunchKernelGGL(bn_stats_kernel<EWVIT_F32>, grid, dim3(rp.threads), 0, s, x, Mg, (int)C, rp.R,
                         rp.rows_per_block, workspace, shifts);
    hipLaunchKernelGGL(bn_finalize_fwd_kernel, dim3(cblocks), dim3(256), 0, s, workspace, rp.nblocks, groups,
                       (int)C, Mg, shifts, gamma, beta, running_mean, running_var, momentum, eps, save_mean,
                       save_invstd, num_batches_tracked, ss);
  } else {
    EWVIT_CHECK_ARG(groups == 1, "bn_fwd: eval mode takes one group");
    hipLaunchKernelGGL(bn_eval_coeff_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, running_mean,
                       running_var, gamma, beta, eps, (int)C, ss);
  }
  const int64_t aMg = training ? Mg : M;
  const BnPlan ap = bn_plan(aMg, C);
  dim3 agrid(ap.nblocks, training ? groups : 1);
#define BN_APPLY(DTV, ACTV) \
  hipLaunchKernelGGL((bn_apply_kernel<DTV, ACTV>), agrid, dim3(ap.threads), 0, s, x, y, ss, aMg, (int)C, ap.R, ap.rows_per_block)
  BN_DISPATCH(BN_APPLY);
#undef BN_APPLY
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
  const BnPlan rp = bn_red_plan(Mg, C, groups);
  float *coef = workspace + ws_part(rp, C, groups) + (int64_t)groups * C;
  dim3 grid(rp.nblocks, groups);
#define BN_RED(DTV, ACTV)                                                                            \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<DTV, ACTV>), grid, dim3(rp.threads), 0, s, dy, x, save_mean, save_invstd, \
                     gamma, beta, Mg, (int)C, rp.R, rp.rows_per_block, workspace)
  BN_DISPATCH(BN_RED);
#undef BN_RED
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3((unsigned)((C + 7) / 8)), dim3(256), 0, s, workspace,
                     rp.nblocks, groups, (int)C, Mg, dgamma, dbeta, accumulate, coef);
  const BnPlan p = bn_plan(Mg, C);
  dim3 dgrid(p.nblocks, groups);
#define BN_DX(DTV, ACTV)                                                                                  \
  hipLaunchKernelGGL((bn_bwd_dx_kernel<DTV, ACTV>), dgrid, dim3(p.threads), 0, s, dy, x, save_mean, save_invstd, gamma, \
                     beta, coef, dx, Mg, (int)C, p.R, p.rows_per_block)
  BN_DISPATCH(BN_DX);
#undef BN_DX
  return launch_status("bn_bwd");
}
