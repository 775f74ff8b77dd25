// BatchNorm2d (train / eval) fused with its activation, channels-last (gfx950).
//
// Every conv of the hot path is followed by BatchNorm2d + activation: ReLU in the
// MWT stack (network/mwt.py:23-72), SiLU / none in the EfficientNetV2-S backbone
// (torchvision Conv2dNormActivation, reached from network/sfe.py:111-113).  On
// MIOpen that was 3 BN kernels + a separate activation kernel each way, per layer.
// Here: forward = statistics pass + one apply pass writing act(bn(x)); backward =
// one reduction pass (sum g, sum g*xhat with g = dy * act'(z)) + one dx pass.  x is
// the only saved activation (the pre-activation z is recomputed from it).  Layout
// [M = N*H*W][C], bf16 or f32; 8 channels (16 B for bf16) per thread.
//
// Blocks own a CHANNEL CHUNK (<= 8 channel vectors = 64 channels, 128 B of a row)
// and a range of rows.  The reduction pass leaves at most 32 partial rows per
// chunk, so the elementwise pass finalises its own chunk's statistics from them
// (a few KB read by the block, from L2) — no separate finalize launch — and the
// blocks of row range 0 keep the books (running stats, saved mean / invstd,
// counter, dgamma / dbeta) for their chunk.
//
// Statistics are numerically stable and deterministic: every block accumulates
// sums shifted by one sample per channel (row 0 of its statistics group, the
// same shift for all blocks), so partials add exactly like plain sums while the
// cancellation in E[(x-K)^2] - E[x-K]^2 stays at the scale of the variance even
// for |mean| >> std.  Partial slabs are reduced in a fixed order.
// Running stats follow torch: running = (1-m)*running + m*stat, with the unbiased
// batch variance for running_var and the biased one for normalisation.
#include "common.h"

#include <cstdlib>

namespace ewvit {

// raw 8-element vector of dtype DT (16 B bf16 / 32 B f32), loaded in one phase and
// unpacked in the next so a batch of rows has its loads in flight together
template <int DT> struct Raw8;
template <> struct Raw8<EWVIT_BF16> { uint4 q; };
template <> struct Raw8<EWVIT_F32> { float4 a, b; };

// NT: the non-temporal hint (global_load / global_store ... nt) on the ReLU instantiations (the
// MWT's BatchNorms over 0.2-2.4 M-row maps, streamed once per pass) — compiled in only with
// EWVIT_MWT_NT=1: measured a net loss with the other MWT hints (common.h)
typedef unsigned bn_v4u __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ldq16(const void *p) {
  if constexpr (NT && EWVIT_MWT_NT) {
    const bn_v4u v = __builtin_nontemporal_load(reinterpret_cast<const bn_v4u *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *reinterpret_cast<const uint4 *>(p);
  }
}
template <bool NT>
__device__ __forceinline__ void stq16(void *p, uint4 v) {
  if constexpr (NT && EWVIT_MWT_NT) {
    __builtin_nontemporal_store(bn_v4u{v.x, v.y, v.z, v.w}, reinterpret_cast<bn_v4u *>(p));
  } else {
    *reinterpret_cast<uint4 *>(p) = v;
  }
}
template <int DT, bool NT = false>
__device__ __forceinline__ Raw8<DT> ldraw(const void *p, int64_t i) {
  Raw8<DT> r;
  if constexpr (DT == EWVIT_BF16) {
    r.q = ldq16<NT>(reinterpret_cast<const bf16_t *>(p) + i);
  } else {
    const float *f = reinterpret_cast<const float *>(p) + i;
    const uint4 a = ldq16<NT>(f), b = ldq16<NT>(f + 4);
    r.a = make_float4(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z), __uint_as_float(a.w));
    r.b = make_float4(__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z), __uint_as_float(b.w));
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
template <int DT, bool NT = false>
__device__ __forceinline__ void st8(void *p, int64_t i, const float (&v)[8]) {
  if (DT == EWVIT_BF16) {
    unsigned w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = (unsigned)f2bf(v[2 * j]) | ((unsigned)f2bf(v[2 * j + 1]) << 16);
    stq16<NT>(reinterpret_cast<bf16_t *>(p) + i, make_uint4(w[0], w[1], w[2], w[3]));
  } else {
    float *f = reinterpret_cast<float *>(p) + i;
    stq16<NT>(f, make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])));
    stq16<NT>(f + 4, make_uint4(__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7])));
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

// ---------------------------------------------------------------- geometry
struct BnGeo {
  int C8;       // channel vectors (8 channels) per row
  int CC8;      // channel vectors per block (chunk)
  int RG;       // row groups per block
  int threads;  // CC8 * RG rounded up to whole waves
  int nch;      // channel chunks
};

static BnGeo bn_geo(int64_t C) {
  BnGeo g;
  g.C8 = (int)(C / 8);
  g.CC8 = g.C8 < 8 ? g.C8 : 8;
  g.RG = 256 / g.CC8;
  g.threads = (g.CC8 * g.RG + 63) / 64 * 64;
  if (g.threads > 256) g.threads = 256;
  g.nch = (g.C8 + g.CC8 - 1) / g.CC8;
  return g;
}

// reduction passes: row chunks per (channel chunk, group) — ~512 blocks in all,
// >= 16 rows per thread, <= 256 partial rows (what an elementwise block finalises
// from: <= 128 KB of L2 reads next to the rows it streams)
// workgroup cap of the BatchNorm passes under ewvit_set_grid_cap: the convs' cap (a separate
// BatchNorm cap, 64 - 640 workgroups, measured no better: DESIGN §5.6)
static int bn_cap() { return g_grid_cap > 0 ? g_grid_cap : 0; }

// (A/B) EWVIT_BN_GEO="reduction blocks:reduction rows per thread:elementwise blocks:elementwise
// rows per thread" overrides the four constants below (read once)
static int bn_knob(int which, int dflt) {
  static int v[4] = {-1, -1, -1, -1};
  static bool init = false;
  if (!init) {
    init = true;
    if (const char *e = getenv("EWVIT_BN_GEO")) sscanf(e, "%d:%d:%d:%d", &v[0], &v[1], &v[2], &v[3]);
  }
  return v[which] > 0 ? v[which] : dflt;
}

static int bn_nrc(const BnGeo &g, int64_t M, int groups) {
  // <= 256 partial rows, >= 16 rows per thread (8 / 32 measured 0.3-2 % slower on the SFE)
  const int cap = 256, minr = bn_knob(1, 16);
  int64_t nrc = (bn_knob(0, 512) + (int64_t)g.nch * groups - 1) / ((int64_t)g.nch * groups);
  if (nrc > cap) nrc = cap;
  const int64_t maxr = M / ((int64_t)g.RG * minr);
  if (nrc > maxr) nrc = maxr;
  if (bn_cap() > 0 && nrc * g.nch * groups > bn_cap()) nrc = bn_cap() / ((int64_t)g.nch * groups);
  if (nrc < 1) nrc = 1;
  return (int)nrc;
}

// elementwise passes: ~512 blocks in all, 8..64 rows per thread (round 6: 512 / 384 against the
// earlier 1024: +0.5-0.7 % at config 2 on three boxes, profiles/r06/s2/ab/bn_geometry.log)
static int64_t bn_rows_per_block(const BnGeo &g, int64_t M, int groups) {
  const int minr = bn_knob(3, 8);  // rows per thread at least (4 / 16 measured slower)
  int64_t rb = (bn_knob(2, 512) + (int64_t)g.nch * groups - 1) / ((int64_t)g.nch * groups);
  int64_t rpt = (M + (int64_t)g.RG * rb - 1) / ((int64_t)g.RG * rb);
  rpt = rpt < minr ? minr : (rpt > 64 ? 64 : rpt);
  if (bn_cap() > 0) {            // capped grid: more rows per block, at most cap blocks in all
    int64_t nb = bn_cap() / ((int64_t)g.nch * groups);
    if (nb < 1) nb = 1;
    const int64_t need = (M + (int64_t)g.RG * nb - 1) / ((int64_t)g.RG * nb);
    if (rpt < need) rpt = need;
  }
  return (int64_t)g.RG * rpt;
}

// workspace (floats): [groups][nrc][2C] partial sums | [groups][C] shifts
static int64_t bn_ws_floats(int64_t M, int64_t C, int groups) {
  const BnGeo g = bn_geo(C);
  return (int64_t)groups * bn_nrc(g, M, groups) * 2 * C + (int64_t)groups * C;
}

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
template <int DT> struct Raw8x2s { Raw8<DT> x, d; float s; };

// StochasticDepth(row) + skip add fused into the apply pass (MBConv block tail):
// y = bn(x) * scale[n] + skip with scale[n] = (u(n) < keep) / keep, n = row / HW, u the
// counter hash of ewvit dropout (common.h); scale_out[n] keeps the factors for backward
struct BnDrop {
  const void *skip = nullptr;
  float keep = 1.f;
  uint64_t seed = 0;
  const int64_t *seed_offset = nullptr;
  float *scale_out = nullptr;
  int HW = 0;
};



// block-reduce the (CC8 x 8) pairs of sums held by every thread over its RG row
// groups (fixed order) and store them to partial row `pr` (2C floats: a | b)
__device__ __forceinline__ void bn_block_sums(float *sm, const float (&a)[8], const float (&b)[8], int cl, int rg,
                                              int CC8, int RG, int c8, int C8, int C, float *pr) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < 8; ++j) { sm[tid * 16 + j] = a[j]; sm[tid * 16 + 8 + j] = b[j]; }
  __syncthreads();
  if (rg == 0 && c8 < C8) {
    float sa[8], sb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { sa[j] = 0.f; sb[j] = 0.f; }
    for (int g = 0; g < RG; ++g) {
      const float *q = sm + (g * CC8 + cl) * 16;
#pragma unroll
      for (int j = 0; j < 8; ++j) { sa[j] += q[j]; sb[j] += q[8 + j]; }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) { pr[c8 * 8 + j] = sa[j]; pr[C + c8 * 8 + j] = sb[j]; }
  }
}

// ---- pass 1 (forward): partial sums of (x - K) and (x - K)^2 per channel;
// grid (row chunks, channel chunks, groups).  K = row 0 of the group (one sample per
// channel, the same for every block): partials add like plain sums while the
// cancellation of E[(x-K)^2] - E[x-K]^2 stays at the scale of the variance.
template <int DT>
__global__ __launch_bounds__(256) void bn_stats_kernel(const void *__restrict__ x, int64_t M, int C, int CC8, int RG,
                                                       int64_t rpc, float *__restrict__ part,
                                                       float *__restrict__ shifts) {
  __shared__ float sm[256 * 16];
  const int grp = blockIdx.z, nrc = gridDim.x;
  x = reinterpret_cast<const char *>(x) + (int64_t)grp * M * C * (DT == EWVIT_BF16 ? 2 : 4);
  const int C8 = C >> 3;
  const int tid = threadIdx.x, cl = tid % CC8, rg = tid / CC8;
  const int c8 = blockIdx.y * CC8 + cl;
  const bool active = rg < RG && c8 < C8;
  const int64_t r0 = (int64_t)blockIdx.x * rpc, r1 = r0 + rpc < M ? r0 + rpc : M;
  float K[8], S[8], SS[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { K[j] = 0.f; S[j] = 0.f; SS[j] = 0.f; }
  if (active) {
    ld8<DT>(x, (int64_t)c8 * 8, K);
    if (blockIdx.x == 0 && rg == 0)
#pragma unroll
      for (int j = 0; j < 8; ++j) shifts[grp * C + c8 * 8 + j] = K[j];
    row_walk<8>(r0, r1, rg, RG, [&](int64_t rr) { return ldraw<DT>(x, rr * C + c8 * 8); },
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
  bn_block_sums(sm, S, SS, cl, rg, CC8, RG, c8, C8, C, part + ((int64_t)grp * nrc + blockIdx.x) * 2 * C);
}

// LDS-only workgroup barrier: waits for this wave's LDS ops, not for its global loads
// (a __syncthreads() fence would also drain the row loads issued ahead of the finalize)
__device__ __forceinline__ void bn_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// the chunk's per-channel sums over the nrc partial rows of group grp: 64 channels x 4
// lanes, each lane its slice of rows (8 loads in flight) -> (a, b); bn_chunk_reduce
// combines the 4 lanes in fixed order into LDS red[0][ch], red[1][ch] (ch < 8*CC8)
__device__ __forceinline__ void bn_chunk_load(const float *__restrict__ part, int grp, int nrc, int C, int ch0,
                                              int nch_c, float &a, float &b) {
  const int tid = threadIdx.x, j = tid & 63, q = tid >> 6;
  a = 0.f; b = 0.f;
  if (j < nch_c && q * 64 < (int)blockDim.x) {
    const float *pg = part + (int64_t)grp * nrc * 2 * C + ch0 + j;
    for (int k0 = q; k0 < nrc; k0 += 32) {
      float va[8], vb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + 4 * u;
        va[u] = k < nrc ? pg[(int64_t)k * 2 * C] : 0.f;
        vb[u] = k < nrc ? pg[(int64_t)k * 2 * C + C] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) { a += va[u]; b += vb[u]; }
    }
  }
}
__device__ __forceinline__ void bn_chunk_reduce(float *red, float a, float b) {
  const int tid = threadIdx.x;
  float *ra = red, *rb = red + 256;
  ra[tid] = a;
  rb[tid] = b;
  bn_sync();
  if (tid < 64) {
    float sa = 0.f, sb = 0.f;
    for (int k = 0; k * 64 < (int)blockDim.x; ++k) { sa += ra[k * 64 + tid]; sb += rb[k * 64 + tid]; }
    ra[tid] = sa;
    rb[tid] = sb;
  }
  bn_sync();
}
__device__ __forceinline__ void bn_chunk_sums(const float *__restrict__ part, int grp, int nrc, int C, int ch0,
                                              int nch_c, float *red) {
  float a, b;
  bn_chunk_load(part, grp, nrc, C, ch0, nch_c, a, b);
  bn_chunk_reduce(red, a, b);
}

// row_walk whose first batch of NB rows is loaded BEFORE fin() (the block's statistics
// finalize, run by every thread) so the two latency chains overlap
template <int NB, typename L, typename U, typename F>
__device__ __forceinline__ void row_walk_pf(bool active, int64_t r0, int64_t r1, int rg, int R, L &&load, U &&use,
                                            F &&fin) {
  using T = decltype(load(int64_t(0)));
  int64_t r = r0 + rg;
  T t[NB];
  const bool full = active && r + (NB - 1) * (int64_t)R < r1;
  if (full) {
#pragma unroll
    for (int q = 0; q < NB; ++q) t[q] = load(r + q * (int64_t)R);
  }
  fin();
  if (!active) return;
  if (full) {
#pragma unroll
    for (int q = 0; q < NB; ++q) use(r + q * (int64_t)R, t[q]);
    r += NB * (int64_t)R;
  }
  for (; r + (NB - 1) * (int64_t)R < r1; r += NB * (int64_t)R) {
    T u[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) u[q] = load(r + q * (int64_t)R);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < NB; ++q) use(r + q * (int64_t)R, u[q]);
  }
  for (; r < r1; r += R) use(r, load(r));
}

// ---- apply: y = act(x * scale + shift).  Training: the block finalises its chunk's
// batch statistics from the partial rows; blocks of row range 0 of group 0 update
// the running statistics group after group (the reference calls the module once per
// group) and save mean / invstd.  Eval: coefficients from the running statistics.
template <int DT, int ACT, bool DROP = false>
__global__ __launch_bounds__(256) void bn_apply_kernel(const void *__restrict__ x, void *__restrict__ y,
                                                       const float *__restrict__ part,
                                                       const float *__restrict__ shifts, int nrc, int64_t Mg, int C,
                                                       int CC8, int RG, int64_t rpb, int training,
                                                       const float *__restrict__ gamma,
                                                       const float *__restrict__ beta, float *running_mean,
                                                       float *running_var, float momentum, float eps, float *save_mean,
                                                       float *save_invstd, int64_t *counter, BnDrop dr = BnDrop(),
                                                       float *coef_out = nullptr) {
  __shared__ float red[512];
  __shared__ float coef[2][64];
  const int grp = blockIdx.z, groups = gridDim.z;
  const int tid = threadIdx.x, C8 = C >> 3;
  const int ch0 = blockIdx.y * CC8 * 8;
  const int nch_c = (C - ch0) < CC8 * 8 ? (C - ch0) : CC8 * 8;
  const float n = (float)Mg;
  const bool book = training && blockIdx.x == 0 && grp == 0;
  // this block's partial-row loads first, then its first batch of rows (row_walk_pf)
  float pa = 0.f, pb = 0.f;
  if (training && !(book && groups > 1)) bn_chunk_load(part, grp, nrc, C, ch0, nch_c, pa, pb);
  const int cl = tid % CC8, rg = tid / CC8;
  const int c8 = blockIdx.y * CC8 + cl;
  const bool active = rg < RG && c8 < C8;
  const int64_t goff = (int64_t)grp * Mg * C;
  const int c = active ? c8 * 8 : 0;
  float sc[8], sh[8];
  auto fin = [&]() {
    if (training) {
      if (book) {
        if (counter && blockIdx.y == 0 && tid == 0) *counter += groups;
        float rm = 0.f, rv = 0.f;
        const int cc = ch0 + tid;
        if (tid < nch_c) { rm = running_mean ? running_mean[cc] : 0.f; rv = running_var ? running_var[cc] : 0.f; }
        for (int g = 0; g < groups; ++g) {
          if (groups > 1) bn_chunk_load(part, g, nrc, C, ch0, nch_c, pa, pb);
          bn_chunk_reduce(red, pa, pb);
          if (tid < nch_c) {
            const float d = red[tid] / n, mu = shifts[g * C + cc] + d;
            const float var = fmaxf(red[256 + tid] / n - d * d, 0.f);
            if (save_mean) save_mean[g * C + cc] = mu;
            if (save_invstd) save_invstd[g * C + cc] = rsqrtf(var + eps);
            rm = (1.f - momentum) * rm + momentum * mu;
            rv = (1.f - momentum) * rv + momentum * (Mg > 1 ? var * (n / (n - 1.f)) : var);
            if (g == grp) {
              const float inv = rsqrtf(var + eps);
              const float ga = gamma ? gamma[cc] : 1.f, be = beta ? beta[cc] : 0.f;
              coef[0][tid] = ga * inv;
              coef[1][tid] = be - mu * ga * inv;
              if (coef_out) {
                coef_out[(2 * grp) * C + cc] = coef[0][tid];
                coef_out[(2 * grp + 1) * C + cc] = coef[1][tid];
              }
            }
          }
          bn_sync();
        }
        if (tid < nch_c) {
          if (running_mean) running_mean[cc] = rm;
          if (running_var) running_var[cc] = rv;
        }
      } else {
        bn_chunk_reduce(red, pa, pb);
        if (tid < nch_c) {
          const int cc = ch0 + tid;
          const float d = red[tid] / n, mu = shifts[grp * C + cc] + d;
          const float var = fmaxf(red[256 + tid] / n - d * d, 0.f);
          const float inv = rsqrtf(var + eps);
          const float ga = gamma ? gamma[cc] : 1.f, be = beta ? beta[cc] : 0.f;
          coef[0][tid] = ga * inv;
          coef[1][tid] = be - mu * ga * inv;
          if (coef_out && blockIdx.x == 0) {
            coef_out[(2 * grp) * C + cc] = coef[0][tid];
            coef_out[(2 * grp + 1) * C + cc] = coef[1][tid];
          }
        }
      }
    } else if (tid < nch_c) {
      const int cc = ch0 + tid;
      const float inv = rsqrtf(running_var[cc] + eps);
      const float ga = gamma ? gamma[cc] : 1.f, be = beta ? beta[cc] : 0.f;
      coef[0][tid] = ga * inv;
      coef[1][tid] = be - running_mean[cc] * ga * inv;
    }
    bn_sync();
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = coef[0][cl * 8 + j]; sh[j] = coef[1][cl * 8 + j]; }
  };
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = r0 + rpb < Mg ? r0 + rpb : Mg;
  if constexpr (!DROP) {
    row_walk_pf<8>(active, r0, r1, rg, RG, [&](int64_t rr) { return ldraw<DT, ACT == 1>(x, goff + rr * C + c); },
                   [&](int64_t rr, const Raw8<DT> &raw) {
      float v[8];
      unpack<DT>(raw, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = act_fwd<ACT>(fmaf(v[j], sc[j], sh[j]));
      st8<DT, ACT == 1>(y, goff + rr * C + c, v);
    }, fin);
  } else {
    const uint64_t sd = step_seed(dr.seed, dr.seed_offset);
    row_walk_pf<8>(active, r0, r1, rg, RG,
                   [&](int64_t rr) { return Raw8x2<DT>{ldraw<DT>(x, rr * C + c), ldraw<DT>(dr.skip, rr * C + c)}; },
                   [&](int64_t rr, const Raw8x2<DT> &raw) {
      const int nn = (int)rr / dr.HW;
      const float ks = uniform01(sd, (uint64_t)nn) < dr.keep ? 1.f / dr.keep : 0.f;
      if (dr.scale_out && (int)rr == nn * dr.HW && c8 == 0) dr.scale_out[nn] = ks;
      float v[8], vs[8];
      unpack<DT>(raw.x, v);
      unpack<DT>(raw.d, vs);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaf(act_fwd<ACT>(fmaf(v[j], sc[j], sh[j])), ks, vs[j]);
      st8<DT>(y, rr * C + c, v);
    }, fin);
  }
}

// SC == 2: the BatchNorm's output gradient is the squeeze-excitation input gradient
// dy * s[n][c] + g[n][c] (ewvit_se_scale's backward, s the excitation, g the squeeze term),
// formed on the fly from the SE output gradient
__device__ __forceinline__ void se_affine(float (&v)[8], const float *__restrict__ s, const float *__restrict__ g,
                                          int64_t n, int C, int c) {
  const float4 *sp = reinterpret_cast<const float4 *>(s + n * C + c);
  const float4 *gp = reinterpret_cast<const float4 *>(g + n * C + c);
  const float4 s0 = sp[0], s1 = sp[1], g0 = gp[0], g1 = gp[1];
  const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j], sv[j], gv[j]);
}

// the se_affine tables of the frames of rows [r0, r1) and the block's channel chunk, staged in
// LDS (tab[0][f][ch] = s, tab[1][f][ch] = g, f relative to frame f0): a row then reads its 8
// channels' factors from LDS instead of four 16-B global loads.  Returns false (use global
// loads) when the rows span more than SE_MAXF frames.
constexpr int SE_MAXF = 16;
__device__ __forceinline__ bool se_stage(float *tab, const float *__restrict__ s, const float *__restrict__ g,
                                         int64_t r0, int64_t r1, int HW, int C, int ch0, int nch_c, int64_t &f0) {
  f0 = r0 / HW;
  const int nf = r1 > r0 ? (int)((r1 - 1) / HW - f0 + 1) : 0;
  if (nf > SE_MAXF) return false;
  for (int i = threadIdx.x; i < nf * 64; i += blockDim.x) {
    const int f = i >> 6, ch = i & 63;
    if (ch < nch_c) {
      tab[f * 64 + ch] = s[(f0 + f) * C + ch0 + ch];
      tab[SE_MAXF * 64 + f * 64 + ch] = g[(f0 + f) * C + ch0 + ch];
    }
  }
  __syncthreads();
  return true;
}
__device__ __forceinline__ void se_affine_lds(float (&v)[8], const float *tab, int f, int cl) {
  const float4 *sp = reinterpret_cast<const float4 *>(tab + f * 64 + cl * 8);
  const float4 *gp = reinterpret_cast<const float4 *>(tab + SE_MAXF * 64 + f * 64 + cl * 8);
  const float4 s0 = sp[0], s1 = sp[1], g0 = gp[0], g1 = gp[1];
  const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j], sv[j], gv[j]);
}

// ---- backward pass 1: partial sums of g and g*xhat, g = dy * act'(z); SC 1: dy scaled
// per row group (rscale[row / HW], the drop-path tail), SC 2: dy -> dy * s + g (se_affine)
template <int DT, int ACT, int SC = 0>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const void *__restrict__ dy, const void *__restrict__ x,
                                                            const float *__restrict__ mean,
                                                            const float *__restrict__ invstd,
                                                            const float *__restrict__ gamma,
                                                            const float *__restrict__ beta, int64_t M, int C, int CC8,
                                                            int RG, int64_t rpc, float *__restrict__ part,
                                                            const float *__restrict__ rscale = nullptr, int HW = 1,
                                                            const float *__restrict__ se_g = nullptr) {
  __shared__ float sm[256 * 16];
  const int grp = blockIdx.z, nrc = gridDim.x;
  {
    const int64_t off = (int64_t)grp * M * C * (DT == EWVIT_BF16 ? 2 : 4);
    x = reinterpret_cast<const char *>(x) + off;
    dy = reinterpret_cast<const char *>(dy) + off;
    mean += grp * C;
    invstd += grp * C;
  }
  const int C8 = C >> 3;
  const int tid = threadIdx.x, cl = tid % CC8, rg = tid / CC8;
  const int c8 = blockIdx.y * CC8 + cl;
  const bool active = rg < RG && c8 < C8;
  const int64_t r0 = (int64_t)blockIdx.x * rpc, r1 = r0 + rpc < M ? r0 + rpc : M;
  __shared__ __attribute__((aligned(16))) float tab[SC == 2 ? 2 * SE_MAXF * 64 : 4];
  int64_t f0 = 0;
  bool ltab = false;
  if constexpr (SC == 2) {
    const int ch0 = blockIdx.y * CC8 * 8;
    ltab = se_stage(tab, rscale, se_g, r0, r1, HW, C, ch0, (C - ch0) < CC8 * 8 ? (C - ch0) : CC8 * 8, f0);
  }
  float sg[8], sgx[8], mu[8], iv[8], ga[8], be[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sg[j] = 0.f; sgx[j] = 0.f;
    const int c = active ? c8 * 8 + j : 0;
    mu[j] = mean[c]; iv[j] = invstd[c];
    ga[j] = gamma ? gamma[c] : 1.f; be[j] = beta ? beta[c] : 0.f;
  }
  if (active) {
    row_walk<8>(r0, r1, rg, RG,
                [&](int64_t rr) {
                  return Raw8x2s<DT>{ldraw<DT, ACT == 1>(x, rr * C + c8 * 8), ldraw<DT, ACT == 1>(dy, rr * C + c8 * 8),
                                     SC == 1 ? rscale[(int)rr / HW] : 1.f};
                },
                [&](int64_t rr, const Raw8x2s<DT> &raw) {
      float vx[8], vd[8];
      unpack<DT>(raw.x, vx);
      unpack<DT>(raw.d, vd);
      if (SC == 2) {
        if (ltab) se_affine_lds(vd, tab, (int)(rr / HW - f0), cl);
        else se_affine(vd, rscale, se_g, rr / HW, C, c8 * 8);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (SC == 1) vd[j] *= raw.s;
        const float xh = (vx[j] - mu[j]) * iv[j];
        const float g = ACT ? vd[j] * act_grad<ACT>(fmaf(xh, ga[j], be[j])) : vd[j];
        sg[j] += g;
        sgx[j] = fmaf(g, xh, sgx[j]);
      }
    });
  }
  bn_block_sums(sm, sg, sgx, cl, rg, CC8, RG, c8, C8, C, part + ((int64_t)grp * nrc + blockIdx.x) * 2 * C);
}

// dx = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat)); the block finalises its chunk's
// two means from the partial rows; blocks of row range 0 of group 0 write
// dgamma = sum g*xhat, dbeta = sum g (over all groups: the parameters are shared)
template <int DT, int ACT, int SC = 0>
__global__ __launch_bounds__(256) void bn_bwd_dx_kernel(const void *__restrict__ dy, const void *__restrict__ x,
                                                        const float *__restrict__ mean,
                                                        const float *__restrict__ invstd,
                                                        const float *__restrict__ gamma,
                                                        const float *__restrict__ beta,
                                                        const float *__restrict__ part, int nrc,
                                                        void *__restrict__ dx, int64_t Mg, int C, int CC8, int RG,
                                                        int64_t rpb, float *dgamma, float *dbeta, int accumulate,
                                                        const float *__restrict__ rscale = nullptr, int HW = 1,
                                                        const float *__restrict__ se_g = nullptr) {
  __shared__ float red[512];
  __shared__ float coef[2][64];
  const int grp = blockIdx.z, groups = gridDim.z;
  const int tid = threadIdx.x, C8 = C >> 3;
  const int ch0 = blockIdx.y * CC8 * 8;
  const int nch_c = (C - ch0) < CC8 * 8 ? (C - ch0) : CC8 * 8;
  const float n = (float)Mg;
  const bool book = blockIdx.x == 0 && grp == 0;
  // partial-row loads first, then the first batch of rows (row_walk_pf), then finalize
  float pa = 0.f, pb = 0.f;
  if (!(book && groups > 1)) bn_chunk_load(part, grp, nrc, C, ch0, nch_c, pa, pb);
  const int cl = tid % CC8, rg = tid / CC8;
  const int c8 = blockIdx.y * CC8 + cl;
  const bool active = rg < RG && c8 < C8;
  const int64_t goff = (int64_t)grp * Mg * C;
  const int c = active ? c8 * 8 : 0;
  float mu[8], iv[8], ga[8], be[8], c0[8], c1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = mean[grp * C + c + j]; iv[j] = invstd[grp * C + c + j];
    ga[j] = gamma ? gamma[c + j] : 1.f; be[j] = beta ? beta[c + j] : 0.f;
  }
  auto fin = [&]() {
    if (book) {
      float sa = 0.f, sb = 0.f;
      for (int g = 0; g < groups; ++g) {
        if (groups > 1) bn_chunk_load(part, g, nrc, C, ch0, nch_c, pa, pb);
        bn_chunk_reduce(red, pa, pb);
        if (tid < nch_c) {
          sa += red[tid];
          sb += red[256 + tid];
          if (g == grp) { coef[0][tid] = red[tid] / n; coef[1][tid] = red[256 + tid] / n; }
        }
        bn_sync();
      }
      if (tid < nch_c) {
        const int cc = ch0 + tid;
        if (dbeta) dbeta[cc] = accumulate ? dbeta[cc] + sa : sa;
        if (dgamma) dgamma[cc] = accumulate ? dgamma[cc] + sb : sb;
      }
    } else {
      bn_chunk_reduce(red, pa, pb);
      if (tid < nch_c) { coef[0][tid] = red[tid] / n; coef[1][tid] = red[256 + tid] / n; }
    }
    bn_sync();
#pragma unroll
    for (int j = 0; j < 8; ++j) { c0[j] = coef[0][cl * 8 + j]; c1[j] = coef[1][cl * 8 + j]; }
  };
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = r0 + rpb < Mg ? r0 + rpb : Mg;
  __shared__ __attribute__((aligned(16))) float tab[SC == 2 ? 2 * SE_MAXF * 64 : 4];
  int64_t f0 = 0;
  bool ltab = false;
  if constexpr (SC == 2) ltab = se_stage(tab, rscale, se_g, r0, r1, HW, C, ch0, nch_c, f0);
  row_walk_pf<8>(active, r0, r1, rg, RG,
                 [&](int64_t rr) {
                   return Raw8x2s<DT>{ldraw<DT, ACT == 1>(x, goff + rr * C + c), ldraw<DT, ACT == 1>(dy, goff + rr * C + c),
                                      SC == 1 ? rscale[(int)rr / HW] : 1.f};
                 },
                 [&](int64_t rr, const Raw8x2s<DT> &raw) {
    float vx[8], vd[8], o[8];
    unpack<DT>(raw.x, vx);
    unpack<DT>(raw.d, vd);
    if (SC == 2) {
      if (ltab) se_affine_lds(vd, tab, (int)(rr / HW - f0), cl);
      else se_affine(vd, rscale, se_g, rr / HW, C, c);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (SC == 1) vd[j] *= raw.s;
      const float xh = (vx[j] - mu[j]) * iv[j];
      const float g = ACT ? vd[j] * act_grad<ACT>(fmaf(xh, ga[j], be[j])) : vd[j];
      o[j] = ga[j] * iv[j] * (g - c0[j] - xh * c1[j]);
    }
    st8<DT, ACT == 1>(dx, goff + rr * C + c, o);
  }, fin);
}

// MBConv's depthwise BatchNorm + SiLU (training, statistics from partial rows, one group)
// and the squeeze of the squeeze-excitation after it in ONE pass: block (frame n, 64-channel
// chunk) finalises its chunk's statistics from the partial rows (the depthwise conv's,
// ewvit_dwconv3x3_fwd_bn) as bn_apply_kernel does (blocks of frame 0 keep the books), applies
// BN + act to the frame's HW rows of its chunk, and sums the stored (rounded) outputs per
// channel — the squeeze s0 = mean_hw y — then leaves the chunk's partial of the SE MLP's
// first layer, part[n][chunk][j] = sum_{c in chunk} W1[j][c] s0[n][c].  The same operations
// in the same order as bn_apply_kernel + se_sq_h1_part_kernel (8 channel vectors x 32 row
// groups, rows rg, rg + 32, ... added in order, then the fixed tree over the row groups), so
// the same bits, one launch and one pass over the tensor fewer.
template <int DT, int ACT>
__global__ __launch_bounds__(256) void bn_act_squeeze_kernel(const void *__restrict__ x, void *__restrict__ y,
                                                             const float *__restrict__ part,
                                                             const float *__restrict__ shifts, int nrc, int HW, int C,
                                                             const float *__restrict__ gamma,
                                                             const float *__restrict__ beta, float *running_mean,
                                                             float *running_var, float momentum, float eps,
                                                             float *save_mean, float *save_invstd, int64_t *counter,
                                                             float inv_hw, const float *__restrict__ w1, int Csq,
                                                             float *__restrict__ s0_out, float *__restrict__ hpart) {
  __shared__ float red[512];
  __shared__ float coef[2][64];
  __shared__ float sm[8 * 256];
  const int tid = threadIdx.x, C8 = C >> 3, nfr = gridDim.x, n = blockIdx.x, cb = blockIdx.y;
  const int ch0 = cb * 64;
  const int nch_c = (C - ch0) < 64 ? (C - ch0) : 64;
  const int64_t Mg = (int64_t)nfr * HW;
  const float nf = (float)Mg;
  const bool book = n == 0;
  float pa = 0.f, pb = 0.f;
  bn_chunk_load(part, 0, nrc, C, ch0, nch_c, pa, pb);
  const int cv = tid & 7, rg = tid >> 3;
  const int c8 = cb * 8 + cv;
  const bool active = c8 < C8;
  const int c = active ? c8 * 8 : 0;
  const int64_t base = (int64_t)n * HW * C + c;
  // first batch of this thread's rows in flight before the statistics finalise
  constexpr int PF = 4;
  Raw8<DT> pre[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q)
    if (active && rg + 32 * q < HW) pre[q] = ldraw<DT>(x, base + (int64_t)(rg + 32 * q) * C);
  bn_chunk_reduce(red, pa, pb);
  if (tid < nch_c) {
    const int cc = ch0 + tid;
    const float d = red[tid] / nf, mu = shifts[cc] + d;
    const float var = fmaxf(red[256 + tid] / nf - d * d, 0.f);
    const float inv = rsqrtf(var + eps);
    const float ga = gamma ? gamma[cc] : 1.f, be = beta ? beta[cc] : 0.f;
    coef[0][tid] = ga * inv;
    coef[1][tid] = be - mu * ga * inv;
    if (book) {
      if (counter && cb == 0 && tid == 0) *counter += 1;
      if (save_mean) save_mean[cc] = mu;
      if (save_invstd) save_invstd[cc] = inv;
      if (running_mean) running_mean[cc] = (1.f - momentum) * running_mean[cc] + momentum * mu;
      if (running_var)
        running_var[cc] = (1.f - momentum) * running_var[cc] + momentum * (Mg > 1 ? var * (nf / (nf - 1.f)) : var);
    }
  }
  bn_sync();
  float sc[8], sh[8], acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = coef[0][cv * 8 + j]; sh[j] = coef[1][cv * 8 + j]; acc[j] = 0.f; }
  auto apply = [&](int h, const Raw8<DT> &raw) {
    float v[8];
    unpack<DT>(raw, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = act_fwd<ACT>(fmaf(v[j], sc[j], sh[j]));
    st8<DT>(y, base + (int64_t)h * C, v);
    float r[8];                                        // the stored values, as the squeeze reads them
    if constexpr (DT == EWVIT_BF16) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = bf2f(f2bf(v[j]));
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = v[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += r[j];
  };
  if (active) {
#pragma unroll
    for (int q = 0; q < PF; ++q)
      if (rg + 32 * q < HW) apply(rg + 32 * q, pre[q]);
    for (int h0 = rg + 32 * PF; h0 < HW; h0 += 32 * PF) {
      Raw8<DT> t[PF];
#pragma unroll
      for (int q = 0; q < PF; ++q)
        if (h0 + 32 * q < HW) t[q] = ldraw<DT>(x, base + (int64_t)(h0 + 32 * q) * C);
#pragma unroll
      for (int q = 0; q < PF; ++q)
        if (h0 + 32 * q < HW) apply(h0 + 32 * q, t[q]);
    }
  }
  // squeeze: the fixed tree of se_chunk_squeeze over the 32 row groups
#pragma unroll
  for (int j = 0; j < 8; ++j) sm[j * 256 + tid] = acc[j];
  __syncthreads();
  for (int st = 16; st >= 1; st >>= 1) {
    if (rg < st)
#pragma unroll
      for (int j = 0; j < 8; ++j) sm[j * 256 + tid] += sm[j * 256 + tid + st * 8];
    __syncthreads();
  }
  const int l = tid & 63, w = tid >> 6;
  const int cl = ch0 + l;
  const float xv = cl < C ? sm[(l & 7) * 256 + (l >> 3)] * inv_hw : 0.f;
  if (w == 0 && cl < C) s0_out[(int64_t)n * C + cl] = xv;
  float *pp = hpart + ((int64_t)n * gridDim.y + cb) * Csq;
  for (int j0 = w; j0 < Csq; j0 += 16) {
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = j0 + 4 * q;
      v[q] = (j < Csq && cl < C) ? w1[(int64_t)j * C + cl] * xv : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = wave_sum(v[q]);
      const int j = j0 + 4 * q;
      if (l == 0 && j < Csq) pp[j] = v[q];
    }
  }
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
  return bn_ws_floats(M / groups, C, groups) * (int64_t)sizeof(float);
}

extern "C" int ewvit_bn_fwd(const void *x, void *y, int dtype, int64_t M, int64_t C, const float *gamma,
                            const float *beta, float *running_mean, float *running_var, int training,
                            float momentum, float eps, int act, float *save_mean, float *save_invstd,
                            int groups, int64_t *num_batches_tracked, float *workspace, void *stream) {
  EWVIT_CHECK_ARG(x && y && workspace && dtype_ok(dtype), "bn_fwd: bad args");
  EWVIT_CHECK_ARG(C > 0 && C % 8 == 0 && C <= 4096, "bn_fwd: C=%lld must be a multiple of 8, <= 4096", (long long)C);
  EWVIT_CHECK_ARG(act >= 0 && act <= 2, "bn_fwd: act=%d", act);
  EWVIT_CHECK_ARG(training || (running_mean && running_var), "bn_fwd: eval needs running stats");
  EWVIT_CHECK_ARG(groups >= 1 && groups <= 65535 && M % groups == 0, "bn_fwd: M=%lld not divisible into %d groups",
                  (long long)M, groups);
  if (M == 0) return 0;
  if (!training) groups = 1;
  hipStream_t s = as_stream(stream);
  const int64_t Mg = M / groups;
  const BnGeo geo = bn_geo(C);
  const int nrc = bn_nrc(geo, Mg, groups);
  float *part = workspace, *shifts = workspace + (int64_t)groups * nrc * 2 * C;
  if (training) {
    const int64_t rpc = (Mg + nrc - 1) / nrc;
    dim3 grid(nrc, geo.nch, groups);
    if (dtype == EWVIT_BF16)
      hipLaunchKernelGGL(bn_stats_kernel<EWVIT_BF16>, grid, dim3(geo.threads), 0, s, x, Mg, (int)C, geo.CC8, geo.RG,
                         rpc, part, shifts);
    else
      hipLaunchKernelGGL(bn_stats_kernel<EWVIT_F32>, grid, dim3(geo.threads), 0, s, x, Mg, (int)C, geo.CC8, geo.RG,
                         rpc, part, shifts);
  }
  const int64_t rpb = bn_rows_per_block(geo, Mg, groups);
  dim3 agrid((unsigned)((Mg + rpb - 1) / rpb), geo.nch, groups);
#define BN_APPLY(DTV, ACTV)                                                                                          \
  hipLaunchKernelGGL((bn_apply_kernel<DTV, ACTV>), agrid, dim3(geo.threads), 0, s, x, y, part, shifts, nrc, Mg,     \
                     (int)C, geo.CC8, geo.RG, rpb, training, gamma, beta, running_mean, running_var, momentum, eps, \
                     save_mean, save_invstd, num_batches_tracked)
  BN_DISPATCH(BN_APPLY);
#undef BN_APPLY
  return launch_status("bn_fwd");
}

// sum consecutive chunks of a group's partial rows: out[g][k][:] = sum of in[g][k*ch ..
// k*ch + ch - 1][:] (fixed order), and the shift [C] replicated per group
__global__ __launch_bounds__(256) void bn_fold_kernel(const float *__restrict__ in, int nin, const float *shift_in,
                                                      float *__restrict__ out, int nout, float *__restrict__ shift_out,
                                                      int C) {
  const int c2 = blockIdx.x * 256 + threadIdx.x, k = blockIdx.y, g = blockIdx.z;
  if (c2 >= 2 * C) return;
  const int ch = (nin + nout - 1) / nout;
  const int r0 = k * ch, r1 = r0 + ch < nin ? r0 + ch : nin;
  const float *p = in + ((int64_t)g * nin) * 2 * C + c2;
  float acc = 0.f;
  int r = r0;
  for (; r + 7 < r1; r += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(r + u) * 2 * C];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; r < r1; ++r) acc += p[(int64_t)r * 2 * C];
  out[((int64_t)g * nout + k) * 2 * C + c2] = acc;
  if (k == 0 && c2 < C) shift_out[g * C + c2] = shift_in[c2];
}

extern "C" int ewvit_bn_fold_partials(const float *part_in, int nin, const float *shift_in, float *part_out,
                                      int nout, float *shift_out, int64_t C, int groups, void *stream) {
  EWVIT_CHECK_ARG(part_in && shift_in && part_out && shift_out && nin >= 1 && nout >= 1 && groups >= 1 &&
                      C > 0 && C <= 4096 && groups <= 65535 && nout <= 65535,
                  "bn_fold_partials: bad args");
  dim3 grid((unsigned)((2 * C + 255) / 256), (unsigned)nout, (unsigned)groups);
  hipLaunchKernelGGL(bn_fold_kernel, grid, dim3(256), 0, as_stream(stream), part_in, nin, shift_in, part_out, nout,
                     shift_out, (int)C);
  return launch_status("bn_fold_partials");
}

// training forward from precomputed partial statistics (per group nrc rows of shifted
// sums [groups][nrc][2C] + the shifts [groups][C], e.g. left by ewvit_conv2d_fwd_bn in
// the producing conv's epilogue): the apply pass only (it finalises from the rows)
extern "C" int ewvit_bn_fwd_partials(const void *x, void *y, int dtype, int64_t M, int64_t C, const float *gamma,
                                     const float *beta, float *running_mean, float *running_var, float momentum,
                                     float eps, int act, float *save_mean, float *save_invstd,
                                     int64_t *num_batches_tracked, const float *part, const float *shifts, int nrc,
                                     int groups, void *stream) {
  EWVIT_CHECK_ARG(x && y && part && shifts && dtype_ok(dtype), "bn_fwd_partials: bad args");
  EWVIT_CHECK_ARG(C > 0 && C % 8 == 0 && C <= 4096, "bn_fwd_partials: C=%lld must be a multiple of 8, <= 4096",
                  (long long)C);
  EWVIT_CHECK_ARG(act >= 0 && act <= 2, "bn_fwd_partials: act=%d", act);
  EWVIT_CHECK_ARG(nrc >= 1 && nrc <= 4096, "bn_fwd_partials: %d partial rows", nrc);
  EWVIT_CHECK_ARG(groups >= 1 && groups <= 65535 && M % groups == 0, "bn_fwd_partials: M=%lld, %d groups",
                  (long long)M, groups);
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  const BnGeo geo = bn_geo(C);
  const int64_t Mg = M / groups;
  const int64_t rpb = bn_rows_per_block(geo, Mg, groups);
  dim3 agrid((unsigned)((Mg + rpb - 1) / rpb), geo.nch, groups);
#define BN_APPLY(DTV, ACTV)                                                                                          \
  hipLaunchKernelGGL((bn_apply_kernel<DTV, ACTV>), agrid, dim3(geo.threads), 0, s, x, y, part, shifts, nrc, Mg,     \
                     (int)C, geo.CC8, geo.RG, rpb, 1, gamma, beta, running_mean, running_var, momentum, eps,        \
                     save_mean, save_invstd, num_batches_tracked)
  BN_DISPATCH(BN_APPLY);
#undef BN_APPLY
  return launch_status("bn_fwd_partials");
}

// the apply pass's coefficients only, for an op that applies the BatchNorm(+act) itself while
// reading x (the windowed conv's input transform, ewvit_conv2d_fwd_bn_xf): the training
// finalisation of ewvit_bn_fwd_partials — same blocks, same reduction order, running statistics,
// counter, save_mean / save_invstd — with no rows, writing coef[g][0][c] = scale, coef[g][1][c]
// = shift (y = act(x * scale + shift) is then bit-identical to that apply pass)
extern "C" int ewvit_bn_coef(int64_t M, int64_t C, const float *gamma, const float *beta, float *running_mean,
                             float *running_var, float momentum, float eps, float *save_mean, float *save_invstd,
                             int64_t *num_batches_tracked, const float *part, const float *shifts, int nrc, int groups,
                             float *coef, void *stream) {
  EWVIT_CHECK_ARG(part && shifts && coef, "bn_coef: bad args");
  EWVIT_CHECK_ARG(C > 0 && C % 8 == 0 && C <= 4096, "bn_coef: C=%lld must be a multiple of 8, <= 4096", (long long)C);
  EWVIT_CHECK_ARG(nrc >= 1 && nrc <= 4096, "bn_coef: %d partial rows", nrc);
  EWVIT_CHECK_ARG(groups >= 1 && groups <= 65535 && M > 0 && M % groups == 0, "bn_coef: M=%lld, %d groups",
                  (long long)M, groups);
  const BnGeo geo = bn_geo(C);
  dim3 grid(1u, geo.nch, groups);
  hipLaunchKernelGGL((bn_apply_kernel<EWVIT_BF16, 1>), grid, dim3(geo.threads), 0, as_stream(stream), nullptr, nullptr,
                     part, shifts, nrc, M / groups, (int)C, geo.CC8, geo.RG, (int64_t)0, 1, gamma, beta, running_mean,
                     running_var, momentum, eps, save_mean, save_invstd, num_batches_tracked, BnDrop(), coef);
  return launch_status("bn_coef");
}

// BatchNorm (no activation) + StochasticDepth(row) + skip add, training, one group:
// y = bn(x) * scale[n] + skip (BnDrop); statistics from `part`/`shifts` (nrc rows, e.g.
// the conv epilogue's) or, when part is NULL, by the stats pass into `workspace`
extern "C" int ewvit_bn_fwd_drop_add(const void *x, void *y, int dtype, int64_t M, int64_t C, const float *gamma,
                                     const float *beta, float *running_mean, float *running_var, float momentum,
                                     float eps, float *save_mean, float *save_invstd, int64_t *num_batches_tracked,
                                     const float *part, const float *shifts, int nrc, const void *skip, int64_t HW,
                                     float keep_prob, uint64_t seed, const int64_t *seed_offset, float *scale_out,
                                     float *workspace, void *stream) {
  EWVIT_CHECK_ARG(x && y && skip && scale_out && dtype_ok(dtype), "bn_fwd_drop_add: bad args");
  EWVIT_CHECK_ARG(C > 0 && C % 8 == 0 && C <= 4096, "bn_fwd_drop_add: C=%lld must be a multiple of 8, <= 4096",
                  (long long)C);
  EWVIT_CHECK_ARG(HW > 0 && M % HW == 0 && M < ((int64_t)1 << 31), "bn_fwd_drop_add: M=%lld rows of %lld", (long long)M,
                  (long long)HW);
  EWVIT_CHECK_ARG(keep_prob > 0.f && keep_prob <= 1.f, "bn_fwd_drop_add: keep_prob %g", (double)keep_prob);
  EWVIT_CHECK_ARG(part ? (shifts && nrc >= 1 && nrc <= 4096) : workspace != nullptr,
                  "bn_fwd_drop_add: partial statistics or a workspace");
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  const BnGeo geo = bn_geo(C);
  if (!part) {
    nrc = bn_nrc(geo, M, 1);
    float *wpart = workspace, *wshift = workspace + (int64_t)nrc * 2 * C;
    const int64_t rpc = (M + nrc - 1) / nrc;
    dim3 grid(nrc, geo.nch, 1);
    if (dtype == EWVIT_BF16)
      hipLaunchKernelGGL(bn_stats_kernel<EWVIT_BF16>, grid, dim3(geo.threads), 0, s, x, M, (int)C, geo.CC8, geo.RG,
                         rpc, wpart, wshift);
    else
      hipLaunchKernelGGL(bn_stats_kernel<EWVIT_F32>, grid, dim3(geo.threads), 0, s, x, M, (int)C, geo.CC8, geo.RG,
                         rpc, wpart, wshift);
    part = wpart;
    shifts = wshift;
  }
  BnDrop dr;
  dr.skip = skip; dr.keep = keep_prob; dr.seed = seed; dr.seed_offset = seed_offset; dr.scale_out = scale_out;
  dr.HW = (int)HW;
  const int64_t rpb = bn_rows_per_block(geo, M, 1);
  dim3 agrid((unsigned)((M + rpb - 1) / rpb), geo.nch, 1);
  if (dtype == EWVIT_BF16)
    hipLaunchKernelGGL((bn_apply_kernel<EWVIT_BF16, 0, true>), agrid, dim3(geo.threads), 0, s, x, y, part, shifts, nrc,
                       M, (int)C, geo.CC8, geo.RG, rpb, 1, gamma, beta, running_mean, running_var, momentum, eps,
                       save_mean, save_invstd, num_batches_tracked, dr);
  else
    hipLaunchKernelGGL((bn_apply_kernel<EWVIT_F32, 0, true>), agrid, dim3(geo.threads), 0, s, x, y, part, shifts, nrc,
                       M, (int)C, geo.CC8, geo.RG, rpb, 1, gamma, beta, running_mean, running_var, momentum, eps,
                       save_mean, save_invstd, num_batches_tracked, dr);
  return launch_status("bn_fwd_drop_add");
}

// backward of ewvit_bn_fwd_drop_add's BatchNorm: g = dy * row_scale[row / HW] (the skip
// gradient is dy itself, no kernel); dgamma / dbeta overwritten
extern "C" int ewvit_bn_bwd_scaled(const void *dy, const void *x, void *dx, int dtype, int64_t M, int64_t C,
                                   const float *gamma, const float *beta, const float *save_mean,
                                   const float *save_invstd, float *dgamma, float *dbeta, const float *row_scale,
                                   int64_t HW, float *workspace, void *stream) {
  EWVIT_CHECK_ARG(dy && x && dx && save_mean && save_invstd && row_scale && workspace && dtype_ok(dtype),
                  "bn_bwd_scaled: bad args");
  EWVIT_CHECK_ARG(C > 0 && C % 8 == 0 && C <= 4096, "bn_bwd_scaled: C=%lld", (long long)C);
  EWVIT_CHECK_ARG(HW > 0 && M % HW == 0 && M < ((int64_t)1 << 31), "bn_bwd_scaled: M=%lld rows of %lld", (long long)M,
                  (long long)HW);
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  const BnGeo geo = bn_geo(C);
  const int nrc = bn_nrc(geo, M, 1);
  const int64_t rpc = (M + nrc - 1) / nrc;
  dim3 grid(nrc, geo.nch, 1);
  const int64_t rpb = bn_rows_per_block(geo, M, 1);
  dim3 dgrid((unsigned)((M + rpb - 1) / rpb), geo.nch, 1);
  if (dtype == EWVIT_BF16) {
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<EWVIT_BF16, 0, 1>), grid, dim3(geo.threads), 0, s, dy, x, save_mean,
                       save_invstd, gamma, beta, M, (int)C, geo.CC8, geo.RG, rpc, workspace, row_scale, (int)HW);
    hipLaunchKernelGGL((bn_bwd_dx_kernel<EWVIT_BF16, 0, 1>), dgrid, dim3(geo.threads), 0, s, dy, x, save_mean,
                       save_invstd, gamma, beta, workspace, nrc, dx, M, (int)C, geo.CC8, geo.RG, rpb, dgamma, dbeta, 0,
                       row_scale, (int)HW);
  } else {
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<EWVIT_F32, 0, 1>), grid, dim3(geo.threads), 0, s, dy, x, save_mean,
                       save_invstd, gamma, beta, M, (int)C, geo.CC8, geo.RG, rpc, workspace, row_scale, (int)HW);
    hipLaunchKernelGGL((bn_bwd_dx_kernel<EWVIT_F32, 0, 1>), dgrid, dim3(geo.threads), 0, s, dy, x, save_mean,
                       save_invstd, gamma, beta, workspace, nrc, dx, M, (int)C, geo.CC8, geo.RG, rpb, dgamma, dbeta, 0,
                       row_scale, (int)HW);
  }
  return launch_status("bn_bwd_scaled");
}

// backward of BatchNorm(+act) followed by squeeze-excitation (the MBConv depthwise BN + SiLU,
// then SE): the BatchNorm's output gradient dy * s[n][c] + g[n][c] is formed from the SE
// output gradient dy inside both passes (s: the excitation [N][C], g: the squeeze term from
// ewvit_se_squeeze_mlp_bwd), so the SE input-gradient pass (ewvit_se_scale) never runs
extern "C" int ewvit_bn_bwd_se(const void *dy, const void *x, void *dx, int dtype, int64_t M, int64_t C,
                               const float *gamma, const float *beta, const float *save_mean, const float *save_invstd,
                               int act, float *dgamma, float *dbeta, const float *se_s, const float *se_g, int64_t HW,
                               float *workspace, void *stream) {
  EWVIT_CHECK_ARG(dy && x && dx && save_mean && save_invstd && se_s && se_g && workspace && dtype_ok(dtype),
                  "bn_bwd_se: bad args");
  EWVIT_CHECK_ARG(C > 0 && C % 8 == 0 && C <= 4096, "bn_bwd_se: C=%lld", (long long)C);
  EWVIT_CHECK_ARG(act >= 0 && act <= 2, "bn_bwd_se: act=%d", act);
  EWVIT_CHECK_ARG(HW > 0 && M % HW == 0 && M < ((int64_t)1 << 31), "bn_bwd_se: M=%lld rows of %lld", (long long)M,
                  (long long)HW);
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  const BnGeo geo = bn_geo(C);
  const int nrc = bn_nrc(geo, M, 1);
  const int64_t rpc = (M + nrc - 1) / nrc;
  dim3 grid(nrc, geo.nch, 1);
  const int64_t rpb = bn_rows_per_block(geo, M, 1);
  dim3 dgrid((unsigned)((M + rpb - 1) / rpb), geo.nch, 1);
#define BN_SE(DTV, ACTV)                                                                                            \
  do {                                                                                                              \
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<DTV, ACTV, 2>), grid, dim3(geo.threads), 0, s, dy, x, save_mean,      \
                       save_invstd, gamma, beta, M, (int)C, geo.CC8, geo.RG, rpc, workspace, se_s, (int)HW, se_g);  \
    hipLaunchKernelGGL((bn_bwd_dx_kernel<DTV, ACTV, 2>), dgrid, dim3(geo.threads), 0, s, dy, x, save_mean,         \
                       save_invstd, gamma, beta, workspace, nrc, dx, M, (int)C, geo.CC8, geo.RG, rpb, dgamma, dbeta, \
                       0, se_s, (int)HW, se_g);                                                                     \
  } while (0)
  BN_DISPATCH(BN_SE);
#undef BN_SE
  return launch_status("bn_bwd_se");
}

namespace ewvit {
// the dx pass of ewvit_bn_bwd_se from partial rows another pass left (ewvit_bn_se_bwd, se.hip)
int bn_bwd_dx_se_launch(const void *dy, const void *x, void *dx, int dtype, int64_t M, int64_t C, const float *gamma,
                        const float *beta, const float *save_mean, const float *save_invstd, int act, float *dgamma,
                        float *dbeta, const float *se_s, const float *se_g, int64_t HW, const float *part, int nrc,
                        hipStream_t s) {
  const BnGeo geo = bn_geo(C);
  const int64_t rpb = bn_rows_per_block(geo, M, 1);
  dim3 dgrid((unsigned)((M + rpb - 1) / rpb), geo.nch, 1);
#define BN_SE_DX(DTV, ACTV)                                                                                          \
  hipLaunchKernelGGL((bn_bwd_dx_kernel<DTV, ACTV, 2>), dgrid, dim3(geo.threads), 0, s, dy, x, save_mean, save_invstd, \
                     gamma, beta, part, nrc, dx, M, (int)C, geo.CC8, geo.RG, rpb, dgamma, dbeta, 0, se_s, (int)HW,   \
                     se_g)
  BN_DISPATCH(BN_SE_DX);
#undef BN_SE_DX
  return launch_status("bn_se_bwd");
}
}  // namespace ewvit

// backward from partial sums left by the kernel that produced dy (the consumer conv's input
// gradient: ewvit_conv2d_bwd_data_bn, ewvit_dwconv3x3_bwd_data_bn): part [nrc][2C] = per
// partial row (sum g, sum g * xhat) with g = dy * act'(...) or, row_scale given (the MBConv
// tail's drop-path, act 0), g = dy * row_scale[row / HW]: the dx pass only (it finalises from
// the rows); dgamma / dbeta overwritten
extern "C" int ewvit_bn_bwd_partials(const void *dy, const void *x, void *dx, int dtype, int64_t M, int64_t C,
                                     const float *gamma, const float *beta, const float *save_mean,
                                     const float *save_invstd, int act, float *dgamma, float *dbeta,
                                     const float *row_scale, int64_t HW, const float *part, int nrc, int groups,
                                     void *stream) {
  EWVIT_CHECK_ARG(dy && x && dx && save_mean && save_invstd && part && dtype_ok(dtype), "bn_bwd_partials: bad args");
  EWVIT_CHECK_ARG(C > 0 && C % 8 == 0 && C <= 4096, "bn_bwd_partials: C=%lld", (long long)C);
  EWVIT_CHECK_ARG(act >= 0 && act <= 2 && !(row_scale && act), "bn_bwd_partials: act=%d (row_scale needs act 0)", act);
  EWVIT_CHECK_ARG(nrc >= 1 && nrc <= 65535, "bn_bwd_partials: %d partial rows", nrc);
  EWVIT_CHECK_ARG(!row_scale || (HW > 0 && M % HW == 0 && M < ((int64_t)1 << 31)), "bn_bwd_partials: M=%lld rows of %lld",
                  (long long)M, (long long)HW);
  EWVIT_CHECK_ARG(groups >= 1 && groups <= 65535 && M % groups == 0 && (groups == 1 || !row_scale),
                  "bn_bwd_partials: %d groups", groups);
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  const BnGeo geo = bn_geo(C);
  const int64_t Mg = M / groups;
  const int64_t rpb = bn_rows_per_block(geo, Mg, groups);
  dim3 dgrid((unsigned)((Mg + rpb - 1) / rpb), geo.nch, groups);
  if (row_scale) {
    if (dtype == EWVIT_BF16)
      hipLaunchKernelGGL((bn_bwd_dx_kernel<EWVIT_BF16, 0, 1>), dgrid, dim3(geo.threads), 0, s, dy, x, save_mean,
                         save_invstd, gamma, beta, part, nrc, dx, M, (int)C, geo.CC8, geo.RG, rpb, dgamma, dbeta, 0,
                         row_scale, (int)HW);
    else
      hipLaunchKernelGGL((bn_bwd_dx_kernel<EWVIT_F32, 0, 1>), dgrid, dim3(geo.threads), 0, s, dy, x, save_mean,
                         save_invstd, gamma, beta, part, nrc, dx, M, (int)C, geo.CC8, geo.RG, rpb, dgamma, dbeta, 0,
                         row_scale, (int)HW);
    return launch_status("bn_bwd_partials");
  }
#define BN_DX(DTV, ACTV)                                                                                              \
  hipLaunchKernelGGL((bn_bwd_dx_kernel<DTV, ACTV>), dgrid, dim3(geo.threads), 0, s, dy, x, save_mean, save_invstd,   \
                     gamma, beta, part, nrc, dx, Mg, (int)C, geo.CC8, geo.RG, rpb, dgamma, dbeta, 0)
  BN_DISPATCH(BN_DX);
#undef BN_DX
  return launch_status("bn_bwd_partials");
}

// The reduction pass of ewvit_bn_bwd alone: part [groups][nrc][2][C] (sum g, sum g * xhat) with
// nrc = ewvit_bn_bwd_reduce_rows(M, C, groups), for a consumer that forms dx itself.
extern "C" int ewvit_bn_bwd_reduce_rows(int64_t M, int64_t C, int groups) {
  if (groups < 1 || M < 1 || C < 8 || C > 4096 || C % 8 || M % groups) return 0;
  return bn_nrc(bn_geo(C), M / groups, groups);
}

extern "C" int ewvit_bn_bwd_reduce(const void *dy, const void *x, int dtype, int64_t M, int64_t C, const float *gamma,
                                   const float *beta, const float *save_mean, const float *save_invstd, int act,
                                   int groups, float *part, void *stream) {
  EWVIT_CHECK_ARG(dy && x && save_mean && save_invstd && part && dtype_ok(dtype), "bn_bwd_reduce: bad args");
  EWVIT_CHECK_ARG(C > 0 && C % 8 == 0 && C <= 4096, "bn_bwd_reduce: C=%lld", (long long)C);
  EWVIT_CHECK_ARG(act >= 0 && act <= 2, "bn_bwd_reduce: act=%d", act);
  EWVIT_CHECK_ARG(groups >= 1 && groups <= 65535 && M % groups == 0, "bn_bwd_reduce: %d groups", groups);
  if (M == 0) return 0;
  const int64_t Mg = M / groups;
  const BnGeo geo = bn_geo(C);
  const int nrc = bn_nrc(geo, Mg, groups);
  const int64_t rpc = (Mg + nrc - 1) / nrc;
  dim3 grid(nrc, geo.nch, groups);
  hipStream_t s = as_stream(stream);
#define BN_RED(DTV, ACTV)                                                                                           \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<DTV, ACTV>), grid, dim3(geo.threads), 0, s, dy, x, save_mean,           \
                     save_invstd, gamma, beta, Mg, (int)C, geo.CC8, geo.RG, rpc, part)
  BN_DISPATCH(BN_RED);
#undef BN_RED
  return launch_status("bn_bwd_reduce");
}

extern "C" int ewvit_bn_bwd(const void *dy, const void *x, void *dx, int dtype, int64_t M, int64_t C,
                            const float *gamma, const float *beta, const float *save_mean,
                            const float *save_invstd, int act, float *dgamma, float *dbeta, int accumulate,
                            int groups, float *workspace, void *stream) {
  EWVIT_CHECK_ARG(dy && x && dx && save_mean && save_invstd && workspace && dtype_ok(dtype), "bn_bwd: bad args");
  EWVIT_CHECK_ARG(C > 0 && C % 8 == 0 && C <= 4096, "bn_bwd: C=%lld must be a multiple of 8, <= 4096", (long long)C);
  EWVIT_CHECK_ARG(act >= 0 && act <= 2, "bn_bwd: act=%d", act);
  EWVIT_CHECK_ARG(groups >= 1 && groups <= 65535 && M % groups == 0, "bn_bwd: M=%lld not divisible into %d groups",
                  (long long)M, groups);
  if (M == 0) return 0;
  hipStream_t s = as_stream(stream);
  const int64_t Mg = M / groups;
  const BnGeo geo = bn_geo(C);
  const int nrc = bn_nrc(geo, Mg, groups);
  const int64_t rpc = (Mg + nrc - 1) / nrc;
  dim3 grid(nrc, geo.nch, groups);
#define BN_RED(DTV, ACTV)                                                                                           \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<DTV, ACTV>), grid, dim3(geo.threads), 0, s, dy, x, save_mean,           \
                     save_invstd, gamma, beta, Mg, (int)C, geo.CC8, geo.RG, rpc, workspace)
  BN_DISPATCH(BN_RED);
#undef BN_RED
  const int64_t rpb = bn_rows_per_block(geo, Mg, groups);
  dim3 dgrid((unsigned)((Mg + rpb - 1) / rpb), geo.nch, groups);
#define BN_DX(DTV, ACTV)                                                                                              \
  hipLaunchKernelGGL((bn_bwd_dx_kernel<DTV, ACTV>), dgrid, dim3(geo.threads), 0, s, dy, x, save_mean, save_invstd,   \
                     gamma, beta, workspace, nrc, dx, Mg, (int)C, geo.CC8, geo.RG, rpb, dgamma, dbeta, accumulate)
  BN_DISPATCH(BN_DX);
#undef BN_DX
  return launch_status("bn_bwd");
}

// MBConv depthwise BatchNorm(+act) from the depthwise conv's partial statistics, fused with the
// SE squeeze and the MLP's first-layer partials (bn_act_squeeze_kernel): x, y [N][HW][C];
// s0 [N][C]; part [N][ceil(C / 64)][Csq] (what ewvit_se_gate_excite finishes); one launch
extern "C" int ewvit_bn_act_se_squeeze(const void *x, void *y, int dtype, int64_t N, int64_t HW, int64_t C,
                                       const float *gamma, const float *beta, float *running_mean, float *running_var,
                                       float momentum, float eps, int act, float *save_mean, float *save_invstd,
                                       int64_t *num_batches_tracked, const float *part, const float *shifts, int nrc,
                                       const float *w1, int64_t Csq, float *s0, float *hpart, void *stream) {
  EWVIT_CHECK_ARG(x && y && part && shifts && w1 && s0 && hpart && dtype_ok(dtype), "bn_act_se_squeeze: bad args");
  EWVIT_CHECK_ARG(C > 0 && C % 8 == 0 && C <= 4096 && N > 0 && N <= 65535 && HW > 0 && HW < (1 << 30),
                  "bn_act_se_squeeze: N=%lld HW=%lld C=%lld", (long long)N, (long long)HW, (long long)C);
  EWVIT_CHECK_ARG(act >= 0 && act <= 2 && nrc >= 1 && nrc <= 65535 && Csq >= 1 && Csq <= 4096,
                  "bn_act_se_squeeze: act=%d nrc=%d Csq=%lld", act, nrc, (long long)Csq);
  const dim3 grid((unsigned)N, (unsigned)((C + 63) / 64));
  hipStream_t s = as_stream(stream);
#define BN_SQ(DTV, ACTV)                                                                                             \
  hipLaunchKernelGGL((bn_act_squeeze_kernel<DTV, ACTV>), grid, dim3(256), 0, s, x, y, part, shifts, nrc, (int)HW,   \
                     (int)C, gamma, beta, running_mean, running_var, momentum, eps, save_mean, save_invstd,         \
                     num_batches_tracked, 1.f / (float)HW, w1, (int)Csq, s0, hpart)
  BN_DISPATCH(BN_SQ);
#undef BN_SQ
  return launch_status("bn_act_se_squeeze");
}
