// Depthwise 3x3 convolution, channels-last (NHWC), forward / input-grad /
// weight-grad (gfx950).
//
// EfficientNetV2-S's 30 MBConv blocks each carry one depthwise 3x3 conv
// (groups = channels = 256..1536, stride 1 or 2, pad 1; torchvision
// Conv2dNormActivation(groups=C), reached from the reference via
// network/sfe.py:111-113,150).  Profiled on MI355X through MIOpen/CK these were
// the step's dominant kernels (naive_conv fwd/bwd-data, ~12 ms per
// grouped-conv weight-grad launch) although the op is purely HBM-bound:
// 9 MACs per element against 2 x 2 bytes of bf16 traffic.
//
// Layout: x [N, H, W, C], y [N, Ho, Wo, C], w [C, 3, 3] (fp32 master weights).
// One thread owns 8 consecutive channels (one 16-B bf16 vector); the 3x3 taps of
// neighbouring pixels are re-read through L1/L2, so HBM traffic stays ~1x in +
// 1x out.  The weight gradient reduces N*Ho*Wo products per (c, tap) in fp32:
// per-block partial slabs (deterministic, no atomics) + a second reduction pass.
#include "common.h"
#include "reduce_jobs.h"

namespace ewvit {

template <int DT>
struct Vec8 {
  __device__ __forceinline__ static void load(const void *p, int64_t i, float (&v)[8]) {
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
  __device__ __forceinline__ static void store(void *p, int64_t i, const float (&v)[8]) {
    if (DT == EWVIT_BF16) {
      unsigned w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w[j] = (unsigned)f2bf(v[2 * j]) | ((unsigned)f2bf(v[2 * j + 1]) << 16);
      *reinterpret_cast<uint4 *>(reinterpret_cast<bf16_t *>(p) + i) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      float4 *q = reinterpret_cast<float4 *>(reinterpret_cast<float *>(p) + i);
      q[0] = make_float4(v[0], v[1], v[2], v[3]);
      q[1] = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
};

struct DwShape {
  int N, H, W, C, Ho, Wo, stride, pad;
};

template <int DT>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const void *__restrict__ x, const float *__restrict__ w,
                                                     void *__restrict__ y, DwShape s) {
  const int C8 = s.C >> 3;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)s.N * s.Ho * s.Wo * C8;
  if (idx >= total) return;
  const int c8 = (int)(idx % C8);
  int64_t t = idx / C8;
  const int wo = (int)(t % s.Wo);
  t /= s.Wo;
  const int ho = (int)(t % s.Ho);
  const int n = (int)(t / s.Ho);
  const int c = c8 * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int hi = ho * s.stride - s.pad + kh;
    if (hi < 0 || hi >= s.H) continue;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int wi = wo * s.stride - s.pad + kw;
      if (wi < 0 || wi >= s.W) continue;
      float v[8];
      Vec8<DT>::load(x, (((int64_t)n * s.H + hi) * s.W + wi) * s.C + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaf(v[j], w[(c + j) * 9 + kh * 3 + kw], acc[j]);
    }
  }
  Vec8<DT>::store(y, idx * 8, acc);
}

template <int DT>
__global__ __launch_bounds__(256) void dw_bwd_data_kernel(const void *__restrict__ dy, const float *__restrict__ w,
                                                          void *__restrict__ dx, DwShape s) {
  const int C8 = s.C >> 3;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)s.N * s.H * s.W * C8;
  if (idx >= total) return;
  const int c8 = (int)(idx % C8);
  int64_t t = idx / C8;
  const int wi = (int)(t % s.W);
  t /= s.W;
  const int hi = (int)(t % s.H);
  const int n = (int)(t / s.H);
  const int c = c8 * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int hn = hi + s.pad - kh;           // = ho * stride
    if (hn < 0 || hn % s.stride) continue;
    const int ho = hn / s.stride;
    if (ho >= s.Ho) continue;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int wn = wi + s.pad - kw;
      if (wn < 0 || wn % s.stride) continue;
      const int wo = wn / s.stride;
      if (wo >= s.Wo) continue;
      float v[8];
      Vec8<DT>::load(dy, (((int64_t)n * s.Ho + ho) * s.Wo + wo) * s.C + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaf(v[j], w[(c + j) * 9 + kh * 3 + kw], acc[j]);
    }
  }
  Vec8<DT>::store(dx, idx * 8, acc);
}

// ---- bf16 row kernel (the hot form): one thread = 8 channels x one output ROW.
// Its 72 weights live in registers (loaded once, 18 x 16-B loads), and the 3x3
// input window slides along the row carrying 3-s columns, so each output costs
// 3*s new 16-B loads instead of 9 (+72 weight loads) in the generic kernel.
// ROT: use the 180-degree-rotated kernel — the input gradient of a stride-1
// conv is the stride-1 conv of dy with the rotated weights (pad 1).
// The row kernels' window loads are buffer loads: a tap outside the map gets the offset DW_OOB
// (>= the resource's size), which the hardware returns as zeros — no branch and no select on
// the loaded value, so the window register carried to the next column is the load's own result
// and its wait lands at the next column's first use.  (A zeroing select after a global load
// made every column wait for its loads before the loop back edge: 7^2 / 14^2 depthwise passes
// 30-60 % slower; the branchy C++ form compiled to FLAT loads from a select between the global
// address and a private zero.)  Offsets are 32-bit bytes: the host takes the row kernels only
// for tensors below 2 GB (dw_bufok).
constexpr uint32_t DW_OOB = 0x80000000u;
typedef __attribute__((ext_vector_type(4))) unsigned dw_u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned dw_u32x2;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t dw_rsrc(const void *p, int64_t elems) {
  const int64_t bytes = elems * 2;
  const uint32_t n = bytes >= (int64_t)DW_OOB ? DW_OOB : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)n, 0x00020000);
}
__device__ __forceinline__ uint4 dw_ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const dw_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 dw_ld8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const dw_u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return make_uint2(v.x, v.y);
}
static inline bool dw_bufok(int64_t elems) { return elems * 2 < (int64_t)DW_OOB; }

__device__ __forceinline__ void bf8_unpack(const uint4 &q, float (&v)[8]) {
  const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}

template <int STRIDE, bool ROT>
__global__ __launch_bounds__(256) void dw_row_bf16_kernel(const bf16_t *__restrict__ x, const float *__restrict__ w,
                                                          bf16_t *__restrict__ y, DwShape s, int rows_per_block,
                                                          int segs) {
  const int C8 = s.C >> 3;
  const int r = threadIdx.x / C8, c8 = threadIdx.x % C8;
  if (r >= rows_per_block) return;
  // a thread walks one column segment of one output row (segs segments per row)
  const int64_t vrow = (int64_t)blockIdx.x * rows_per_block + r;
  if (vrow >= (int64_t)s.N * s.Ho * segs) return;
  const int64_t row = vrow / segs;                                   // n*Ho + ho
  const int wseg = (s.Wo + segs - 1) / segs;
  const int wo0 = (int)(vrow - row * segs) * wseg;
  const int wo1 = wo0 + wseg < s.Wo ? wo0 + wseg : s.Wo;
  const int ho = (int)(row % s.Ho);
  const int n = (int)(row / s.Ho);
  const int c = c8 * 8;
  float wr[9][8];  // [tap][channel]
  {
    const float4 *wp = reinterpret_cast<const float4 *>(w + (int64_t)c * 9);
    float t[72];
#pragma unroll
    for (int i = 0; i < 18; ++i) {
      const float4 q = wp[i];
      t[4 * i] = q.x; t[4 * i + 1] = q.y; t[4 * i + 2] = q.z; t[4 * i + 3] = q.w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int k = 0; k < 9; ++k) wr[ROT ? 8 - k : k][j] = t[j * 9 + k];
  }
  bool rok[3];
  int64_t rbase[3];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int hi = ho * STRIDE - s.pad + kh;
    rok[kh] = hi >= 0 && hi < s.H;
    rbase[kh] = (((int64_t)n * s.H + (rok[kh] ? hi : 0)) * s.W) * s.C + c;
  }
  const __amdgpu_buffer_rsrc_t xr = dw_rsrc(x, (int64_t)s.N * s.H * s.W * s.C);
  auto ld = [&](int kh, int col) -> uint4 {     // zeros outside the map (DW_OOB)
    return dw_ld16(xr, rok[kh] && col >= 0 && col < s.W ? (uint32_t)((rbase[kh] + (int64_t)col * s.C) * 2) : DW_OOB);
  };
  uint4 win[3][3];  // [kw][kh], column ci = wo*STRIDE - pad + kw
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) win[kw][kh] = ld(kh, wo0 * STRIDE - s.pad + kw);
  // stride 1: the window's next column loaded one column ahead (its wait lands a column later)
  uint4 nx[3];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) nx[kh] = STRIDE == 1 ? ld(kh, wo0 + 3 - s.pad) : make_uint4(0u, 0u, 0u, 0u);
  bf16_t *yrow = y + (row * s.Wo) * s.C + c;
  for (int wo = wo0; wo < wo1; ++wo) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        float v[8];
        bf8_unpack(win[kw][kh], v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(v[j], wr[kh * 3 + kw][j], acc[j]);
      }
    unsigned o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (unsigned)f2bf(acc[2 * j]) | ((unsigned)f2bf(acc[2 * j + 1]) << 16);
    *reinterpret_cast<uint4 *>(yrow + (int64_t)wo * s.C) = make_uint4(o[0], o[1], o[2], o[3]);
    const int nb = (wo + 1) * STRIDE - s.pad;  // first column of the next window
    if (STRIDE == 1) {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        win[0][kh] = win[1][kh];
        win[1][kh] = win[2][kh];
        win[2][kh] = nx[kh];
        nx[kh] = ld(kh, nb + 3);
      }
    } else {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        win[0][kh] = win[2][kh];
        win[1][kh] = ld(kh, nb + 1);
        win[2][kh] = ld(kh, nb + 2);
      }
    }
  }
}

// ---- the row kernel with the BatchNorm sums of what it stores (MBConv: the BN after the
// depthwise conv in the forward, the BN before it in the backward), so the BN needs no
// statistics pass of its own.  Block = 32 output rows (n*Ho + ho, across frames) x 64
// channels: thread tid walks row tid / 8 for channel vector tid % 8, exactly as
// dw_row_bf16_kernel walks a row, and keeps its 8 channels' sums of the bf16-rounded
// outputs; the block leaves ONE partial row (its 64 channels) at part[blockIdx.x]:
//   ST 1 (forward): sum (y - K), sum (y - K)^2 with K = shift (or 0) — the shifted sums
//        ewvit_bn_fwd_partials finalises; block row 0 copies K to shift_out
//   ST 2 (input gradient of a stride-1 conv, ROT): sum g, sum g * xhat (BnBwdStats: g =
//        dx * act'(xhat * gamma + beta), the gradient of the BN(+act) whose output the conv
//        read) — what ewvit_bn_bwd_partials finalises
// The 32 row sums of a channel are added in row order through LDS (deterministic).  Launched
// for the stride-2 forward only (the first block of stages 4 and 6); the stride-1 forms run on
// dw_row4_kernel below.
struct DwBnFwd {
  float *part = nullptr;
  const float *shift = nullptr;
  float *shift_out = nullptr;
};
// The BatchNorm(+act) + squeeze-excitation backward of the conv's OUTPUT, folded into the
// stride-1 fused backward (dw_row4_kernel SE): the conv's output gradient
//   dz = gamma*invstd*(act'(zhat*gamma + beta) * (dy*s + g) - row/n - zhat * row'/n),
// zhat = (z - mean)*invstd, is formed from the SE output gradient dy and z as the window loads
// them — the same operations in the same order as bn_bwd_dx_kernel<bf16, act, 2>, rounded to
// bf16 as it stores dz — so the dz tensor is never written or read (ewvit_bn_se_bwd with dx
// NULL leaves `row` and dgamma / dbeta).
struct DwSe {
  const bf16_t *z = nullptr;                     // the BatchNorm's input (the conv's output)
  const float *mean = nullptr, *invstd = nullptr, *gamma = nullptr, *beta = nullptr;
  const float *row = nullptr;                    // [2C]: sum g', sum g' zhat
  const float *s = nullptr, *g = nullptr;        // [N][C]: excitation, squeeze term
  float n = 1.f;                                 // rows N*H*W
  int act = 0;
};
template <int STRIDE, bool ROT, int ST, int ACT>
__global__ __launch_bounds__(256) void dw_row_bn_kernel(const bf16_t *__restrict__ x, const float *__restrict__ w,
                                                        bf16_t *__restrict__ y, DwShape s, DwBnFwd f, BnBwdStats b) {
  __shared__ float red[32 * 8 * 16];
  const int tid = threadIdx.x, cv = tid & 7, r = tid >> 3;
  const int C8 = s.C >> 3;
  const int c8 = blockIdx.y * 8 + cv;
  const int64_t row = (int64_t)blockIdx.x * 32 + r;          // n*Ho + ho
  const bool active = c8 < C8 && row < (int64_t)s.N * s.Ho;
  float sa[8], sb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sa[j] = 0.f; sb[j] = 0.f; }
  if (active) {
    const int ho = (int)(row % s.Ho);
    const int n = (int)(row / s.Ho);
    const int c = c8 * 8;
    float wr[9][8];
    {
      const float4 *wp = reinterpret_cast<const float4 *>(w + (int64_t)c * 9);
      float t[72];
#pragma unroll
      for (int i = 0; i < 18; ++i) {
        const float4 q = wp[i];
        t[4 * i] = q.x; t[4 * i + 1] = q.y; t[4 * i + 2] = q.z; t[4 * i + 3] = q.w;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < 9; ++k) wr[ROT ? 8 - k : k][j] = t[j * 9 + k];
    }
    float p0[8], p1[8], p2[8], p3[8];     // ST 1: K | ST 2: mean, invstd, gamma, beta
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (ST == 1) {
        p0[j] = f.shift ? f.shift[c + j] : 0.f;
      } else {
        p0[j] = b.mean[c + j]; p1[j] = b.invstd[c + j];
        p2[j] = b.gamma ? b.gamma[c + j] : 1.f; p3[j] = b.beta ? b.beta[c + j] : 0.f;
      }
    }
      bool rok[3];
    int64_t rbase[3];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int hi = ho * STRIDE - s.pad + kh;
      rok[kh] = hi >= 0 && hi < s.H;
      rbase[kh] = (((int64_t)n * s.H + (rok[kh] ? hi : 0)) * s.W) * s.C + c;
    }
    const __amdgpu_buffer_rsrc_t xr = dw_rsrc(x, (int64_t)s.N * s.H * s.W * s.C);
    auto ld = [&](int kh, int col) -> uint4 {   // zeros outside the map (DW_OOB)
      return dw_ld16(xr, rok[kh] && col >= 0 && col < s.W ? (uint32_t)((rbase[kh] + (int64_t)col * s.C) * 2) : DW_OOB);
    };
    const int64_t ybase = (row * s.Wo) * s.C + c;
    // one output pixel from the window columns (w0, w1, w2) and the BN input bq (ST 2)
    auto pixel = [&](const uint4 (&w0)[3], const uint4 (&w1)[3], const uint4 (&w2)[3], const uint4 &bq, int wo) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const uint4 *cols[3] = {w0, w1, w2};
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          float v[8];
          bf8_unpack(cols[kw][kh], v);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = fmaf(v[j], wr[kh * 3 + kw][j], acc[j]);
        }
      unsigned o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (unsigned)f2bf(acc[2 * j]) | ((unsigned)f2bf(acc[2 * j + 1]) << 16);
      const uint4 oq = make_uint4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<uint4 *>(y + ybase + (int64_t)wo * s.C) = oq;
      float v[8];
      bf8_unpack(oq, v);
      if (ST == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[j] - p0[j];
          sa[j] += d;
          sb[j] = fmaf(d, d, sb[j]);
        }
      } else {
        float xv[8];
        bf8_unpack(bq, xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (xv[j] - p0[j]) * p1[j];
          const float g = ACT ? v[j] * bn_act_grad(ACT, fmaf(xh, p2[j], p3[j])) : v[j];
          sa[j] += g;
          sb[j] = fmaf(g, xh, sb[j]);
        }
      }
    };
    {
      uint4 win[3][3];
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) win[kw][kh] = ld(kh, -s.pad + kw);
      for (int wo = 0; wo < s.Wo; ++wo) {
        pixel(win[0], win[1], win[2], make_uint4(0u, 0u, 0u, 0u), wo);
        const int nb = (wo + 1) * STRIDE - s.pad;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          win[0][kh] = win[2][kh];
          win[1][kh] = ld(kh, nb + 1);
          win[2][kh] = ld(kh, nb + 2);
        }
      }
    }
  }
  float *q = red + (r * 8 + cv) * 16;
#pragma unroll
  for (int j = 0; j < 8; ++j) { q[j] = sa[j]; q[8 + j] = sb[j]; }
  __syncthreads();
  if (tid < 64) {
    const int v = tid >> 3, j = tid & 7;
    const int c = (blockIdx.y * 8 + v) * 8 + j;
    float A = 0.f, B = 0.f;
    for (int rr = 0; rr < 32; ++rr) {
      A += red[(rr * 8 + v) * 16 + j];
      B += red[(rr * 8 + v) * 16 + 8 + j];
    }
    if (c < s.C) {
      float *pr = (ST == 1 ? f.part : b.part) + (int64_t)blockIdx.x * 2 * s.C;
      pr[c] = A;
      pr[s.C + c] = B;
      if (ST == 1 && blockIdx.x == 0 && f.shift_out) f.shift_out[c] = f.shift ? f.shift[c] : 0.f;
    }
  }
}

// ---- stride-1 pad-1 row kernel with 4-channel threads: the MBConv depthwise conv of blocks
// after the first of stages 4-6 (7^2 / 14^2 maps, 28 of the step's 30 depthwise convs).
//   ST 1: forward + the BatchNorm statistics of y (as dw_row_bn_kernel ST 1);
//   ST 2: input gradient (the rotated-kernel conv of dy) + the backward sums of the
//         BatchNorm(+act ACT) whose output the conv read (as dw_row_bn_kernel ST 2), and with
//         WG also the weight gradient dW[c][kh][kw] = sum dy[h][w] x[h - 1 + kh][w - 1 + kw] —
//         whose dy is the centre of the dx window, so the whole backward reads dy once, plus an
//         x window sliding in step, in one launch instead of two.
// The 8-channel row kernels were latency-bound (0.9-1.9 TB/s: 448 / 896 rows of 7 / 14 columns,
// ~230 VGPRs, 2 waves per SIMD); a 4-channel thread halves the weights, windows and sums it
// holds and doubles the waves.  The window's next column is loaded a column ahead.  Block = 32 rows x 8 channel quads (32 channels): one
// partial row of BN sums per block (part[blockIdx.x][2C], its 32 channels) and with WG one dW
// slab wpart[blockIdx.x][C][9] for dw_bwd_weight_reduce_kernel; the block's sums over its rows
// go lane bits 3..5 by DPP / permlane, then the 4 waves in order through LDS (deterministic).
__device__ __forceinline__ void bf4_unpack(const uint2 &q, float (&v)[4]) {
  v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
  v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
}
#ifndef DW_PD
#define DW_PD 1          // columns loaded ahead (2 / 3 measured slower: profiles/r06/s2/ab/dw_prefetch.log)
#endif
#ifndef DW_Q16
#define DW_Q16 0         // 1: 16 channel quads (128 B of a row) per block row, 512-thread blocks
#endif
constexpr int DW_NQ = DW_Q16 ? 16 : 8;           // channel quads per block row
constexpr int DW_THREADS = 32 * DW_NQ;            // 32 rows per block (ewvit_dwconv3x3_bn_rows)
template <int ST, int ACT, bool WG, bool SE = false>
__global__ __launch_bounds__(DW_THREADS, (WG ? 2 : 4) * 256 / DW_THREADS) void dw_row4_kernel(
    const bf16_t *__restrict__ in, const bf16_t *__restrict__ x, const float *__restrict__ w, bf16_t *__restrict__ out,
    DwShape s, DwBnFwd f, BnBwdStats b, float *__restrict__ wpart, DwSe e = DwSe()) {
  static_assert(!SE || (ST == 2 && DW_PD == 1), "the SE fold is the stride-1 backward with one column ahead");
  constexpr int NV = 8 + (WG ? 36 : 0);        // per quad: 4 + 4 BN sums (+ 36 dW)
  constexpr int NW = DW_THREADS / 64;
  __shared__ float red[NW][DW_NQ * NV];
  const int tid = threadIdx.x, q = tid % DW_NQ, r = tid / DW_NQ, wv = tid >> 6;
  const int C4 = s.C >> 2;
  const int c4 = blockIdx.y * DW_NQ + q;
  const int64_t row = (int64_t)blockIdx.x * 32 + r;          // n*H + h
  const bool active = c4 < C4 && row < (int64_t)s.N * s.H;
  float sa[4], sb[4], acc[WG ? 9 : 1][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sa[j] = 0.f; sb[j] = 0.f;
#pragma unroll
    for (int k = 0; k < (WG ? 9 : 1); ++k) acc[k][j] = 0.f;
  }
  if (active) {
    const int h = (int)(row % s.H);
    const int n = (int)(row / s.H);
    const int c = c4 * 4;
    float wr[9][4];                            // [window tap][channel]; ST 2 rotated
    {
      const float4 *wp = reinterpret_cast<const float4 *>(w + (int64_t)c * 9);
      float t[36];
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        const float4 v = wp[i];
        t[4 * i] = v.x; t[4 * i + 1] = v.y; t[4 * i + 2] = v.z; t[4 * i + 3] = v.w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 9; ++k) wr[ST == 2 ? 8 - k : k][j] = t[j * 9 + k];
    }
    float p0[4], p1[4], p2[4], p3[4];          // ST 1: K | ST 2: mean, invstd, gamma, beta
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (ST == 1) {
        p0[j] = f.shift ? f.shift[c + j] : 0.f;
      } else {
        p0[j] = b.mean[c + j]; p1[j] = b.invstd[c + j];
        p2[j] = b.gamma ? b.gamma[c + j] : 1.f; p3[j] = b.beta ? b.beta[c + j] : 0.f;
      }
    }
    bool rok[3];
    int64_t rbase[3];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int hi = h - 1 + kh;
      rok[kh] = hi >= 0 && hi < s.H;
      rbase[kh] = (((int64_t)n * s.H + (rok[kh] ? hi : 0)) * s.W) * s.C + c;
    }
    const int64_t total = (int64_t)s.N * s.H * s.W * s.C;
    const __amdgpu_buffer_rsrc_t ir = dw_rsrc(in, total);
    const __amdgpu_buffer_rsrc_t xr = dw_rsrc(WG ? (const void *)x : (const void *)in, total);
    const __amdgpu_buffer_rsrc_t br = dw_rsrc(ST == 2 ? (const void *)b.x : (const void *)in, total);
    auto off = [&](int kh, int col) -> uint32_t {  // zeros outside the map (DW_OOB)
      return rok[kh] && col >= 0 && col < s.W ? (uint32_t)((rbase[kh] + (int64_t)col * s.C) * 2) : DW_OOB;
    };
    const int64_t base = (row * s.W) * s.C + c;
    auto boff = [&](int col) -> uint32_t {
      return col < s.W ? (uint32_t)((base + (int64_t)col * s.C) * 2) : DW_OOB;
    };
    // SE: the folded BN + SE backward's per-channel (and, for this row's frame, per-frame) factors
    float e_mu[4], e_iv[4], e_ga[4], e_be[4], e_c0[4], e_c1[4], e_sv[4], e_gv[4];
    if constexpr (SE) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        e_mu[j] = e.mean[c + j]; e_iv[j] = e.invstd[c + j];
        e_ga[j] = e.gamma ? e.gamma[c + j] : 1.f; e_be[j] = e.beta ? e.beta[c + j] : 0.f;
        e_c0[j] = e.row[c + j] / e.n; e_c1[j] = e.row[s.C + c + j] / e.n;
        e_sv[j] = e.s[(int64_t)n * s.C + c + j]; e_gv[j] = e.g[(int64_t)n * s.C + c + j];
      }
    }
    const __amdgpu_buffer_rsrc_t zr = dw_rsrc(SE ? (const void *)e.z : (const void *)in, total);
    // dz of one window element from dy and z (zero outside the map, as the dz tensor's load was)
    auto xf = [&](uint2 dq, uint2 zq, bool ok) -> uint2 {
      float vd[4], vz[4], o[4];
      bf4_unpack(dq, vd);
      bf4_unpack(zq, vz);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        vd[j] = fmaf(vd[j], e_sv[j], e_gv[j]);
        const float xh = (vz[j] - e_mu[j]) * e_iv[j];
        const float g = e.act ? vd[j] * bn_act_grad(e.act, fmaf(xh, e_ga[j], e_be[j])) : vd[j];
        o[j] = e_ga[j] * e_iv[j] * (g - e_c0[j] - xh * e_c1[j]);
      }
      return ok ? make_uint2((unsigned)f2bf(o[0]) | ((unsigned)f2bf(o[1]) << 16),
                             (unsigned)f2bf(o[2]) | ((unsigned)f2bf(o[3]) << 16))
                : make_uint2(0u, 0u);
    };
    // window columns col - 1 .. col + 1 ([kw][kh]; G the conv input's, X (WG) x's) and the
    // next DW_PD columns col + 2 .. loaded ahead, like the BN input (ST 2) — DW_PD columns of
    // loads in flight behind the current one's FMAs; every load is a buffer load (zeros outside
    // the map), so the loop has no branch
    uint2 G[3][3], X[3][3], Gn[DW_PD][3], Xn[DW_PD][3], bq[DW_PD], Zn[3];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const uint32_t o = off(kh, kw - 1);
        G[kw][kh] = dw_ld8(ir, o);
        if constexpr (SE) G[kw][kh] = xf(G[kw][kh], dw_ld8(zr, o), o != DW_OOB);
        if (WG) X[kw][kh] = dw_ld8(xr, o);
      }
#pragma unroll
      for (int p = 0; p < DW_PD; ++p) {
        Gn[p][kh] = dw_ld8(ir, off(kh, 2 + p));
        if (WG) Xn[p][kh] = dw_ld8(xr, off(kh, 2 + p));
      }
      if constexpr (SE) Zn[kh] = dw_ld8(zr, off(kh, 2));
    }
#pragma unroll
    for (int p = 0; p < DW_PD; ++p) bq[p] = ST == 2 ? dw_ld8(br, boff(p)) : make_uint2(0u, 0u);
#pragma unroll 1
    for (int col = 0; col < s.W; ++col) {
      float o4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          float v[4];
          bf4_unpack(G[kw][kh], v);
#pragma unroll
          for (int j = 0; j < 4; ++j) o4[j] = fmaf(v[j], wr[kh * 3 + kw][j], o4[j]);
        }
      if (WG) {
        float g[4];
        bf4_unpack(G[1][1], g);                // dy[h][col]: the weight gradient's dy
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int kh = 0; kh < 3; ++kh) {
            float v[4];
            bf4_unpack(X[kw][kh], v);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[WG ? kh * 3 + kw : 0][j] = fmaf(g[j], v[j], acc[WG ? kh * 3 + kw : 0][j]);
          }
      }
      const uint2 oq = make_uint2((unsigned)f2bf(o4[0]) | ((unsigned)f2bf(o4[1]) << 16),
                                  (unsigned)f2bf(o4[2]) | ((unsigned)f2bf(o4[3]) << 16));
      *reinterpret_cast<uint2 *>(out + base + (int64_t)col * s.C) = oq;
      float v[4];
      bf4_unpack(oq, v);
      if (ST == 1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = v[j] - p0[j];
          sa[j] += d;
          sb[j] = fmaf(d, d, sb[j]);
        }
      } else {
        float xv[4];
        bf4_unpack(bq[0], xv);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float xh = (xv[j] - p0[j]) * p1[j];
          const float gg = ACT ? v[j] * bn_act_grad(ACT, fmaf(xh, p2[j], p3[j])) : v[j];
          sa[j] += gg;
          sb[j] = fmaf(gg, xh, sb[j]);
        }
#pragma unroll
        for (int p = 0; p + 1 < DW_PD; ++p) bq[p] = bq[p + 1];
        bq[DW_PD - 1] = dw_ld8(br, boff(col + DW_PD));
      }
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const uint32_t o = off(kh, col + 2 + DW_PD);
        G[0][kh] = G[1][kh]; G[1][kh] = G[2][kh];
        if constexpr (SE) {
          G[2][kh] = xf(Gn[0][kh], Zn[kh], off(kh, col + 2) != DW_OOB);
          Zn[kh] = dw_ld8(zr, o);
        } else {
          G[2][kh] = Gn[0][kh];
        }
#pragma unroll
        for (int p = 0; p + 1 < DW_PD; ++p) Gn[p][kh] = Gn[p + 1][kh];
        Gn[DW_PD - 1][kh] = dw_ld8(ir, o);
        if (WG) {
          X[0][kh] = X[1][kh]; X[1][kh] = X[2][kh]; X[2][kh] = Xn[0][kh];
#pragma unroll
          for (int p = 0; p + 1 < DW_PD; ++p) Xn[p][kh] = Xn[p + 1][kh];
          Xn[DW_PD - 1][kh] = dw_ld8(xr, o);
        }
      }
    }
  }
  // the wave's rows of each quad (lane bits 3..5, or 4..5 with 16 quads), then the waves in order
  float *mine = red[wv] + q * NV;
  const int lane = tid & 63;
  auto put = [&](int i, float v) {
    if constexpr (DW_NQ == 8) v += dpp_mov<0x128>(v);    // row_ror:8 = lane ^ 8 within the row
    v = rows_sum4(v);
    if (lane < DW_NQ) mine[i] = v;
  };
#pragma unroll
  for (int j = 0; j < 4; ++j) { put(j, sa[j]); put(4 + j, sb[j]); }
  if (WG) {
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) put(8 + j * 9 + k, acc[WG ? k : 0][j]);
  }
  __syncthreads();
  for (int i = tid; i < DW_NQ * NV; i += DW_THREADS) {
    const int qq = i / NV, k = i - qq * NV;
    const int cq = blockIdx.y * DW_NQ + qq;
    if (cq >= C4) continue;
    float t = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
    if constexpr (NW == 8) t += (red[4 % NW][i] + red[5 % NW][i]) + (red[6 % NW][i] + red[7 % NW][i]);
    if (k < 8) {
      float *pr = (ST == 1 ? f.part : b.part) + (int64_t)blockIdx.x * 2 * s.C;
      pr[(k < 4 ? 0 : s.C) + cq * 4 + (k & 3)] = t;
      if (ST == 1 && k < 4 && blockIdx.x == 0 && f.shift_out) f.shift_out[cq * 4 + k] = f.shift ? f.shift[cq * 4 + k] : 0.f;
    } else {
      wpart[(int64_t)blockIdx.x * s.C * 9 + (int64_t)cq * 36 + (k - 8)] = t;   // [c][tap]
    }
  }
}

// ---- bf16 input gradient of a STRIDE-2 pad-1 conv, row form (the first block of stages 4
// and 6).  dx[hi][wi] only meets the taps with kh = hi+1 (mod 2), kw = wi+1 (mod 2): an even
// dx row one dy row (kh = 1), an odd one two (kh = 0, 2); likewise along the row, so a thread
// (8 channels x one dx row segment) walks dx columns in pairs (2j, 2j+1): the even column
// takes dy column j (kw = 1), the odd one dy columns j+1 (kw = 0) and j (kw = 2) — one new
// 16-B dy load per dy row per pair, the 72 weights in registers.  (The generic kernel this
// replaces gathered its weights per lane and tested every tap: 0.5 TB/s.)
__global__ __launch_bounds__(256) void dw_row_s2_bwd_kernel(const bf16_t *__restrict__ dy, const float *__restrict__ w,
                                                            bf16_t *__restrict__ dx, DwShape s, int rows_per_block,
                                                            int segs) {
  const int C8 = s.C >> 3;
  const int r = threadIdx.x / C8, c8 = threadIdx.x % C8;
  if (r >= rows_per_block) return;
  const int64_t vrow = (int64_t)blockIdx.x * rows_per_block + r;
  if (vrow >= (int64_t)s.N * s.H * segs) return;
  const int64_t row = vrow / segs;                                   // n*H + hi
  const int npair = (s.W + 1) / 2;                                   // dx column pairs
  const int pseg = (npair + segs - 1) / segs;
  const int j0 = (int)(vrow - row * segs) * pseg;
  const int j1 = j0 + pseg < npair ? j0 + pseg : npair;
  const int hi = (int)(row % s.H);
  const int n = (int)(row / s.H);
  const int c = c8 * 8;
  float wr[9][8];  // [tap][channel]
  {
    const float4 *wp = reinterpret_cast<const float4 *>(w + (int64_t)c * 9);
    float t[72];
#pragma unroll
    for (int i = 0; i < 18; ++i) {
      const float4 q = wp[i];
      t[4 * i] = q.x; t[4 * i + 1] = q.y; t[4 * i + 2] = q.z; t[4 * i + 3] = q.w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int k = 0; k < 9; ++k) wr[k][j] = t[j * 9 + k];
  }
  // dy rows: even hi -> ho = hi/2 (kh 1); odd hi -> ho = (hi+1)/2 (kh 0), (hi-1)/2 (kh 2)
  const bool odd = hi & 1;
  const int hoA = odd ? (hi + 1) >> 1 : hi >> 1, khA = odd ? 0 : 1;
  const int hoB = (hi - 1) >> 1, khB = 2;                            // odd rows only
  const bool okA = hoA < s.Ho, okB = odd && hoB >= 0;
  const int64_t rA = (((int64_t)n * s.Ho + (okA ? hoA : 0)) * s.Wo) * s.C + c;
  const int64_t rB = (((int64_t)n * s.Ho + (okB ? hoB : 0)) * s.Wo) * s.C + c;
  const __amdgpu_buffer_rsrc_t gr = dw_rsrc(dy, (int64_t)s.N * s.Ho * s.Wo * s.C);
  auto ld = [&](int64_t rp, bool ok, int col) -> uint4 {   // zeros outside the map (DW_OOB)
    return dw_ld16(gr, ok && col >= 0 && col < s.Wo ? (uint32_t)((rp + (int64_t)col * s.C) * 2) : DW_OOB);
  };
  uint4 a0 = ld(rA, okA, j0), b0 = ld(rB, okB, j0);                  // dy column j of rows A, B
  bf16_t *xrow = dx + (row * s.W) * s.C + c;
  for (int j = j0; j < j1; ++j) {
    const uint4 a1 = ld(rA, okA, j + 1), b1 = ld(rB, okB, j + 1);    // dy column j+1
    float va0[8], va1[8], vb0[8], vb1[8];
    bf8_unpack(a0, va0); bf8_unpack(a1, va1); bf8_unpack(b0, vb0); bf8_unpack(b1, vb1);
    float e[8], o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      // even column 2j: kw = 1 on dy column j;  odd column 2j+1: kw = 0 on j+1, kw = 2 on j
      // (row B is all zeros for an even dx row: its terms add nothing, no branch)
      e[q] = fmaf(vb0[q], wr[khB * 3 + 1][q], va0[q] * wr[khA * 3 + 1][q]);
      o[q] = fmaf(va1[q], wr[khA * 3 + 0][q], va0[q] * wr[khA * 3 + 2][q]);
      o[q] = fmaf(vb1[q], wr[khB * 3 + 0][q], fmaf(vb0[q], wr[khB * 3 + 2][q], o[q]));
    }
    unsigned pe[4], po[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      pe[q] = (unsigned)f2bf(e[2 * q]) | ((unsigned)f2bf(e[2 * q + 1]) << 16);
      po[q] = (unsigned)f2bf(o[2 * q]) | ((unsigned)f2bf(o[2 * q + 1]) << 16);
    }
    *reinterpret_cast<uint4 *>(xrow + (int64_t)(2 * j) * s.C) = make_uint4(pe[0], pe[1], pe[2], pe[3]);
    if (2 * j + 1 < s.W)
      *reinterpret_cast<uint4 *>(xrow + (int64_t)(2 * j + 1) * s.C) = make_uint4(po[0], po[1], po[2], po[3]);
    a0 = a1; b0 = b1;
  }
}

// ---- bf16 weight gradient, row form.  Thread = 8 channels; it walks whole output
// rows (row += gridDim.x * R) accumulating its 72 (tap, channel) products in fp32
// registers over a sliding x window (one dy + 3*s x loads per output).  The R row
// groups of a block are summed through one LDS buffer, then the block writes one
// partial slab [C][9]; dw_bwd_weight_reduce_kernel adds the slabs in block order
// (deterministic).
template <int STRIDE>
__global__ __launch_bounds__(512) void dw_wgrad_row_bf16_kernel(const bf16_t *__restrict__ x,
                                                                const bf16_t *__restrict__ dy,
                                                                float *__restrict__ part, DwShape s, int R) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // C8 * 72 floats (dynamic)
  const int C8 = s.C >> 3;
  const int r = threadIdx.x / C8, c8 = threadIdx.x % C8;
  const bool active = r < R;
  const int c = c8 * 8;
  float acc[9][8];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  const int64_t nrows = (int64_t)s.N * s.Ho;
  for (int64_t row = (int64_t)blockIdx.x * R + r; active && row < nrows; row += (int64_t)gridDim.x * R) {
    const int ho = (int)(row % s.Ho);
    const int n = (int)(row / s.Ho);
    bool rok[3];
    int64_t rbase[3];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int hi = ho * STRIDE - s.pad + kh;
      rok[kh] = hi >= 0 && hi < s.H;
      rbase[kh] = (((int64_t)n * s.H + (rok[kh] ? hi : 0)) * s.W) * s.C + c;
    }
    const __amdgpu_buffer_rsrc_t xr = dw_rsrc(x, (int64_t)s.N * s.H * s.W * s.C);
    auto ld = [&](int kh, int col) -> uint4 {   // zeros outside the map (DW_OOB)
      return dw_ld16(xr, rok[kh] && col >= 0 && col < s.W ? (uint32_t)((rbase[kh] + (int64_t)col * s.C) * 2) : DW_OOB);
    };
    uint4 win[3][3];
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) win[kw][kh] = ld(kh, -s.pad + kw);
    uint4 nx[3];                           // stride 1: the next column, one column ahead
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) nx[kh] = STRIDE == 1 ? ld(kh, 3 - s.pad) : make_uint4(0u, 0u, 0u, 0u);
    // dy of this output pixel, loaded one column ahead too
    const __amdgpu_buffer_rsrc_t gr = dw_rsrc(dy, (int64_t)s.N * s.Ho * s.Wo * s.C);
    const uint32_t gb = (uint32_t)(((row * s.Wo) * s.C + c) * 2), gstep = (uint32_t)s.C * 2;
    uint4 gq = dw_ld16(gr, gb);
    for (int wo = 0; wo < s.Wo; ++wo) {
      float g[8];
      bf8_unpack(gq, g);
      gq = dw_ld16(gr, wo + 1 < s.Wo ? gb + (uint32_t)(wo + 1) * gstep : DW_OOB);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          float v[8];
          bf8_unpack(win[kw][kh], v);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[kh * 3 + kw][j] = fmaf(g[j], v[j], acc[kh * 3 + kw][j]);
        }
      const int nb = (wo + 1) * STRIDE - s.pad;
      if (STRIDE == 1) {
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          win[0][kh] = win[1][kh];
          win[1][kh] = win[2][kh];
          win[2][kh] = nx[kh];
          nx[kh] = ld(kh, nb + 3);
        }
      } else {
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          win[0][kh] = win[2][kh];
          win[1][kh] = ld(kh, nb + 1);
          win[2][kh] = ld(kh, nb + 2);
        }
      }
    }
  }
  // sum the R row groups: group 0 stores, groups 1..R-1 add in order
  float *mine = red + c8 * 72;  // [c8][channel j][tap k] = layout of dw [C][9]
  for (int g = 0; g < R; ++g) {
    if (active && r == g) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < 9; ++k) mine[j * 9 + k] = (g == 0 ? 0.f : mine[j * 9 + k]) + acc[k][j];
    }
    __syncthreads();
  }
  float *dst = part + (int64_t)blockIdx.x * s.C * 9;
  for (int i = threadIdx.x; i < C8 * 72; i += blockDim.x) dst[i] = red[i];
}

// Weight gradient, pass 1: block = 64 channels x a slab of output pixels.
// tid = pl*8 + cg: 8 channel groups (8 channels each) x 32 pixel lanes.
constexpr int DWW_PIX_PER_BLOCK = 256;

template <int DT>
__global__ __launch_bounds__(256) void dw_bwd_weight_partial_kernel(const void *__restrict__ x,
                                                                    const void *__restrict__ dy,
                                                                    float *__restrict__ part, DwShape s,
                                                                    int64_t npix) {
  __shared__ float red[4][64 * 9];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int cg = tid & 7, pl = tid >> 3;  // pl 0..31
  const int c = blockIdx.y * 64 + cg * 8;
  const bool cok = c < s.C;
  float acc[9][8];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  const int64_t p0 = (int64_t)blockIdx.x * DWW_PIX_PER_BLOCK;
  if (cok) {
    for (int64_t p = p0 + pl; p < p0 + DWW_PIX_PER_BLOCK && p < npix; p += 32) {
      const int wo = (int)(p % s.Wo);
      const int64_t t = p / s.Wo;
      const int ho = (int)(t % s.Ho);
      const int n = (int)(t / s.Ho);
      float g[8];
      Vec8<DT>::load(dy, p * s.C + c, g);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int hi = ho * s.stride - s.pad + kh;
        if (hi < 0 || hi >= s.H) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int wi = wo * s.stride - s.pad + kw;
          if (wi < 0 || wi >= s.W) continue;
          float v[8];
          Vec8<DT>::load(x, (((int64_t)n * s.H + hi) * s.W + wi) * s.C + c, v);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[kh * 3 + kw][j] = fmaf(g[j], v[j], acc[kh * 3 + kw][j]);
        }
      }
    }
  }
  // reduce the 8 pixel lanes of this wave (lane bits 3..5), then the 4 waves via LDS
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = acc[k][j];
      v += dpp_mov<0x128>(v);   // row_ror:8 = lane ^ 8 within the row
      v = rows_sum4(v);
      acc[k][j] = v;
    }
  if (lane < 8) {
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wv][(cg * 8 + j) * 9 + k] = acc[k][j];
  }
  __syncthreads();
  for (int i = tid; i < 64 * 9; i += 256) {
    const int cc = blockIdx.y * 64 + i / 9;
    if (cc < s.C)
      part[(int64_t)blockIdx.x * s.C * 9 + (int64_t)blockIdx.y * 64 * 9 + i] =
          red[0][i] + red[1][i] + red[2][i] + red[3][i];
  }
}

// Sum the per-block slabs: block = 64 outputs x 4 slab groups (one wave each,
// every wave reading 256 contiguous bytes per slab, 4 loads in flight), then the
// 4 groups are added through LDS in a fixed order (deterministic).
__global__ __launch_bounds__(256) void dw_bwd_weight_reduce_kernel(const float *__restrict__ part,
                                                                   float *__restrict__ dw, int64_t n,
                                                                   int slabs, int accumulate) {
  __shared__ float red[256];
  dw_slab_reduce_block(part, dw, n, slabs, accumulate, (int)blockIdx.x, red);   // (reduce_jobs.h)
}

static int check_shape(const DwShape &s, const char *nm) {
  EWVIT_CHECK_ARG(s.N > 0 && s.H > 0 && s.W > 0 && s.C > 0, "%s: empty shape", nm);
  EWVIT_CHECK_ARG(s.C % 8 == 0, "%s: C=%d must be a multiple of 8 (16-B channel vectors)", nm, s.C);
  EWVIT_CHECK_ARG(s.stride == 1 || s.stride == 2, "%s: stride %d", nm, s.stride);
  EWVIT_CHECK_ARG(s.pad >= 0 && s.pad <= 2, "%s: pad %d", nm, s.pad);
  EWVIT_CHECK_ARG(s.Ho == (s.H + 2 * s.pad - 3) / s.stride + 1 && s.Wo == (s.W + 2 * s.pad - 3) / s.stride + 1,
                  "%s: output size mismatch", nm);
  return 0;
}

}  // namespace ewvit

using namespace ewvit;

static DwShape mk(int64_t N, int64_t H, int64_t W, int64_t C, int stride, int pad) {
  DwShape s;
  s.N = (int)N; s.H = (int)H; s.W = (int)W; s.C = (int)C; s.stride = stride; s.pad = pad;
  s.Ho = (int)((H + 2 * pad - 3) / stride + 1);
  s.Wo = (int)((W + 2 * pad - 3) / stride + 1);
  return s;
}

// The row kernels walk whole output rows (segs = 1).  Measured and removed: column segments
// per row for the 7^2 / 14^2 maps (2682 vs 2703 frames/s: one more 3x3 window fill per
// segment) and a per-pixel kernel for them (SFE piece 14.29-14.32 -> 15.09-15.12 ms: the 9 tap
// loads of a pixel re-read each input vector 9 times through L1/L2 where the row kernel's
// window re-reads it 3 times).
extern "C" int ewvit_dwconv3x3_fwd(const void *x, const float *w, void *y, int64_t N, int64_t H, int64_t W,
                                   int64_t C, int stride, int pad, int dtype, void *stream) {
  EWVIT_CHECK_ARG(x && w && y && dtype_ok(dtype), "dwconv3x3_fwd: bad args");
  DwShape s = mk(N, H, W, C, stride, pad);
  if (int rc = check_shape(s, "dwconv3x3_fwd")) return rc;
  const bool buf = dw_bufok((int64_t)s.N * s.H * s.W * s.C) && dw_bufok((int64_t)s.N * s.Ho * s.Wo * s.C);
  if (dtype == EWVIT_BF16 && s.C / 8 <= 256 && (s.stride == 1 || s.stride == 2) && buf) {
    const int rpb = 256 / (s.C / 8), segs = 1;
    dim3 grid((unsigned)(((int64_t)s.N * s.Ho + rpb - 1) / rpb));
    if (s.stride == 1)
      hipLaunchKernelGGL((dw_row_bf16_kernel<1, false>), grid, dim3(256), 0, as_stream(stream),
                         (const bf16_t *)x, w, (bf16_t *)y, s, rpb, segs);
    else
      hipLaunchKernelGGL((dw_row_bf16_kernel<2, false>), grid, dim3(256), 0, as_stream(stream),
                         (const bf16_t *)x, w, (bf16_t *)y, s, rpb, segs);
  } else {
    const int64_t total = (int64_t)s.N * s.Ho * s.Wo * (s.C / 8);
    dim3 grid((unsigned)((total + 255) / 256));
    if (dtype == EWVIT_BF16)
      hipLaunchKernelGGL(dw_fwd_kernel<EWVIT_BF16>, grid, dim3(256), 0, as_stream(stream), x, w, y, s);
    else
      hipLaunchKernelGGL(dw_fwd_kernel<EWVIT_F32>, grid, dim3(256), 0, as_stream(stream), x, w, y, s);
  }
  return launch_status("dwconv3x3_fwd");
}

extern "C" int ewvit_dwconv3x3_bwd_data(const void *dy, const float *w, void *dx, int64_t N, int64_t H,
                                        int64_t W, int64_t C, int stride, int pad, int dtype, void *stream) {
  EWVIT_CHECK_ARG(dy && w && dx && dtype_ok(dtype), "dwconv3x3_bwd_data: bad args");
  DwShape s = mk(N, H, W, C, stride, pad);
  if (int rc = check_shape(s, "dwconv3x3_bwd_data")) return rc;
  const bool buf = dw_bufok((int64_t)s.N * s.H * s.W * s.C) && dw_bufok((int64_t)s.N * s.Ho * s.Wo * s.C);
  if (dtype == EWVIT_BF16 && s.stride == 1 && s.pad == 1 && s.C / 8 <= 256 && buf) {
    // input gradient of a stride-1 pad-1 conv = stride-1 pad-1 conv of dy with the rotated kernel
    DwShape t = s;
    t.H = s.Ho; t.W = s.Wo; t.Ho = s.H; t.Wo = s.W;
    const int rpb = 256 / (s.C / 8), segs = 1;
    dim3 grid((unsigned)(((int64_t)t.N * t.Ho + rpb - 1) / rpb));
    hipLaunchKernelGGL((dw_row_bf16_kernel<1, true>), grid, dim3(256), 0, as_stream(stream),
                       (const bf16_t *)dy, w, (bf16_t *)dx, t, rpb, segs);
  } else if (dtype == EWVIT_BF16 && s.stride == 2 && s.pad == 1 && s.C / 8 <= 256 && buf && s.Ho == (s.H + 1) / 2 &&
             s.Wo == (s.W + 1) / 2) {
    // stride 2: dx rows in column pairs (dw_row_s2_bwd_kernel)
    const int rpb = 256 / (s.C / 8), segs = 1;
    dim3 grid((unsigned)(((int64_t)s.N * s.H + rpb - 1) / rpb));
    hipLaunchKernelGGL(dw_row_s2_bwd_kernel, grid, dim3(256), 0, as_stream(stream), (const bf16_t *)dy, w,
                       (bf16_t *)dx, s, rpb, segs);
  } else {
    const int64_t total = (int64_t)s.N * s.H * s.W * (s.C / 8);
    dim3 grid((unsigned)((total + 255) / 256));
    if (dtype == EWVIT_BF16)
      hipLaunchKernelGGL(dw_bwd_data_kernel<EWVIT_BF16>, grid, dim3(256), 0, as_stream(stream), dy, w, dx, s);
    else
      hipLaunchKernelGGL(dw_bwd_data_kernel<EWVIT_F32>, grid, dim3(256), 0, as_stream(stream), dy, w, dx, s);
  }
  return launch_status("dwconv3x3_bwd_data");
}

// partial rows the BatchNorm-sum forms below leave (one per 32 output rows n*Ho + ho of
// the output they store), or 0 when the shape does not take them (bf16 only, pad 1,
// stride 1 | 2 forward / stride 1 input gradient, C % 8 == 0)

extern "C" int64_t ewvit_dwconv3x3_bn_rows(int64_t N, int64_t H, int64_t W, int64_t C, int stride, int bwd) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || C > 65536 * 8 || (stride != 1 && stride != 2) ||
      (bwd && stride != 1) || !dw_bufok(N * H * W * C))
    return 0;
  const int64_t Ho = bwd ? H : (H - 1) / stride + 1;
  return (N * Ho + 31) / 32;
}

// forward + the BatchNorm statistics of y (shifted sums, ewvit_bn_fwd_partials): part
// [ewvit_dwconv3x3_bn_rows(..., 0)][2C], shift_out [C] (= shift, or zeros)
extern "C" int ewvit_dwconv3x3_fwd_bn(const void *x, const float *w, void *y, int64_t N, int64_t H, int64_t W,
                                      int64_t C, int stride, const float *shift, float *part, float *shift_out,
                                      void *stream) {
  EWVIT_CHECK_ARG(x && w && y && part && shift_out, "dwconv3x3_fwd_bn: null pointer");
  const int64_t nrc = ewvit_dwconv3x3_bn_rows(N, H, W, C, stride, 0);
  EWVIT_CHECK_ARG(nrc > 0 && nrc < 65536, "dwconv3x3_fwd_bn: shape not supported");
  DwShape s = mk(N, H, W, C, stride, 1);
  if (int rc = check_shape(s, "dwconv3x3_fwd_bn")) return rc;
  DwBnFwd f;
  f.part = part; f.shift = shift; f.shift_out = shift_out;
  BnBwdStats b;
  if (stride == 1) {
    hipLaunchKernelGGL((dw_row4_kernel<1, 0, false>), dim3((unsigned)nrc, (unsigned)((C / 4 + DW_NQ - 1) / DW_NQ)),
                       dim3(DW_THREADS), 0,
                       as_stream(stream), (const bf16_t *)x, nullptr, w, (bf16_t *)y, s, f, b, nullptr, DwSe());
    return launch_status("dwconv3x3_fwd_bn");
  }
  hipLaunchKernelGGL((dw_row_bn_kernel<2, false, 1, 0>), dim3((unsigned)nrc, (unsigned)((C / 8 + 7) / 8)), dim3(256), 0,
                     as_stream(stream), (const bf16_t *)x, w, (bf16_t *)y, s, f, b);
  return launch_status("dwconv3x3_fwd_bn");
}

// stride-1 input gradient + the backward statistics of the BatchNorm(+act) whose output the
// conv read (bx: that BN's input, mean / invstd its saved batch statistics, gamma / beta its
// affine parameters or null, act 0 / 1 / 2): part [ewvit_dwconv3x3_bn_rows(..., 1)][2C]
// for ewvit_bn_bwd_partials
extern "C" int ewvit_dwconv3x3_bwd_data_bn(const void *dy, const float *w, void *dx, int64_t N, int64_t H, int64_t W,
                                           int64_t C, const void *bx, const float *mean, const float *invstd,
                                           const float *gamma, const float *beta, int act, float *part,
                                           void *stream) {
  EWVIT_CHECK_ARG(dy && w && dx && bx && mean && invstd && part && act >= 0 && act <= 2,
                  "dwconv3x3_bwd_data_bn: bad args");
  const int64_t nrc = ewvit_dwconv3x3_bn_rows(N, H, W, C, 1, 1);
  EWVIT_CHECK_ARG(nrc > 0 && nrc < 65536, "dwconv3x3_bwd_data_bn: shape not supported");
  DwShape s = mk(N, H, W, C, 1, 1);
  if (int rc = check_shape(s, "dwconv3x3_bwd_data_bn")) return rc;
  DwBnFwd f;
  BnBwdStats b;
  b.part = part; b.x = (const bf16_t *)bx; b.mean = mean; b.invstd = invstd; b.gamma = gamma; b.beta = beta;
  b.act = act;
  auto kern = act == 2 ? dw_row4_kernel<2, 2, false> : act == 1 ? dw_row4_kernel<2, 1, false> : dw_row4_kernel<2, 0, false>;
  hipLaunchKernelGGL(kern, dim3((unsigned)nrc, (unsigned)((C / 4 + DW_NQ - 1) / DW_NQ)), dim3(DW_THREADS), 0,
                     as_stream(stream), (const bf16_t *)dy, nullptr, w, (bf16_t *)dx, s, f, b, nullptr, DwSe());
  return launch_status("dwconv3x3_bwd_data_bn");
}

// bytes of f32 workspace ewvit_dwconv3x3_bwd_fused needs: one [C][9] slab per 32 rows
extern "C" int64_t ewvit_dwconv3x3_bwd_fused_workspace(int64_t N, int64_t H, int64_t W, int64_t C) {
  const int64_t nrc = ewvit_dwconv3x3_bn_rows(N, H, W, C, 1, 1);
  return nrc * C * 9 * (int64_t)sizeof(float);
}

// the stride-1 pad-1 backward in one pass (dw_row4_kernel WG): dx, the producing BatchNorm's
// backward sums (as ewvit_dwconv3x3_bwd_data_bn: part [ewvit_dwconv3x3_bn_rows(..., 1)][2C])
// and dW [C][9] (= or += with accumulate) from x, the conv's bf16 input
extern "C" int ewvit_dwconv3x3_bwd_fused(const void *dy, const float *w, void *dx, const void *x, float *dw,
                                         int accumulate, int64_t N, int64_t H, int64_t W, int64_t C, const void *bx,
                                         const float *mean, const float *invstd, const float *gamma,
                                         const float *beta, int act, float *part, float *workspace, void *stream) {
  const bool defer_mark = reduce_take_defer();      // (reduce_jobs.h; consumed by every call)
  EWVIT_CHECK_ARG(dy && w && dx && x && dw && bx && mean && invstd && part && workspace && act >= 0 && act <= 2,
                  "dwconv3x3_bwd_fused: bad args");
  const int64_t nrc = ewvit_dwconv3x3_bn_rows(N, H, W, C, 1, 1);
  EWVIT_CHECK_ARG(nrc > 0 && nrc < 65536, "dwconv3x3_bwd_fused: shape not supported");
  DwShape s = mk(N, H, W, C, 1, 1);
  if (int rc = check_shape(s, "dwconv3x3_bwd_fused")) return rc;
  BnBwdStats b;
  b.part = part; b.x = (const bf16_t *)bx; b.mean = mean; b.invstd = invstd; b.gamma = gamma; b.beta = beta;
  b.act = act;
  hipStream_t st = as_stream(stream);
  DwBnFwd f;
  auto kern = act == 2 ? dw_row4_kernel<2, 2, true> : act == 1 ? dw_row4_kernel<2, 1, true> : dw_row4_kernel<2, 0, true>;
  hipLaunchKernelGGL(kern, dim3((unsigned)nrc, (unsigned)((C / 4 + DW_NQ - 1) / DW_NQ)), dim3(DW_THREADS), 0, st,
                     (const bf16_t *)dy, (const bf16_t *)x, w, (bf16_t *)dx, s, f, b, workspace, DwSe());
  if (int rc = launch_status("dwconv3x3_bwd_fused")) return rc;
  const int64_t n = C * 9;
  if (defer_mark) {                 // the slab sum runs in front of a later weight-gradient launch
    RedJob j;
    j.kind = 2; j.part = workspace; j.dw = dw; j.n = n; j.splits = (int)nrc; j.accumulate = accumulate;
    reduce_defer(st, j);
    return 0;
  }
  hipLaunchKernelGGL(dw_bwd_weight_reduce_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, workspace, dw, n,
                     (int)nrc, accumulate);
  return launch_status("dwconv3x3_bwd_fused reduce");
}

// ewvit_dwconv3x3_bwd_fused with the BatchNorm(+act) + squeeze-excitation backward of the conv's
// output folded in (DwSe): `dy` is the SE OUTPUT gradient, z / se_* the BN's input, saved
// statistics, affine and the sums row (ewvit_bn_se_bwd with dx NULL), se_s / se_g [N][C]
extern "C" int ewvit_dwconv3x3_bwd_fused_se(const void *dy, const float *w, void *dx, const void *x, float *dw,
                                            int accumulate, int64_t N, int64_t H, int64_t W, int64_t C, const void *bx,
                                            const float *mean, const float *invstd, const float *gamma,
                                            const float *beta, int act, float *part, float *workspace, const void *z,
                                            const float *se_mean, const float *se_invstd, const float *se_gamma,
                                            const float *se_beta, int se_act, const float *se_row, const float *se_s,
                                            const float *se_g, void *stream) {
  const bool defer_mark = reduce_take_defer();      // (reduce_jobs.h; consumed by every call)
  EWVIT_CHECK_ARG(dy && w && dx && x && dw && bx && mean && invstd && part && workspace && act >= 0 && act <= 2 &&
                      z && se_mean && se_invstd && se_row && se_s && se_g && se_act >= 0 && se_act <= 2,
                  "dwconv3x3_bwd_fused_se: bad args");
  const int64_t nrc = ewvit_dwconv3x3_bn_rows(N, H, W, C, 1, 1);
  EWVIT_CHECK_ARG(nrc > 0 && nrc < 65536, "dwconv3x3_bwd_fused_se: shape not supported");
  DwShape s = mk(N, H, W, C, 1, 1);
  if (int rc = check_shape(s, "dwconv3x3_bwd_fused_se")) return rc;
  BnBwdStats b;
  b.part = part; b.x = (const bf16_t *)bx; b.mean = mean; b.invstd = invstd; b.gamma = gamma; b.beta = beta;
  b.act = act;
  DwSe e;
  e.z = (const bf16_t *)z; e.mean = se_mean; e.invstd = se_invstd; e.gamma = se_gamma; e.beta = se_beta;
  e.row = se_row; e.s = se_s; e.g = se_g; e.n = (float)(N * H * W); e.act = se_act;
  hipStream_t st = as_stream(stream);
  DwBnFwd f;
  auto kern = act == 2 ? dw_row4_kernel<2, 2, true, true> : act == 1 ? dw_row4_kernel<2, 1, true, true>
                                                                   : dw_row4_kernel<2, 0, true, true>;
  hipLaunchKernelGGL(kern, dim3((unsigned)nrc, (unsigned)((C / 4 + DW_NQ - 1) / DW_NQ)), dim3(DW_THREADS), 0, st,
                     (const bf16_t *)dy, (const bf16_t *)x, w, (bf16_t *)dx, s, f, b, workspace, e);
  if (int rc = launch_status("dwconv3x3_bwd_fused_se")) return rc;
  const int64_t n = C * 9;
  if (defer_mark) {
    RedJob j;
    j.kind = 2; j.part = workspace; j.dw = dw; j.n = n; j.splits = (int)nrc; j.accumulate = accumulate;
    reduce_defer(st, j);
    return 0;
  }
  hipLaunchKernelGGL(dw_bwd_weight_reduce_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, workspace, dw, n,
                     (int)nrc, accumulate);
  return launch_status("dwconv3x3_bwd_fused_se reduce");
}

// weight-gradient plan: row kernel (bf16, C/8 <= 256) with `slabs` blocks, or the
// generic pixel-slab kernel; the workspace holds one [C][9] f32 slab per block
static void wgrad_plan(const DwShape &s, int dtype, bool *row, int *R, int64_t *slabs) {
  const int C8 = s.C / 8;
  *row = dtype == EWVIT_BF16 && C8 <= 256 && (s.stride == 1 || s.stride == 2) &&
         dw_bufok((int64_t)s.N * s.H * s.W * s.C) && dw_bufok((int64_t)s.N * s.Ho * s.Wo * s.C);
  if (*row) {
    *R = 512 / C8;
    const int64_t nrows = (int64_t)s.N * s.Ho;
    int64_t nb = (nrows + (int64_t)(*R) - 1) / (int64_t)(*R);   // one row per thread, 512-thread blocks
    *slabs = nb < 1 ? 1 : (nb > 2048 ? 2048 : nb);
  } else {
    *R = 0;
    const int64_t npix = (int64_t)s.N * s.Ho * s.Wo;
    *slabs = (npix + DWW_PIX_PER_BLOCK - 1) / DWW_PIX_PER_BLOCK;
  }
}

extern "C" int64_t ewvit_dwconv3x3_bwd_weight_workspace(int64_t N, int64_t H, int64_t W, int64_t C, int stride,
                                                        int pad) {
  DwShape s = mk(N, H, W, C, stride, pad);
  bool row; int R; int64_t slabs, slabs_f32;
  wgrad_plan(s, EWVIT_BF16, &row, &R, &slabs);
  wgrad_plan(s, EWVIT_F32, &row, &R, &slabs_f32);
  if (slabs_f32 > slabs) slabs = slabs_f32;
  return slabs * C * 9 * (int64_t)sizeof(float);
}

extern "C" int ewvit_dwconv3x3_bwd_weight(const void *x, const void *dy, float *dw, int accumulate, int64_t N,
                                          int64_t H, int64_t W, int64_t C, int stride, int pad, int dtype,
                                          float *workspace, void *stream) {
  EWVIT_CHECK_ARG(x && dy && dw && workspace && dtype_ok(dtype), "dwconv3x3_bwd_weight: bad args");
  DwShape s = mk(N, H, W, C, stride, pad);
  if (int rc = check_shape(s, "dwconv3x3_bwd_weight")) return rc;
  bool row; int R; int64_t nslab;
  wgrad_plan(s, dtype, &row, &R, &nslab);
  const int slabs = (int)nslab;
  const int64_t npix = (int64_t)s.N * s.Ho * s.Wo;
  hipStream_t st = as_stream(stream);
  if (row) {
    const size_t lds = (size_t)(s.C / 8) * 72 * sizeof(float);
    if (s.stride == 1)
      hipLaunchKernelGGL(dw_wgrad_row_bf16_kernel<1>, dim3((unsigned)slabs), dim3(512), lds, st,
                         (const bf16_t *)x, (const bf16_t *)dy, workspace, s, R);
    else
      hipLaunchKernelGGL(dw_wgrad_row_bf16_kernel<2>, dim3((unsigned)slabs), dim3(512), lds, st,
                         (const bf16_t *)x, (const bf16_t *)dy, workspace, s, R);
  } else {
    dim3 grid((unsigned)slabs, (unsigned)((s.C + 63) / 64));
    if (dtype == EWVIT_BF16)
      hipLaunchKernelGGL(dw_bwd_weight_partial_kernel<EWVIT_BF16>, grid, dim3(256), 0, st, x, dy, workspace, s, npix);
    else
      hipLaunchKernelGGL(dw_bwd_weight_partial_kernel<EWVIT_F32>, grid, dim3(256), 0, st, x, dy, workspace, s, npix);
  }
  if (int rc = launch_status("dwconv3x3_bwd_weight")) return rc;
  const int64_t n = (int64_t)s.C * 9;
  hipLaunchKernelGGL(dw_bwd_weight_reduce_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, workspace,
                     dw, n, slabs, accumulate);
  return launch_status("dwconv3x3_bwd_weight reduce");
}
