// Squeeze-excitation and stochastic-depth residual passes of the EfficientNetV2-S
// MBConv blocks (torchvision SqueezeExcitation / StochasticDepth, reached from
// network/sfe.py:111-113), channels-last [N][HW][C], bf16 or f32.
//
//   squeeze   s0[n, c]  = mean_hw x                      (se_reduce, PROD = 0)
//   excite    y         = x * s[n, c]                     (se_scale, g = null)
//   backward  ds[n, c]  = sum_hw dy * x                   (se_reduce, PROD = 1)
//             dx        = dy * s[n, c] + g[n, c]          (se_scale; g = dsqueeze / HW)
//   residual  y         = r * scale[n] (+ x)              (scale_add: drop-path + skip)
//
// The squeeze MLP (C -> C/4 -> C on [N, C]) is tiny and runs as plain GEMMs on the
// host side; these kernels are the four HBM passes over the [N, HW, C] tensors
// (torch issues ~10 for the same block: mean, mul, two mul-backwards, the
// squeeze backward's expand and the autograd accumulation add).
// Reductions are deterministic: per-(split, n) partial slabs summed in a fixed order.
#include "common.h"

namespace ewvit {

template <int DT>
__device__ __forceinline__ void se_ld8(const void *p, int64_t i, float (&v)[8]) {
  if constexpr (DT == EWVIT_BF16) {
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
__device__ __forceinline__ void se_st8(void *p, int64_t i, const float (&v)[8]) {
  if constexpr (DT == EWVIT_BF16) {
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

struct SePlan {
  int C8, LC, R, cblocks, S;
  int rows_per_split;
};

// block = LC channel vectors x R row groups; grid (N * S, cblocks).  Narrow channel
// chunks (LC <= 32 vectors, R >= 8 row groups) give >= 2 blocks per frame and short
// per-thread row walks; the rows are split (S > 1, then a fold launch sums the
// slabs) only when a thread would otherwise walk more than 32 rows — never for the
// backbone's SE shapes (HW <= 196), which therefore take one launch.
static SePlan se_plan(int64_t N, int64_t HW, int64_t C) {
  SePlan p;
  p.C8 = (int)(C / 8);
  p.LC = p.C8 < 32 ? p.C8 : 32;
  p.R = 256 / p.LC;
  p.cblocks = (p.C8 + p.LC - 1) / p.LC;
  int64_t s = (HW + 32 * p.R - 1) / (32 * p.R);                 // <= 32 rows per thread
  if (N * p.cblocks * s < 256) {                                // fill the chip when rows allow
    int64_t want = (256 + N * p.cblocks - 1) / (N * p.cblocks);
    const int64_t maxs = HW / (8 * p.R);                        // >= 8 rows per thread
    if (want > maxs) want = maxs;
    if (want > s) s = want;
  }
  if (s < 1) s = 1;
  p.S = (int)s;
  p.rows_per_split = (int)((HW + s - 1) / s);
  return p;
}

// part[split][n][c] = sum over this split's rows of a (PROD=0) or a*b (PROD=1);
// with one split the block writes out[n][c] = scale * sum directly
template <int DT, int PROD>
__global__ __launch_bounds__(256) void se_reduce_kernel(const void *__restrict__ a, const void *__restrict__ b,
                                                        int HW, int C, int R, int LC, int S, int rps,
                                                        float *__restrict__ part, int N, float scale,
                                                        float *__restrict__ out) {
  __shared__ float sm[256 * 8];
  const int n = blockIdx.x / S, split = blockIdx.x % S;
  const int tid = threadIdx.x, rg = tid / LC, cl = tid % LC;
  const int c8 = blockIdx.y * LC + cl;
  const bool active = rg < R && c8 < (C >> 3);
  const int h0 = split * rps, h1 = h0 + rps < HW ? h0 + rps : HW;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (active) {
    const int64_t base = (int64_t)n * HW * C + c8 * 8;
    int h = h0 + rg;
    for (; h + 7 * R < h1; h += 8 * R) {     // 8 rows' loads in flight
      float va[8][8], vb[8][8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        se_ld8<DT>(a, base + (int64_t)(h + q * R) * C, va[q]);
        if (PROD) se_ld8<DT>(b, base + (int64_t)(h + q * R) * C, vb[q]);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = PROD ? fmaf(va[q][j], vb[q][j], acc[j]) : acc[j] + va[q][j];
    }
    for (; h < h1; h += R) {
      float va[8], vb[8];
      se_ld8<DT>(a, base + (int64_t)h * C, va);
      if (PROD) se_ld8<DT>(b, base + (int64_t)h * C, vb);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = PROD ? fmaf(va[j], vb[j], acc[j]) : acc[j] + va[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) sm[tid * 8 + j] = acc[j];
  __syncthreads();
  if (rg == 0 && active) {
    for (int g = 1; g < R; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += sm[(g * LC + cl) * 8 + j];
    if (S == 1) {
      float *dst = out + (int64_t)n * C + c8 * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[j] = acc[j] * scale;
    } else {
      float *dst = part + ((int64_t)split * N + n) * C + c8 * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[j] = acc[j];
    }
  }
}

// out[n][c] = scale * sum_split part[split][n][c]
__global__ __launch_bounds__(256) void se_fold_kernel(const float *__restrict__ part, int S, int64_t NC, float scale,
                                                      float *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= NC) return;
  float s = 0.f;
  for (int k = 0; k < S; ++k) s += part[(int64_t)k * NC + i];
  out[i] = s * scale;
}

// y = x * s[n, c] (+ g[n, c]); one 8-channel vector per thread
template <int DT>
__global__ __launch_bounds__(256) void se_scale_kernel(const void *__restrict__ x, const float *__restrict__ s,
                                                       const float *__restrict__ g, void *__restrict__ y,
                                                       int64_t nvec, int HW, int C) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nvec) return;
  const int C8 = C >> 3;
  const int64_t row = v / C8;
  const int c = (int)(v - row * C8) * 8;
  const int64_t n = row / HW;
  const float4 *sp = reinterpret_cast<const float4 *>(s + n * C + c);
  const float4 s0 = sp[0], s1 = sp[1];
  const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  float gv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (g) {
    const float4 *gp = reinterpret_cast<const float4 *>(g + n * C + c);
    const float4 g0 = gp[0], g1 = gp[1];
    gv[0] = g0.x; gv[1] = g0.y; gv[2] = g0.z; gv[3] = g0.w; gv[4] = g1.x; gv[5] = g1.y; gv[6] = g1.z; gv[7] = g1.w;
  }
  float vx[8];
  se_ld8<DT>(x, v * 8, vx);
#pragma unroll
  for (int j = 0; j < 8; ++j) vx[j] = fmaf(vx[j], sc[j], gv[j]);
  se_st8<DT>(y, v * 8, vx);
}

// y = r * scale[n] (+ x): StochasticDepth(mode='row') times its keep/(1-p) factor,
// plus the block's skip connection
template <int DT>
__global__ __launch_bounds__(256) void scale_add_kernel(const void *__restrict__ r, const void *__restrict__ x,
                                                        const float *__restrict__ scale, void *__restrict__ y,
                                                        int64_t nvec, int64_t row_vec) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nvec) return;
  const float sc = scale[v / row_vec];
  float vr[8], vx[8];
  se_ld8<DT>(r, v * 8, vr);
  if (x) se_ld8<DT>(x, v * 8, vx);
#pragma unroll
  for (int j = 0; j < 8; ++j) vr[j] = x ? fmaf(vr[j], sc, vx[j]) : vr[j] * sc;
  se_st8<DT>(y, v * 8, vr);
}

// StochasticDepth(row) drawn in-kernel: scale[n] = (u(n) < keep) / keep with u the
// counter hash of (seed, step counter, n) — every thread draws its row's value, the
// thread holding the row's first vector stores it for the backward pass
template <int DT>
__global__ __launch_bounds__(256) void scale_add_drop_kernel(const void *__restrict__ r, const void *__restrict__ x,
                                                             float keep, uint64_t seed,
                                                             const int64_t *__restrict__ seed_offset,
                                                             float *__restrict__ scale_out, void *__restrict__ y,
                                                             int64_t nvec, int64_t row_vec) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nvec) return;
  const int64_t n = v / row_vec;
  const float sc = uniform01(step_seed(seed, seed_offset), (uint64_t)n) < keep ? 1.f / keep : 0.f;
  if (v == n * row_vec) scale_out[n] = sc;
  float vr[8], vx[8];
  se_ld8<DT>(r, v * 8, vr);
  se_ld8<DT>(x, v * 8, vx);
#pragma unroll
  for (int j = 0; j < 8; ++j) vr[j] = fmaf(vr[j], sc, vx[j]);
  se_st8<DT>(y, v * 8, vr);
}

// ---------------------------------------------------------------- squeeze MLP
// s0 [N, C] -> h1 = W1 s0 + b1 [N, Csq] -> a1 = silu(h1) -> s = sigmoid(W2 a1 + b2) [N, C]
// (torchvision SqueezeExcitation fc1 / fc2 as 1x1 convs, fp32 like the reference).
// The vectors are tiny (N = 64 frames); what costs is load latency, so every kernel
// spreads a frame over many blocks and issues all of a thread's loads back to back.
// Reductions over c go through fixed-order partial slabs (deterministic).
//   F1 se_mlp_h1_part  grid (N, C/64):  part[n][cb][j] = sum_{c in cb} W1[j][c] s0[n][c]
//   F2 se_mlp_gate     grid (N, C/64):  h1 = b1 + sum_cb part; s = sigmoid(W2 silu(h1) + b2)
//   B1 se_mlp_dh_part  grid (N, C/64):  dz2 = ds s(1-s); part[n][cb][j] = sum_c W2[c][j] dz2
//   B2 se_mlp_g        grid (N, C/64):  dz1 = (sum_cb part) silu'(h1); g = W1^T dz1 / HW
//   B3 se_mlp_wgrad    64 dW1 / dW2 / db elements per block, the 4 waves on quarters of n
constexpr int SE_CB = 64;

// lanes = 64 consecutive channels of chunk cb, waves take outputs j = w, w+4, ...
__global__ __launch_bounds__(256) void se_mlp_h1_part_kernel(const float *__restrict__ s0,
                                                             const float *__restrict__ w1, int C, int Csq,
                                                             float *__restrict__ part) {
  const int n = blockIdx.x, cb = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = cb * SE_CB + lane;
  const float xv = c < C ? s0[(int64_t)n * C + c] : 0.f;
  float *pp = part + ((int64_t)n * gridDim.y + cb) * Csq;
  for (int j0 = w; j0 < Csq; j0 += 16) {
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = j0 + 4 * q;
      v[q] = (j < Csq && c < C) ? w1[(int64_t)j * C + c] * xv : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = wave_sum(v[q]);
      const int j = j0 + 4 * q;
      if (lane == 0 && j < Csq) pp[j] = v[q];
    }
  }
}

__device__ __forceinline__ float silu_f(float h) { return h * __builtin_amdgcn_rcpf(1.f + __expf(-h)); }
__device__ __forceinline__ float sigmoid_f(float z) { return __builtin_amdgcn_rcpf(1.f + __expf(-z)); }

// sum the nb partial rows of output j (up to 32 loads in flight per thread)
__device__ __forceinline__ float se_part_sum(const float *__restrict__ pp, int nb, int Csq, int j) {
  float acc = 0.f;
  for (int k0 = 0; k0 < nb; k0 += 8) {
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = k0 + q < nb ? pp[(int64_t)(k0 + q) * Csq + j] : 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) acc += v[q];
  }
  return acc;
}

// the pre-activations of a block's 64 gates: z[c] = b2[c] + sum_j W2[c][j] a[j] (a in LDS), lane
// = channel, the 4 waves on quarters of j, the quarters combined in a fixed order through red —
// every thread of the block returns its lane's z (one barrier inside)
__device__ __forceinline__ float se_gate64(const float *__restrict__ w2, const float *__restrict__ b2,
                                          const float *a, int C, int Csq, int c, float (*red)[64]) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int q = (Csq + 3) >> 2, ja = w * q, jb = ja + q < Csq ? ja + q : Csq;
  float acc0 = 0.f, acc1 = 0.f;
  if (c < C) {
    const float *row = w2 + (int64_t)c * Csq;
    int j = ja;
    for (; j + 8 <= jb; j += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = row[j + u];
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        acc0 = fmaf(v[u], a[j + u], acc0);
        acc1 = fmaf(v[u + 1], a[j + u + 1], acc1);
      }
    }
    for (; j < jb; ++j) acc0 = fmaf(row[j], a[j], acc0);
  }
  red[w][lane] = acc0 + acc1;
  __syncthreads();
  return ((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane])) + (b2 && c < C ? b2[c] : 0.f);
}

__global__ __launch_bounds__(256) void se_mlp_gate_kernel(const float *__restrict__ part, int nb,
                                                          const float *__restrict__ b1,
                                                          const float *__restrict__ w2,
                                                          const float *__restrict__ b2, int C, int Csq,
                                                          float *__restrict__ h1_out, float *__restrict__ s_out) {
  extern __shared__ float a1[];
  __shared__ float red[4][64];
  const int n = blockIdx.x, tid = threadIdx.x;
  const float *pp = part + (int64_t)n * nb * Csq;
  for (int j = tid; j < Csq; j += 256) {
    const float h = se_part_sum(pp, nb, Csq, j) + (b1 ? b1[j] : 0.f);
    a1[j] = silu_f(h);
    if (blockIdx.y == 0) h1_out[(int64_t)n * Csq + j] = h;
  }
  __syncthreads();
  const int c = blockIdx.y * 64 + (tid & 63);
  const float z = se_gate64(w2, b2, a1, C, Csq, c, red);
  if (tid < 64 && c < C) s_out[(int64_t)n * C + c] = sigmoid_f(z);
}

// F2 + the excite pass in one launch: block (n, 64-channel chunk) forms the frame's hidden
// vector and its chunk's gates exactly as se_mlp_gate_kernel does, then scales the chunk's
// HW rows of x (y = x * s, as se_scale_kernel) — 8 channel vectors x 32 row groups, the first
// 2 rows of every thread loaded before the gate is known (they do not depend on it)
template <int DT>
__global__ __launch_bounds__(256) void se_gate_scale_kernel(const float *__restrict__ part, int nb,
                                                            const float *__restrict__ b1,
                                                            const float *__restrict__ w2,
                                                            const float *__restrict__ b2, int C, int Csq,
                                                            float *__restrict__ h1_out, float *__restrict__ s_out,
                                                            const void *__restrict__ x, void *__restrict__ y, int HW) {
  extern __shared__ float gsm[];
  __shared__ float red[4][64];
  float *a1 = gsm, *sv = gsm + ((Csq + 3) & ~3);
  const int n = blockIdx.x, tid = threadIdx.x;
  const int cv = tid & 7, rg = tid >> 3;             // 8 channel vectors x 32 row groups
  const int c0 = blockIdx.y * 64 + cv * 8;
  const bool active = c0 < C;
  const int64_t base = (int64_t)n * HW * C + c0;
  constexpr int PF = 2, RS = 32;
  float pre[PF][8];
#pragma unroll
  for (int q = 0; q < PF; ++q) {
    const int r = rg + RS * q;
    if (active && r < HW) se_ld8<DT>(x, base + (int64_t)r * C, pre[q]);
  }
  const float *pp = part + (int64_t)n * nb * Csq;
  for (int j = tid; j < Csq; j += 256) {
    const float h = se_part_sum(pp, nb, Csq, j) + (b1 ? b1[j] : 0.f);
    a1[j] = silu_f(h);
    if (blockIdx.y == 0) h1_out[(int64_t)n * Csq + j] = h;
  }
  __syncthreads();
  const int c = blockIdx.y * 64 + (tid & 63);
  const float z = se_gate64(w2, b2, a1, C, Csq, c, red);
  if (tid < 64) {
    const float sg = sigmoid_f(z);
    if (c < C) s_out[(int64_t)n * C + c] = sg;
    sv[tid] = sg;
  }
  __syncthreads();
  if (!active) return;
  float sc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sc[j] = sv[cv * 8 + j];
#pragma unroll
  for (int q = 0; q < PF; ++q) {
    const int r = rg + RS * q;
    if (r < HW) {
#pragma unroll
      for (int j = 0; j < 8; ++j) pre[q][j] = fmaf(pre[q][j], sc[j], 0.f);
      se_st8<DT>(y, base + (int64_t)r * C, pre[q]);
    }
  }
  for (int r0 = rg + RS * PF; r0 < HW; r0 += RS * PF) {
    float v[PF][8];
#pragma unroll
    for (int q = 0; q < PF; ++q)
      if (r0 + RS * q < HW) se_ld8<DT>(x, base + (int64_t)(r0 + RS * q) * C, v[q]);
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      if (r0 + RS * q < HW) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[q][j] = fmaf(v[q][j], sc[j], 0.f);
        se_st8<DT>(y, base + (int64_t)(r0 + RS * q) * C, v[q]);
      }
    }
  }
}

__global__ __launch_bounds__(256) void se_mlp_dh_part_kernel(const float *__restrict__ ds,
                                                             const float *__restrict__ s,
                                                             const float *__restrict__ w2, int C, int Csq,
                                                             float *__restrict__ dz2_out, float *__restrict__ part) {
  const int n = blockIdx.x, cb = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = cb * SE_CB + lane;
  float d = 0.f;
  if (c < C) {
    const float sv = s[(int64_t)n * C + c];
    d = ds[(int64_t)n * C + c] * sv * (1.f - sv);
    if (w == 0) dz2_out[(int64_t)n * C + c] = d;
  }
  float *pp = part + ((int64_t)n * gridDim.y + cb) * Csq;
  for (int j0 = w; j0 < Csq; j0 += 16) {
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = j0 + 4 * q;
      v[q] = (j < Csq && c < C) ? w2[(int64_t)c * Csq + j] * d : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = wave_sum(v[q]);
      const int j = j0 + 4 * q;
      if (lane == 0 && j < Csq) pp[j] = v[q];
    }
  }
}

// block (n, 64-channel chunk): dz1 for the frame (every block of the frame forms it), then
// g[c] = sum_j W1[j][c] dz1[j] / HW with the 4 waves on quarters of j, combined in order
__global__ __launch_bounds__(256) void se_mlp_g_kernel(const float *__restrict__ part, int nb,
                                                       const float *__restrict__ h1,
                                                       const float *__restrict__ w1, int C, int Csq, float inv_hw,
                                                       float *__restrict__ dz1_out, float *__restrict__ g_out) {
  extern __shared__ float dz1[];
  __shared__ float red[4][64];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float *pp = part + (int64_t)n * nb * Csq;
  for (int j = tid; j < Csq; j += 256) {
    const float dh = se_part_sum(pp, nb, Csq, j);
    const float h = h1[(int64_t)n * Csq + j];
    const float sg = sigmoid_f(h);
    const float d = dh * sg * (1.f + h * (1.f - sg));
    dz1[j] = d;
    if (blockIdx.y == 0) dz1_out[(int64_t)n * Csq + j] = d;
  }
  __syncthreads();
  const int c = blockIdx.y * 64 + lane;
  const int q = (Csq + 3) >> 2, ja = w * q, jb = ja + q < Csq ? ja + q : Csq;
  float acc0 = 0.f, acc1 = 0.f;
  if (c < C) {
    int j = ja;
    for (; j + 8 <= jb; j += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = w1[(int64_t)(j + u) * C + c];
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        acc0 = fmaf(v[u], dz1[j + u], acc0);
        acc1 = fmaf(v[u + 1], dz1[j + u + 1], acc1);
      }
    }
    for (; j < jb; ++j) acc0 = fmaf(w1[(int64_t)j * C + c], dz1[j], acc0);
  }
  red[w][lane] = acc0 + acc1;
  __syncthreads();
  if (w == 0 && c < C) g_out[(int64_t)n * C + c] = ((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane])) * inv_hw;
}

// the BN's two channel sums from the per-frame sums (see se_sq_dh_bn_part_kernel): out[c] =
// sum g', out[C + c] = sum g' xhat — one partial row for bn_bwd_dx_kernel.  Lanes over channels,
// the 4 waves over quarters of the frames, combined in a fixed order (deterministic).
// (Extra blocks of se_mlp_wgrad_kernel: no launch of its own.)
__device__ __forceinline__ void se_bn_sums_block(int bx, const float *__restrict__ bnsum, const float *__restrict__ s,
                                                 const float *__restrict__ g, int N, int C, float *__restrict__ out,
                                                 float (*red)[64], float *__restrict__ dbeta = nullptr,
                                                 float *__restrict__ dgamma = nullptr) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k = bx * 64 + lane;                  // 0 .. 2C - 1
  const int which = k >= C, c = which ? k - C : k;
  const int q = (N + 3) >> 2, na = w * q, nb = na + q < N ? na + q : N;
  float acc0 = 0.f, acc1 = 0.f;
  if (k < 2 * C) {
    const float *pa = bnsum + (int64_t)(which ? 2 : 0) * N * C + c;    // A or Q
    const float *pb = bnsum + (int64_t)(which ? 3 : 1) * N * C + c;    // B or D
    for (int n0 = na; n0 < nb; n0 += 4) {
      float vs[4], vg[4], va[4], vb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = n0 + u < nb;
        const int64_t o = (int64_t)(ok ? n0 + u : na) * C;
        vs[u] = ok ? s[o + c] : 0.f; vg[u] = ok ? g[o + c] : 0.f;
        va[u] = pa[o]; vb[u] = pb[o];
      }
#pragma unroll
      for (int u = 0; u < 4; u += 2) {
        acc0 = fmaf(vg[u], vb[u], fmaf(vs[u], va[u], acc0));
        acc1 = fmaf(vg[u + 1], vb[u + 1], fmaf(vs[u + 1], va[u + 1], acc1));
      }
    }
  }
  red[w][lane] = acc0 + acc1;
  __syncthreads();
  if (w == 0 && k < 2 * C) {
    const float v = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    out[k] = v;
    // the BN's parameter gradients are these sums (dbeta = sum g', dgamma = sum g' xhat): written
    // here when the dx pass is folded into the depthwise backward (ewvit_bn_se_bwd, dx NULL)
    float *d = which ? dgamma : dbeta;
    if (d) d[c] = v;
  }
}



// dW2[c][j] = sum_n dz2[n][c] silu(h1[n][j]),  db2[c] = sum_n dz2[n][c]
// dW1[j][c] = sum_n dz1[n][j] s0[n][c],        db1[j] = sum_n dz1[n][j]
// block: 64 consecutive outputs (lanes) x 4 waves on quarters of the frames, the quarters
// combined in a fixed order through LDS (deterministic); a thread's loads of its quarter are
// issued 8 at a time
__global__ __launch_bounds__(256) void se_mlp_wgrad_kernel(const float *__restrict__ dz2,
                                                           const float *__restrict__ dz1,
                                                           const float *__restrict__ h1,
                                                           const float *__restrict__ s0, int N, int C, int Csq,
                                                           float *__restrict__ dw1, float *__restrict__ db1,
                                                           float *__restrict__ dw2, float *__restrict__ db2,
                                                           const float *__restrict__ bnsum = nullptr,
                                                           const float *__restrict__ exc = nullptr,
                                                           const float *__restrict__ gsq = nullptr,
                                                           float *__restrict__ bnout = nullptr, int nwb = 0,
                                                           float *__restrict__ bn_dbeta = nullptr,
                                                           float *__restrict__ bn_dgamma = nullptr) {
  __shared__ float red[4][64];
  if (bnsum && (int)blockIdx.x >= nwb) {         // the BN sums' blocks (ewvit_bn_se_bwd)
    se_bn_sums_block((int)blockIdx.x - nwb, bnsum, exc, gsq, N, C, bnout, red, bn_dbeta, bn_dgamma);
    return;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  const int64_t P = (int64_t)C * Csq;
  const float *pa = nullptr, *pb = nullptr;
  int64_t sa = 0, sb = 0;
  bool silu_b = false;
  float *dst = nullptr;
  if (i < P) {                    // dW2[c][j], j fastest
    const int c = (int)(i / Csq), j = (int)(i % Csq);
    pa = dz2 + c; sa = C; pb = h1 + j; sb = Csq; silu_b = true; dst = dw2 + i;
  } else if (i < 2 * P) {         // dW1[j][c], c fastest
    const int64_t k = i - P;
    const int j = (int)(k / C), c = (int)(k % C);
    pa = dz1 + j; sa = Csq; pb = s0 + c; sb = C; dst = dw1 + k;
  } else if (i < 2 * P + C) {
    const int c = (int)(i - 2 * P);
    pa = dz2 + c; sa = C; dst = db2 ? db2 + c : nullptr;
  } else if (i < 2 * P + C + Csq) {
    const int j = (int)(i - 2 * P - C);
    pa = dz1 + j; sa = Csq; dst = db1 ? db1 + j : nullptr;
  }
  const int q = (N + 3) >> 2, na = w * q, nb = na + q < N ? na + q : N;
  float acc0 = 0.f, acc1 = 0.f;
  if (dst) {
    for (int n0 = na; n0 < nb; n0 += 8) {
      float va[8], vb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool ok = n0 + u < nb;
        va[u] = ok ? pa[(int64_t)(n0 + u) * sa] : 0.f;
        vb[u] = ok ? (pb ? pb[(int64_t)(n0 + u) * sb] : 1.f) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        const float b0 = silu_b ? silu_f(vb[u]) : vb[u], b1v = silu_b ? silu_f(vb[u + 1]) : vb[u + 1];
        acc0 = fmaf(va[u], b0, acc0);
        acc1 = fmaf(va[u + 1], b1v, acc1);
      }
    }
  }
  red[w][lane] = acc0 + acc1;
  __syncthreads();
  if (w == 0 && dst) *dst = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// The squeeze folded into the MLP's first kernel: block (n, chunk) reduces its 64
// channels of frame n over the HW rows itself (8 channel vectors x 32 row groups, 4
// rows' loads in flight, fixed-order tree) instead of reading a vector a separate
// launch produced.  PROD = 0: mean_hw a (the forward squeeze s0, written out for the
// backward); PROD = 1: sum_hw a * b (the backward's ds = sum dy * x).
template <int DT, int PROD>
__device__ __forceinline__ float se_chunk_squeeze(const void *__restrict__ a, const void *__restrict__ b, int n,
                                                  int cb, int HW, int C, float scale, float *sm) {
  const int tid = threadIdx.x, cv = tid & 7, rg = tid >> 3;
  const int c = cb * SE_CB + cv * 8;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (c < C) {
    const int64_t base = (int64_t)n * HW * C + c;
    int h = rg;
    for (; h + 96 < HW; h += 128) {
      float va[4][8], vb[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        se_ld8<DT>(a, base + (int64_t)(h + 32 * q) * C, va[q]);
        if (PROD) se_ld8<DT>(b, base + (int64_t)(h + 32 * q) * C, vb[q]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = PROD ? fmaf(va[q][j], vb[q][j], acc[j]) : acc[j] + va[q][j];
    }
    for (; h < HW; h += 32) {
      float va[8], vb[8];
      se_ld8<DT>(a, base + (int64_t)h * C, va);
      if (PROD) se_ld8<DT>(b, base + (int64_t)h * C, vb);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = PROD ? fmaf(va[j], vb[j], acc[j]) : acc[j] + va[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) sm[j * 256 + tid] = acc[j];
  __syncthreads();
  for (int st = 16; st >= 1; st >>= 1) {
    if (rg < st)
#pragma unroll
      for (int j = 0; j < 8; ++j) sm[j * 256 + tid] += sm[j * 256 + tid + st * 8];
    __syncthreads();
  }
  // lane l of every wave: channel cb*64 + l = vector l>>3, element l&7
  const int l = tid & 63;
  return sm[(l & 7) * 256 + (l >> 3)] * scale;
}

template <int DT>
__global__ __launch_bounds__(256) void se_sq_h1_part_kernel(const void *__restrict__ x, int HW, float inv_hw,
                                                            const float *__restrict__ w1, int C, int Csq,
                                                            float *__restrict__ s0_out, float *__restrict__ part) {
  __shared__ float sm[8 * 256];
  const int n = blockIdx.x, cb = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = cb * SE_CB + lane;
  const float sq = se_chunk_squeeze<DT, 0>(x, nullptr, n, cb, HW, C, inv_hw, sm);
  const float xv = c < C ? sq : 0.f;
  if (w == 0 && c < C) s0_out[(int64_t)n * C + c] = xv;
  float *pp = part + ((int64_t)n * gridDim.y + cb) * Csq;
  for (int j0 = w; j0 < Csq; j0 += 16) {
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = j0 + 4 * q;
      v[q] = (j < Csq && c < C) ? w1[(int64_t)j * C + c] * xv : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = wave_sum(v[q]);
      const int j = j0 + 4 * q;
      if (lane == 0 && j < Csq) pp[j] = v[q];
    }
  }
}

template <int DT>
__global__ __launch_bounds__(256) void se_sq_dh_part_kernel(const void *__restrict__ dy, const void *__restrict__ x,
                                                            int HW, const float *__restrict__ s,
                                                            const float *__restrict__ w2, int C, int Csq,
                                                            float *__restrict__ dz2_out, float *__restrict__ part) {
  __shared__ float sm[8 * 256];
  const int n = blockIdx.x, cb = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = cb * SE_CB + lane;
  const float dsv = se_chunk_squeeze<DT, 1>(dy, x, n, cb, HW, C, 1.f, sm);
  float d = 0.f;
  if (c < C) {
    const float sv = s[(int64_t)n * C + c];
    d = dsv * sv * (1.f - sv);
    if (w == 0) dz2_out[(int64_t)n * C + c] = d;
  }
  // part[j] = sum_c w2[c][j] * d[c] over the chunk's channels: w2 is [C][Csq], so lanes run
  // over j (coalesced rows of w2) and the 4 waves over interleaved channels, d from LDS
  __shared__ float dsh[SE_CB];
  __shared__ float red[4][64];
  if (w == 0) dsh[lane] = d;
  __syncthreads();
  float *pp = part + ((int64_t)n * gridDim.y + cb) * Csq;
  const int c0 = cb * SE_CB;
  const int nc = C - c0 < SE_CB ? C - c0 : SE_CB;
  for (int j0 = 0; j0 < Csq; j0 += 64) {
    const int j = j0 + lane;
    float acc = 0.f;
    if (j < Csq) {
      // the wave's 16 channels k = w, w + 4, .. (nc <= SE_CB = 64): all 16 loads issued before
      // the first FMA (a load-FMA loop waited out each load's latency: 16 serial L2 round
      // trips), then the FMAs in the same k order (the same bits)
      // (branch-free: past the chunk's nc channels the load repeats channel nc - 1 and meets
      // dsh[k] = 0 — d is 0 for channels >= C — so the FMA adds an exact zero)
      const float *wr = w2 + (int64_t)c0 * Csq + j;
      float wv[SE_CB / 4];
#pragma unroll
      for (int u = 0; u < SE_CB / 4; ++u) {
        const int k = w + 4 * u;
        wv[u] = wr[(int64_t)(k < nc ? k : nc - 1) * Csq];
      }
#pragma unroll
      for (int u = 0; u < SE_CB / 4; ++u) acc = fmaf(wv[u], dsh[w + 4 * u], acc);
    }
    red[w][lane] = acc;
    __syncthreads();
    if (w == 0 && j < Csq) pp[j] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    __syncthreads();
  }
}

// the BatchNorm(+act) backward's reduction folded into the SE backward's squeeze pass
// (ewvit_bn_se_bwd): the BN's output gradient is dy*s[n][c] + g[n][c] (s the excitation, g the
// squeeze term the MLP backward forms later), so its two channel sums split per frame as
//   sum g'      = sum_n s[n][c] A[n][c] + g[n][c] B[n][c]
//   sum g' xhat = sum_n s[n][c] Q[n][c] + g[n][c] D[n][c]
// with g' = (dy s + g) act'(xhat gamma + beta) and the per-frame sums
//   A = sum_hw dy t,  B = sum_hw t,  Q = sum_hw dy t xhat,  D = sum_hw t xhat,  t = act'(.).
// This pass (block: frame n, 64-channel chunk) forms them beside ds = sum_hw dy * a while it
// streams dy and a anyway; se_mlp_wgrad_kernel, which already sums over the frames, adds the
// two channel sums; the BN's own reduction pass over dy and z never runs.
template <int ACT>
__device__ __forceinline__ float se_act_grad(float z) {   // = batchnorm.hip act_grad
  if (ACT == 1) return z > 0.f ? 1.f : 0.f;
  if (ACT == 2) {
    const float s = __builtin_amdgcn_rcpf(1.f + __expf(-z));
    return s * (1.f + z * (1.f - s));
  }
  return 1.f;
}

template <int V> struct se_ic { static constexpr int value = V; };
// raw 8-channel vectors (bf16: one 16-B load, unpacked at use) for the batched row walks
template <int DT> struct SeRaw { uint4 a, b; };
template <int DT>
__device__ __forceinline__ SeRaw<DT> se_ldraw(const void *p, int64_t i) {
  SeRaw<DT> r;
  if constexpr (DT == EWVIT_BF16) {
    r.a = *reinterpret_cast<const uint4 *>(reinterpret_cast<const bf16_t *>(p) + i);
    r.b = r.a;
  } else {
    const uint4 *q = reinterpret_cast<const uint4 *>(reinterpret_cast<const float *>(p) + i);
    r.a = q[0];
    r.b = q[1];
  }
  return r;
}
template <int DT>
__device__ __forceinline__ void se_unpack(const SeRaw<DT> &r, float (&v)[8]) {
  if constexpr (DT == EWVIT_BF16) {
    const unsigned w[4] = {r.a.x, r.a.y, r.a.z, r.a.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(w[j] << 16);
      v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
    }
  } else {
    const unsigned w[8] = {r.a.x, r.a.y, r.a.z, r.a.w, r.b.x, r.b.y, r.b.z, r.b.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = __uint_as_float(w[j]);
  }
}
__device__ __forceinline__ void ld8f(const float *p, float (&v)[8]) {
  const float4 a = reinterpret_cast<const float4 *>(p)[0], b = reinterpret_cast<const float4 *>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// v + v[lane ^ 8], v + v[lane ^ 16], v + v[lane ^ 32] (fp addition commutes: both lanes
// of a pair get the same bits)
__device__ __forceinline__ float xsum8(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
}
__device__ __forceinline__ float xsum16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <int DT, int ACT>
__global__ __launch_bounds__(256) void se_sq_dh_bn_part_kernel(const void *__restrict__ dy, const void *__restrict__ x,
                                                               const void *__restrict__ z, int HW,
                                                               const float *__restrict__ s,
                                                               const float *__restrict__ w2, int C, int Csq,
                                                               const float *__restrict__ mean,
                                                               const float *__restrict__ invstd,
                                                               const float *__restrict__ gamma,
                                                               const float *__restrict__ beta,
                                                               float *__restrict__ dz2_out, float *__restrict__ part,
                                                               float *__restrict__ bnsum, int N) {
  __shared__ float wred[4][5][SE_CB];
  const int n = blockIdx.x, cb = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = cb * SE_CB + lane;
  const int c0 = cb * SE_CB;
  const int nc = C - c0 < SE_CB ? C - c0 : SE_CB;
  {
    const int cv = tid & 7, rg = tid >> 3;
    const int cc = cb * SE_CB + cv * 8;
    float acc[5][8];
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
    if (cc < C) {
      float mu[8], iv[8], ga[8], be[8];
      ld8f(mean + cc, mu);
      ld8f(invstd + cc, iv);
      if (gamma) ld8f(gamma + cc, ga);
      else
#pragma unroll
        for (int j = 0; j < 8; ++j) ga[j] = 1.f;
      if (beta) ld8f(beta + cc, be);
      else
#pragma unroll
        for (int j = 0; j < 8; ++j) be[j] = 0.f;
      const int64_t base = (int64_t)n * HW * C + cc;
      auto use = [&](const SeRaw<DT> &rd, const SeRaw<DT> &ra, const SeRaw<DT> &rz) {
        float vd[8], va[8], vz[8];
        se_unpack<DT>(rd, vd);
        se_unpack<DT>(ra, va);
        se_unpack<DT>(rz, vz);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          acc[0][j] = fmaf(vd[j], va[j], acc[0][j]);
          const float xh = (vz[j] - mu[j]) * iv[j];
          const float t = ACT ? se_act_grad<ACT>(fmaf(xh, ga[j], be[j])) : 1.f;
          const float dt = vd[j] * t;
          acc[1][j] += dt;
          acc[2][j] += t;
          acc[3][j] = fmaf(dt, xh, acc[3][j]);
          acc[4][j] = fmaf(t, xh, acc[4][j]);
        }
      };
      // NB rows' 3 NB loads issued before any is used (the sched_barrier keeps hipcc from
      // sinking them into the uses, where each would wait out its own latency)
      auto batch = [&](int h0, auto NBc) {
        constexpr int NB = decltype(NBc)::value;
        SeRaw<DT> rd[NB], ra[NB], rz[NB];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const int64_t o = base + (int64_t)(h0 + 32 * q) * C;
          rd[q] = se_ldraw<DT>(dy, o);
          ra[q] = se_ldraw<DT>(x, o);
          rz[q] = se_ldraw<DT>(z, o);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < NB; ++q) use(rd[q], ra[q], rz[q]);
      };
      int h = rg;
      for (; h + 32 < HW; h += 64) batch(h, se_ic<2>{});
      if (h < HW) batch(h, se_ic<1>{});
    }
    // the wave's 8 row groups (lanes cv, cv + 8, .., cv + 56) summed in registers: xor 8 by DPP
    // row_ror:8, xor 16 / 32 by gfx950's v_permlane16/32_swap (no LDS traffic — an LDS tree over
    // 40 values per thread was LDS-bandwidth bound), then the 4 waves through LDS in a fixed order
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[k][j] = xsum32(xsum16(xsum8(acc[k][j])));
    if (lane < 8)
#pragma unroll
      for (int k = 0; k < 5; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) wred[w][k][lane * 8 + j] = acc[k][j];
  }
  __syncthreads();
  float tot[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) tot[k] = (wred[0][k][lane] + wred[1][k][lane]) + (wred[2][k][lane] + wred[3][k][lane]);
  const float dsv = tot[0];
  if (w == 0 && c < C) {
#pragma unroll
    for (int k = 0; k < 4; ++k) bnsum[((int64_t)k * N + n) * C + c] = tot[k + 1];
  }
  float d = 0.f;
  if (c < C) {
    const float sv = s[(int64_t)n * C + c];
    d = dsv * sv * (1.f - sv);
    if (w == 0) dz2_out[(int64_t)n * C + c] = d;
  }
  __shared__ float dsh[SE_CB];
  __shared__ float red[4][64];
  if (w == 0) dsh[lane] = d;
  __syncthreads();
  float *pp = part + ((int64_t)n * gridDim.y + cb) * Csq;
  for (int j0 = 0; j0 < Csq; j0 += 64) {     // as se_sq_dh_part_kernel
    const int j = j0 + lane;
    float acc = 0.f;
    if (j < Csq) {
      float wv[SE_CB / 4];
      const float *wr = w2 + (int64_t)c0 * Csq + j;
#pragma unroll
      for (int u = 0; u < SE_CB / 4; ++u) {
        const int k = w + 4 * u;
        wv[u] = wr[(int64_t)(k < nc ? k : nc - 1) * Csq];
      }
#pragma unroll
      for (int u = 0; u < SE_CB / 4; ++u) acc = fmaf(wv[u], dsh[w + 4 * u], acc);
    }
    red[w][lane] = acc;
    __syncthreads();
    if (w == 0 && j < Csq) pp[j] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    __syncthreads();
  }
}

// bn_bwd_dx_kernel<DT, ACT, 2> over one partial row (batchnorm.hip)
int bn_bwd_dx_se_launch(const void *dy, const void *x, void *dx, int dtype, int64_t M, int64_t C, const float *gamma,
                        const float *beta, const float *save_mean, const float *save_invstd, int act, float *dgamma,
                        float *dbeta, const float *se_s, const float *se_g, int64_t HW, const float *part, int nrc,
                        hipStream_t s);

}  // namespace ewvit

using namespace ewvit;

static int se_check(int dtype, int64_t N, int64_t HW, int64_t C, const char *nm) {
  EWVIT_CHECK_ARG(dtype_ok(dtype), "%s: dtype %d", nm, dtype);
  EWVIT_CHECK_ARG(N > 0 && HW > 0 && C > 0 && C % 8 == 0, "%s: N=%lld HW=%lld C=%lld (C %% 8 == 0)", nm,
                  (long long)N, (long long)HW, (long long)C);
  return 0;
}

extern "C" int64_t ewvit_se_reduce_workspace(int64_t N, int64_t HW, int64_t C) {
  const SePlan p = se_plan(N, HW, C);
  return (int64_t)p.S * N * C * (int64_t)sizeof(float);
}

extern "C" int ewvit_se_reduce(const void *a, const void *b, int dtype, int64_t N, int64_t HW, int64_t C,
                               float scale, float *out, float *workspace, void *stream) {
  if (int rc = se_check(dtype, N, HW, C, "se_reduce")) return rc;
  EWVIT_CHECK_ARG(a && out && workspace, "se_reduce: null pointer");
  const SePlan p = se_plan(N, HW, C);
  hipStream_t s = as_stream(stream);
  dim3 grid((unsigned)(N * p.S), (unsigned)p.cblocks);
#define SE_RED(DTV, PV)                                                                                        \
  hipLaunchKernelGGL((se_reduce_kernel<DTV, PV>), grid, dim3(256), 0, s, a, b, (int)HW, (int)C, p.R, p.LC, p.S, \
                     p.rows_per_split, workspace, (int)N, scale, out)
  if (dtype == EWVIT_BF16) { if (b) SE_RED(EWVIT_BF16, 1); else SE_RED(EWVIT_BF16, 0); }
  else { if (b) SE_RED(EWVIT_F32, 1); else SE_RED(EWVIT_F32, 0); }
#undef SE_RED
  if (p.S > 1) {
    const int64_t NC = N * C;
    hipLaunchKernelGGL(se_fold_kernel, dim3((unsigned)((NC + 255) / 256)), dim3(256), 0, s, workspace, p.S, NC,
                       scale, out);
  }
  return launch_status("se_reduce");
}

extern "C" int ewvit_se_scale(const void *x, int dtype, const float *s, const float *g, void *y, int64_t N,
                              int64_t HW, int64_t C, void *stream) {
  if (int rc = se_check(dtype, N, HW, C, "se_scale")) return rc;
  EWVIT_CHECK_ARG(x && s && y, "se_scale: null pointer");
  const int64_t nvec = N * HW * C / 8;
  dim3 grid((unsigned)((nvec + 255) / 256));
  if (dtype == EWVIT_BF16)
    hipLaunchKernelGGL(se_scale_kernel<EWVIT_BF16>, grid, dim3(256), 0, as_stream(stream), x, s, g, y, nvec,
                       (int)HW, (int)C);
  else
    hipLaunchKernelGGL(se_scale_kernel<EWVIT_F32>, grid, dim3(256), 0, as_stream(stream), x, s, g, y, nvec,
                       (int)HW, (int)C);
  return launch_status("se_scale");
}

extern "C" int ewvit_scale_add(const void *r, const void *x, int dtype, const float *scale, void *y, int64_t N,
                               int64_t row_elems, void *stream) {
  EWVIT_CHECK_ARG(dtype_ok(dtype), "scale_add: dtype %d", dtype);
  EWVIT_CHECK_ARG(r && scale && y && N > 0 && row_elems > 0 && row_elems % 8 == 0,
                  "scale_add: bad args (row_elems %% 8 == 0)");
  const int64_t nvec = N * row_elems / 8;
  dim3 grid((unsigned)((nvec + 255) / 256));
  if (dtype == EWVIT_BF16)
    hipLaunchKernelGGL(scale_add_kernel<EWVIT_BF16>, grid, dim3(256), 0, as_stream(stream), r, x, scale, y, nvec,
                       row_elems / 8);
  else
    hipLaunchKernelGGL(scale_add_kernel<EWVIT_F32>, grid, dim3(256), 0, as_stream(stream), r, x, scale, y, nvec,
                       row_elems / 8);
  return launch_status("scale_add");
}

extern "C" int ewvit_scale_add_drop(const void *r, const void *x, int dtype, float keep_prob, uint64_t seed,
                                    const int64_t *seed_offset, float *scale_out, void *y, int64_t N,
                                    int64_t row_elems, void *stream) {
  EWVIT_CHECK_ARG(dtype_ok(dtype), "scale_add_drop: dtype %d", dtype);
  EWVIT_CHECK_ARG(r && x && scale_out && y && N > 0 && row_elems > 0 && row_elems % 8 == 0,
                  "scale_add_drop: bad args (row_elems %% 8 == 0)");
  EWVIT_CHECK_ARG(keep_prob > 0.f && keep_prob <= 1.f, "scale_add_drop: keep_prob %g", (double)keep_prob);
  const int64_t nvec = N * row_elems / 8;
  dim3 grid((unsigned)((nvec + 255) / 256));
  if (dtype == EWVIT_BF16)
    hipLaunchKernelGGL(scale_add_drop_kernel<EWVIT_BF16>, grid, dim3(256), 0, as_stream(stream), r, x, keep_prob,
                       seed, seed_offset, scale_out, y, nvec, row_elems / 8);
  else
    hipLaunchKernelGGL(scale_add_drop_kernel<EWVIT_F32>, grid, dim3(256), 0, as_stream(stream), r, x, keep_prob,
                       seed, seed_offset, scale_out, y, nvec, row_elems / 8);
  return launch_status("scale_add_drop");
}

static int se_mlp_check(int64_t N, int64_t C, int64_t Csq, const char *nm) {
  EWVIT_CHECK_ARG(N > 0 && C > 0 && Csq > 0 && C <= 65535 * 64 && Csq <= 8192, "%s: N=%lld C=%lld Csq=%lld", nm,
                  (long long)N, (long long)C, (long long)Csq);
  return 0;
}

static int se_nb(int64_t C) { return (int)((C + SE_CB - 1) / SE_CB); }

extern "C" int64_t ewvit_se_mlp_fwd_workspace(int64_t N, int64_t C, int64_t Csq) {
  return N * se_nb(C) * Csq * (int64_t)sizeof(float);
}

extern "C" int ewvit_se_mlp_fwd(const float *s0, const float *w1, const float *b1, const float *w2, const float *b2,
                                float *h1, float *s, int64_t N, int64_t C, int64_t Csq, float *workspace,
                                void *stream) {
  if (int rc = se_mlp_check(N, C, Csq, "se_mlp_fwd")) return rc;
  EWVIT_CHECK_ARG(s0 && w1 && w2 && h1 && s && workspace, "se_mlp_fwd: null pointer");
  hipStream_t st = as_stream(stream);
  const int nb = se_nb(C);
  hipLaunchKernelGGL(se_mlp_h1_part_kernel, dim3((unsigned)N, (unsigned)nb), dim3(256), 0, st, s0, w1, (int)C,
                     (int)Csq, workspace);
  hipLaunchKernelGGL(se_mlp_gate_kernel, dim3((unsigned)N, (unsigned)((C + 63) / 64)), dim3(256),
                     (size_t)Csq * sizeof(float), st, workspace, nb, b1, w2, b2, (int)C, (int)Csq, h1, s);
  return launch_status("se_mlp_fwd");
}

extern "C" int64_t ewvit_se_mlp_bwd_workspace(int64_t N, int64_t C, int64_t Csq) {
  return N * (C + Csq + se_nb(C) * Csq) * (int64_t)sizeof(float);
}

extern "C" int ewvit_se_mlp_bwd(const float *ds, const float *s, const float *h1, const float *s0, const float *w1,
                                const float *w2, float inv_hw, float *g, float *dw1, float *db1, float *dw2,
                                float *db2, int64_t N, int64_t C, int64_t Csq, float *workspace, void *stream) {
  if (int rc = se_mlp_check(N, C, Csq, "se_mlp_bwd")) return rc;
  EWVIT_CHECK_ARG(ds && s && h1 && s0 && w1 && w2 && g && dw1 && dw2 && workspace, "se_mlp_bwd: null pointer");
  hipStream_t st = as_stream(stream);
  const int nb = se_nb(C);
  float *dz2 = workspace, *dz1 = workspace + N * C, *part = dz1 + N * Csq;
  hipLaunchKernelGGL(se_mlp_dh_part_kernel, dim3((unsigned)N, (unsigned)nb), dim3(256), 0, st, ds, s, w2, (int)C,
                     (int)Csq, dz2, part);
  hipLaunchKernelGGL(se_mlp_g_kernel, dim3((unsigned)N, (unsigned)((C + 63) / 64)), dim3(256),
                     (size_t)Csq * sizeof(float), st, part, nb, h1, w1, (int)C, (int)Csq, inv_hw, dz1, g);
  const int64_t tot = 2 * C * Csq + C + Csq;
  hipLaunchKernelGGL(se_mlp_wgrad_kernel, dim3((unsigned)((tot + 63) / 64)), dim3(256), 0, st, dz2, dz1, h1, s0,
                     (int)N, (int)C, (int)Csq, dw1, db1, dw2, db2);
  return launch_status("se_mlp_bwd");
}

// squeeze + MLP forward: s0 = mean_hw x (written out), then h1 and s as ewvit_se_mlp_fwd;
// the squeeze runs inside the MLP's first kernel (2 launches for the excite vector)
extern "C" int ewvit_se_squeeze_mlp_fwd(const void *x, int dtype, int64_t N, int64_t HW, int64_t C, const float *w1,
                                        const float *b1, const float *w2, const float *b2, int64_t Csq, float *s0,
                                        float *h1, float *s, float *workspace, void *stream) {
  if (int rc = se_check(dtype, N, HW, C, "se_squeeze_mlp_fwd")) return rc;
  if (int rc = se_mlp_check(N, C, Csq, "se_squeeze_mlp_fwd")) return rc;
  EWVIT_CHECK_ARG(x && w1 && w2 && s0 && h1 && s && workspace && HW < (1 << 30), "se_squeeze_mlp_fwd: bad args");
  hipStream_t st = as_stream(stream);
  const int nb = se_nb(C);
  const dim3 g1((unsigned)N, (unsigned)nb);
  if (dtype == EWVIT_BF16)
    hipLaunchKernelGGL(se_sq_h1_part_kernel<EWVIT_BF16>, g1, dim3(256), 0, st, x, (int)HW, 1.f / (float)HW, w1,
                       (int)C, (int)Csq, s0, workspace);
  else
    hipLaunchKernelGGL(se_sq_h1_part_kernel<EWVIT_F32>, g1, dim3(256), 0, st, x, (int)HW, 1.f / (float)HW, w1,
                       (int)C, (int)Csq, s0, workspace);
  hipLaunchKernelGGL(se_mlp_gate_kernel, dim3((unsigned)N, (unsigned)((C + 63) / 64)), dim3(256),
                     (size_t)Csq * sizeof(float), st, workspace, nb, b1, w2, b2, (int)C, (int)Csq, h1, s);
  return launch_status("se_squeeze_mlp_fwd");
}

// the whole squeeze-excitation forward in two launches: ewvit_se_squeeze_mlp_fwd's squeeze +
// hidden-partials kernel, then the gate and the excite pass y = x * s together
extern "C" int ewvit_se_forward(const void *x, int dtype, int64_t N, int64_t HW, int64_t C, const float *w1,
                                const float *b1, const float *w2, const float *b2, int64_t Csq, float *s0, float *h1,
                                float *s, void *y, float *workspace, void *stream) {
  if (int rc = se_check(dtype, N, HW, C, "se_forward")) return rc;
  if (int rc = se_mlp_check(N, C, Csq, "se_forward")) return rc;
  EWVIT_CHECK_ARG(x && w1 && w2 && s0 && h1 && s && y && workspace && HW < (1 << 30), "se_forward: bad args");
  hipStream_t st = as_stream(stream);
  const int nb = se_nb(C);
  const dim3 g1((unsigned)N, (unsigned)nb);
  const dim3 g2((unsigned)N, (unsigned)((C + 63) / 64));
  const size_t lds = (size_t)(((Csq + 3) & ~3) + 256) * sizeof(float);
  if (dtype == EWVIT_BF16) {
    hipLaunchKernelGGL(se_sq_h1_part_kernel<EWVIT_BF16>, g1, dim3(256), 0, st, x, (int)HW, 1.f / (float)HW, w1,
                       (int)C, (int)Csq, s0, workspace);
    hipLaunchKernelGGL(se_gate_scale_kernel<EWVIT_BF16>, g2, dim3(256), lds, st, workspace, nb, b1, w2, b2, (int)C,
                       (int)Csq, h1, s, x, y, (int)HW);
  } else {
    hipLaunchKernelGGL(se_sq_h1_part_kernel<EWVIT_F32>, g1, dim3(256), 0, st, x, (int)HW, 1.f / (float)HW, w1,
                       (int)C, (int)Csq, s0, workspace);
    hipLaunchKernelGGL(se_gate_scale_kernel<EWVIT_F32>, g2, dim3(256), lds, st, workspace, nb, b1, w2, b2, (int)C,
                       (int)Csq, h1, s, x, y, (int)HW);
  }
  return launch_status("se_forward");
}

// the second half of ewvit_se_forward alone: the gates from the MLP's first-layer partials
// (part [N][ceil(C / 64)][Csq], e.g. from ewvit_bn_act_se_squeeze) and the excite pass
extern "C" int ewvit_se_gate_excite(const float *part, const float *b1, const float *w2, const float *b2,
                                    const void *x, int dtype, int64_t N, int64_t HW, int64_t C, int64_t Csq, float *h1,
                                    float *s, void *y, void *stream) {
  if (int rc = se_check(dtype, N, HW, C, "se_gate_excite")) return rc;
  if (int rc = se_mlp_check(N, C, Csq, "se_gate_excite")) return rc;
  EWVIT_CHECK_ARG(part && w2 && h1 && s && x && y && HW < (1 << 30), "se_gate_excite: bad args");
  const dim3 g2((unsigned)N, (unsigned)((C + 63) / 64));
  const size_t lds = (size_t)(((Csq + 3) & ~3) + 256) * sizeof(float);
  if (dtype == EWVIT_BF16)
    hipLaunchKernelGGL(se_gate_scale_kernel<EWVIT_BF16>, g2, dim3(256), lds, as_stream(stream), part, se_nb(C), b1, w2,
                       b2, (int)C, (int)Csq, h1, s, x, y, (int)HW);
  else
    hipLaunchKernelGGL(se_gate_scale_kernel<EWVIT_F32>, g2, dim3(256), lds, as_stream(stream), part, se_nb(C), b1, w2,
                       b2, (int)C, (int)Csq, h1, s, x, y, (int)HW);
  return launch_status("se_gate_excite");
}

extern "C" int ewvit_se_squeeze_mlp_bwd(const void *dy, const void *x, int dtype, int64_t N, int64_t HW, int64_t C,
                                        const float *s, const float *h1, const float *s0, const float *w1,
                                        const float *w2, int64_t Csq, float *g, float *dw1, float *db1, float *dw2,
                                        float *db2, float *workspace, void *stream) {
  if (int rc = se_check(dtype, N, HW, C, "se_squeeze_mlp_bwd")) return rc;
  if (int rc = se_mlp_check(N, C, Csq, "se_squeeze_mlp_bwd")) return rc;
  EWVIT_CHECK_ARG(dy && x && s && h1 && s0 && w1 && w2 && g && dw1 && dw2 && workspace && HW < (1 << 30),
                  "se_squeeze_mlp_bwd: bad args");
  hipStream_t st = as_stream(stream);
  const int nb = se_nb(C);
  float *dz2 = workspace, *dz1 = workspace + N * C, *part = dz1 + N * Csq;
  const dim3 g1((unsigned)N, (unsigned)nb);
  if (dtype == EWVIT_BF16)
    hipLaunchKernelGGL(se_sq_dh_part_kernel<EWVIT_BF16>, g1, dim3(256), 0, st, dy, x, (int)HW, s, w2, (int)C,
                       (int)Csq, dz2, part);
  else
    hipLaunchKernelGGL(se_sq_dh_part_kernel<EWVIT_F32>, g1, dim3(256), 0, st, dy, x, (int)HW, s, w2, (int)C,
                       (int)Csq, dz2, part);
  hipLaunchKernelGGL(se_mlp_g_kernel, dim3((unsigned)N, (unsigned)((C + 63) / 64)), dim3(256),
                     (size_t)Csq * sizeof(float), st, part, nb, h1, w1, (int)C, (int)Csq, 1.f / (float)HW, dz1, g);
  const int64_t tot = 2 * C * Csq + C + Csq;
  hipLaunchKernelGGL(se_mlp_wgrad_kernel, dim3((unsigned)((tot + 63) / 64)), dim3(256), 0, st, dz2, dz1, h1, s0,
                     (int)N, (int)C, (int)Csq, dw1, db1, dw2, db2);
  return launch_status("se_squeeze_mlp_bwd");
}

extern "C" int64_t ewvit_bn_se_bwd_workspace(int64_t N, int64_t C, int64_t Csq) {
  return ewvit_se_mlp_bwd_workspace(N, C, Csq) + (4 * N * C + 2 * C) * (int64_t)sizeof(float);
}

// where ewvit_bn_se_bwd leaves the BN's sums row [2C] (sum g', sum g' zhat) in its workspace (floats)
extern "C" int64_t ewvit_bn_se_bwd_row_offset(int64_t N, int64_t C, int64_t Csq) {
  return ewvit_se_mlp_bwd_workspace(N, C, Csq) / (int64_t)sizeof(float) + 4 * N * C;
}

// the dx pass alone, from the sums row ewvit_bn_se_bwd (dx NULL) left: dx = the BN input gradient
// of SE(act(BN(z))) given the SE output gradient dy (the form ewvit_dwconv3x3_bwd_fused_se folds)
extern "C" int ewvit_bn_se_bwd_dx(const void *dy, const void *z, void *dx, int dtype, int64_t N, int64_t HW, int64_t C,
                                  const float *gamma, const float *beta, const float *save_mean,
                                  const float *save_invstd, int act, const float *s, const float *g, const float *row,
                                  void *stream) {
  if (int rc = se_check(dtype, N, HW, C, "bn_se_bwd_dx")) return rc;
  EWVIT_CHECK_ARG(dy && z && dx && save_mean && save_invstd && s && g && row && act >= 0 && act <= 2 && C <= 4096,
                  "bn_se_bwd_dx: bad args");
  return bn_bwd_dx_se_launch(dy, z, dx, dtype, N * HW, C, gamma, beta, save_mean, save_invstd, act, nullptr, nullptr,
                             s, g, HW, row, 1, as_stream(stream));
}

// The backward of SE(act(BatchNorm(z))) in 4 launches: the SE squeeze pass with the BN's
// per-frame sums (se_sq_dh_bn_part_kernel), the MLP's g, its weight gradients + the BN's two
// channel sums (extra blocks), and the BN's dx pass from that one partial row.  Replaces
// ewvit_se_squeeze_mlp_bwd + ewvit_bn_bwd_se (whose reduction pass re-read dy and z).
extern "C" int ewvit_bn_se_bwd(const void *dy, const void *a, const void *z, void *dx, int dtype, int64_t N,
                               int64_t HW, int64_t C, const float *gamma, const float *beta, const float *save_mean,
                               const float *save_invstd, int act, float *dgamma, float *dbeta, const float *s,
                               const float *h1, const float *s0, const float *w1, const float *w2, int64_t Csq,
                               float *g, float *dw1, float *db1, float *dw2, float *db2, float *workspace,
                               void *stream) {
  if (int rc = se_check(dtype, N, HW, C, "bn_se_bwd")) return rc;
  if (int rc = se_mlp_check(N, C, Csq, "bn_se_bwd")) return rc;
  // dx NULL: the dx pass is left to the depthwise conv's backward (ewvit_dwconv3x3_bwd_fused_se, which
  // forms dz from dy and z); dgamma / dbeta come from the sums blocks, the sums row stays in the
  // workspace at ewvit_bn_se_bwd_row_offset floats
  EWVIT_CHECK_ARG(dy && a && z && save_mean && save_invstd && s && h1 && s0 && w1 && w2 && g && dw1 && dw2 &&
                      workspace && HW < (1 << 30),
                  "bn_se_bwd: bad args");
  EWVIT_CHECK_ARG(act >= 0 && act <= 2 && C <= 4096 && N * HW < ((int64_t)1 << 31), "bn_se_bwd: act=%d C=%lld", act,
                  (long long)C);
  hipStream_t st = as_stream(stream);
  const int nb = se_nb(C);
  float *dz2 = workspace, *dz1 = workspace + N * C, *part = dz1 + N * Csq;
  float *bnsum = part + N * nb * Csq, *bnrow = bnsum + 4 * N * C;
  const dim3 g1((unsigned)N, (unsigned)nb);
#define SE_BN_DH(DTV, ACTV)                                                                                          \
  hipLaunchKernelGGL((se_sq_dh_bn_part_kernel<DTV, ACTV>), g1, dim3(256), 0, st, dy, a, z, (int)HW, s, w2, (int)C,  \
                     (int)Csq, save_mean, save_invstd, gamma, beta, dz2, part, bnsum, (int)N)
  if (dtype == EWVIT_BF16) {
    if (act == 0) SE_BN_DH(EWVIT_BF16, 0);
    else if (act == 1) SE_BN_DH(EWVIT_BF16, 1);
    else SE_BN_DH(EWVIT_BF16, 2);
  } else {
    if (act == 0) SE_BN_DH(EWVIT_F32, 0);
    else if (act == 1) SE_BN_DH(EWVIT_F32, 1);
    else SE_BN_DH(EWVIT_F32, 2);
  }
#undef SE_BN_DH
  hipLaunchKernelGGL(se_mlp_g_kernel, dim3((unsigned)N, (unsigned)((C + 63) / 64)), dim3(256),
                     (size_t)Csq * sizeof(float), st, part, nb, h1, w1, (int)C, (int)Csq, 1.f / (float)HW, dz1, g);
  const int64_t tot = 2 * C * Csq + C + Csq;
  const int nwb = (int)((tot + 63) / 64), nbn = (int)((2 * C + 63) / 64);
  hipLaunchKernelGGL(se_mlp_wgrad_kernel, dim3((unsigned)(nwb + nbn)), dim3(256), 0, st, dz2, dz1, h1, s0, (int)N,
                     (int)C, (int)Csq, dw1, db1, dw2, db2, bnsum, s, g, bnrow, nwb, dx ? nullptr : dbeta,
                     dx ? nullptr : dgamma);
  if (int rc = launch_status("bn_se_bwd")) return rc;
  if (!dx) return 0;
  return bn_bwd_dx_se_launch(dy, z, dx, dtype, N * HW, C, gamma, beta, save_mean, save_invstd, act, dgamma, dbeta, s,
                             g, HW, bnrow, 1, st);
}
