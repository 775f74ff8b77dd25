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

// block = LC channel vectors x R row groups; grid (N * S, cblocks)
static SePlan se_plan(int64_t N, int64_t HW, int64_t C) {
  SePlan p;
  p.C8 = (int)(C / 8);
  p.LC = p.C8 < 256 ? p.C8 : 256;
  p.R = 256 / p.LC;
  p.cblocks = (p.C8 + p.LC - 1) / p.LC;
  int64_t s = (512 + N * p.cblocks - 1) / (N * p.cblocks);     // ~512 blocks
  const int64_t maxs = HW / (4 * p.R);                          // >= 4 rows per thread
  if (s > maxs) s = maxs;
  if (s < 1) s = 1;
  p.S = (int)s;
  p.rows_per_split = (int)((HW + s - 1) / s);
  return p;
}

// part[split][n][c] = sum over this split's rows of a (PROD=0) or a*b (PROD=1)
template <int DT, int PROD>
__global__ __launch_bounds__(256) void se_reduce_kernel(const void *__restrict__ a, const void *__restrict__ b,
                                                        int HW, int C, int R, int LC, int S, int rps,
                                                        float *__restrict__ part, int N) {
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
    for (; h + 3 * R < h1; h += 4 * R) {     // 4 rows' loads in flight
      float va[4][8], vb[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        se_ld8<DT>(a, base + (int64_t)(h + q * R) * C, va[q]);
        if (PROD) se_ld8<DT>(b, base + (int64_t)(h + q * R) * C, vb[q]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
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
    float *dst = part + ((int64_t)split * N + n) * C + c8 * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[j] = acc[j];
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
                     p.rows_per_split, workspace, (int)N)
  if (dtype == EWVIT_BF16) { if (b) SE_RED(EWVIT_BF16, 1); else SE_RED(EWVIT_BF16, 0); }
  else { if (b) SE_RED(EWVIT_F32, 1); else SE_RED(EWVIT_F32, 0); }
#undef SE_RED
  const int64_t NC = N * C;
  hipLaunchKernelGGL(se_fold_kernel, dim3((unsigned)((NC + 255) / 256)), dim3(256), 0, s, workspace, p.S, NC, scale,
                     out);
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
