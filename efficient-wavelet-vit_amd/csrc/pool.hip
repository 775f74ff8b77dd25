// 2x2 / stride-2 max pooling over channels-last tensors — the MaxPool2d(2) of the MWT's
// freq_pool (network/mwt.py:38-44) on the freq_conv output [N, H, W, C] (bf16 or f32).
//
//   fwd  y[n,i,j,c] = max over the 2x2 window (first maximum in (0,0) (0,1) (1,0) (1,1)
//        order, NaN wins — torch's max_pool2d tie/NaN rule); arg[n,i,j,c] = window slot
//   bwd  dx = dy at the recorded slot, 0 at the other three: every dx element is written
//        once (no zero fill, no scatter)
// One thread per 8-channel vector of an output pixel: 4 (fwd) / 1 (bwd) 16-B loads.
// Odd H / W: the last input row / column is not covered (floor mode) and gets dx = 0.
#include "common.h"

namespace ewvit {

template <int DT>
__device__ __forceinline__ void pl_ld8(const void *p, int64_t i, float (&v)[8]) {
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
__device__ __forceinline__ void pl_st8(void *p, int64_t i, const float (&v)[8]) {
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

template <int DT>
__global__ __launch_bounds__(256) void maxpool2_fwd_kernel(const void *__restrict__ x, void *__restrict__ y,
                                                           uint8_t *__restrict__ arg, int H, int W, int C,
                                                           int64_t nvec) {
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= nvec) return;
  const int C8 = C >> 3, Ho = H >> 1, Wo = W >> 1;
  const int c = (int)(v % C8) * 8;
  const int64_t p = v / C8;                       // output pixel
  const int j = (int)(p % Wo);
  const int64_t t = p / Wo;
  const int i = (int)(t % Ho);
  const int64_t n = t / Ho;
  const int64_t b = ((n * H + 2 * i) * W + 2 * j) * C + c;
  float a[4][8];
  pl_ld8<DT>(x, b, a[0]);
  pl_ld8<DT>(x, b + C, a[1]);
  pl_ld8<DT>(x, b + (int64_t)W * C, a[2]);
  pl_ld8<DT>(x, b + (int64_t)W * C + C, a[3]);
  float m[8];
  uint32_t s[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    m[e] = a[0][e];
    s[e] = 0;
#pragma unroll
    for (int k = 1; k < 4; ++k)
      if (a[k][e] > m[e] || (a[k][e] != a[k][e] && m[e] == m[e])) { m[e] = a[k][e]; s[e] = k; }
  }
  pl_st8<DT>(y, p * C + c, m);
  uint2 pk;
  pk.x = s[0] | (s[1] << 8) | (s[2] << 16) | (s[3] << 24);
  pk.y = s[4] | (s[5] << 8) | (s[6] << 16) | (s[7] << 24);
  *reinterpret_cast<uint2 *>(arg + p * C + c) = pk;
}

template <int DT>
__global__ __launch_bounds__(256) void maxpool2_bwd_kernel(const void *__restrict__ dy,
                                                           const uint8_t *__restrict__ arg, void *__restrict__ dx,
                                                           int H, int W, int C, int64_t nvec) {
  // one thread per 8-channel vector of an INPUT pixel pair-row: covers the 2x2 window of
  // output pixel (i, j) — rows 2i, 2i+1, columns 2j, 2j+1 — plus the floor-mode remainder
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= nvec) return;
  const int C8 = C >> 3, Hc = (H + 1) >> 1, Wc = (W + 1) >> 1, Ho = H >> 1, Wo = W >> 1;
  const int c = (int)(v % C8) * 8;
  const int64_t p = v / C8;                       // window index over the ceil grid
  const int j = (int)(p % Wc);
  const int64_t t = p / Wc;
  const int i = (int)(t % Hc);
  const int64_t n = t / Hc;
  float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  uint32_t s[8] = {4, 4, 4, 4, 4, 4, 4, 4};
  if (i < Ho && j < Wo) {
    const int64_t o = ((n * Ho + i) * Wo + j) * C + c;
    pl_ld8<DT>(dy, o, g);
    const uint2 pk = *reinterpret_cast<const uint2 *>(arg + o);
#pragma unroll
    for (int e = 0; e < 4; ++e) { s[e] = (pk.x >> (8 * e)) & 0xff; s[4 + e] = (pk.y >> (8 * e)) & 0xff; }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int hi = 2 * i + (k >> 1), wi = 2 * j + (k & 1);
    if (hi >= H || wi >= W) continue;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = s[e] == (uint32_t)k ? g[e] : 0.f;
    pl_st8<DT>(dx, ((n * H + hi) * W + wi) * C + c, o);
  }
}

}  // namespace ewvit

using namespace ewvit;

extern "C" int ewvit_maxpool2_fwd(const void *x, void *y, uint8_t *argmax, int dtype, int64_t N, int64_t H,
                                  int64_t W, int64_t C, void *stream) {
  EWVIT_CHECK_ARG(x && y && argmax && dtype_ok(dtype), "maxpool2_fwd: bad args");
  EWVIT_CHECK_ARG(N > 0 && H >= 2 && W >= 2 && C > 0 && C % 8 == 0 && N * H * W * C < ((int64_t)1 << 40),
                  "maxpool2_fwd: shape N=%lld H=%lld W=%lld C=%lld (C %% 8 == 0)", (long long)N, (long long)H,
                  (long long)W, (long long)C);
  const int64_t nvec = N * (H / 2) * (W / 2) * (C / 8);
  const dim3 grid((unsigned)((nvec + 255) / 256));
  if (dtype == EWVIT_BF16)
    hipLaunchKernelGGL(maxpool2_fwd_kernel<EWVIT_BF16>, grid, dim3(256), 0, as_stream(stream), x, y, argmax, (int)H,
                       (int)W, (int)C, nvec);
  else
    hipLaunchKernelGGL(maxpool2_fwd_kernel<EWVIT_F32>, grid, dim3(256), 0, as_stream(stream), x, y, argmax, (int)H,
                       (int)W, (int)C, nvec);
  return launch_status("maxpool2_fwd");
}

extern "C" int ewvit_maxpool2_bwd(const void *dy, const uint8_t *argmax, void *dx, int dtype, int64_t N, int64_t H,
                                  int64_t W, int64_t C, void *stream) {
  EWVIT_CHECK_ARG(dy && dx && argmax && dtype_ok(dtype), "maxpool2_bwd: bad args");
  EWVIT_CHECK_ARG(N > 0 && H >= 2 && W >= 2 && C > 0 && C % 8 == 0 && N * H * W * C < ((int64_t)1 << 40),
                  "maxpool2_bwd: shape N=%lld H=%lld W=%lld C=%lld (C %% 8 == 0)", (long long)N, (long long)H,
                  (long long)W, (long long)C);
  const int64_t nvec = N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  const dim3 grid((unsigned)((nvec + 255) / 256));
  if (dtype == EWVIT_BF16)
    hipLaunchKernelGGL(maxpool2_bwd_kernel<EWVIT_BF16>, grid, dim3(256), 0, as_stream(stream), dy, argmax, dx,
                       (int)H, (int)W, (int)C, nvec);
  else
    hipLaunchKernelGGL(maxpool2_bwd_kernel<EWVIT_F32>, grid, dim3(256), 0, as_stream(stream), dy, argmax, dx,
                       (int)H, (int)W, (int)C, nvec);
  return launch_status("maxpool2_bwd");
}
