// The backbone stem: Conv2d(3 -> 24, 3x3, stride 2, pad 1) over the frames (EfficientNetV2-S
// features.0.0, reference network/sfe.py:111-119 — frozen there: parameters 0-5 of the
// backbone take no gradient, so the stem is forward-only on the training path).
//
// K = 27 is too short for an MFMA tile (a 64-deep K-tile would be 58 % zeros) and the
// frames arrive as fp32 NCHW, so this is a direct conv on the vector ALU: a lane owns one
// output pixel, loads its 3x3x3 window straight from the frames, holds the 27 values in
// registers and forms all Cout outputs with packed fp32 FMAs (channel pairs, x broadcast)
// whose weight operand is an SGPR pair: the weights, tap-major, come in two taps at a time
// by scalar loads.  (Read from LDS as broadcasts instead, every ds_read_b128 returns 1 KiB
// per wave: the LDS return path held that form at 46 us.)  Operands stay fp32
// (the autocast reference rounds them to bf16: this is the more precise of the two, at the
// same cost); only the output is rounded.  The output is channels-last bf16 — what the backbone's kernels take — stored 16 B at a time, and the
// BatchNorm batch statistics of the rounded output are summed on the way (per block,
// shifted by the running mean), so the stem BN runs its apply pass only.
// HBM-bound: 64 frames x 3 x 224^2 x 4 B in + 64 x 112^2 x 24 x 2 B out = 77 MB per launch.
#include "common.h"

namespace ewvit {

constexpr int STEM_T = 16;                 // 16 x 16 output pixels per tile, one per lane

struct StemArgs {
  const void *x;
  int64_t sn, sc, sh, sw;                  // element strides of x
  int64_t xbytes;                          // bytes addressable from x (< 2 GiB)
  const float *w;                          // fp32 [Cin*9 (+1: bias)][Cout] tap-major, + >= 64 floats
  int has_bias;                            // w holds a (Cin*9+1)-th tap row: the bias
  bf16_t *y;                               // [N][Ho][Wo][Cout]
  int N, Cin, H, W, Ho, Wo, stride, tw, ntiles;
  const float *bn_shift;
  float *bn_part;                          // [gridDim.x][2][Cout] shifted sums, or null
  float *bn_shift_out;
};

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// One tap's Cout weights in SGPRs: `sissue` starts the scalar loads (reads only; up to 32
// floats as x16 + x8 pieces — the buffer is padded by 64 floats, so an over-read stays
// inside it), `swait` waits for them and re-defines the registers, so nothing reads them
// before they land.  Loading all taps' weights at once spills the scalar file; double-
// buffering two taps also spills it at this kernel's SGPR use, so taps go one at a time
// (measured: 40-43 us for the config-2 stem, against 46 us for LDS-broadcast weights).
typedef float f32x8 __attribute__((ext_vector_type(8)));
struct TapW {
  f32x16 a;
  f32x8 b;                 // COUT > 16: channels 16..23
  f32x8 c;                 // COUT 32: channels 24..31
};
template <int COUT>
__device__ __forceinline__ void sissue(const float *base, int off, TapW &w) {
  if constexpr (COUT <= 16)
    asm volatile("s_load_dwordx16 %0, %1, %2" : "=s"(w.a) : "s"(base), "s"(off) : "memory");
  else if constexpr (COUT <= 24)
    asm volatile("s_load_dwordx16 %0, %2, %3\n\ts_load_dwordx8 %1, %2, %4"
                 : "=s"(w.a), "=s"(w.b) : "s"(base), "s"(off), "s"(off + 64) : "memory");
  else
    asm volatile("s_load_dwordx16 %0, %3, %4\n\ts_load_dwordx8 %1, %3, %5\n\ts_load_dwordx8 %2, %3, %6"
                 : "=s"(w.a), "=s"(w.b), "=s"(w.c) : "s"(base), "s"(off), "s"(off + 64), "s"(off + 96) : "memory");
}
template <int COUT>
__device__ __forceinline__ void swait(TapW &w) {
  if constexpr (COUT <= 16)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(w.a) :: "memory");
  else if constexpr (COUT <= 24)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(w.a), "+s"(w.b) :: "memory");
  else
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(w.a), "+s"(w.b), "+s"(w.c) :: "memory");
}
template <int COUT>
__device__ __forceinline__ float tapw(const TapW &w, int c) {
  return c < 16 ? w.a[c] : (c < 24 ? w.b[c - 16] : w.c[c - 24]);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t stem_rsrc(const void *p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}

template <int COUT, int CIN, bool F32>
__global__ __launch_bounds__(256) void stem_conv_kernel(StemArgs a) {
  constexpr int K = CIN * 9, CP = COUT / 2;
  constexpr uint32_t OOBX = 0x80000000u;     // any offset >= num_records reads 0
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ty = tid >> 4, tx = tid & 15;
  const float *__restrict__ wt = a.w;
  bf16_t *__restrict__ yout = a.y;
  const __amdgpu_buffer_rsrc_t rx = stem_rsrc(a.x, a.xbytes);
  // BN shift K (pairs) read from LDS where the statistics use it; the bias is the weight
  // buffer's extra tap (x = 1), so neither holds registers across the tile loop
  __shared__ f32x2 shl[CP];
  if (tid < CP) shl[tid] = a.bn_shift ? f32x2{a.bn_shift[2 * tid], a.bn_shift[2 * tid + 1]} : f32x2{0.f, 0.f};
  __syncthreads();
  f32x2 s2[CP], q2[CP];
#pragma unroll
  for (int c = 0; c < CP; ++c) { s2[c] = f32x2{0.f, 0.f}; q2[c] = s2[c]; }
  const bool has_bias = a.has_bias != 0;
  const int tpi = a.tw * ((a.Ho + STEM_T - 1) / STEM_T);    // tiles per image
  for (int t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
    const int n = t / tpi, r = t - n * tpi;
    const int oh = (r / a.tw) * STEM_T + ty, ow = (r % a.tw) * STEM_T + tx;
    if (oh >= a.Ho || ow >= a.Wo) continue;
    // the 3x3xCIN window: element offsets (32-bit: the frames are < 2 GiB) from per-row and
    // per-column parts; taps outside the frame (zero padding) read through an offset past
    // the buffer's end, which the descriptor returns as 0 — no branch, no select
    const int ih0 = oh * a.stride - 1, iw0 = ow * a.stride - 1;
    uint32_t ro[3], co[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const int ih = ih0 + d, iw = iw0 + d;
      ro[d] = (unsigned)ih < (unsigned)a.H ? (uint32_t)(n * a.sn + ih * a.sh) : OOBX;
      co[d] = (unsigned)iw < (unsigned)a.W ? (uint32_t)(iw * a.sw) : OOBX;
    }
    float xv[K];
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const uint32_t e = (ro[kh] | co[kw]) & OOBX ? OOBX : ro[kh] + co[kw] + (uint32_t)(ci * a.sc);
          float v;
          if constexpr (F32)
            v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, e == OOBX ? OOBX : e * 4, 0, 0));
          else
            v = bf2f(__builtin_amdgcn_raw_buffer_load_b16(rx, e == OOBX ? OOBX : e * 2, 0, 0));
          xv[(ci * 3 + kh) * 3 + kw] = v;
        }
    // y[c] = b[c] + sum_k x[k] w[k][c]: weights tap-major ([K][Cout]), two taps per scalar
    // load step, channel pairs on packed fp32 FMAs (x broadcast, the weight pair an SGPR pair)
    f32x2 y2[CP];
#pragma unroll
    for (int c = 0; c < CP; ++c) y2[c] = f32x2{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < K; ++k) {
      TapW w;
      asm volatile("" : "+v"(y2[CP - 1]));      // tap k's loads after tap k-1's FMAs
      sissue<COUT>(wt, k * COUT * 4, w);
      swait<COUT>(w);
      const f32x2 xx = f32x2{xv[k], xv[k]};
#pragma unroll
      for (int c = 0; c < CP; ++c)
        y2[c] = __builtin_elementwise_fma(xx, f32x2{tapw<COUT>(w, 2 * c), tapw<COUT>(w, 2 * c + 1)}, y2[c]);
    }
    if (has_bias) {                        // the bias tap (x = 1)
      TapW w;
      asm volatile("" : "+v"(y2[CP - 1]));
      sissue<COUT>(wt, K * COUT * 4, w);
      swait<COUT>(w);
#pragma unroll
      for (int c = 0; c < CP; ++c) y2[c] += f32x2{tapw<COUT>(w, 2 * c), tapw<COUT>(w, 2 * c + 1)};
    }
    uint32_t pk[CP];
#pragma unroll
    for (int c = 0; c < CP; ++c) {
      const bf16x2 h = __builtin_convertvector(y2[c], bf16x2);
      pk[c] = __builtin_bit_cast(uint32_t, h);
      const f32x2 d = f32x2{__uint_as_float(pk[c] << 16), __uint_as_float(pk[c] & 0xffff0000u)} - shl[c];
      s2[c] += d;
      q2[c] = __builtin_elementwise_fma(d, d, q2[c]);
    }
    uint4 *dst = reinterpret_cast<uint4 *>(yout + (((int64_t)n * a.Ho + oh) * a.Wo + ow) * COUT);
#pragma unroll
    for (int v = 0; v < COUT / 8; ++v) dst[v] = make_uint4(pk[4 * v], pk[4 * v + 1], pk[4 * v + 2], pk[4 * v + 3]);
  }
  if (!a.bn_part) return;
  // this block's partial row: wave sums (DPP / permlane), then the 4 waves through LDS
  __shared__ float red[4][2 * COUT];
#pragma unroll
  for (int c = 0; c < CP; ++c) {
    const float S0 = wave_sum(s2[c].x), S1 = wave_sum(s2[c].y), Q0 = wave_sum(q2[c].x), Q1 = wave_sum(q2[c].y);
    if (lane == 0) {
      red[wv][2 * c] = S0; red[wv][2 * c + 1] = S1;
      red[wv][COUT + 2 * c] = Q0; red[wv][COUT + 2 * c + 1] = Q1;
    }
  }
  __syncthreads();
  if (tid < 2 * COUT) {
    a.bn_part[(int64_t)blockIdx.x * 2 * COUT + tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
    if (blockIdx.x == 0 && tid < COUT && a.bn_shift_out) a.bn_shift_out[tid] = a.bn_shift ? a.bn_shift[tid] : 0.f;
  }
}

static int stem_grid(int64_t ntiles) {
  constexpr int64_t cap = 1024;                  // workgroups; each walks its tiles
  const int64_t g = ntiles < cap ? ntiles : cap;
  return (int)(g < 1 ? 1 : g);
}

static int64_t stem_tiles(int64_t N, int64_t Ho, int64_t Wo) {
  return N * ((Ho + STEM_T - 1) / STEM_T) * ((Wo + STEM_T - 1) / STEM_T);
}

}  // namespace ewvit

using namespace ewvit;

extern "C" int64_t ewvit_conv2d_stem_parts(int64_t N, int64_t H, int64_t W, int stride) {
  if (N <= 0 || H <= 0 || W <= 0 || (stride != 1 && stride != 2)) return 0;
  return stem_grid(stem_tiles(N, (H - 1) / stride + 1, (W - 1) / stride + 1));
}

extern "C" int ewvit_conv2d_stem_fwd(const void *x, int x_dtype, int64_t N, int64_t Cin, int64_t H, int64_t W,
                                     int64_t sx_n, int64_t sx_c, int64_t sx_h, int64_t sx_w, const float *w,
                                     int has_bias, void *y, int64_t Cout, int stride, const float *bn_shift,
                                     float *bn_part, float *bn_shift_out, void *stream) {
  EWVIT_CHECK_ARG(x && w && y && dtype_ok(x_dtype), "conv2d_stem_fwd: bad args");
  EWVIT_CHECK_ARG(Cin >= 1 && Cin <= 4 && (Cout == 8 || Cout == 16 || Cout == 24 || Cout == 32),
                  "conv2d_stem_fwd: Cin=%lld (1..4), Cout=%lld (8/16/24/32)", (long long)Cin, (long long)Cout);
  EWVIT_CHECK_ARG(stride == 1 || stride == 2, "conv2d_stem_fwd: stride %d", stride);
  EWVIT_CHECK_ARG(N >= 1 && H >= 1 && W >= 1 && N * Cin * H * W < ((int64_t)1 << 40) && H < 65536 && W < 65536,
                  "conv2d_stem_fwd: shape");
  EWVIT_CHECK_ARG(!bn_part || bn_shift_out, "conv2d_stem_fwd: bn_part needs bn_shift_out");
  EWVIT_CHECK_ARG(sx_n >= 0 && sx_c >= 0 && sx_h >= 0 && sx_w >= 0, "conv2d_stem_fwd: negative strides");
  const int64_t xbytes = ((N - 1) * sx_n + (Cin - 1) * sx_c + (H - 1) * sx_h + (W - 1) * sx_w + 1) *
                         (x_dtype == EWVIT_F32 ? 4 : 2);
  EWVIT_CHECK_ARG(xbytes < ((int64_t)1 << 31), "conv2d_stem_fwd: x spans %lld bytes (< 2 GiB: 32-bit offsets)",
                  (long long)xbytes);
  StemArgs a;
  a.x = x; a.sn = sx_n; a.sc = sx_c; a.sh = sx_h; a.sw = sx_w; a.xbytes = xbytes;
  a.w = w; a.has_bias = has_bias; a.y = (bf16_t *)y;
  a.N = (int)N; a.Cin = (int)Cin; a.H = (int)H; a.W = (int)W;
  a.Ho = (int)((H - 1) / stride + 1); a.Wo = (int)((W - 1) / stride + 1); a.stride = stride;
  a.tw = (a.Wo + STEM_T - 1) / STEM_T;
  const int64_t nt = stem_tiles(N, a.Ho, a.Wo);
  EWVIT_CHECK_ARG(nt < ((int64_t)1 << 31), "conv2d_stem_fwd: %lld tiles", (long long)nt);
  a.ntiles = (int)nt;
  a.bn_shift = bn_shift; a.bn_part = bn_part; a.bn_shift_out = bn_shift_out;
  const dim3 grid((unsigned)stem_grid(nt));
  hipStream_t s = as_stream(stream);
  const bool f32 = x_dtype == EWVIT_F32;
#define STEM_LAUNCH(CO, CI)                                                                             \
  do {                                                                                                  \
    if (f32) hipLaunchKernelGGL((stem_conv_kernel<CO, CI, true>), grid, dim3(256), 0, s, a);           \
    else hipLaunchKernelGGL((stem_conv_kernel<CO, CI, false>), grid, dim3(256), 0, s, a);              \
  } while (0)
#define STEM_CO(CI)                          \
  switch (Cout) {                            \
    case 8: STEM_LAUNCH(8, CI); break;       \
    case 16: STEM_LAUNCH(16, CI); break;     \
    case 24: STEM_LAUNCH(24, CI); break;     \
    default: STEM_LAUNCH(32, CI); break;     \
  }
  switch (Cin) {
    case 1: STEM_CO(1); break;
    case 2: STEM_CO(2); break;
    case 3: STEM_CO(3); break;
    default: STEM_CO(4); break;
  }
#undef STEM_CO
#undef STEM_LAUNCH
  return launch_status("conv2d_stem_fwd");
}
