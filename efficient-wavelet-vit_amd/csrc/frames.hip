// Frame transform chain on the GPU (gfx950): the input side of the hot path.
//
// The reference prepares every frame on the host (config/data_loader.py:325-337 per frame,
// config/transforms.py:81-113): face crop -> Resize(450) (Pillow bilinear, 8-bpc fixed point)
// -> CenterCrop(224) -> [ColorJitter(0.01, 0.01)] -> ToTensor -> Normalize, then stacks the
// frames.  Here a batch of raw uint8 RGB frames (ragged sizes, one device buffer) becomes the
// model's [N, 3, S, S] fp32 input in one launch (two with ColorJitter), bit-identical to
// Pillow + torchvision:
//
// * only the S x S pixels CenterCrop keeps are computed: the 450-pixel image is never formed;
// * a workgroup owns `rb` output rows of one frame.  It derives the Pillow coefficients of its
//   S columns and rb rows itself, in double with no FMA contraction (Resample.c
//   precompute_coeffs + normalize_coeffs_8bpc: same IEEE operations, same results), runs the
//   horizontal pass over the source rows its rows need into LDS (uint8, rounded as Pillow's
//   intermediate image), then the vertical pass from LDS, and writes either normalised fp32
//   planes (coalesced along x) or the uint8 HWC image (for the jitter pass);
// * ColorJitter (brightness / contrast blends of ImageEnhance, float32 arithmetic, the
//   contrast level from the frame's integer luma mean) + ToTensor + Normalize: one workgroup
//   per frame (the luma mean is a whole-frame reduction).
//
// Byte-gather work (taps of 3-byte pixels), HBM / latency bound: no MFMA.
#include "common.h"

namespace ewvit {

constexpr int FR_KMAX = 17;            // taps per output sample: 2 * ceil(support) + 1, scale <= 8
constexpr int FR_SMAX = 256;           // output size S (CenterCrop) at most
constexpr int FR_LDS_CAP = 160 * 1024; // the most dynamic LDS one workgroup may be given (gfx950)
constexpr int FR_PREC = 22;            // Pillow PRECISION_BITS for 8-bpc images
constexpr int FR_GEOM = 10;            // int64 per frame (include/ewvit.h)

#pragma clang fp contract(off)

// Pillow precompute_coeffs for output sample xx of in_size -> out_size (box = whole input),
// normalised to int32 fixed point; returns xmin, writes n coefficients (+ zeros to kmax).
__host__ __device__ inline int fr_coeffs(int in_size, int out_size, int xx, int *k, int kstride, int &n) {
  const double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const double center = (xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) {
    double t = (x + xmin - center + 0.5) * ss;
    if (t < 0.0) t = -t;
    ww += t < 1.0 ? 1.0 - t : 0.0;
  }
  for (int x = 0; x < xmax; ++x) {
    double t = (x + xmin - center + 0.5) * ss;
    if (t < 0.0) t = -t;
    double w = t < 1.0 ? 1.0 - t : 0.0;
    if (ww != 0.0) w /= ww;
    const double f = w * (double)(1 << FR_PREC);
    if (k) k[x * kstride] = w < 0 ? (int)(-0.5 + f) : (int)(0.5 + f);
  }
  n = xmax;
  return xmin;
}

__device__ __forceinline__ unsigned fr_clip8(int acc) {
  const int v = acc >> FR_PREC;
  return v < 0 ? 0u : v > 255 ? 255u : (unsigned)v;
}

struct FrGeom {
  int64_t off, stride;       // frame's first byte in the batch buffer, bytes per source row
  int l, t, w, h;            // crop box (left, top, width, height) inside the frame
  int nw, nh, ox, oy;        // Resize output size, CenterCrop offsets
};

__device__ __forceinline__ FrGeom fr_geom(const int64_t *g, int n) {
  const int64_t *p = g + (int64_t)n * FR_GEOM;
  FrGeom r;
  r.off = p[0]; r.stride = p[1];
  r.l = (int)p[2]; r.t = (int)p[3]; r.w = (int)p[4]; r.h = (int)p[5];
  r.nw = (int)p[6]; r.nh = (int)p[7]; r.ox = (int)p[8]; r.oy = (int)p[9];
  return r;
}

struct FrNorm { float mean[3], inv[3]; };   // inv = std (division, as torchvision)

// LDS layout of a resize workgroup (ints, then pixels): hk [kmax][S] column weights, hx / hn [S]
// first tap / taps per column, vk [kmax][rb], vy / vn [rb]; then the horizontal pass's rows
// tmp [rmax][S] and, when the plan stages the source (pitch > 0), the source rows
// src [rmax][pitch] — one 4-byte word per RGB pixel (R | G << 8 | B << 16), so a tap is one LDS
// read and three byte extracts.
struct FrPlan { int rb, kmax, rmax, pitch; };

__host__ __device__ inline int fr_ints(int S, const FrPlan &p) { return (p.kmax + 2) * (S + p.rb); }
__host__ __device__ inline int fr_lds_bytes(int S, const FrPlan &p) {
  return (fr_ints(S, p) + p.rmax * S + p.rmax * p.pitch) * 4;
}

// acc += weight * (8-bit channels of a packed pixel); weights and bytes fit the 24-bit multiply
__device__ __forceinline__ void fr_tap(uint32_t px, uint32_t w, uint32_t &a0, uint32_t &a1, uint32_t &a2) {
  a0 += __umul24(px & 0xffu, w);   // (Pillow's weights are >= 0 and <= 2^22)
  a1 += __umul24((px >> 8) & 0xffu, w);
  a2 += __umul24(px >> 16, w);
}
__device__ __forceinline__ uint32_t fr_pack(uint32_t a0, uint32_t a1, uint32_t a2) {
  const uint32_t r = min(a0 >> FR_PREC, 255u), g = min(a1 >> FR_PREC, 255u), b = min(a2 >> FR_PREC, 255u);
  return r | (g << 8) | (b << 16);
}

// grid (ceil(S / rb), N), 256 threads, fr_lds_bytes of dynamic LDS; KT >= the plan's taps.
// out: TO_F32 -> [N][3][S][S] normalised fp32, else [N][S][S][3] uint8.
template <int KT, bool TO_F32>
__global__ __launch_bounds__(256) void frames_resize_crop_kernel(const uint8_t *__restrict__ src,
                                                                 const int64_t *__restrict__ geom, int S, FrPlan pl,
                                                                 FrNorm nm, void *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) int fr_smem[];
  const int rb = pl.rb, kmax = pl.kmax;
  int *hk = fr_smem, *hx = hk + kmax * S, *hn = hx + S;
  int *vk = hn + S, *vy = vk + kmax * rb, *vn = vy + rb;
  uint32_t *tmp = reinterpret_cast<uint32_t *>(fr_smem + fr_ints(S, pl));
  uint32_t *stg = tmp + pl.rmax * S;
  const int tid = threadIdx.x, n = blockIdx.y;
  const int y_beg = blockIdx.x * rb;
  const int rows = S - y_beg < rb ? S - y_beg : rb;
  if (rows <= 0) return;
  const FrGeom g = fr_geom(geom, n);
  for (int c = tid; c < S; c += blockDim.x) {
    int cnt;
    hx[c] = fr_coeffs(g.w, g.nw, g.ox + c, hk + c, S, cnt);
    hn[c] = cnt;
  }
  for (int r = tid; r < rows; r += blockDim.x) {
    int cnt;
    vy[r] = fr_coeffs(g.h, g.nh, g.oy + y_beg + r, vk + r, rb, cnt);
    vn[r] = cnt;
  }
  __syncthreads();
  const int y0 = vy[0], R = vy[rows - 1] + vn[rows - 1] - y0;   // both bounds monotone in the row
  const int x0 = hx[0], npx = hx[S - 1] + hn[S - 1] - x0;
  if (R > pl.rmax) return;                                       // the planner bounds R
  const uint8_t *base = src + g.off + (int64_t)(g.t + y0) * g.stride + (int64_t)(g.l + x0) * 3;
  const bool staged = npx <= pl.pitch;
  if (staged) {
    // 4 pixels (12 bytes) per item from the 4 aligned dwords that hold them (a dword holding
    // one of the frame's bytes never leaves its allocation; dwords past the span are not read)
    const int groups = (npx + 3) >> 2, items = R * groups;
    for (int i = tid; i < items; i += blockDim.x) {
      const int r = i / groups, j = i - r * groups;
      const uintptr_t a = (uintptr_t)(base + (int64_t)r * g.stride);
      const uintptr_t al = a & ~(uintptr_t)3, last = (a + 3 * npx - 1) & ~(uintptr_t)3;
      const uint32_t lead = (uint32_t)(a & 3);
      uint32_t d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uintptr_t ad = al + 12 * j + 4 * q;
        d[q] = ad <= last ? *reinterpret_cast<const uint32_t *>(ad) : 0u;
      }
      const uint32_t w0 = __builtin_amdgcn_alignbyte(d[1], d[0], lead);
      const uint32_t w1 = __builtin_amdgcn_alignbyte(d[2], d[1], lead);
      const uint32_t w2 = __builtin_amdgcn_alignbyte(d[3], d[2], lead);
      uint4 v;
      v.x = w0 & 0xffffffu;
      v.y = (w0 >> 24) | ((w1 & 0xffffu) << 8);
      v.z = (w1 >> 16) | ((w2 & 0xffu) << 16);
      v.w = w2 >> 8;
      *reinterpret_cast<uint4 *>(stg + r * pl.pitch + 4 * j) = v;
    }
    __syncthreads();
  }
  // horizontal pass, a thread per output column: its taps in registers, down the R rows
  for (int c = tid; c < S; c += blockDim.x) {
    const int cnt = hn[c], xo = hx[c] - x0;
    uint32_t w[KT];
#pragma unroll
    for (int k = 0; k < KT; ++k) w[k] = k < cnt ? (uint32_t)hk[k * S + c] : 0u;
    for (int r = 0; r < R; ++r) {
      uint32_t a0 = 1u << (FR_PREC - 1), a1 = a0, a2 = a0;
      if (staged) {
        const uint32_t *p = stg + r * pl.pitch + xo;
#pragma unroll
        for (int k = 0; k < KT; ++k)
          if (k < cnt) fr_tap(p[k], w[k], a0, a1, a2);
      } else {
        const uint8_t *p = base + (int64_t)r * g.stride + xo * 3;
#pragma unroll
        for (int k = 0; k < KT; ++k)
          if (k < cnt) fr_tap(p[3 * k] | (p[3 * k + 1] << 8) | (p[3 * k + 2] << 16), w[k], a0, a1, a2);
      }
      tmp[r * S + c] = fr_pack(a0, a1, a2);
    }
  }
  __syncthreads();
  // vertical pass from LDS, a thread per output column
  for (int c = tid; c < S; c += blockDim.x) {
    for (int r = 0; r < rows; ++r) {
      const int cnt = vn[r];
      const uint32_t *p = tmp + (vy[r] - y0) * S + c;
      uint32_t a0 = 1u << (FR_PREC - 1), a1 = a0, a2 = a0;
#pragma unroll
      for (int k = 0; k < KT; ++k)
        if (k < cnt) fr_tap(p[k * S], (uint32_t)vk[k * rb + r], a0, a1, a2);
      const uint32_t px = fr_pack(a0, a1, a2);
      const int y = y_beg + r;
      if (TO_F32) {
        float *o = reinterpret_cast<float *>(out) + (int64_t)n * 3 * S * S + (int64_t)y * S + c;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch)
          o[(int64_t)ch * S * S] = ((float)((px >> (8 * ch)) & 0xffu) / 255.0f - nm.mean[ch]) / nm.inv[ch];
      } else {
        uint8_t *o = reinterpret_cast<uint8_t *>(out) + (((int64_t)n * S + y) * S + c) * 3;
        o[0] = (uint8_t)px;
        o[1] = (uint8_t)(px >> 8);
        o[2] = (uint8_t)(px >> 16);
      }
    }
  }
}

// Pillow ImagingBlend(in1, in2, alpha) for one uint8 sample, float32 arithmetic
__device__ __forceinline__ unsigned fr_blend(int in1, int in2, float alpha) {
  const float v = (float)in1 + alpha * (float)(in2 - in1);
  if (v <= 0.0f) return 0u;
  if (v >= 255.0f) return 255u;
  return (unsigned)v;
}

// ColorJitter(brightness, contrast) + ToTensor + Normalize, one workgroup per frame.
// jit [N][4] f32: brightness factor (< 0: none), contrast factor (< 0: none), order (0:
// brightness first, 1: contrast first), unused.
__global__ __launch_bounds__(1024) void frames_jitter_kernel(const uint8_t *__restrict__ img,
                                                             const float *__restrict__ jit, int S, FrNorm nm,
                                                             float *__restrict__ out) {
  __shared__ int red[16];
  const int n = blockIdx.x, tid = threadIdx.x;
  const float bf = jit[n * 4 + 0], cf = jit[n * 4 + 1];
  const bool bfirst = jit[n * 4 + 2] == 0.0f;
  const bool has_b = bf >= 0.0f, has_c = cf >= 0.0f;
  const int npx = S * S;
  const uint8_t *p = img + (int64_t)n * npx * 3;
  int level = 0;
  if (has_c) {
    int s = 0;
    for (int i = tid; i < npx; i += blockDim.x) {
      int v[3] = {p[3 * i], p[3 * i + 1], p[3 * i + 2]};
      if (has_b && bfirst)
        for (int ch = 0; ch < 3; ++ch) v[ch] = (int)fr_blend(0, v[ch], bf);
      s += (v[0] * 19595 + v[1] * 38470 + v[2] * 7471 + 0x8000) >> 16;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if ((tid & 63) == 0) red[tid >> 6] = s;
    __syncthreads();
    int64_t tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += red[w];
    level = (int)((2 * tot + npx) / (2 * (int64_t)npx));   // int(mean + 0.5), exact
  }
  float *o = out + (int64_t)n * 3 * npx;
  for (int i = tid; i < npx; i += blockDim.x) {
    int v[3] = {p[3 * i], p[3 * i + 1], p[3 * i + 2]};
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      if (has_b && bfirst) v[ch] = (int)fr_blend(0, v[ch], bf);
      if (has_c) v[ch] = (int)fr_blend(level, v[ch], cf);
      if (has_b && !bfirst) v[ch] = (int)fr_blend(0, v[ch], bf);
      o[(int64_t)ch * npx + i] = ((float)v[ch] / 255.0f - nm.mean[ch]) / nm.inv[ch];
    }
  }
}

// rows of the horizontal pass one band of rb output rows needs, at most, for a frame
static int fr_band_rows(int h, int nh, int oy, int S, int rb) {
  int worst = 0;
  for (int y = 0; y < S; y += rb) {
    const int last = (y + rb < S ? y + rb : S) - 1;
    int n0, n1;
    const int a = fr_coeffs(h, nh, oy + y, nullptr, 0, n0);
    const int b = fr_coeffs(h, nh, oy + last, nullptr, 0, n1);
    if (b + n1 - a > worst) worst = b + n1 - a;
  }
  return worst;
}

// dynamic LDS budget per workgroup
static int fr_lds_max() { return 64 * 1024; }

static FrNorm fr_norm(const float *mean_std) {
  FrNorm nm;
  for (int c = 0; c < 3; ++c) { nm.mean[c] = mean_std[c]; nm.inv[c] = mean_std[3 + c]; }
  return nm;
}

}  // namespace ewvit

using namespace ewvit;

extern "C" int ewvit_frames_plan(const int64_t *geom, int64_t n, int S, int64_t nbytes, int *plan) {
  if (!geom || !plan || n <= 0 || S <= 0 || S > FR_SMAX) {
    set_error("frames_plan: bad arguments (n %lld, S %d; S <= %d)", (long long)n, S, FR_SMAX);
    return EWVIT_EINVAL;
  }
  int kmax = 3, words = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t *p = geom + i * FR_GEOM;
    const int l = (int)p[2], t = (int)p[3], w = (int)p[4], h = (int)p[5];
    const int nw = (int)p[6], nh = (int)p[7], ox = (int)p[8], oy = (int)p[9];
    if (w <= 0 || h <= 0 || l < 0 || t < 0 || p[0] < 0 || p[1] < 3 * (int64_t)(l + w) || nw < S || nh < S ||
        ox < 0 || oy < 0 || ox + S > nw || oy + S > nh || p[0] + (t + h - 1) * p[1] + 3 * (int64_t)(l + w) > nbytes) {
      set_error("frames_plan: frame %lld: bad geometry (box %d,%d %dx%d, resize %dx%d, crop at %d,%d, S %d)",
                (long long)i, l, t, w, h, nw, nh, ox, oy, S);
      return EWVIT_EINVAL;
    }
    // taps per output sample: support = max(scale, 1) -> 2 * ceil(support) + 1 <= FR_KMAX
    if (w > 8 * (int64_t)nw || h > 8 * (int64_t)nh) {
      set_error("frames_plan: frame %lld: downscale %dx%d -> %dx%d beyond 8x", (long long)i, w, h, nw, nh);
      return EWVIT_EINVAL;
    }
    const int kx = 2 * ((w + nw - 1) / nw) + 1, ky = 2 * ((h + nh - 1) / nh) + 1;
    kmax = kx > kmax ? kx : kmax;
    kmax = ky > kmax ? ky : kmax;
    int n0, n1;
    const int a = fr_coeffs(w, nw, ox, nullptr, 0, n0), b = fr_coeffs(w, nw, ox + S - 1, nullptr, 0, n1);
    const int wd = (b + n1 - a + 3) / 4 * 4;       // staged pixels per source row (16-B rows)
    words = wd > words ? wd : words;
  }
  auto rmax_of = [&](int rb) {
    int r = 0;
    for (int64_t i = 0; i < n; ++i) {
      const int64_t *p = geom + i * FR_GEOM;
      const int v = fr_band_rows((int)p[5], (int)p[7], (int)p[9], S, rb);
      r = v > r ? v : r;
    }
    return r;
  };
  // staged source rows at the tallest band that fits, else bands read the source from global
  // the tallest band (<= 4 rows) whose LDS fits: 64-frame 720p clip with face boxes, 2 / 4 / 8 /
  // 16-row bands 38.5 / 31.7 / 32.6 / 44.4 us (tools/frames_lds_ab.sh: the column-per-thread
  // horizontal pass walks the band's source rows serially)
  constexpr int rbmax = 4;
  for (int staged = 1; staged >= 0; --staged)
    for (int rb = rbmax; rb >= 1; rb >>= 1) {
      const FrPlan pl{rb, kmax, rmax_of(rb), staged ? words : 0};
      if (fr_lds_bytes(S, pl) <= fr_lds_max()) {
        plan[0] = pl.rb; plan[1] = pl.kmax; plan[2] = pl.rmax; plan[3] = pl.pitch;
        return 0;
      }
    }
  set_error("frames_plan: one output row needs more source rows than LDS holds");
  return EWVIT_EINVAL;
}

extern "C" int ewvit_frames_resize_crop(const uint8_t *frames, const int64_t *geom, int64_t n, int S, const int *plan,
                                        int to_f32, const float *mean_std, void *out, void *stream) {
  EWVIT_CHECK_ARG(frames && geom && out && plan && n > 0, "frames_resize_crop: null pointer or empty batch");
  const FrPlan pl{plan[0], plan[1], plan[2], plan[3]};
  EWVIT_CHECK_ARG(S > 0 && S <= FR_SMAX && pl.rb >= 1 && pl.rb <= 64 && pl.kmax >= 1 && pl.kmax <= FR_KMAX &&
                      pl.rmax >= 1 && pl.pitch >= 0 && fr_lds_bytes(S, pl) <= FR_LDS_CAP,
                  "frames_resize_crop: S %d / plan (%d, %d, %d, %d) out of range (use ewvit_frames_plan)", S, pl.rb,
                  pl.kmax, pl.rmax, pl.pitch);
  EWVIT_CHECK_ARG(!to_f32 || mean_std, "frames_resize_crop: normalised output needs mean_std");
  const float one[6] = {0.f, 0.f, 0.f, 1.f, 1.f, 1.f};
  const FrNorm nm = fr_norm(mean_std ? mean_std : one);
  EWVIT_CHECK_ARG(pl.pitch % 4 == 0, "frames_resize_crop: plan pitch %d not a multiple of 4", pl.pitch);
  const dim3 grid((unsigned)((S + pl.rb - 1) / pl.rb), (unsigned)n);
  const size_t lds = (size_t)fr_lds_bytes(S, pl);
  hipStream_t st = as_stream(stream);
#define EWVIT_FR_LAUNCH(KT_)                                                                                        \
  do {                                                                                                            \
    static const bool attr = [] {      /* more than 64 KB of dynamic LDS needs the attribute */                  \
      return hipFuncSetAttribute(reinterpret_cast<const void *>(frames_resize_crop_kernel<KT_, true>),            \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, FR_LDS_CAP) == hipSuccess &&         \
             hipFuncSetAttribute(reinterpret_cast<const void *>(frames_resize_crop_kernel<KT_, false>),           \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, FR_LDS_CAP) == hipSuccess;           \
    }();                                                                                                          \
    (void)attr;                                                                                                   \
    if (to_f32)                                                                                                   \
      hipLaunchKernelGGL((frames_resize_crop_kernel<KT_, true>), grid, dim3(256), lds, st, frames, geom, S, pl, nm, out); \
    else                                                                                                          \
      hipLaunchKernelGGL((frames_resize_crop_kernel<KT_, false>), grid, dim3(256), lds, st, frames, geom, S, pl, nm, out); \
  } while (0)
  if (pl.kmax <= 5) EWVIT_FR_LAUNCH(5);
  else if (pl.kmax <= 9) EWVIT_FR_LAUNCH(9);
  else EWVIT_FR_LAUNCH(FR_KMAX);
#undef EWVIT_FR_LAUNCH
  return launch_status("frames_resize_crop");
}

extern "C" int ewvit_frames_jitter_normalize(const uint8_t *img, const float *jitter, int64_t n, int S,
                                             const float *mean_std, float *out, void *stream) {
  EWVIT_CHECK_ARG(img && jitter && mean_std && out && n > 0, "frames_jitter_normalize: null pointer or empty batch");
  EWVIT_CHECK_ARG(S > 0 && S <= 4096, "frames_jitter_normalize: S %d out of range", S);
  hipLaunchKernelGGL(frames_jitter_kernel, dim3((unsigned)n), dim3(1024), 0, as_stream(stream), img, jitter, S,
                     fr_norm(mean_std), out);
  return launch_status("frames_jitter_normalize");
}
