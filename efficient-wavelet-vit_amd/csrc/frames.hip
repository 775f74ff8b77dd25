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
constexpr int FR_TMP = 40 * 1024;      // LDS bytes of the horizontal pass's rows (2 workgroups per CU)
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

// grid (ceil(S / rb), N), 256 threads.  out: TO_F32 -> [N][3][S][S] normalised fp32,
// else [N][S][S][3] uint8.
template <bool TO_F32>
__global__ __launch_bounds__(256) void frames_resize_crop_kernel(const uint8_t *__restrict__ src,
                                                                 const int64_t *__restrict__ geom, int S, int rb,
                                                                 FrNorm nm, void *__restrict__ out) {
  __shared__ int hk[FR_KMAX * FR_SMAX];      // [k][column] (lanes read consecutive columns)
  __shared__ int hx[FR_SMAX], hn[FR_SMAX];
  __shared__ int vk[FR_KMAX * 64];
  __shared__ int vy[64], vn[64];
  __shared__ __attribute__((aligned(16))) uint8_t tmp[FR_TMP];
  const int tid = threadIdx.x, n = blockIdx.y;
  const int y_beg = blockIdx.x * rb;
  const int rows = S - y_beg < rb ? S - y_beg : rb;
  if (rows <= 0) return;
  const FrGeom g = fr_geom(geom, n);
  for (int c = tid; c < S; c += blockDim.x) {
    int cnt;
    hx[c] = fr_coeffs(g.w, g.nw, g.ox + c, hk + c, FR_SMAX, cnt);
    hn[c] = cnt;
  }
  for (int r = tid; r < rows; r += blockDim.x) {
    int cnt;
    vy[r] = fr_coeffs(g.h, g.nh, g.oy + y_beg + r, vk + r, 64, cnt);
    vn[r] = cnt;
  }
  __syncthreads();
  const int y0 = vy[0], y1 = vy[rows - 1] + vn[rows - 1];   // both monotone in the row
  const int R = y1 - y0;
  if (R * S * 3 > FR_TMP) return;                           // the planner keeps R within LDS
  // horizontal pass: source rows y0 .. y1 of the crop, the S output columns
  const uint8_t *base = src + g.off + (int64_t)g.t * g.stride + (int64_t)g.l * 3;
  for (int i = tid; i < R * S; i += blockDim.x) {
    const int r = i / S, c = i - r * S;
    const uint8_t *p = base + (int64_t)(y0 + r) * g.stride + hx[c] * 3;
    int a0 = 1 << (FR_PREC - 1), a1 = a0, a2 = a0;
    const int cnt = hn[c];
    for (int k = 0; k < cnt; ++k) {
      const int w = hk[k * FR_SMAX + c];
      a0 += (int)p[3 * k] * w;
      a1 += (int)p[3 * k + 1] * w;
      a2 += (int)p[3 * k + 2] * w;
    }
    uint8_t *q = tmp + i * 3;
    q[0] = (uint8_t)fr_clip8(a0);
    q[1] = (uint8_t)fr_clip8(a1);
    q[2] = (uint8_t)fr_clip8(a2);
  }
  __syncthreads();
  // vertical pass from LDS
  for (int i = tid; i < rows * S; i += blockDim.x) {
    const int r = i / S, c = i - r * S;
    const uint8_t *p = tmp + ((vy[r] - y0) * S + c) * 3;
    int a0 = 1 << (FR_PREC - 1), a1 = a0, a2 = a0;
    const int cnt = vn[r];
    for (int k = 0; k < cnt; ++k) {
      const int w = vk[k * 64 + r];
      a0 += (int)p[k * S * 3] * w;
      a1 += (int)p[k * S * 3 + 1] * w;
      a2 += (int)p[k * S * 3 + 2] * w;
    }
    const unsigned u[3] = {fr_clip8(a0), fr_clip8(a1), fr_clip8(a2)};
    const int y = y_beg + r;
    if (TO_F32) {
      float *o = reinterpret_cast<float *>(out) + (int64_t)n * 3 * S * S + (int64_t)y * S + c;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) o[(int64_t)ch * S * S] = ((float)u[ch] / 255.0f - nm.mean[ch]) / nm.inv[ch];
    } else {
      uint8_t *o = reinterpret_cast<uint8_t *>(out) + (((int64_t)n * S + y) * S + c) * 3;
      o[0] = (uint8_t)u[0];
      o[1] = (uint8_t)u[1];
      o[2] = (uint8_t)u[2];
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

static FrNorm fr_norm(const float *mean_std) {
  FrNorm nm;
  for (int c = 0; c < 3; ++c) { nm.mean[c] = mean_std[c]; nm.inv[c] = mean_std[3 + c]; }
  return nm;
}

}  // namespace ewvit

using namespace ewvit;

extern "C" int ewvit_frames_plan(const int64_t *geom, int64_t n, int S, int64_t nbytes) {
  if (!geom || n <= 0 || S <= 0 || S > FR_SMAX) {
    set_error("frames_plan: bad arguments (n %lld, S %d; S <= %d)", (long long)n, S, FR_SMAX);
    return -EWVIT_EINVAL;
  }
  int rb = 16;   // 14 bands of a 224-row output: ~900 workgroups for 64 frames
  for (int64_t i = 0; i < n; ++i) {
    const int64_t *p = geom + i * FR_GEOM;
    const int l = (int)p[2], t = (int)p[3], w = (int)p[4], h = (int)p[5];
    const int nw = (int)p[6], nh = (int)p[7], ox = (int)p[8], oy = (int)p[9];
    if (w <= 0 || h <= 0 || l < 0 || t < 0 || p[0] < 0 || p[1] < 3 * (int64_t)(l + w) || nw < S || nh < S ||
        ox < 0 || oy < 0 || ox + S > nw || oy + S > nh || p[0] + (t + h - 1) * p[1] + 3 * (int64_t)(l + w) > nbytes) {
      set_error("frames_plan: frame %lld: bad geometry (box %d,%d %dx%d, resize %dx%d, crop at %d,%d, S %d)",
                (long long)i, l, t, w, h, nw, nh, ox, oy, S);
      return -EWVIT_EINVAL;
    }
    // taps per output sample: support = max(scale, 1) -> 2 * ceil(support) + 1 <= FR_KMAX
    if (w > 8 * (int64_t)nw || h > 8 * (int64_t)nh) {
      set_error("frames_plan: frame %lld: downscale %dx%d -> %dx%d beyond 8x", (long long)i, w, h, nw, nh);
      return -EWVIT_EINVAL;
    }
    while (rb > 1 && fr_band_rows(h, nh, oy, S, rb) * S * 3 > FR_TMP) rb >>= 1;
    if (fr_band_rows(h, nh, oy, S, rb) * S * 3 > FR_TMP) {
      set_error("frames_plan: frame %lld: one output row needs more source rows than LDS holds", (long long)i);
      return -EWVIT_EINVAL;
    }
  }
  return rb;
}

extern "C" int ewvit_frames_resize_crop(const uint8_t *frames, const int64_t *geom, int64_t n, int S, int rb,
                                        int to_f32, const float *mean_std, void *out, void *stream) {
  EWVIT_CHECK_ARG(frames && geom && out && n > 0, "frames_resize_crop: null pointer or empty batch");
  EWVIT_CHECK_ARG(S > 0 && S <= FR_SMAX && rb >= 1 && rb <= 64, "frames_resize_crop: S %d / rb %d out of range", S, rb);
  EWVIT_CHECK_ARG(!to_f32 || mean_std, "frames_resize_crop: normalised output needs mean_std");
  const float one[6] = {0.f, 0.f, 0.f, 1.f, 1.f, 1.f};
  const FrNorm nm = fr_norm(mean_std ? mean_std : one);
  const dim3 grid((unsigned)((S + rb - 1) / rb), (unsigned)n);
  if (to_f32)
    hipLaunchKernelGGL(frames_resize_crop_kernel<true>, grid, dim3(256), 0, as_stream(stream), frames, geom, S, rb, nm,
                       out);
  else
    hipLaunchKernelGGL(frames_resize_crop_kernel<false>, grid, dim3(256), 0, as_stream(stream), frames, geom, S, rb, nm,
                       out);
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
