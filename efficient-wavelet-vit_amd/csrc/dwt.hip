// Multi-level Haar DWT and the fused HF bilinear upsample (gfx950).
//
// Replaces network/mwt.py:20,76-81 (pytorch_wavelets DWTForward(J=1,'haar','zero')
// per level + reshape + F.interpolate(bilinear, align_corners=False)).
//
// dwt_multilevel_kernel: one workgroup = one 32x32 input tile of one (n,c)
// plane.  The tile is read from HBM once (coalesced 16-B loads) into LDS; every
// level is then an LDS-staged row pass followed by a column pass, its LL
// written back to LDS for the next level, its three HF bands stored straight to
// their planes.  Algorithmic HBM traffic = one read of x + one write of every
// band (602,112 B/frame at 224^2, bf16 out, fp32 in adds 301,056).
#include "common.h"

namespace ewvit {

constexpr int DWT_TILE = 32;
// float32(1/sqrt(2)), the haar dec_lo/dec_hi magnitude pytorch_wavelets stores
constexpr float HAAR_S = 0.70710677f;

template <int XDT, int ODT>
__global__ __launch_bounds__(256) void dwt_multilevel_kernel(const void *__restrict__ x,
                                                             void *__restrict__ yh,
                                                             void *__restrict__ ll, int H,
                                                             int W, int C, int levels,
                                                             int64_t nplanes) {
  __shared__ float tile[2][DWT_TILE][DWT_TILE + 1];
  const int tid = threadIdx.x;
  const int64_t plane = blockIdx.z;  // n*C + c
  const int y0 = blockIdx.y * DWT_TILE, x0 = blockIdx.x * DWT_TILE;

  // ---- load: 32 rows x 32 cols, 4 consecutive pixels per thread
  {
    const int r = tid >> 3, c4 = (tid & 7) * 4;
    const int gy = y0 + r, gx = x0 + c4;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (gy < H) {
      const int64_t base = (plane * H + gy) * (int64_t)W + gx;
      if (XDT == EWVIT_F32 && gx + 3 < W && ((base & 3) == 0)) {
        const float4 q = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(x) + base);
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
      } else if (XDT == EWVIT_BF16 && gx + 3 < W && ((base & 3) == 0)) {
        const uint2 q = *reinterpret_cast<const uint2 *>(reinterpret_cast<const bf16_t *>(x) + base);
        v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
        v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (gx + i < W) v[i] = Elem<XDT>::load(x, base + i);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) tile[0][r][c4 + i] = v[i];
  }
  __syncthreads();

  // ---- levels: row pass then column pass, exactly AFB2D's two fp32 passes
  const int n = (int)(plane / C), c = (int)(plane % C);
  int hl = H, wl = W;     // size of this level's input plane
  int64_t yh_off = 0;     // offset of this level's yh block
  int S = DWT_TILE;       // tile extent at this level's input
  int ty = y0, tx = x0;   // tile origin at this level's input resolution
  int buf = 0;
  for (int lv = 0; lv < levels; ++lv) {
    const int ho = (hl + 1) >> 1, wo = (wl + 1) >> 1;
    const int So = S >> 1;
    const int oy0 = ty >> 1, ox0 = tx >> 1;
    if (tid < So * So) {
      const int i = tid / So, j = tid % So;
      const float a = tile[buf][2 * i][2 * j], b = tile[buf][2 * i][2 * j + 1];
      const float cc = tile[buf][2 * i + 1][2 * j], d = tile[buf][2 * i + 1][2 * j + 1];
      const float s = HAAR_S;
      // row pass (dim 3): even row 2i and odd row 2i+1
      const float lo0 = __fadd_rn(__fmul_rn(s, a), __fmul_rn(s, b));
      const float hi0 = __fsub_rn(__fmul_rn(s, a), __fmul_rn(s, b));
      const float lo1 = __fadd_rn(__fmul_rn(s, cc), __fmul_rn(s, d));
      const float hi1 = __fsub_rn(__fmul_rn(s, cc), __fmul_rn(s, d));
      // column pass (dim 2)
      const float LL = __fadd_rn(__fmul_rn(s, lo0), __fmul_rn(s, lo1));
      const float B0 = __fsub_rn(__fmul_rn(s, lo0), __fmul_rn(s, lo1));  // (W-lo,H-hi)
      const float B1 = __fadd_rn(__fmul_rn(s, hi0), __fmul_rn(s, hi1));  // (W-hi,H-lo)
      const float B2 = __fsub_rn(__fmul_rn(s, hi0), __fmul_rn(s, hi1));  // (W-hi,H-hi)
      tile[buf ^ 1][i][j] = LL;
      const int gy = oy0 + i, gx = ox0 + j;
      if (gy < ho && gx < wo) {
        const int64_t hw = (int64_t)ho * wo;
        const int64_t o = yh_off + ((int64_t)(n * C + c) * 3) * hw + (int64_t)gy * wo + gx;
        Elem<ODT>::store(yh, o, B0);
        Elem<ODT>::store(yh, o + hw, B1);
        Elem<ODT>::store(yh, o + 2 * hw, B2);
        if (lv == levels - 1) Elem<ODT>::store(ll, plane * hw + (int64_t)gy * wo + gx, LL);
      }
    }
    __syncthreads();
    yh_off += nplanes * 3 * (int64_t)ho * wo;
    hl = ho; wl = wo; S = So; ty = oy0; tx = ox0; buf ^= 1;
  }
}

// ---- fused HF reshape + bilinear upsample to (OH, OW), channels-last output.
// One thread = one output pixel of one level, all 3C channels.  Source index
// arithmetic is PyTorch's upsample_bilinear2d (align_corners=False): src =
// max(scale*(dst+0.5)-0.5, 0), scale = in/out in f32.
template <int IDT, int ODT, int CH>
__global__ __launch_bounds__(256) void hf_upsample_kernel(const void *__restrict__ yh,
                                                          void *__restrict__ out, int N, int C,
                                                          int H, int W, int levels, int OH,
                                                          int OW, int64_t total, int ocs) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int ox = (int)(idx % OW);
  int64_t t = idx / OW;
  const int oy = (int)(t % OH);
  t /= OH;
  const int n = (int)(t % N);
  const int lv = (int)(t / N);
  // level geometry + yh offset
  int hl = H, wl = W;
  int64_t off = 0;
  for (int l = 0; l < lv; ++l) {
    hl = (hl + 1) >> 1; wl = (wl + 1) >> 1;
    off += (int64_t)N * C * 3 * hl * wl;
  }
  hl = (hl + 1) >> 1; wl = (wl + 1) >> 1;
  const float sh = (float)hl / (float)OH, sw = (float)wl / (float)OW;
  float fy = sh * ((float)oy + 0.5f) - 0.5f;
  float fx = sw * ((float)ox + 0.5f) - 0.5f;
  fy = fy < 0.f ? 0.f : fy;
  fx = fx < 0.f ? 0.f : fx;
  const int y0 = (int)fy, x0 = (int)fx;
  const int yp = y0 < hl - 1 ? 1 : 0, xp = x0 < wl - 1 ? 1 : 0;
  const float ly1 = fy - (float)y0, ly0 = 1.f - ly1;
  const float lx1 = fx - (float)x0, lx0 = 1.f - lx1;
  const int64_t hw = (int64_t)hl * wl;
  const int64_t p00 = (int64_t)y0 * wl + x0;
  const int64_t base = off + (int64_t)n * 3 * C * hw;
  const int nch = (CH > 0) ? CH : 3 * C;
  const int64_t obase = idx * ocs;          // ocs >= 3C: padded channel stride, pad = 0
  if (CH == 9 && ODT == EWVIT_BF16 && ocs == 16) {
    // the 9 bands + 7 zero channels of the hf_conv input: two 16-B stores per pixel
    float v[9];
#pragma unroll
    for (int ch = 0; ch < 9; ++ch) {
      const int64_t pb = base + ch * hw + p00;
      const float v00 = Elem<IDT>::load(yh, pb), v01 = Elem<IDT>::load(yh, pb + xp);
      const float v10 = Elem<IDT>::load(yh, pb + yp * wl), v11 = Elem<IDT>::load(yh, pb + yp * wl + xp);
      v[ch] = ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11);
    }
    unsigned w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float a = 2 * k < 9 ? v[2 * k] : 0.f, b = 2 * k + 1 < 9 ? v[2 * k + 1] : 0.f;
      w[k] = (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
    }
    uint4 *o = reinterpret_cast<uint4 *>(reinterpret_cast<bf16_t *>(out) + obase);
    o[0] = make_uint4(w[0], w[1], w[2], w[3]);
    o[1] = make_uint4(w[4], w[5], w[6], w[7]);
    return;
  }
  for (int ch = 0; ch < nch; ++ch) {
    const int64_t pb = base + ch * hw + p00;
    const float v00 = Elem<IDT>::load(yh, pb), v01 = Elem<IDT>::load(yh, pb + xp);
    const float v10 = Elem<IDT>::load(yh, pb + yp * wl), v11 = Elem<IDT>::load(yh, pb + yp * wl + xp);
    const float v = ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11);
    Elem<ODT>::store(out, obase + ch, v);
  }
  for (int ch = nch; ch < ocs; ++ch) Elem<ODT>::store(out, obase + ch, 0.f);
}

}  // namespace ewvit

using namespace ewvit;

extern "C" int ewvit_dwt_haar_fwd(const void *x, void *yh, void *ll, int64_t N, int64_t C,
                                  int64_t H, int64_t W, int levels, int x_dtype, int out_dtype,
                                  void *stream) {
  EWVIT_CHECK_ARG(x && yh && ll, "dwt_haar_fwd: null pointer");
  EWVIT_CHECK_ARG(N > 0 && C > 0 && H > 0 && W > 0, "dwt_haar_fwd: empty input [%lld,%lld,%lld,%lld]",
                  (long long)N, (long long)C, (long long)H, (long long)W);
  EWVIT_CHECK_ARG(levels >= 1 && levels <= 5, "dwt_haar_fwd: levels=%d not in [1,5]", levels);
  EWVIT_CHECK_ARG(dtype_ok(x_dtype) && dtype_ok(out_dtype), "dwt_haar_fwd: bad dtype");
  EWVIT_CHECK_ARG(H < (1 << 30) && W < (1 << 30), "dwt_haar_fwd: plane too large");
  const int64_t planes = N * C;
  EWVIT_CHECK_ARG(planes <= 65535, "dwt_haar_fwd: N*C=%lld exceeds 65535", (long long)planes);
  dim3 block(256);
  dim3 grid((unsigned)((W + DWT_TILE - 1) / DWT_TILE), (unsigned)((H + DWT_TILE - 1) / DWT_TILE),
            (unsigned)planes);
  hipStream_t s = as_stream(stream);
#define DWT_LAUNCH(XD, OD)                                                                     \
  hipLaunchKernelGGL((dwt_multilevel_kernel<XD, OD>), grid, block, 0, s, x, yh, ll, (int)H,   \
                     (int)W, (int)C, levels, planes)
  if (x_dtype == EWVIT_F32 && out_dtype == EWVIT_F32) DWT_LAUNCH(EWVIT_F32, EWVIT_F32);
  else if (x_dtype == EWVIT_F32 && out_dtype == EWVIT_BF16) DWT_LAUNCH(EWVIT_F32, EWVIT_BF16);
  else if (x_dtype == EWVIT_BF16 && out_dtype == EWVIT_F32) DWT_LAUNCH(EWVIT_BF16, EWVIT_F32);
  else DWT_LAUNCH(EWVIT_BF16, EWVIT_BF16);
#undef DWT_LAUNCH
  return launch_status("dwt_haar_fwd");
}

extern "C" int ewvit_hf_upsample(const void *yh, void *out, int64_t N, int64_t C, int64_t H,
                                 int64_t W, int levels, int64_t OH, int64_t OW, int in_dtype,
                                 int out_dtype, int64_t out_channels, void *stream) {
  EWVIT_CHECK_ARG(yh && out, "hf_upsample: null pointer");
  if (out_channels == 0) out_channels = 3 * C;
  EWVIT_CHECK_ARG(out_channels >= 3 * C && out_channels <= 4096, "hf_upsample: out_channels %lld < 3C",
                  (long long)out_channels);
  EWVIT_CHECK_ARG(N > 0 && C > 0 && H > 0 && W > 0 && OH > 0 && OW > 0, "hf_upsample: empty shape");
  EWVIT_CHECK_ARG(levels >= 1 && levels <= 5, "hf_upsample: levels=%d not in [1,5]", levels);
  EWVIT_CHECK_ARG(dtype_ok(in_dtype) && dtype_ok(out_dtype), "hf_upsample: bad dtype");
  const int64_t total = (int64_t)levels * N * OH * OW;
  dim3 block(256), grid((unsigned)((total + 255) / 256));
  hipStream_t s = as_stream(stream);
#define UP_LAUNCH(ID, OD, CHN)                                                                  \
  hipLaunchKernelGGL((hf_upsample_kernel<ID, OD, CHN>), grid, block, 0, s, yh, out, (int)N,    \
                     (int)C, (int)H, (int)W, levels, (int)OH, (int)OW, total, (int)out_channels)
  const bool c3 = (C == 3);
  if (in_dtype == EWVIT_F32 && out_dtype == EWVIT_F32) { if (c3) UP_LAUNCH(EWVIT_F32, EWVIT_F32, 9); else UP_LAUNCH(EWVIT_F32, EWVIT_F32, 0); }
  else if (in_dtype == EWVIT_F32) { if (c3) UP_LAUNCH(EWVIT_F32, EWVIT_BF16, 9); else UP_LAUNCH(EWVIT_F32, EWVIT_BF16, 0); }
  else if (out_dtype == EWVIT_F32) { if (c3) UP_LAUNCH(EWVIT_BF16, EWVIT_F32, 9); else UP_LAUNCH(EWVIT_BF16, EWVIT_F32, 0); }
  else { if (c3) UP_LAUNCH(EWVIT_BF16, EWVIT_BF16, 9); else UP_LAUNCH(EWVIT_BF16, EWVIT_BF16, 0); }
#undef UP_LAUNCH
  return launch_status("hf_upsample");
}
