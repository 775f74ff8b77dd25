// Multi-level Haar DWT and the fused HF bilinear upsample (gfx950).
//
// Replaces network/mwt.py:20,76-81 (pytorch_wavelets DWTForward(J=1,'haar','zero')
// per level + reshape + F.interpolate(bilinear, align_corners=False)).
//
// dwt_multilevel_kernel: one workgroup = one 32-row strip (up to 256 columns) of one
// (n,c) plane.  The strip is read from HBM once (coalesced 16-B loads) into LDS; every
// level is then an LDS-staged row pass followed by a column pass, its LL
// written back to LDS for the next level, its three HF bands stored straight to
// their planes.  Algorithmic HBM traffic = one read of x + one write of every
// band (602,112 B/frame at 224^2, bf16 out, fp32 in adds 301,056).
#include "common.h"

namespace ewvit {

constexpr int DWT_TH = 32;      // strip height: a multiple of 2^levels (levels <= 5)
constexpr int DWT_TWMAX = 256;  // strip width (runtime, a multiple of 32)
// float32(1/sqrt(2)), the haar dec_lo/dec_hi magnitude pytorch_wavelets stores
constexpr float HAAR_S = 0.70710677f;

// store v[0..1] at o, o+1 (second only if two): one 4-B bf16x2 / 8-B f32x2 store
// when both are present and the pair is aligned
template <int ODT>
__device__ __forceinline__ void store_pair(void *p, int64_t o, float v0, float v1, bool two) {
  if (two && (o & 1) == 0) {
    if (ODT == EWVIT_BF16) {
      const uint32_t w = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
      *reinterpret_cast<uint32_t *>(reinterpret_cast<bf16_t *>(p) + o) = w;
    } else {
      *reinterpret_cast<float2 *>(reinterpret_cast<float *>(p) + o) = make_float2(v0, v1);
    }
    return;
  }
  Elem<ODT>::store(p, o, v0);
  if (two) Elem<ODT>::store(p, o + 1, v1);
}

// 4 consecutive pixels of row gy from column gx (zero outside the plane)
template <int XDT>
__device__ __forceinline__ float4 load4(const void *x, int64_t plane, int gy, int gx, int H, int W) {
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (gy >= H || gx >= W) return r;
  const int64_t base = (plane * H + gy) * (int64_t)W + gx;
  if (XDT == EWVIT_F32 && gx + 3 < W && ((base & 3) == 0))
    return *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(x) + base);
  if (XDT == EWVIT_BF16 && gx + 3 < W && ((base & 3) == 0)) {
    const uint2 q = *reinterpret_cast<const uint2 *>(reinterpret_cast<const bf16_t *>(x) + base);
    return make_float4(__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                       __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u));
  }
  r.x = Elem<XDT>::load(x, base);
  if (gx + 1 < W) r.y = Elem<XDT>::load(x, base + 1);
  if (gx + 2 < W) r.z = Elem<XDT>::load(x, base + 2);
  if (gx + 3 < W) r.w = Elem<XDT>::load(x, base + 3);
  return r;
}

// one Haar 2x2 step, AFB2D's two fp32 passes in their order: row pass (dim 3) over
// (a b / c d), then the column pass (dim 2).  Every product rounded before its sum (no FMA
// contraction: the result must not depend on the calling kernel)
__device__ __forceinline__ void haar2x2(float a, float b, float cc, float d, float &LL, float &B0, float &B1,
                                        float &B2) {
#pragma clang fp contract(off)
  const float s = HAAR_S;
  const float lo0 = s * a + s * b;
  const float hi0 = s * a - s * b;
  const float lo1 = s * cc + s * d;
  const float hi1 = s * cc - s * d;
  LL = s * lo0 + s * lo1;
  B0 = s * lo0 - s * lo1;  // (W-lo,H-hi)
  B1 = s * hi0 + s * hi1;  // (W-hi,H-lo)
  B2 = s * hi0 - s * hi1;  // (W-hi,H-hi)
}

// One workgroup = one 32-row x tw-column strip of one (n,c) plane (tw = the whole
// 224-pixel row at config 2: 1344 workgroups).  Level 1 runs from registers: an item
// is a 2-row x 4-column patch (two coalesced 16-B loads, up to 4 items = 8 loads in
// flight per thread) -> 2 output pixels, bands stored as 4-B bf16x2 pairs along output
// rows, LL to LDS.  Levels 2.. run over LDS (<= 10 KB per workgroup, so ~8 resident per
// CU and the whole grid in one round), ping-ponging between two LL buffers.
template <int XDT, int ODT>
__global__ __launch_bounds__(256) void dwt_multilevel_kernel(const void *__restrict__ x,
                                                             void *__restrict__ yh,
                                                             void *__restrict__ ll, int H,
                                                             int W, int C, int levels,
                                                             int64_t nplanes, int tw) {
  __shared__ float bufB[(DWT_TH / 2) * (DWT_TWMAX / 2 + 1)];
  __shared__ float bufA[(DWT_TH / 4) * (DWT_TWMAX / 4 + 1)];
  const int tid = threadIdx.x;
  const int64_t plane = blockIdx.z;  // n*C + c
  const int y0 = blockIdx.y * DWT_TH, x0 = blockIdx.x * tw;
  const int n = (int)(plane / C), c = (int)(plane % C);

  // ---- level 1 from registers
  int hl = H, wl = W;
  int ho = (hl + 1) >> 1, wo = (wl + 1) >> 1;
  {
    const int nq = tw >> 2, items = (DWT_TH / 2) * nq, dp = (tw >> 1) + 1;
    float4 r0[4], r1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int it = tid + k * 256;
      if (it < items) {
        const int i = it / nq, q = it - i * nq;
        r0[k] = load4<XDT>(x, plane, y0 + 2 * i, x0 + 4 * q, H, W);
        r1[k] = load4<XDT>(x, plane, y0 + 2 * i + 1, x0 + 4 * q, H, W);
      }
    }
    const int64_t hw = (int64_t)ho * wo;
    const int64_t ob = ((int64_t)(n * C + c) * 3) * hw;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int it = tid + k * 256;
      if (it >= items) continue;
      const int i = it / nq, q = it - i * nq;
      float L0, L1, a0, a1, b0, b1, c0, c1;
      haar2x2(r0[k].x, r0[k].y, r1[k].x, r1[k].y, L0, a0, b0, c0);
      haar2x2(r0[k].z, r0[k].w, r1[k].z, r1[k].w, L1, a1, b1, c1);
      bufB[i * dp + 2 * q] = L0;
      bufB[i * dp + 2 * q + 1] = L1;
      const int gy = (y0 >> 1) + i, gx = (x0 >> 1) + 2 * q;
      if (gy < ho && gx < wo) {
        const bool two = gx + 1 < wo;
        const int64_t o = ob + (int64_t)gy * wo + gx;
        store_pair<ODT>(yh, o, a0, a1, two);
        store_pair<ODT>(yh, o + hw, b0, b1, two);
        store_pair<ODT>(yh, o + 2 * hw, c0, c1, two);
        if (levels == 1) store_pair<ODT>(ll, plane * hw + (int64_t)gy * wo + gx, L0, L1, two);
      }
    }
  }
  __syncthreads();

  // ---- levels 2..: row pass then column pass over LDS
  int64_t yh_off = nplanes * 3 * (int64_t)ho * wo;   // offset of this level's yh block
  hl = ho; wl = wo;
  int Sh = DWT_TH / 2, Sw = tw >> 1;   // strip extent at this level's input
  int ty = y0 >> 1, tx = x0 >> 1;      // strip origin at this level's input resolution
  for (int lv = 1; lv < levels; ++lv) {
    const float *src = (lv & 1) ? bufB : bufA;
    float *dst = (lv & 1) ? bufA : bufB;
    const int sp = Sw + 1, Soh = Sh >> 1, Sow = Sw >> 1, dp = Sow + 1;
    ho = (hl + 1) >> 1; wo = (wl + 1) >> 1;
    const int oy0 = ty >> 1, ox0 = tx >> 1;
    const int npair = (Sow + 1) >> 1, items = Soh * npair;
    const int64_t hw = (int64_t)ho * wo;
    const int64_t ob = yh_off + ((int64_t)(n * C + c) * 3) * hw;
    for (int it = tid; it < items; it += 256) {
      const int i = it / npair, j0 = (it - i * npair) * 2;
      float L[2], B0[2], B1[2], B2[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int j = j0 + e < Sow ? j0 + e : j0;
        haar2x2(src[(2 * i) * sp + 2 * j], src[(2 * i) * sp + 2 * j + 1], src[(2 * i + 1) * sp + 2 * j],
                src[(2 * i + 1) * sp + 2 * j + 1], L[e], B0[e], B1[e], B2[e]);
      }
      dst[i * dp + j0] = L[0];
      if (j0 + 1 < Sow) dst[i * dp + j0 + 1] = L[1];
      const int gy = oy0 + i, gx = ox0 + j0;
      if (gy < ho && gx < wo) {
        const bool two = j0 + 1 < Sow && gx + 1 < wo;
        const int64_t o = ob + (int64_t)gy * wo + gx;
        store_pair<ODT>(yh, o, B0[0], B0[1], two);
        store_pair<ODT>(yh, o + hw, B1[0], B1[1], two);
        store_pair<ODT>(yh, o + 2 * hw, B2[0], B2[1], two);
        if (lv == levels - 1) store_pair<ODT>(ll, plane * hw + (int64_t)gy * wo + gx, L[0], L[1], two);
      }
    }
    __syncthreads();
    yh_off += nplanes * 3 * (int64_t)ho * wo;
    hl = ho; wl = wo; Sh = Soh; Sw = Sow; ty = oy0; tx = ox0;
  }
}

// PyTorch upsample_bilinear2d (align_corners=False) source coordinate of output index o:
// src = max(scale*(o+0.5)-0.5, 0), scale = in/out in f32; explicit FMAs so the two-launch
// path and the fused kernel below round identically
struct Lerp {
  int i0, ip;      // first source index, step to the second (0 at the last index)
  float w0, w1;
};
__device__ __forceinline__ Lerp lerp_src(int o, int in, int out) {
  const float sc = (float)in / (float)out;
  float f = fmaf(sc, (float)o + 0.5f, -0.5f);
  f = f < 0.f ? 0.f : f;
  Lerp l;
  l.i0 = (int)f;
  l.ip = l.i0 < in - 1 ? 1 : 0;
  l.w1 = f - (float)l.i0;
  l.w0 = 1.f - l.w1;
  return l;
}
__device__ __forceinline__ float bilerp(float v00, float v01, float v10, float v11, const Lerp &ly, const Lerp &lx) {
  const float r0 = fmaf(lx.w0, v00, lx.w1 * v01);
  const float r1 = fmaf(lx.w0, v10, lx.w1 * v11);
  return fmaf(ly.w0, r0, ly.w1 * r1);
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
  const Lerp ly = lerp_src(oy, hl, OH), lx = lerp_src(ox, wl, OW);
  const int yp = ly.ip, xp = lx.ip;
  const int64_t hw = (int64_t)hl * wl;
  const int64_t p00 = (int64_t)ly.i0 * wl + lx.i0;
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
      v[ch] = bilerp(v00, v01, v10, v11, ly, lx);
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
    Elem<ODT>::store(out, obase + ch, bilerp(v00, v01, v10, v11, ly, lx));
  }
  for (int ch = nch; ch < ocs; ++ch) Elem<ODT>::store(out, obase + ch, 0.f);
}

// ---- fused DWT -> HF bilinear upsample (3 colour planes): the MWT's hf_conv
// input of every level, [levels][N][H/2][W/2][ocs] channels-last (9 band channels, the rest
// zero), straight from the frames — the bands never go to HBM.  Same values, bit for bit,
// as dwt_multilevel_kernel (bands rounded to the output type) + hf_upsample_kernel.
//
// One workgroup = 16 level-1 output rows of one frame, full width.  Level l's bilinear
// upsample to level-1 resolution (scale 2^(1-l)) reads one level-l row beyond the strip on
// each side, so the workgroup computes a window of 16 + 2*HALO level-1 rows (HALO = 2^(L-1)
// level-1 rows = one level-L row): 48 input rows for L = 3, the halo rows' loads mostly
// L2 hits of the neighbouring strips.  Level 1 runs from registers (a thread = one level-1
// pixel of all 3 planes: six 8-B loads, 9 bands -> one 32-B store for the strip's own rows,
// LL to LDS); levels 2..L run over LDS (bands rounded to the output type, LL in fp32); the
// upsample pass then gathers 4 x 9 band values per output pixel from LDS.
constexpr int DWTF_ROWS = 16;       // level-1 output rows per workgroup

template <int ODT>
__device__ __forceinline__ float rnd_out(float v) {
  return ODT == EWVIT_BF16 ? bf2f(f2bf(v)) : v;
}

// 9 (or 16 with zero padding) channels of one output pixel
template <int ODT>
__device__ __forceinline__ void store_px9(void *out, int64_t o, const float (&v)[9], int ocs) {
  if (ODT == EWVIT_BF16 && ocs == 9) {
    // the 9 band channels only (18 B per pixel): four 4-B stores and one 2-B store, the 2-B one
    // first or last as the pixel's offset is odd or even
    unsigned short h[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) h[k] = f2bf(v[k]);
    bf16_t *b = reinterpret_cast<bf16_t *>(out) + o;
    const int s = (int)(o & 1);             // 1: channel 0 alone, then pairs (1,2) .. (7,8)
    if (s) b[0] = h[0];
    else b[8] = h[8];
    unsigned *w = reinterpret_cast<unsigned *>(b + s);
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = (unsigned)h[s + 2 * k] | ((unsigned)h[s + 2 * k + 1] << 16);
    return;
  }
  if (ODT == EWVIT_BF16 && ocs == 16) {
    unsigned w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float a = 2 * k < 9 ? v[2 * k] : 0.f, b = 2 * k + 1 < 9 ? v[2 * k + 1] : 0.f;
      w[k] = (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
    }
    uint4 *q = reinterpret_cast<uint4 *>(reinterpret_cast<bf16_t *>(out) + o);
    q[0] = make_uint4(w[0], w[1], w[2], w[3]);
    q[1] = make_uint4(w[4], w[5], w[6], w[7]);
    return;
  }
#pragma unroll
  for (int ch = 0; ch < 9; ++ch) Elem<ODT>::store(out, o + ch, v[ch]);
  for (int ch = 9; ch < ocs; ++ch) Elem<ODT>::store(out, o + ch, 0.f);
}

// two consecutive pixels of a row (an 8-B / 4-B load: W even, column even)
template <int XDT>
__device__ __forceinline__ float2 load2(const void *x, int64_t i) {
  if (XDT == EWVIT_F32) return *reinterpret_cast<const float2 *>(reinterpret_cast<const float *>(x) + i);
  const unsigned q = *reinterpret_cast<const unsigned *>(reinterpret_cast<const bf16_t *>(x) + i);
  return make_float2(__uint_as_float(q << 16), __uint_as_float(q & 0xffff0000u));
}

template <int XDT, int ODT, int L, int OWMAX, int NT, int ROWS = DWTF_ROWS, int PF = 2>
__global__ __launch_bounds__(NT) void dwt_hf_fused_kernel(const void *__restrict__ x, void *__restrict__ out,
                                                           int N, int H, int W, int ocs) {
  constexpr int HALO = L > 1 ? (1 << (L - 1)) : 0;      // level-1 rows
  constexpr int R1 = ROWS + 2 * HALO;              // level-1 window rows
  constexpr int R2 = L >= 2 ? R1 / 2 : 1, R3 = L >= 3 ? R1 / 4 : 1;
  constexpr int O2 = OWMAX / 2, O3 = OWMAX / 4;
  constexpr int S1 = L >= 2 ? R1 * OWMAX * 3 : 1, S2 = L >= 2 ? R2 * O2 * 9 : 1, S3 = L >= 3 ? R2 * O2 * 3 : 1;
  constexpr int S4 = L >= 3 ? R3 * O3 * 9 : 1;
  __shared__ __attribute__((aligned(16))) float sm[S1 + S2 + S3 + S4];
  float *ll1 = sm, *b2 = sm + S1, *ll2 = b2 + S2, *b3 = ll2 + S3;
  const int OH = H >> 1, OW = W >> 1;
  // one-dimensional grid, XCD-aware: the blocks one XCD receives (b, b + 8, ...) take consecutive
  // (frame, strip) ids, so a strip's halo rows are mostly the L2 lines its neighbour strip, on the
  // same XCD, loads (round-robin strips put every neighbour on another XCD's L2)
  const int nstrip = (OH + ROWS - 1) / ROWS;
  int sid;
  {
    const int bid = blockIdx.x, nwg = gridDim.x;
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    sid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int tid = threadIdx.x, n = sid / nstrip;
  const int y0 = (sid - n * nstrip) * ROWS;        // first level-1 output row
  const int ws1 = y0 - HALO;                            // window origin, level-1 rows
  const int64_t plane = (int64_t)H * W;
  const char *xn = reinterpret_cast<const char *>(x) + (int64_t)n * 3 * plane * (XDT == EWVIT_BF16 ? 2 : 4);
  const int64_t lvl = (int64_t)N * OH * OW * ocs;       // one level's output block
  // 9 output channels (18 B per pixel): a strip level's ROWS x OW x 9 bf16 output is staged in LDS
  // and written as 16-B vectors (the strip is contiguous in the output) — level 1 through the
  // b2 / ll2 space (free until level 2), the upsampled levels through ll1 (free after level 2)
  constexpr int STG = ROWS * OWMAX * 9 / 2;             // staged floats per strip level
  const bool stg9 = ODT == EWVIT_BF16 && L == 3 && S2 + S3 >= STG && S1 >= STG && ocs == 9 && (OW % 8) == 0;
  unsigned short *st1 = reinterpret_cast<unsigned short *>(b2), *stu = reinterpret_cast<unsigned short *>(ll1);
  const int srows = OH - y0 < ROWS ? OH - y0 : ROWS;
  // copy a staged strip level (srows x OW x 9 bf16) to its contiguous place in the output
  auto flush9 = [&](const unsigned short *src, int64_t dst_elem) {
    const int n16 = srows * OW * 9 / 8;
    const uint4 *sp = reinterpret_cast<const uint4 *>(src);
    uint4 *dp = reinterpret_cast<uint4 *>(reinterpret_cast<bf16_t *>(out) + dst_elem);
    for (int t = tid; t < n16; t += NT) dp[t] = sp[t];
  };

  // ---- level 1 (registers): PF pixels per thread in flight
  {
    const int items = R1 * OW;
    for (int i0 = tid; i0 < items; i0 += PF * NT) {
      float2 r[PF][3][2];
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        const int it = i0 + k * NT;
        const int i = it / OW, j = it - i * OW, y = ws1 + i;
        if (it < items && y >= 0 && y < OH) {
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const int64_t b = c * plane + (int64_t)(2 * y) * W + 2 * j;
            r[k][c][0] = load2<XDT>(xn, b);
            r[k][c][1] = load2<XDT>(xn, b + W);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        const int it = i0 + k * NT;
        const int i = it / OW, j = it - i * OW, y = ws1 + i;
        if (!(it < items && y >= 0 && y < OH)) continue;
        float v[9];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          float LL, B0, B1, B2;
          haar2x2(r[k][c][0].x, r[k][c][0].y, r[k][c][1].x, r[k][c][1].y, LL, B0, B1, B2);
          v[3 * c] = B0; v[3 * c + 1] = B1; v[3 * c + 2] = B2;
          if (L >= 2) ll1[(i * OWMAX + j) * 3 + c] = LL;
        }
        if (i >= HALO && i < HALO + ROWS) {
          if (stg9) {
            unsigned short *q = st1 + ((i - HALO) * OW + j) * 9;
#pragma unroll
            for (int ch = 0; ch < 9; ++ch) q[ch] = f2bf(v[ch]);
          } else {
            store_px9<ODT>(out, (((int64_t)n * OH + y) * OW + j) * ocs, v, ocs);
          }
        }
      }
    }
  }
  if constexpr (L >= 2) {
    __syncthreads();
    if (stg9) {
      flush9(st1, ((int64_t)n * OH + y0) * OW * 9);
      __syncthreads();                              // b2 / ll2 staged data read before level 2 writes them
    }
    // ---- level 2 over LDS: window rows ws2 .. ws2 + R2
    const int OH2 = OH >> 1, OW2 = OW >> 1, ws2 = ws1 >> 1;
    for (int it = tid; it < R2 * OW2; it += NT) {
      const int i = it / OW2, j = it - i * OW2, y = ws2 + i;
      if (y < 0 || y >= OH2) continue;
      const float *p0 = ll1 + ((2 * i) * OWMAX + 2 * j) * 3, *p1 = p0 + OWMAX * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float LL, B0, B1, B2;
        haar2x2(p0[c], p0[3 + c], p1[c], p1[3 + c], LL, B0, B1, B2);
        float *q = b2 + (i * O2 + j) * 9 + 3 * c;
        q[0] = rnd_out<ODT>(B0); q[1] = rnd_out<ODT>(B1); q[2] = rnd_out<ODT>(B2);
        if (L >= 3) ll2[(i * O2 + j) * 3 + c] = LL;
      }
    }
    if constexpr (L >= 3) {
      __syncthreads();
      const int OH3 = OH2 >> 1, OW3 = OW2 >> 1, ws3 = ws2 >> 1;
      for (int it = tid; it < R3 * OW3; it += NT) {
        const int i = it / OW3, j = it - i * OW3, y = ws3 + i;
        if (y < 0 || y >= OH3) continue;
        const float *p0 = ll2 + ((2 * i) * O2 + 2 * j) * 3, *p1 = p0 + O2 * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          float LL, B0, B1, B2;
          haar2x2(p0[c], p0[3 + c], p1[c], p1[3 + c], LL, B0, B1, B2);
          float *q = b3 + (i * O3 + j) * 9 + 3 * c;
          q[0] = rnd_out<ODT>(B0); q[1] = rnd_out<ODT>(B1); q[2] = rnd_out<ODT>(B2);
        }
      }
    }
    __syncthreads();
    // ---- levels 2..L upsampled to the strip's level-1 rows
    const int rows = OH - y0 < ROWS ? OH - y0 : ROWS;
    const int items = rows * OW;
    if (stg9) {
      // one level at a time through ll1 (free now: level 2 has read it)
      for (int l = 2; l <= L; ++l) {
        for (int r = tid; r < items; r += NT) {
          const int oy = y0 + r / OW, ox = r - (r / OW) * OW;
          const int hl = OH >> (l - 1), wl = OW >> (l - 1);
          const Lerp ly = lerp_src(oy, hl, OH), lx = lerp_src(ox, wl, OW);
          const float *bb = l == 2 ? b2 : b3;
          const int ow = l == 2 ? O2 : O3, ws = l == 2 ? ws2 : (ws1 >> 2);
          const float *q00 = bb + ((ly.i0 - ws) * ow + lx.i0) * 9;
          const float *q01 = q00 + lx.ip * 9, *q10 = q00 + ly.ip * ow * 9, *q11 = q10 + lx.ip * 9;
          unsigned short *q = stu + r * 9;
#pragma unroll
          for (int ch = 0; ch < 9; ++ch) q[ch] = f2bf(bilerp(q00[ch], q01[ch], q10[ch], q11[ch], ly, lx));
        }
        __syncthreads();
        flush9(stu, (l - 1) * lvl + ((int64_t)n * OH + y0) * OW * 9);
        __syncthreads();
      }
      return;
    }
    for (int it = tid; it < (L - 1) * items; it += NT) {
      const int l = 2 + it / items, r = it - (l - 2) * items;
      const int oy = y0 + r / OW, ox = r - (r / OW) * OW;
      const int hl = OH >> (l - 1), wl = OW >> (l - 1);
      const Lerp ly = lerp_src(oy, hl, OH), lx = lerp_src(ox, wl, OW);
      const float *bb = l == 2 ? b2 : b3;
      const int ow = l == 2 ? O2 : O3, ws = l == 2 ? ws2 : (ws1 >> 2);
      const float *q00 = bb + ((ly.i0 - ws) * ow + lx.i0) * 9;
      const float *q01 = q00 + lx.ip * 9, *q10 = q00 + ly.ip * ow * 9, *q11 = q10 + lx.ip * 9;
      float v[9];
#pragma unroll
      for (int ch = 0; ch < 9; ++ch) v[ch] = bilerp(q00[ch], q01[ch], q10[ch], q11[ch], ly, lx);
      store_px9<ODT>(out, (l - 1) * lvl + (((int64_t)n * OH + oy) * OW + ox) * ocs, v, ocs);
    }
  }
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
  // strip width: the whole row when it fits (rounded up to 32), else the multiple of 32 in
  // [128, 256] that wastes the fewest columns
  int tw = (int)((W + 31) / 32 * 32);
  if (tw > DWT_TWMAX) {
    int64_t best = -1;
    for (int c = DWT_TWMAX; c >= 128; c -= 32) {
      const int64_t waste = (W + c - 1) / c * c - W;
      if (best < 0 || waste < best) { best = waste; tw = c; }
    }
  }
  dim3 block(256);
  dim3 grid((unsigned)((W + tw - 1) / tw), (unsigned)((H + DWT_TH - 1) / DWT_TH), (unsigned)planes);
  hipStream_t s = as_stream(stream);
#define DWT_LAUNCH(XD, OD)                                                                     \
  hipLaunchKernelGGL((dwt_multilevel_kernel<XD, OD>), grid, block, 0, s, x, yh, ll, (int)H,   \
                     (int)W, (int)C, levels, planes, tw)
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

// the fused DWT -> HF upsample applies: 3 planes, every level halves exactly (H, W multiples
// of 2^levels), output at level-1 resolution, levels <= 3, W/2 <= 112, 9..16 output channels.
// (A 192-column form for config 4's 384^2 frames needed 121 KB of LDS — one workgroup per CU
// — and ran 61 us against the two launches' 58 us: wider frames keep the two launches.)
extern "C" int ewvit_dwt_hf_fused_ok(int64_t N, int64_t C, int64_t H, int64_t W, int levels, int64_t OH, int64_t OW,
                                     int64_t out_channels) {
  const int64_t m = (int64_t)1 << (levels < 1 ? 1 : levels);
  return N > 0 && N <= 65535 && C == 3 && levels >= 1 && levels <= 3 && H > 0 && W > 0 && H % m == 0 &&
         W % m == 0 && OH == H / 2 && OW == W / 2 && OW <= 112 && out_channels >= 9 && out_channels <= 16;
}

// level-1 pixels per thread in flight: 2 (104 VGPRs: two 512-thread workgroups per CU, so the 448
// strips of config 2 are resident at once) measured 30.2 -> 23.5 us (9 channels) and 32.2 -> 25.7 us
// (16) against 4 (196 VGPRs, one workgroup per CU); EWVIT_DWTF_PF=4: the A/B
static int g_dwtf_pf = 2;
extern "C" int ewvit_dwt_set_pf(int pf) {
  const int prev = g_dwtf_pf;
  g_dwtf_pf = pf == 4 ? 4 : 2;
  return prev;
}

extern "C" int ewvit_dwt_hf_upsample_fused(const void *x, void *out, int64_t N, int64_t C, int64_t H, int64_t W,
                                           int levels, int x_dtype, int out_dtype, int64_t out_channels,
                                           void *stream) {
  EWVIT_CHECK_ARG(x && out, "dwt_hf_upsample_fused: null pointer");
  EWVIT_CHECK_ARG(dtype_ok(x_dtype) && dtype_ok(out_dtype), "dwt_hf_upsample_fused: bad dtype");
  EWVIT_CHECK_ARG(ewvit_dwt_hf_fused_ok(N, C, H, W, levels, H / 2, W / 2, out_channels),
                  "dwt_hf_upsample_fused: unsupported shape [%lld,%lld,%lld,%lld] levels=%d channels=%lld",
                  (long long)N, (long long)C, (long long)H, (long long)W, levels, (long long)out_channels);
  const int OH = (int)(H / 2);
  // 512 threads over 16-row strips (29.9 -> 26.5 us at config 2 against 256 threads; 1024: 29.7;
  // 8-row strips 31-33 us, 32-row strips on 1024 threads 26.3 us: profiles/r02/ab/dwtf_rows.log)
  constexpr int nt = 512, rows = 16;
  dim3 grid((unsigned)((OH + rows - 1) / rows * N)), block(nt);
  hipStream_t s = as_stream(stream);
#define DWTF_L(XD, OD, LV)                                                                                    \
  do {                                                                                                        \
    if (g_dwtf_pf == 4)                                                                                       \
      hipLaunchKernelGGL((dwt_hf_fused_kernel<XD, OD, LV, 112, nt, rows, 4>), grid, block, 0, s, x, out, (int)N, \
                         (int)H, (int)W, (int)out_channels);                                                  \
    else                                                                                                      \
      hipLaunchKernelGGL((dwt_hf_fused_kernel<XD, OD, LV, 112, nt, rows, 2>), grid, block, 0, s, x, out, (int)N, \
                         (int)H, (int)W, (int)out_channels);                                                  \
  } while (0)
#define DWTF_D(XD, OD)                        \
  do {                                        \
    if (levels == 1) DWTF_L(XD, OD, 1);       \
    else if (levels == 2) DWTF_L(XD, OD, 2);  \
    else DWTF_L(XD, OD, 3);                   \
  } while (0)
  if (x_dtype == EWVIT_F32 && out_dtype == EWVIT_BF16) DWTF_D(EWVIT_F32, EWVIT_BF16);
  else if (x_dtype == EWVIT_F32) DWTF_D(EWVIT_F32, EWVIT_F32);
  else if (out_dtype == EWVIT_BF16) DWTF_D(EWVIT_BF16, EWVIT_BF16);
  else DWTF_D(EWVIT_BF16, EWVIT_F32);
#undef DWTF_D
#undef DWTF_L
  return launch_status("dwt_hf_upsample_fused");
}
