// The MWT "seperate" convs — reference network/mwt.py:48-59 builds three
// Conv2d(3, 18, 3, padding=1) + BatchNorm2d(18) + ReLU, and mwt.py:84-86 applies
// hf_conv['seperate'][g] to hf[:, 3g:3g+3], colour g's three HF bands (channel c*3+band of
// the reshaped yh, mwt.py:77), with the weights shared by every DWT level (mwt.py:108).
//
// Layouts (all levels in one launch, level-major images, NI = levels * N):
//   x  [NI][H][W][16] bf16 — the fused DWT -> upsample output: channel 3g+ci real for
//      g, ci < 3, channels 9..15 zero
//   y  [NI][H][W][64] bf16 — channel 18g+o for o < 18 (54 real), channels 54..63 zero: whole
//      64-channel K slices for the fusion conv that reads it
//   w_g [18][3][3][3] fp32 (the modules' own parameters), b_g [18] fp32
//
// Arithmetic per pixel: 3 groups x 18 outputs x 27 taps = 1458 MACs.  Both directions are
// HBM-bound (the forward reads 32 B and writes 128 B per pixel, the weight gradient reads
// 128 + 32 B), so the MFMA tiles run dense over the 16 x 64 channel block (the zero lanes
// ride along in tiles the bandwidth already pays for) and what the kernels save is HBM
// passes:
//   fwd    y and, per level, the BatchNorm partial sums of the rounded y (shifted by the
//          running mean) for ewvit_bn_fwd_partials — the statistics pass over y never runs;
//          weights read straight from the three fp32 parameters (no pack launch, no
//          block-diagonal weight assembled by the host);
//   wgrad  one pass over dy and x: a workgroup stages a band of TH rows (dy rows and the x
//          rows with their halo) in LDS, its 4 waves each own 16 dy channels and reduce over
//          the band's pixels with v_mfma_f32_16x16x32_bf16 (A = dy^T, B = x per tap, both
//          read transposed with ds_read_b64_tr_b16 from the natural [pixel][channel]
//          images); the bias gradient comes from a ones channel (x channel 15 set to 1.0 in
//          LDS: its centre-tap column is sum dy).  Persistent over bands; per-workgroup
//          partial slabs summed in a fixed order by one small reduce launch (deterministic)
//          that also scatters the three groups' blocks into the parameters' gradients.
#include "common.h"

#include <cstdlib>

namespace ewvit {

typedef __attribute__((ext_vector_type(8))) __bf16 hbf16x8;
typedef __attribute__((ext_vector_type(4))) float hf32x4;
typedef __attribute__((ext_vector_type(4))) short hs4;

constexpr int HS_CIN = 16, HS_COUT = 64, HS_G = 3, HS_GO = 18, HS_GI = 3;
constexpr int HS_REAL = HS_G * HS_GO;            // 54
constexpr int HS_K = 9 * HS_CIN;                 // 144 GEMM columns of the weight gradient

struct HsParams {
  const float *w[3];
  const float *b[3];
};

// ---------------------------------------------------------------- forward (+ BN partials)
// grid (G, L): block (bx, l) walks bands bx, bx + G, ... of level l (TH output rows of one
// image each).  A lane ends each 16-pixel group with 4 consecutive output channels of one
// pixel per 16-channel tile (weights-first MFMA operands), which it stores (8 B) and adds
// into its running shifted sums; the block reduces them over its pixels at the end:
// part[l][bx][c] = sum (y - K_c), part[l][bx][64 + c] = sum (y - K_c)^2.
template <int TH>
__global__ __launch_bounds__(256) void hfsep_fwd_kernel(const bf16_t *__restrict__ x, bf16_t *__restrict__ y,
                                                        HsParams p, int Nl, int H, int W,
                                                        const float *__restrict__ shift, float *__restrict__ part,
                                                        float *__restrict__ shift_out) {
  constexpr int CC = HS_CIN / 8, NCH = 9 * CC, KSTEPS = (NCH + 3) / 4, NT = HS_COUT / 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char hs_smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lvl = blockIdx.y;
  const int Wp = W + 2, rowb = Wp * HS_CIN * 2;
  // weights as the MFMA A operand: lane -> output channel n = 16t + (lane & 15), 8-channel
  // chunk kc = 4s + (lane >> 4) of tap kc / 2; w_g[o][ci][tap] sits at input channel 3g + ci
  hbf16x8 wf[NT][KSTEPS];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      const int n = t * 16 + (lane & 15), kc = 4 * s + (lane >> 4);
      const int tap = kc / CC, c0 = (kc % CC) * 8;
      unsigned short e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        float v = 0.f;
        if (n < HS_REAL && kc < NCH && c < HS_G * HS_GI) {
          const int g = n / HS_GO, o = n - g * HS_GO;
          if (c / HS_GI == g) v = p.w[g][(o * HS_GI + (c - g * HS_GI)) * 9 + tap];
        }
        e[j] = f2bf(v);
      }
      const uint4 u = make_uint4(e[0] | ((unsigned)e[1] << 16), e[2] | ((unsigned)e[3] << 16),
                                 e[4] | ((unsigned)e[5] << 16), e[6] | ((unsigned)e[7] << 16));
      wf[t][s] = __builtin_bit_cast(hbf16x8, u);
    }
  float bias[NT][4], K[NT][4], s1[NT][4], s2[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = t * 16 + 4 * (lane >> 4) + i;
      const int g = n / HS_GO;
      bias[t][i] = n < HS_REAL ? p.b[g][n - g * HS_GO] : 0.f;
      K[t][i] = (shift && n < HS_REAL) ? shift[n] : 0.f;
      s1[t][i] = 0.f;
      s2[t][i] = 0.f;
    }
  const int nbh = (H + TH - 1) / TH, nbands = Nl * nbh;
  for (int band = blockIdx.x; band < nbands; band += gridDim.x) {
    const int img = lvl * Nl + band / nbh, r0 = (band % nbh) * TH;
    const int rows = H - r0 < TH ? H - r0 : TH;
    const int items = (TH + 2) * Wp * CC;
    __syncthreads();                               // the previous band's readers are done
    for (int i = tid; i < items; i += 256) {
      const int c8 = i % CC, px = i / CC;
      const int tr = px / Wp, tc = px - tr * Wp;
      const int ir = r0 - 1 + tr, ic = tc - 1;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if ((unsigned)ir < (unsigned)H && (unsigned)ic < (unsigned)W && tr < rows + 2)
        v = *reinterpret_cast<const uint4 *>(x + (((int64_t)img * H + ir) * W + ic) * HS_CIN + c8 * 8);
      *reinterpret_cast<uint4 *>(hs_smem + (size_t)tr * rowb + (tc * HS_CIN + c8 * 8) * 2) = v;
    }
    __syncthreads();
    const int npx = rows * W, ngr = (npx + 15) / 16;
    for (int gi = w; gi < ngr; gi += 4) {
      const int q = gi * 16 + (lane & 15);
      const int qq = q < npx ? q : npx - 1;
      const int r = qq / W, c = qq - r * W;
      hf32x4 acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = hf32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        const int kc = 4 * s + (lane >> 4);
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (kc < NCH) {
          const int tap = kc / CC, c8 = kc - tap * CC;
          const int kh = tap / 3, kw = tap - kh * 3;
          v = *reinterpret_cast<const uint4 *>(hs_smem + (size_t)(r + kh) * rowb + ((c + kw) * HS_CIN + c8 * 8) * 2);
        }
        const hbf16x8 xf = __builtin_bit_cast(hbf16x8, v);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][s], xf, acc[t], 0, 0, 0);
      }
      if (q < npx) {
        bf16_t *o = y + (((int64_t)img * H + r0 + r) * W + c) * HS_COUT;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          bf16_t h[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            h[i] = f2bf(acc[t][i] + bias[t][i]);
            const float d = bf2f(h[i]) - K[t][i];
            s1[t][i] += d;
            s2[t][i] += d * d;
          }
          const int n = t * 16 + 4 * (lane >> 4);
          *reinterpret_cast<uint2 *>(o + n) =
              make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
        }
      }
    }
  }
  if (!part) return;
  // the 16 lanes of a DPP row hold the same 4 channels of different pixels
  __syncthreads();
  float *red = reinterpret_cast<float *>(hs_smem);   // [4 waves][64 channels][2]
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float a = row_sum16(s1[t][i]), b = row_sum16(s2[t][i]);
      if ((lane & 15) == 0) {
        const int n = t * 16 + 4 * (lane >> 4) + i;
        red[(w * HS_COUT + n) * 2] = a;
        red[(w * HS_COUT + n) * 2 + 1] = b;
      }
    }
  __syncthreads();
  if (tid < HS_COUT) {
    const float a = (red[(0 * HS_COUT + tid) * 2] + red[(1 * HS_COUT + tid) * 2]) +
                    (red[(2 * HS_COUT + tid) * 2] + red[(3 * HS_COUT + tid) * 2]);
    const float b = (red[(0 * HS_COUT + tid) * 2 + 1] + red[(1 * HS_COUT + tid) * 2 + 1]) +
                    (red[(2 * HS_COUT + tid) * 2 + 1] + red[(3 * HS_COUT + tid) * 2 + 1]);
    float *dst = part + ((int64_t)lvl * gridDim.x + blockIdx.x) * 2 * HS_COUT;
    dst[tid] = a;
    dst[HS_COUT + tid] = b;
    if (blockIdx.x == 0) shift_out[lvl * HS_COUT + tid] = (shift && tid < HS_REAL) ? shift[tid] : 0.f;
  }
}

// ---------------------------------------------------------------- weight gradient
// GEMM view: C[co][tap*16 + c] = sum_p dy[p][co] x[pix(p, tap)][c] over the band's pixels.
// K order inside a 32-pixel K-step: MFMA k = 8g + 4hh + q (g = lane >> 4, hh = lo / hi
// read, q < 4) is pixel p0 + 4g + 16hh + q, so the two 16-lane groups of a 32-lane half
// read 8 consecutive pixels — x rows (32 B) then hit 64 distinct banks without a swizzle,
// and the dy rows (128 B) with the chunk XOR dsw(r) = 2((r >> 1) & 3).
// dy image: Pk rows (the band's TH*W pixels rounded up to 32; rows past the band zero).
// x image: the band's rows plus a halo row above and below, each W + 2 pixels with a zero
// column either side, 32 B per pixel; one zero pixel after them for the padding rows.
// The next band's global loads are issued into registers before the current band's MFMAs
// (one register stage), then written to LDS after them.
__device__ __forceinline__ int hs_dsw(int r) { return ((r >> 1) & 3) << 1; }

// DYI / XI: register-staged 16-B pieces per thread (dy, x): 7 / 4 cover W <= 112 at TH = 2
// (the MWT's 112^2 levels), 13 / 7 cover W <= 200 (config 4's 192^2)
template <int TH, int DYI, int XI>
__global__ __launch_bounds__(256) void hfsep_wgrad_kernel(const bf16_t *__restrict__ x, const bf16_t *__restrict__ dy,
                                                          float *__restrict__ part, int NI, int H, int W) {
  extern __shared__ __attribute__((aligned(16))) unsigned char hs_smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);    // dy channels 16 wv .. 16 wv + 15
  const int Wp = W + 2;
  const int Pk = (TH * W + 31) & ~31;
  const int nhalo = (TH + 2) * Wp;
  unsigned char *dimg = hs_smem;
  unsigned char *ximg = hs_smem + Pk * 128;
  const int zoff = nhalo * 32;                                // the zero pixel
  const int gq = (lane & 15) >> 2, gp = lane & 3, grp = lane >> 4;
  const int chk = 2 * wv + (gp >> 1);
  hf32x4 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = hf32x4{0.f, 0.f, 0.f, 0.f};
  if (tid < 2) *reinterpret_cast<uint4 *>(ximg + zoff + tid * 16) = make_uint4(0u, 0u, 0u, 0u);
  const int nbh = (H + TH - 1) / TH, nbands = NI * nbh;
  const int ndy = Pk * 8, nx = nhalo * 2;
  uint4 rd[DYI], rx[XI];
  auto fetch = [&](int band) {
    const int img = band / nbh, r0 = (band % nbh) * TH;
    const int rows = H - r0 < TH ? H - r0 : TH;
    const int Pb = rows * W;
    const bf16_t *dsrc = dy + ((int64_t)img * H + r0) * W * HS_COUT;
#pragma unroll
    for (int k = 0; k < DYI; ++k) {
      const int i = tid + 256 * k;
      rd[k] = make_uint4(0u, 0u, 0u, 0u);
      if (i < ndy && (i >> 3) < Pb) rd[k] = *reinterpret_cast<const uint4 *>(dsrc + (int64_t)(i >> 3) * HS_COUT + (i & 7) * 8);
    }
#pragma unroll
    for (int k = 0; k < XI; ++k) {
      const int i = tid + 256 * k;
      rx[k] = make_uint4(0u, 0u, 0u, 0u);
      if (i < nx) {
        const int h = i >> 1, c = i & 1;
        const int hr = h / Wp, hc = h - hr * Wp;
        const int ir = r0 - 1 + hr, ic = hc - 1;
        if ((unsigned)ir < (unsigned)H && (unsigned)ic < (unsigned)W && hr < rows + 2) {
          rx[k] = *reinterpret_cast<const uint4 *>(x + (((int64_t)img * H + ir) * W + ic) * HS_CIN + c * 8);
          if (c == 1) rx[k].w = (rx[k].w & 0xffffu) | 0x3f800000u;   // channel 15 := 1.0 (bias column)
        }
      }
    }
  };
  if ((int)blockIdx.x < nbands) fetch(blockIdx.x);
  for (int band = blockIdx.x; band < nbands; band += gridDim.x) {
    const int rows = H - (band % nbh) * TH < TH ? H - (band % nbh) * TH : TH;
    const int Pb = rows * W;
    __syncthreads();                               // the previous band's readers are done
#pragma unroll
    for (int k = 0; k < DYI; ++k) {
      const int i = tid + 256 * k;
      if (i < ndy) *reinterpret_cast<uint4 *>(dimg + (i >> 3) * 128 + 16 * ((i & 7) ^ hs_dsw(i >> 3))) = rd[k];
    }
#pragma unroll
    for (int k = 0; k < XI; ++k) {
      const int i = tid + 256 * k;
      if (i < nx) *reinterpret_cast<uint4 *>(ximg + i * 16) = rx[k];
    }
    __syncthreads();
    if (band + (int)gridDim.x < nbands) fetch(band + gridDim.x);   // in flight under the MFMAs
    // this lane's pixels of K-step 0: lo p = 4 grp + gq, hi p + 16; tracked as (row, col)
    int pr[2], rr[2], cc[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      pr[hh] = 4 * grp + 16 * hh + gq;
      rr[hh] = pr[hh] / W;
      cc[hh] = pr[hh] - rr[hh] * W;
    }
    for (int k0 = 0; k0 < Pk; k0 += 32) {
      hs4 av[2];
      int xb[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int r = pr[hh];
        av[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) hs4 *)(dimg + r * 128 + 16 * (chk ^ hs_dsw(r)) + 8 * (gp & 1)));
        xb[hh] = r < Pb ? (rr[hh] * Wp + cc[hh]) * 32 + 8 * gp : zoff + 8 * gp;   // tap (0, 0)
      }
      const hbf16x8 af = __builtin_bit_cast(hbf16x8, (__attribute__((ext_vector_type(8))) short){
                                                         av[0][0], av[0][1], av[0][2], av[0][3], av[1][0], av[1][1], av[1][2], av[1][3]});
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int kh = tap / 3, kw = tap - kh * 3;
        const int toff = (kh * Wp + kw) * 32;
        hs4 b[2];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
          b[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) hs4 *)(ximg + (pr[hh] < Pb ? xb[hh] + toff : xb[hh])));
        const hbf16x8 bf = __builtin_bit_cast(hbf16x8, (__attribute__((ext_vector_type(8))) short){
                                                           b[0][0], b[0][1], b[0][2], b[0][3], b[1][0], b[1][1], b[1][2], b[1][3]});
        acc[tap] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[tap], 0, 0, 0);
      }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        pr[hh] += 32;
        cc[hh] += 32;
        while (cc[hh] >= W) {
          cc[hh] -= W;
          ++rr[hh];
        }
      }
    }
  }
  // C[16 wv + 4 grp + r][tap * 16 + (lane & 15)]
  float *dst = part + (int64_t)blockIdx.x * HS_COUT * HS_K;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      dst[(int64_t)(16 * wv + 4 * grp + r) * HS_K + tap * 16 + (lane & 15)] = acc[tap][r];
}

// dW_g[o][ci][tap] = sum_b part[b][18g + o][tap * 16 + 3g + ci]; db_g[o] = sum_b
// part[b][18g + o][4 * 16 + 15] (the ones channel at the centre tap).  Block: 64 outputs x
// 4 slab quarters, combined in a fixed order.
__global__ __launch_bounds__(256) void hfsep_wgrad_reduce_kernel(const float *__restrict__ part, int G, HsParams out) {
  __shared__ float red[4][64];
  const int tid = threadIdx.x, o64 = tid & 63, qtr = tid >> 6;
  const int idx = blockIdx.x * 64 + o64;              // 0 .. 54*27 + 54
  constexpr int NW = HS_REAL * 27;
  int co = 0, col = 0;
  const bool live = idx < NW + HS_REAL;
  if (live) {
    if (idx < NW) {
      co = idx / 27;
      const int k = idx - co * 27, ci = k / 9, tap = k - ci * 9;
      col = tap * 16 + (co / HS_GO) * HS_GI + ci;
    } else {
      co = idx - NW;
      col = 4 * 16 + 15;
    }
  }
  float s = 0.f;
  if (live)
    for (int b = qtr; b < G; b += 4) s += part[((int64_t)b * HS_COUT + co) * HS_K + col];
  red[qtr][o64] = s;
  __syncthreads();
  if (qtr == 0 && live) {
    const float v = (red[0][o64] + red[1][o64]) + (red[2][o64] + red[3][o64]);
    const int g = co / HS_GO, o = co - g * HS_GO;
    if (idx < NW) {
      if (out.w[g]) const_cast<float *>(out.w[g])[o * 27 + (idx - co * 27)] = v;
    } else if (out.b[g]) {
      const_cast<float *>(out.b[g])[o] = v;
    }
  }
}

static int hs_blocks(int64_t work, int cap_default) {
  int64_t g = work < cap_default ? work : cap_default;
  if (g_grid_cap > 0 && g > g_grid_cap) g = g_grid_cap;
  return g < 1 ? 1 : (int)g;
}

static int hs_fwd_th() { return 8; }
static int hs_wg_th() { return 2; }        // rows per band (1-row bands measured slower)
static int hs_wg_blocks(int64_t NI, int64_t H) {
  constexpr int maxb = 768;                     // 3 resident per CU
  const int th = hs_wg_th();
  return hs_blocks(NI * ((H + th - 1) / th), maxb);
}

}  // namespace ewvit

using namespace ewvit;

static bool hs_geom_ok(int64_t NI, int64_t H, int64_t W) {
  return NI > 0 && H > 0 && W > 0 && W <= 512 && H <= 4096 && NI * H * W < ((int64_t)1 << 31);
}

extern "C" int64_t ewvit_hfsep_fwd_parts(int64_t L, int64_t N, int64_t H, int64_t W) {
  if (L < 1 || N < 1 || !hs_geom_ok(L * N, H, W)) return 0;
  const int th = hs_fwd_th();
  const int64_t bands = N * ((H + th - 1) / th);
  // one partial row per workgroup of the level (<= 256: the BatchNorm apply pass finalises
  // from them directly); all levels together one round of resident workgroups (2 per CU at
  // this kernel's register use), so no level's tail waits for a second round; under a grid
  // cap the levels share it
  constexpr int fwdb = 512;
  int64_t g = fwdb / L > 0 ? fwdb / L : 1;
  if (g > 256) g = 256;
  if (g > bands) g = bands;
  if (g_grid_cap > 0 && g * L > g_grid_cap) g = g_grid_cap / L > 0 ? g_grid_cap / L : 1;
  return g;
}

extern "C" int ewvit_hfsep_fwd(const void *x, void *y, int64_t L, int64_t N, int64_t H, int64_t W, const float *w0,
                               const float *w1, const float *w2, const float *b0, const float *b1, const float *b2,
                               const float *bn_shift, float *bn_part, float *bn_shift_out, int nparts,
                               void *stream) {
  EWVIT_CHECK_ARG(x && y && w0 && w1 && w2 && b0 && b1 && b2, "hfsep_fwd: null pointer");
  EWVIT_CHECK_ARG(L >= 1 && L <= 65535 && N >= 1 && hs_geom_ok(L * N, H, W), "hfsep_fwd: bad geometry L=%lld N=%lld %lldx%lld",
                  (long long)L, (long long)N, (long long)H, (long long)W);
  const int64_t g = ewvit_hfsep_fwd_parts(L, N, H, W);
  EWVIT_CHECK_ARG(!bn_part || (bn_shift_out && nparts == g), "hfsep_fwd: %d partial rows, the launch gives %lld",
                  nparts, (long long)g);
  const int th = hs_fwd_th();
  const size_t lds = (size_t)(th + 2) * (W + 2) * HS_CIN * 2;
  EWVIT_CHECK_ARG(lds <= 64 * 1024, "hfsep_fwd: W=%lld too wide", (long long)W);
  HsParams p{{w0, w1, w2}, {b0, b1, b2}};
  hipLaunchKernelGGL(hfsep_fwd_kernel<8>, dim3((unsigned)g, (unsigned)L), dim3(256), lds, as_stream(stream),
                     (const bf16_t *)x, (bf16_t *)y, p, (int)N, (int)H, (int)W, bn_shift, bn_part, bn_shift_out);
  return launch_status("hfsep_fwd");
}

extern "C" int64_t ewvit_hfsep_bwd_weight_workspace(int64_t NI, int64_t H, int64_t W) {
  if (!hs_geom_ok(NI, H, W)) return 0;
  return (int64_t)hs_wg_blocks(NI, H) * HS_COUT * HS_K * 4;
}

extern "C" int ewvit_hfsep_bwd_weight(const void *x, const void *dy, int64_t NI, int64_t H, int64_t W, float *dw0,
                                      float *dw1, float *dw2, float *db0, float *db1, float *db2, float *workspace,
                                      void *stream) {
  EWVIT_CHECK_ARG(x && dy && workspace, "hfsep_bwd_weight: null pointer");
  EWVIT_CHECK_ARG(hs_geom_ok(NI, H, W), "hfsep_bwd_weight: bad geometry");
  const int th = hs_wg_th();
  const int G = hs_wg_blocks(NI, H);
  const int Pk = (int)((th * W + 31) & ~31);
  // the register stage holds a band's pieces: DYI x 256 dy pieces, XI x 256 x pieces
  const bool small = Pk * 8 <= 7 * 256 && (th + 2) * (W + 2) * 2 <= 4 * 256;
  EWVIT_CHECK_ARG(small || (Pk * 8 <= 13 * 256 && (th + 2) * (W + 2) * 2 <= 7 * 256),
                  "hfsep_bwd_weight: W=%lld too wide for TH=%d", (long long)W, th);
  const size_t lds = (size_t)Pk * 128 + ((size_t)(th + 2) * (W + 2) + 1) * 32;
  hipStream_t s = as_stream(stream);
#define EWVIT_HS_WG(TH_, D_, X_)                                                                                 \
  do {                                                                                                           \
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void *>(hfsep_wgrad_kernel<TH_, D_, X_>), \
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) == hipSuccess; \
    (void)attr;                                                                                                  \
    hipLaunchKernelGGL((hfsep_wgrad_kernel<TH_, D_, X_>), dim3(G), dim3(256), lds, s, (const bf16_t *)x,           \
                       (const bf16_t *)dy, workspace, (int)NI, (int)H, (int)W);                                  \
  } while (0)
  if (small) EWVIT_HS_WG(2, 7, 4); else EWVIT_HS_WG(2, 13, 7);
#undef EWVIT_HS_WG
  int rc = launch_status("hfsep_bwd_weight");
  if (rc) return rc;
  HsParams out{{dw0, dw1, dw2}, {db0, db1, db2}};
  const int nout = HS_REAL * 27 + HS_REAL;
  hipLaunchKernelGGL(hfsep_wgrad_reduce_kernel, dim3((nout + 63) / 64), dim3(256), 0, s, workspace, G, out);
  return launch_status("hfsep_bwd_weight reduce");
}
