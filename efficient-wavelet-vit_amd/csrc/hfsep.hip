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

// non-temporal 16-B load / 8-B store (global ... nt): the MWT's 0.3 GB maps stream through once
typedef __attribute__((ext_vector_type(2))) uint32_t hs_v2u;
typedef __attribute__((ext_vector_type(4))) uint32_t hs_v4u;
__device__ __forceinline__ uint4 hs_ldnt(const bf16_t *p) {
#if EWVIT_MWT_NT
  const hs_v4u v = __builtin_nontemporal_load(reinterpret_cast<const hs_v4u *>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return *reinterpret_cast<const uint4 *>(p);
#endif
}
__device__ __forceinline__ void hs_stnt(bf16_t *p, hs_v2u v) {
#if EWVIT_MWT_NT
  __builtin_nontemporal_store(v, reinterpret_cast<hs_v2u *>(p));
#else
  *reinterpret_cast<hs_v2u *>(p) = v;
#endif
}

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

// 9-channel input (XS 9: the fused DWT front end's 9 real band channels, 18 B per pixel, no zero
// channels in HBM): a pixel PAIR (2q, 2q+1) of a row is 36 B = 9 dwords at a 4-B aligned offset
// (W even).  hs_pair9 rewrites it as the two pixels' 16-channel LDS rows (channels 9..15 zero; one
// = 1.0 at channel 15 for the weight gradient's bias column).
__device__ __forceinline__ void hs_pair9(const unsigned (&w)[9], uint4 &a0, uint4 &a1, uint4 &b0, uint4 &b1,
                                         unsigned c15) {
  a0 = make_uint4(w[0], w[1], w[2], w[3]);
  a1 = make_uint4(w[4] & 0xffffu, 0u, 0u, c15);
  b0 = make_uint4((w[4] >> 16) | (w[5] << 16), (w[5] >> 16) | (w[6] << 16), (w[6] >> 16) | (w[7] << 16),
                  (w[7] >> 16) | (w[8] << 16));
  b1 = make_uint4(w[8] >> 16, 0u, 0u, c15);
}

// ---------------------------------------------------------------- forward (+ BN partials)
// grid (G, L): block (bx, l) walks bands bx, bx + G, ... of level l (TH output rows of one
// image each).  A lane ends each 16-pixel group with 4 consecutive output channels of one
// pixel per 16-channel tile (weights-first MFMA operands), which it stores (8 B) and adds
// into its running shifted sums; the block reduces them over its pixels at the end:
// part[l][bx][c] = sum (y - K_c), part[l][bx][64 + c] = sum (y - K_c)^2.
// A band's x rows are staged through registers: XP 16-B pieces per thread, all issued together
// from clamped in-range addresses (one memory round trip per band, not one per piece).
// XS 9: x has 9 channels per pixel; the band is staged as pixel-pair items (hs_pair9), XP of
// them per thread, plus one zero item per halo row for its two border pixels.
template <int TH, int XP, int XS = 16>
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
  const int items = (TH + 2) * Wp * CC;
  uint4 rx[XP];                                     // (the unused form's registers are dead code)
  unsigned rq[XP][9];
  unsigned okm = 0;                                 // which of this thread's pieces lie in the image
  const int npair = W / 2 + 1, items9 = (TH + 2) * npair;
  auto fetch9 = [&](int band) {
    const int img = lvl * Nl + band / nbh, r0 = (band % nbh) * TH;
    const int rows = H - r0 < TH ? H - r0 : TH;
    okm = 0;
    const unsigned *ximg = reinterpret_cast<const unsigned *>(x + (int64_t)img * H * W * 9);
#pragma unroll
    for (int k = 0; k < XP; ++k) {
      const int i = tid + 256 * k;
      const int tr = i / npair, q = i - tr * npair, ir = r0 - 1 + tr;
      const bool ok = i < items9 && q < W / 2 && (unsigned)ir < (unsigned)H && tr < rows + 2;
      okm |= (unsigned)ok << k;
      const unsigned *p = ximg + (ok ? ((int64_t)ir * W + 2 * q) * 9 / 2 : 0);
#pragma unroll
      for (int e = 0; e < 9; ++e) rq[k][e] = p[e];
    }
  };
  auto stage9 = [&]() {
#pragma unroll
    for (int k = 0; k < XP; ++k) {
      const int i = tid + 256 * k;
      if (i >= items9) continue;
      const int tr = i / npair, q = i - tr * npair;
      uint4 a0, a1, b0, b1;
      if ((okm >> k) & 1u) {
        hs_pair9(rq[k], a0, a1, b0, b1, 0u);
      } else {
        a0 = a1 = b0 = b1 = make_uint4(0u, 0u, 0u, 0u);
      }
      // halo pixels 2q + 1, 2q + 2 (q = W / 2: the row's two border pixels 0 and W + 1, zero)
      const int pa = tr * Wp + (q < W / 2 ? 2 * q + 1 : 0), pb = q < W / 2 ? pa + 1 : tr * Wp + W + 1;
      uint4 *da = reinterpret_cast<uint4 *>(hs_smem + (size_t)pa * HS_CIN * 2);
      uint4 *db = reinterpret_cast<uint4 *>(hs_smem + (size_t)pb * HS_CIN * 2);
      da[0] = a0; da[1] = a1; db[0] = b0; db[1] = b1;
    }
  };
  auto fetch = [&](int band) {
    const int img = lvl * Nl + band / nbh, r0 = (band % nbh) * TH;
    const int rows = H - r0 < TH ? H - r0 : TH;
    okm = 0;
    // piece i = tid + 256 k: pixel px = i / CC of the (TH + 2) x Wp halo image, walked
    // incrementally (256 / CC pixels per step)
    const int c8 = tid % CC;
    int tr = (tid / CC) / Wp, tc = (tid / CC) - tr * Wp;
    const bf16_t *ximg = x + (int64_t)img * H * W * HS_CIN + c8 * 8;
#pragma unroll
    for (int k = 0; k < XP; ++k) {
      const int i = tid + 256 * k;
      const int ir = r0 - 1 + tr, ic = tc - 1;
      const bool ok = i < items && (unsigned)ir < (unsigned)H && (unsigned)ic < (unsigned)W && tr < rows + 2;
      okm |= (unsigned)ok << k;
      // unconditional load from a clamped address (no branch around the load), zeroed below
      rx[k] = *reinterpret_cast<const uint4 *>(ximg + (ok ? ((int64_t)ir * W + ic) * HS_CIN : 0));
      tc += 256 / CC;
      while (tc >= Wp) { tc -= Wp; ++tr; }
    }
  };
  for (int band = blockIdx.x; band < nbands; band += gridDim.x) {
    const int img = lvl * Nl + band / nbh, r0 = (band % nbh) * TH;
    const int rows = H - r0 < TH ? H - r0 : TH;
    if constexpr (XS == 9) fetch9(band);
    else fetch(band);
    __syncthreads();                               // the previous band's readers are done
    if constexpr (XS == 9) {
      stage9();
    } else {
      // LDS image offset of piece i: px * 32 + c8 * 16 bytes (rows of Wp pixels, 16 channels)
      const int c8 = tid % CC;
#pragma unroll
      for (int k = 0; k < XP; ++k) {
        const int i = tid + 256 * k;
        if (i < items) {
          const uint4 v = ((okm >> k) & 1u) ? rx[k] : make_uint4(0u, 0u, 0u, 0u);
          *reinterpret_cast<uint4 *>(hs_smem + (size_t)(i / CC) * HS_CIN * 2 + c8 * 16) = v;
        }
      }
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
          // (non-temporal: the 0.3 GB output map streams to the fusion conv, no L2 reuse)
          hs_stnt(o + n, hs_v2u{(uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16)});
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
// BNB: dy is not given but recomputed per element from the BatchNorm + ReLU that follows the conv
// (the grouped seperate BN, per-level statistics): dz (the gradient of the BN output), yb (the
// BN input = this conv's output) and the per-(level, channel) table `bnt` [L][64][8] give
// dy = gamma invstd (g' - mean(g') - xhat mean(g' xhat)), g' = dz [gamma xhat + beta > 0],
// xhat = (y - mean) invstd, folded to dy = A g' + B y + C and the mask to P y + Q > 0 (table
// {A, B, C, P, Q}) — the BN backward's dx pass, so dy never goes through memory.
// XS 9: 9-channel x staged as pixel-pair items (hs_pair9), XI of them per thread.
template <int TH, int DYI, int XI, bool BNB, int XS = 16>
__global__ __launch_bounds__(256) void hfsep_wgrad_kernel(const bf16_t *__restrict__ x, const bf16_t *__restrict__ dy,
                                                          float *__restrict__ part, int NI, int H, int W,
                                                          const bf16_t *__restrict__ yb, const float *__restrict__ bnt,
                                                          int L, int Nl) {
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
  float *tab = reinterpret_cast<float *>(hs_smem + Pk * 128 + (nhalo + 1) * 32);   // BNB: [L][64][8]
  if (BNB)
    for (int e = tid; e < L * 64 * 8; e += 256) tab[e] = bnt[e];
  const int nbh = (H + TH - 1) / TH, nbands = NI * nbh;
  const int ndy = Pk * 8, nx = nhalo * 2;
  uint4 rd[DYI], ry[BNB ? DYI : 1], rx[XI];
  unsigned rq[XI][9];                          // XS 9 (the unused form's registers are dead code)
  unsigned dok = 0, xok = 0;                   // which pieces are real (the loads are unconditional)
  const int npair = W / 2 + 1, items9 = (TH + 2) * npair;
  auto fetch = [&](int band) {
    const int img = band / nbh, r0 = (band % nbh) * TH;
    const int rows = H - r0 < TH ? H - r0 : TH;
    const int Pb = rows * W;
    const int64_t dbase = ((int64_t)img * H + r0) * W * HS_COUT;
    dok = 0;
    xok = 0;
#pragma unroll
    for (int k = 0; k < DYI; ++k) {
      const int i = tid + 256 * k;
      const bool ok = i < ndy && (i >> 3) < Pb;
      dok |= (unsigned)ok << k;
      const int64_t off = ok ? dbase + (int64_t)(i >> 3) * HS_COUT + (i & 7) * 8 : 0;
      rd[k] = hs_ldnt(dy + off);
      if constexpr (BNB) ry[k] = hs_ldnt(yb + off);
    }
    if constexpr (XS == 9) {
      // pixel pairs (2q, 2q + 1) of the halo rows; item q = W / 2 of a row: its two border pixels
      const unsigned *xi = reinterpret_cast<const unsigned *>(x + (int64_t)img * H * W * 9);
#pragma unroll
      for (int k = 0; k < XI; ++k) {
        const int i = tid + 256 * k;
        const int tr = i / npair, q = i - tr * npair, ir = r0 - 1 + tr;
        const bool ok = i < items9 && q < W / 2 && (unsigned)ir < (unsigned)H && tr < rows + 2;
        xok |= (unsigned)ok << k;
        const unsigned *p = xi + (ok ? ((int64_t)ir * W + 2 * q) * 9 / 2 : 0);
#pragma unroll
        for (int e = 0; e < 9; ++e) rq[k][e] = p[e];
      }
      return;
    }
    // x halo pieces: pixel h = i / 2 of the (TH + 2) x Wp image, walked incrementally
    int hr = (tid >> 1) / Wp, hc = (tid >> 1) - hr * Wp;
    const int c = tid & 1;
#pragma unroll
    for (int k = 0; k < XI; ++k) {
      const int i = tid + 256 * k;
      const int ir = r0 - 1 + hr, ic = hc - 1;
      const bool ok = i < nx && (unsigned)ir < (unsigned)H && (unsigned)ic < (unsigned)W && hr < rows + 2;
      xok |= (unsigned)ok << k;
      rx[k] = *reinterpret_cast<const uint4 *>(x + (ok ? (((int64_t)img * H + ir) * W + ic) * HS_CIN + c * 8 : 0));
      hc += 128;
      while (hc >= Wp) { hc -= Wp; ++hr; }
    }
  };
  if ((int)blockIdx.x < nbands) fetch(blockIdx.x);
  for (int band = blockIdx.x; band < nbands; band += gridDim.x) {
    const int rows = H - (band % nbh) * TH < TH ? H - (band % nbh) * TH : TH;
    const int Pb = rows * W;
    const int lvl = (band / nbh) / Nl;
    // BNB: this thread's 8 channels ((tid & 7) * 8 + j: a piece's channels never change with k)
    // as dy = A g' + B y + C, g' = g [P y + Q > 0]
    float cst[BNB ? 8 : 1][5];
    if constexpr (BNB) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int m = 0; m < 5; ++m) cst[j][m] = tab[(lvl * 64 + (tid & 7) * 8 + j) * 8 + m];
    }
    __syncthreads();                               // the previous band's readers are done
#pragma unroll
    for (int k = 0; k < DYI; ++k) {
      const int i = tid + 256 * k;
      if (i < ndy) {
        uint4 v = ((dok >> k) & 1u) ? rd[k] : make_uint4(0u, 0u, 0u, 0u);
        if constexpr (BNB) {
          if ((dok >> k) & 1u) {
            const unsigned dz[4] = {rd[k].x, rd[k].y, rd[k].z, rd[k].w};
            const unsigned yv[4] = {ry[k].x, ry[k].y, ry[k].z, ry[k].w};
            unsigned o[4];
#pragma unroll
            for (int h = 0; h < 4; ++h) {
              float d2[2];
#pragma unroll
              for (int u = 0; u < 2; ++u) {
                const int j = 2 * h + u;
                const float g = __uint_as_float(u ? dz[h] & 0xffff0000u : dz[h] << 16);
                const float yy = __uint_as_float(u ? yv[h] & 0xffff0000u : yv[h] << 16);
                const float gp = fmaf(cst[j][3], yy, cst[j][4]) > 0.f ? g : 0.f;
                d2[u] = fmaf(cst[j][0], gp, fmaf(cst[j][1], yy, cst[j][2]));
              }
              o[h] = (unsigned)f2bf(d2[0]) | ((unsigned)f2bf(d2[1]) << 16);
            }
            v = make_uint4(o[0], o[1], o[2], o[3]);
          }
        }
        *reinterpret_cast<uint4 *>(dimg + (i >> 3) * 128 + 16 * ((i & 7) ^ hs_dsw(i >> 3))) = v;
      }
    }
    if constexpr (XS == 9) {
#pragma unroll
      for (int k = 0; k < XI; ++k) {
        const int i = tid + 256 * k;
        if (i >= items9) continue;
        const int tr = i / npair, q = i - tr * npair;
        uint4 a0, a1, b0, b1;
        if ((xok >> k) & 1u) {
          hs_pair9(rq[k], a0, a1, b0, b1, 0x3f800000u);   // channel 15 := 1.0 (bias column)
        } else {
          a0 = a1 = b0 = b1 = make_uint4(0u, 0u, 0u, 0u);
        }
        const int pa = tr * Wp + (q < W / 2 ? 2 * q + 1 : 0), pb = q < W / 2 ? pa + 1 : tr * Wp + W + 1;
        uint4 *da = reinterpret_cast<uint4 *>(ximg + pa * 32), *db = reinterpret_cast<uint4 *>(ximg + pb * 32);
        da[0] = a0; da[1] = a1; db[0] = b0; db[1] = b1;
      }
    } else {
#pragma unroll
      for (int k = 0; k < XI; ++k) {
        const int i = tid + 256 * k;
        if (i < nx) {
          uint4 v = ((xok >> k) & 1u) ? rx[k] : make_uint4(0u, 0u, 0u, 0u);
          if ((i & 1) && ((xok >> k) & 1u)) v.w = (v.w & 0xffffu) | 0x3f800000u;   // channel 15 := 1.0 (bias column)
          *reinterpret_cast<uint4 *>(ximg + i * 16) = v;
        }
      }
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
// 16 slab groups (8 loads in flight per thread), combined in a fixed order.
// BNB launches: the last 2 blocks write the grouped BatchNorm's affine gradients, dbeta[c] =
// sum_l sum g', dgamma[c] = sum_l sum g' xhat (lsum [L][128], levels in order).
__global__ __launch_bounds__(1024) void hfsep_wgrad_reduce_kernel(const float *__restrict__ part, int G, HsParams out,
                                                                 const float *__restrict__ lsum = nullptr, int L = 0,
                                                                 float *dgamma = nullptr, float *dbeta = nullptr) {
  __shared__ float red[16][64];
  const int tid = threadIdx.x, o64 = tid & 63, qtr = tid >> 6;   // 16 slab groups of 64 outputs
  const int idx = blockIdx.x * 64 + o64;              // 0 .. 54*27 + 54
  constexpr int NW = HS_REAL * 27;
  if (lsum && (int)blockIdx.x >= (int)gridDim.x - 2) {
    const int which = (int)gridDim.x - 1 - (int)blockIdx.x;      // 1: dbeta, 0: dgamma
    if (qtr == 0) {
      float v = 0.f;
      for (int l = 0; l < L; ++l) v += lsum[l * 128 + (which ? 0 : 64) + o64];   // levels in order
      float *dst = which ? dbeta : dgamma;
      if (dst) dst[o64] = v;
    }
    return;
  }
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
  if (live) {
    // slabs b = qtr + 16 i, 8 loads in flight per step (fixed order)
    const float *src = part + (int64_t)co * HS_K + col;
    const int64_t sstr = (int64_t)HS_COUT * HS_K;
    int b = qtr;
    for (; b + 7 * 16 < G; b += 8 * 16) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(b + 16 * u) * sstr];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < G; b += 16) s += src[(int64_t)b * sstr];
  }
  red[qtr][o64] = s;
  __syncthreads();
  if (qtr == 0 && live) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) v += red[q][o64];
    const int g = co / HS_GO, o = co - g * HS_GO;
    if (idx < NW) {
      if (out.w[g]) const_cast<float *>(out.w[g])[o * 27 + (idx - co * 27)] = v;
    } else if (out.b[g]) {
      const_cast<float *>(out.b[g])[o] = v;
    }
  }
}

// The grouped seperate BatchNorm's backward coefficients per (level, channel) from the partial
// sums left by the fusion conv's input-gradient epilogue (part [L][nrc][128]: sum g' and sum
// g' xhat per channel): the table the BNB weight-gradient kernel reads, and the per-level sums
// for the affine gradients.  One workgroup per level: 8 row slices x 4 loads in flight per
// thread (a latency-bound launch on the MWT's critical path otherwise), summed in a fixed order.
__global__ __launch_bounds__(1024) void hfsep_bn_coef_kernel(const float *__restrict__ part, int nrc, float n,
                                                             const float *__restrict__ mean,
                                                             const float *__restrict__ invstd,
                                                             const float *__restrict__ gamma,
                                                             const float *__restrict__ beta, float *__restrict__ tab,
                                                             float *__restrict__ lsum) {
  __shared__ float red[8][128];
  const int l = blockIdx.x, tid = threadIdx.x, col = tid & 127, q = tid >> 7;
  const float *p = part + (int64_t)l * nrc * 128 + col;
  float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
  int r = q;
  for (; r + 24 < nrc; r += 32) {
    v0 += p[(int64_t)r * 128];
    v1 += p[(int64_t)(r + 8) * 128];
    v2 += p[(int64_t)(r + 16) * 128];
    v3 += p[(int64_t)(r + 24) * 128];
  }
  for (; r < nrc; r += 8) v0 += p[(int64_t)r * 128];
  red[q][col] = (v0 + v1) + (v2 + v3);
  __syncthreads();
  if (tid < 128) {
    const float t = ((red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid])) +
                    ((red[4][tid] + red[5][tid]) + (red[6][tid] + red[7][tid]));
    lsum[l * 128 + tid] = t;
    red[0][tid] = t;                  // (this thread's column only)
  }
  __syncthreads();
  if (tid < 64) {
    const int c = tid;
    const float mu = mean[l * 64 + c], iv = invstd[l * 64 + c];
    const float ga = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
    // dy = gi (g' - a - xhat b) with xhat = (y - mu) iv, gi = gamma iv: A g' + B y + C; the ReLU
    // mask gamma xhat + beta > 0 as P y + Q > 0
    const float a = red[0][c] / n, b = red[0][64 + c] / n, gi = ga * iv;
    float *t = tab + (l * 64 + c) * 8;
    t[0] = gi; t[1] = -gi * b * iv; t[2] = -gi * a + gi * b * iv * mu; t[3] = gi; t[4] = be - gi * mu;
    t[5] = 0.f; t[6] = 0.f; t[7] = 0.f;
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

extern "C" int ewvit_hfsep_fwd(const void *x, void *y, int64_t L, int64_t N, int64_t H, int64_t W, int x_channels, const float *w0,
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
  EWVIT_CHECK_ARG(x_channels == 16 || (x_channels == 9 && W % 2 == 0), "hfsep_fwd: x_channels %d (16, or 9 with W even)",
                  x_channels);
  HsParams p{{w0, w1, w2}, {b0, b1, b2}};
  if (x_channels == 9) {
    // pixel-pair items: (TH + 2) x (W / 2 + 1)
    const int64_t items9 = (int64_t)(th + 2) * (W / 2 + 1);
    EWVIT_CHECK_ARG(items9 <= 4 * 256, "hfsep_fwd: W=%lld too wide for the 9-channel staging", (long long)W);
    if (items9 <= 3 * 256)
      hipLaunchKernelGGL((hfsep_fwd_kernel<8, 3, 9>), dim3((unsigned)g, (unsigned)L), dim3(256), lds, as_stream(stream),
                         (const bf16_t *)x, (bf16_t *)y, p, (int)N, (int)H, (int)W, bn_shift, bn_part, bn_shift_out);
    else
      hipLaunchKernelGGL((hfsep_fwd_kernel<8, 4, 9>), dim3((unsigned)g, (unsigned)L), dim3(256), lds, as_stream(stream),
                         (const bf16_t *)x, (bf16_t *)y, p, (int)N, (int)H, (int)W, bn_shift, bn_part, bn_shift_out);
    return launch_status("hfsep_fwd");
  }
  // the register stage holds a band's (TH + 2) x (W + 2) x 2 x pieces
  const int64_t items = (int64_t)(th + 2) * (W + 2) * 2;
  if (items <= 9 * 256)
    hipLaunchKernelGGL((hfsep_fwd_kernel<8, 9>), dim3((unsigned)g, (unsigned)L), dim3(256), lds, as_stream(stream),
                       (const bf16_t *)x, (bf16_t *)y, p, (int)N, (int)H, (int)W, bn_shift, bn_part, bn_shift_out);
  else
    hipLaunchKernelGGL((hfsep_fwd_kernel<8, 16>), dim3((unsigned)g, (unsigned)L), dim3(256), lds, as_stream(stream),
                       (const bf16_t *)x, (bf16_t *)y, p, (int)N, (int)H, (int)W, bn_shift, bn_part, bn_shift_out);
  return launch_status("hfsep_fwd");
}

extern "C" int64_t ewvit_hfsep_bwd_weight_workspace(int64_t NI, int64_t H, int64_t W) {
  if (!hs_geom_ok(NI, H, W)) return 0;
  return (int64_t)hs_wg_blocks(NI, H) * HS_COUT * HS_K * 4;
}

extern "C" int ewvit_hfsep_bwd_weight(const void *x, const void *dy, int64_t NI, int64_t H, int64_t W, int x_channels, float *dw0,
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
  EWVIT_CHECK_ARG(x_channels == 16 || (x_channels == 9 && W % 2 == 0), "hfsep_bwd_weight: x_channels %d", x_channels);
  const size_t lds = (size_t)Pk * 128 + ((size_t)(th + 2) * (W + 2) + 1) * 32;
  hipStream_t s = as_stream(stream);
#define EWVIT_HS_WG(TH_, D_, X_, XS_)                                                                            \
  do {                                                                                                           \
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void *>(hfsep_wgrad_kernel<TH_, D_, X_, false, XS_>), \
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) == hipSuccess; \
    (void)attr;                                                                                                  \
    hipLaunchKernelGGL((hfsep_wgrad_kernel<TH_, D_, X_, false, XS_>), dim3(G), dim3(256), lds, s, (const bf16_t *)x, \
                       (const bf16_t *)dy, workspace, (int)NI, (int)H, (int)W, nullptr, nullptr, 0, 1);          \
  } while (0)
  // (XS 9: pixel-pair items (TH + 2) x (W / 2 + 1): 1 per thread for W <= 126, 2 for W <= 254)
  if (x_channels == 9) { if (small) EWVIT_HS_WG(2, 7, 1, 9); else EWVIT_HS_WG(2, 13, 2, 9); }
  else if (small) EWVIT_HS_WG(2, 7, 4, 16); else EWVIT_HS_WG(2, 13, 7, 16);
#undef EWVIT_HS_WG
  int rc = launch_status("hfsep_bwd_weight");
  if (rc) return rc;
  HsParams out{{dw0, dw1, dw2}, {db0, db1, db2}};
  const int nout = HS_REAL * 27 + HS_REAL;
  hipLaunchKernelGGL(hfsep_wgrad_reduce_kernel, dim3((nout + 63) / 64), dim3(1024), 0, s, workspace, G, out);
  return launch_status("hfsep_bwd_weight reduce");
}

extern "C" int64_t ewvit_hfsep_bn_bwd_weight_workspace(int64_t L, int64_t N, int64_t H, int64_t W) {
  if (L < 1 || L > 8 || N < 1 || !hs_geom_ok(L * N, H, W)) return 0;
  return (int64_t)hs_wg_blocks(L * N, H) * HS_COUT * HS_K * 4 + (int64_t)L * (64 * 8 + 128) * 4;
}

extern "C" int ewvit_hfsep_bn_bwd_weight(const void *x, const void *y, const void *dz, int64_t L, int64_t N, int64_t H,
                                         int64_t W, int x_channels, const float *mean, const float *invstd, const float *gamma,
                                         const float *beta, const float *part, int nrc, float *dw0, float *dw1,
                                         float *dw2, float *db0, float *db1, float *db2, float *dgamma, float *dbeta,
                                         float *workspace, void *stream) {
  EWVIT_CHECK_ARG(x && y && dz && mean && invstd && part && workspace, "hfsep_bn_bwd_weight: null pointer");
  EWVIT_CHECK_ARG(L >= 1 && L <= 8 && N >= 1 && hs_geom_ok(L * N, H, W), "hfsep_bn_bwd_weight: bad geometry");
  EWVIT_CHECK_ARG(nrc >= 1 && nrc <= 65535, "hfsep_bn_bwd_weight: %d partial rows", nrc);
  const int64_t NI = L * N;
  const int th = hs_wg_th();
  const int G = hs_wg_blocks(NI, H);
  const int Pk = (int)((th * W + 31) & ~31);
  const bool small = Pk * 8 <= 7 * 256 && (th + 2) * (W + 2) * 2 <= 4 * 256;
  EWVIT_CHECK_ARG(small || (Pk * 8 <= 13 * 256 && (th + 2) * (W + 2) * 2 <= 7 * 256),
                  "hfsep_bn_bwd_weight: W=%lld too wide for TH=%d", (long long)W, th);
  EWVIT_CHECK_ARG(x_channels == 16 || (x_channels == 9 && W % 2 == 0), "hfsep_bn_bwd_weight: x_channels %d", x_channels);
  const size_t lds = (size_t)Pk * 128 + ((size_t)(th + 2) * (W + 2) + 1) * 32 + (size_t)L * 64 * 8 * 4;
  hipStream_t s = as_stream(stream);
  float *tab = workspace + (int64_t)G * HS_COUT * HS_K;
  float *lsum = tab + L * 64 * 8;
  hipLaunchKernelGGL(hfsep_bn_coef_kernel, dim3((unsigned)L), dim3(1024), 0, s, part, nrc, (float)(N * H * W), mean,
                     invstd, gamma, beta, tab, lsum);
  if (int rc = launch_status("hfsep_bn_bwd_weight coef")) return rc;
#define EWVIT_HS_WGB(TH_, D_, X_, XS_)                                                                            \
  do {                                                                                                            \
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void *>(hfsep_wgrad_kernel<TH_, D_, X_, true, XS_>), \
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) == hipSuccess; \
    (void)attr;                                                                                                   \
    hipLaunchKernelGGL((hfsep_wgrad_kernel<TH_, D_, X_, true, XS_>), dim3(G), dim3(256), lds, s, (const bf16_t *)x, \
                       (const bf16_t *)dz, workspace, (int)NI, (int)H, (int)W, (const bf16_t *)y, tab, (int)L,    \
                       (int)N);                                                                                   \
  } while (0)
  if (x_channels == 9) { if (small) EWVIT_HS_WGB(2, 7, 1, 9); else EWVIT_HS_WGB(2, 13, 2, 9); }
  else if (small) EWVIT_HS_WGB(2, 7, 4, 16); else EWVIT_HS_WGB(2, 13, 7, 16);
#undef EWVIT_HS_WGB
  if (int rc = launch_status("hfsep_bn_bwd_weight")) return rc;
  HsParams out{{dw0, dw1, dw2}, {db0, db1, db2}};
  const int nout = HS_REAL * 27 + HS_REAL;
  hipLaunchKernelGGL(hfsep_wgrad_reduce_kernel, dim3((nout + 63) / 64 + 2), dim3(1024), 0, s, workspace, G, out, lsum,
                     (int)L, dgamma, dbeta);
  return launch_status("hfsep_bn_bwd_weight reduce");
}
