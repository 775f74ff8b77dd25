// Dense 2-D convolution (kernel 1x1 or 3x3, pad k/2, stride 1|2) as an MFMA
// implicit GEMM, channels-last bf16 (gfx950).
//
// Callers: the MWT conv stack of network/mwt.py:23-72 — hf_conv['fusion'] (all 3
// levels batched), multiscale_fusion (384 -> 128, 112^2, reading the three
// level-major fusion outputs in place), freq_conv / freq_pool (stride 2) — 74 % of
// the model's FLOPs (SURVEY §8 note 3), and the EfficientNetV2-S backbone's dense
// convs (FusedMBConv 3x3, MBConv expand/project 1x1, head 1x1).  Three kernels:
//
//   fwd    y[m, co]  = sum_{tap, ci} x[pix(m, tap), ci] * W[co, ci, tap]   (+ bias)
//   dgrad  dx[m, ci] = sum_{tap, co} dy[pix^T(m, tap), co] * W[co, ci, tap]
//          (same kernel: A gathers dy through the transposed pixel map, B = W packed
//           [ci][tap][co]; stride 2 handled by the parity test of pix^T)
//   wgrad  dW[co, tap, ci] = sum_m dy[m, co] * x[pix(m, tap), ci]   (split over m)
//
// GEMM tile 128xBNx32, 256 threads = 4 waves (2x2), each wave 64x(BN/2) =
// 4x(BN/32) v_mfma_f32_16x16x32_bf16 tiles, fp32 accumulate.  Operands are staged
// global -> registers -> LDS with the next K-tile's loads in flight during the
// current tile's MFMAs.  When the per-tap channel count is a multiple of 32 every
// K-tile lies inside one tap, so the tap (and the pixel offset it implies) is a
// wave-uniform scalar and the gather costs a handful of VALU ops per vector.
// fwd/dgrad images are [row][k] (k contiguous, padded 80-B rows) read with
// ds_read_b128; wgrad's operands both have the reduction (pixel) index outermost
// in HBM, so they are staged as natural [k][row] images (256-B rows, XOR-swizzled
// 16-B chunks) and read as MFMA fragments with ds_read_b64_tr_b16.
//
// Grouped channels-last layout (gc, gs): channel c of pixel p lives at
// (c / gc) * gs + p * gc + c % gc.  gc = C is plain NHWC; gc = 128, gs = B*H*W*128
// is the MWT's level-major fusion output [L][B][H][W][128] read as the
// [B][H][W][3*128] concatenation (mwt.py:112) without materialising it.
#include "conv_common.h"
#include "reduce_jobs.h"

#include <cstdlib>
#include <deque>
#include <mutex>
#include <unordered_map>

namespace ewvit {

template <bool DGRAD, int BN_, int KS, int BK, int PF>
__global__ __launch_bounds__(256) void conv_fwd_kernel(FwdArgs a) {
  // BK: K-tile depth (32 | 64); PF: K-tiles of register prefetch (1 | 2)
  constexpr int WN = BN_ / 2, J = WN / 16;  // per-wave columns, 16-wide MFMA tiles
  constexpr int LD = BK + 8;                 // padded [row][k] image row (bf16)
  constexpr int CPR = BK / 8;                // 16-B chunks per image row
  constexpr int VA = CBM * CPR / 256;        // A vectors staged per thread per K-tile
  constexpr int VB = BN_ * CPR / 256;        // B vectors
  constexpr int A_EL = 2 * CBM * LD, B_EL = 2 * BN_ * LD;
  constexpr int CST = BN_ + 8;               // epilogue image row (bf16)
  static_assert(CBM * CST <= A_EL + B_EL, "epilogue tile must fit the staging LDS");
  static_assert(VB >= 1, "tile too narrow for the staging map");
  // one LDS array: double-buffered A / B images, reused as the output tile image
  __shared__ __attribute__((aligned(16))) bf16_t smem[A_EL + B_EL];
  auto As = reinterpret_cast<bf16_t (*)[CBM][LD]>(smem);
  auto Bs = reinterpret_cast<bf16_t (*)[BN_][LD]>(smem + A_EL);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int64_t ntm = (a.M + CBM - 1) / CBM;
  // one M-tile per workgroup, or a grid-stride walk when the grid is capped (g_grid_cap)
  for (int64_t mt = blockIdx.x; mt < ntm; mt += gridDim.x) {
  const int64_t m0 = mt * CBM;
  const int n0 = blockIdx.y * BN_;
  const int K = KS * KS * a.KC;
  const int nk = (K + BK - 1) / BK;
  const bool fastk = (a.KC % BK) == 0;    // every K-tile inside one tap / one src group
  const int cbn = a.KC / BK;              // channel blocks per tap (fastk)
  const int ls = a.g.stride >> 1;         // log2(stride)
  const int smask = a.g.stride - 1;

  // staged vector v = tid + 256*u covers image row v / CPR, chunk v % CPR
  int arow[VA], ach[VA];
  int py[VA], px[VA];    // fwd: oh*s - pad, ow*s - pad;  dgrad: oh + pad, ow + pad
  int64_t pbase[VA];     // n * srcH * srcW
  bool avalid[VA];
#pragma unroll
  for (int u = 0; u < VA; ++u) {
    const int v = tid + 256 * u;
    arow[u] = v / CPR;
    ach[u] = (v % CPR) * 8;
    const int64_t m = m0 + arow[u];
    avalid[u] = m < a.M;
    const int64_t mm = avalid[u] ? m : 0;
    const int ow = (int)(mm % a.outW);
    const int64_t t = mm / a.outW;
    const int oh = (int)(t % a.outH);
    const int n = (int)(t / a.outH);
    if (!DGRAD) { py[u] = oh * a.g.stride - a.g.pad; px[u] = ow * a.g.stride - a.g.pad; }
    else        { py[u] = oh + a.g.pad;               px[u] = ow + a.g.pad; }
    pbase[u] = (int64_t)n * a.srcH * a.srcW;
  }
  // pixel index of tap (kh, kw) for staged row u, or -1 when it falls outside src
  auto src_pix = [&](int u, int kh, int kw) -> int64_t {
    int sh, sw;
    if (!DGRAD) {
      sh = py[u] + kh; sw = px[u] + kw;
    } else {
      const int th = py[u] - kh, tw = px[u] - kw;
      if (th < 0 || tw < 0 || ((th | tw) & smask)) return -1;
      sh = th >> ls; sw = tw >> ls;
    }
    if ((unsigned)sh >= (unsigned)a.srcH || (unsigned)sw >= (unsigned)a.srcW) return -1;
    return pbase[u] + (int64_t)sh * a.srcW + sw;
  };
  int ltap = 0, lcb = 0;   // fastk: tap / channel block of the next K-tile to load
  auto load_tile = [&](int kt, uint4 (&ra)[VA], uint4 (&rb)[VB]) {
    int kh = 0, kw = 0;
    int64_t goff = 0;      // group offset (elements) of this tile's channel block
    int cin0 = 0;          // channel within the group for ach == 0
    if (fastk) {
      kh = ltap / KS; kw = ltap - kh * KS;
      const int c0 = lcb * BK;
      const int gi = c0 / a.sgc;
      goff = (int64_t)gi * a.sgs;
      cin0 = c0 - gi * a.sgc;
      if (++lcb == cbn) { lcb = 0; ++ltap; }
    }
#pragma unroll
    for (int u = 0; u < VA; ++u) {
      const int k = kt * BK + ach[u];
      int64_t off, p;
      if (fastk) {
        p = src_pix(u, kh, kw);
        off = goff + p * a.sgc + cin0 + ach[u];
      } else {   // KC % BK != 0 (ungrouped src): per-thread tap
        const int tap = KS == 1 ? 0 : k / a.KC;
        const int c = k - tap * a.KC;
        const int th = tap / KS;
        p = src_pix(u, th, tap - th * KS);
        off = p * a.KC + c;
      }
      uint4 va = make_uint4(0u, 0u, 0u, 0u);
      if (avalid[u] && k < K && p >= 0) va = *reinterpret_cast<const uint4 *>(a.src + off);
      ra[u] = va;
    }
#pragma unroll
    for (int u = 0; u < VB; ++u) {
      const int v = tid + 256 * u;
      const int n = n0 + v / CPR, k = kt * BK + (v % CPR) * 8;
      uint4 vb = make_uint4(0u, 0u, 0u, 0u);
      if (n < a.Ncol && k < K) vb = *reinterpret_cast<const uint4 *>(a.wp + (int64_t)n * K + k);
      rb[u] = vb;
    }
  };
  auto store_tile = [&](int buf, const uint4 (&ra)[VA], const uint4 (&rb)[VB]) {
#pragma unroll
    for (int u = 0; u < VA; ++u) *reinterpret_cast<uint4 *>(&As[buf][arow[u]][ach[u]]) = ra[u];
#pragma unroll
    for (int u = 0; u < VB; ++u) {
      const int v = tid + 256 * u;
      *reinterpret_cast<uint4 *>(&Bs[buf][v / CPR][(v % CPR) * 8]) = rb[u];
    }
  };

  cf32x4 acc[4][J];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = cf32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fk = (lane >> 4) * 8;
  auto compute = [&](int cur) {
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      cbf16x8 af[4], bfr[J];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const cbf16x8 *>(&As[cur][wm * 64 + i * 16 + fr][ks * 32 + fk]);
#pragma unroll
      for (int j = 0; j < J; ++j)
        bfr[j] = *reinterpret_cast<const cbf16x8 *>(&Bs[cur][wn * WN + j * 16 + fr][ks * 32 + fk]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (PF == 1) {
    // K-tile kt+1 is loaded into registers while kt is computed from LDS
    uint4 ra[VA], rb[VB];
    load_tile(0, ra, rb);
    store_tile(0, ra, rb);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nk;
      if (more) load_tile(kt + 1, ra, rb);
      compute(cur);
      if (more) store_tile(cur ^ 1, ra, rb);
      __syncthreads();
    }
  } else {
    // K-tile kt+2 is loaded into registers while kt is computed from LDS and kt+1
    // (loaded one step earlier) is written to the other LDS buffer
    auto step = [&](int kt, uint4 (&na)[VA], uint4 (&nb)[VB], const uint4 (&ra)[VA], const uint4 (&rb)[VB]) {
      const int cur = kt & 1;
      if (kt + 2 < nk) load_tile(kt + 2, na, nb);
      compute(cur);
      if (kt + 1 < nk) store_tile(cur ^ 1, ra, rb);
      __syncthreads();
    };
    uint4 pa[VA], pb[VB], qa[VA], qb[VB];
    load_tile(0, pa, pb);
    if (nk > 1) load_tile(1, qa, qb);
    store_tile(0, pa, pb);
    __syncthreads();
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      step(kt, pa, pb, qa, qb);
      step(kt + 1, qa, qb, pa, pb);
    }
    if (kt < nk) step(kt, pa, pb, qa, qb);
  }
  // epilogue: accumulators (+ bias) -> bf16 tile image in LDS (C/D map col = lane&15,
  // row = (lane>>4)*4 + r), then 16-B row-contiguous stores of 8 output channels
  // (the loop above ended with a barrier, so the staging images are free)
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int cl = wn * WN + j * 16 + (lane & 15);
    const float b = (a.bias && n0 + cl < a.Ncol) ? a.bias[n0 + cl] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) smem[(wm * 64 + i * 16 + (lane >> 4) * 4 + r) * CST + cl] = f2bf(acc[i][j][r] + b);
  }
  __syncthreads();
  constexpr int VPR = BN_ / 8;               // 16-B vectors per tile row
#pragma unroll
  for (int k = 0; k < CBM * VPR / 256; ++k) {
    const int v = tid + 256 * k;
    const int rl = v / VPR, cv = v % VPR;
    const int64_t row = m0 + rl;
    const int col = n0 + cv * 8;
    if (row < a.M && col < a.Ncol) {
      const int gi = col / a.ogc;
      *reinterpret_cast<uint4 *>(a.out + (int64_t)gi * a.ogs + row * a.ogc + (col - gi * a.ogc)) =
          *reinterpret_cast<const uint4 *>(&smem[rl * CST + cv * 8]);
    }
  }
  __syncthreads();         // the output image is read before the next tile stages into smem
  }
}

// ---------------------------------------------------------------- wgrad
// C[co][n'] with n' = tap*Cin + ci, reduction over output pixels m.
template <int KS>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2][2][CBK * 256];  // [buf][A/B][32 rows x 256 B]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int co0 = blockIdx.y * CBM;
  const int np0 = blockIdx.x * CBN;
  const int NP = KS * KS * a.g.Cin;
  const int64_t mbeg = (int64_t)blockIdx.z * a.mper;
  const int64_t mend = mbeg + a.mper < a.M ? mbeg + a.mper : a.M;
  const int nk = (int)((mend - mbeg + CBK - 1) / CBK);

  // staging: 32 rows x 16 chunks per operand = 512 vectors -> 2 per thread
  // vector v: row = v >> 4, chunk = v & 15
  int vrow[2], vch[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int v = tid + 256 * u;
    vrow[u] = v >> 4;
    vch[u] = v & 15;
  }
  // the B chunk's (tap, ci) is fixed per thread
  int tkh[2], tkw[2];
  int64_t bgoff[2];      // grouped-layout offset of this chunk's channel
  bool bok[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int np = np0 + vch[u] * 8;
    bok[u] = np < NP;
    const int btap = bok[u] ? np / a.g.Cin : 0;
    const int bci = bok[u] ? np - btap * a.g.Cin : 0;
    tkh[u] = btap / KS - a.g.pad;
    tkw[u] = btap % KS - a.g.pad;
    const int gi = bci / a.xgc;
    bgoff[u] = (int64_t)gi * a.xgs + (bci - gi * a.xgc);
  }
  // pixel coordinates of each staged row, advanced by CBK pixels per K-tile
  // (no 64-bit div/mod in the loop)
  int pn[2], poh[2], pow_[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int64_t m = mbeg + vrow[u];
    pow_[u] = (int)(m % a.g.Wo);
    const int64_t t = m / a.g.Wo;
    poh[u] = (int)(t % a.g.Ho);
    pn[u] = (int)(t / a.g.Ho);
  }
  const bool do_bias = a.dbias_part != nullptr && blockIdx.x == 0;
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto load_tile = [&](int kt, uint4 (&ra)[2], uint4 (&rb)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t m = mbeg + (int64_t)kt * CBK + vrow[u];
      const int co = co0 + vch[u] * 8;
      uint4 va = make_uint4(0u, 0u, 0u, 0u), vb = va;
      if (m < mend && co < a.g.Cout) va = *reinterpret_cast<const uint4 *>(a.dy + m * a.g.Cout + co);
      const int ih = poh[u] * a.g.stride + tkh[u], iw = pow_[u] * a.g.stride + tkw[u];
      if (m < mend && bok[u] && (unsigned)ih < (unsigned)a.g.H && (unsigned)iw < (unsigned)a.g.W)
        vb = *reinterpret_cast<const uint4 *>(a.x + bgoff[u] + (((int64_t)pn[u] * a.g.H + ih) * a.g.W + iw) * a.xgc);
      ra[u] = va;
      rb[u] = vb;
      pow_[u] += CBK;
      while (pow_[u] >= a.g.Wo) {
        pow_[u] -= a.g.Wo;
        if (++poh[u] == a.g.Ho) { poh[u] = 0; ++pn[u]; }
      }
    }
  };
  auto bias_acc = [&](const uint4 (&ra)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const unsigned wv[4] = {ra[u].x, ra[u].y, ra[u].z, ra[u].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bsum[2 * j] += __uint_as_float(wv[j] << 16);
        bsum[2 * j + 1] += __uint_as_float(wv[j] & 0xffff0000u);
      }
    }
  };
  auto store_tile = [&](int buf, const uint4 (&ra)[2], const uint4 (&rb)[2]) {
    if (do_bias) bias_acc(ra);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      *reinterpret_cast<uint4 *>(&smem[buf][0][swz_off(vrow[u], vch[u])]) = ra[u];
      *reinterpret_cast<uint4 *>(&smem[buf][1][swz_off(vrow[u], vch[u])]) = rb[u];
    }
  };
  // transposed fragment read: rows k0..k0+3 of an image, columns c0..c0+15 (16-lane group);
  // lane 4q+p supplies row k0+q, columns c0+4p..c0+4p+3
  auto tr_read = [&](const unsigned char *img, int k0, int c0) -> cs4 {
    const int i = lane & 15, q = i >> 2, p = i & 3;
    const int col = c0 + 4 * p;
    const int off = swz_off(k0 + q, col >> 3) + 2 * (col & 7);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) cs4 *)(img + off));
  };

  cf32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = cf32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4;  // k rows 8g .. 8g+7 of the 32-row tile
  // same two-deep register prefetch as the fwd kernel
  auto step = [&](int kt, uint4 (&na)[2], uint4 (&nb)[2], const uint4 (&ra)[2], const uint4 (&rb)[2]) {
    const int cur = kt & 1;
    if (kt + 2 < nk) load_tile(kt + 2, na, nb);
    cbf16x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const cs4 lo = tr_read(smem[cur][0], 8 * g, wm * 64 + i * 16);
      const cs4 hi = tr_read(smem[cur][0], 8 * g + 4, wm * 64 + i * 16);
      af[i] = __builtin_bit_cast(cbf16x8, (__attribute__((ext_vector_type(8))) short){
                                              lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const cs4 lo = tr_read(smem[cur][1], 8 * g, wn * 64 + j * 16);
      const cs4 hi = tr_read(smem[cur][1], 8 * g + 4, wn * 64 + j * 16);
      bfr[j] = __builtin_bit_cast(cbf16x8, (__attribute__((ext_vector_type(8))) short){
                                               lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) store_tile(cur ^ 1, ra, rb);
    __syncthreads();
  };
  uint4 pa[2], pb[2], qa[2], qb[2];
  if (nk > 0) {
    load_tile(0, pa, pb);
    if (nk > 1) load_tile(1, qa, qb);
    store_tile(0, pa, pb);
  }
  __syncthreads();
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(kt, pa, pb, qa, qb);
    step(kt + 1, qa, qb, pa, pb);
  }
  if (kt < nk) step(kt, pa, pb, qa, qb);
  if (do_bias) {
    // threads with equal (tid & 15) hold the same 8 channels: lanes l, l^16, l^32, l^48
    // in a wave, then the 4 waves through LDS (the staging buffers are free now)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bsum[j] = rows_sum4(bsum[j]);
    }
    float *red = reinterpret_cast<float *>(&smem[0][0][0]);  // [4 waves][16 chunks][8]
    if (lane < 16)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[(w * 16 + lane) * 8 + j] = bsum[j];
    __syncthreads();
    if (tid < 128) {
      const int ch = tid >> 3, j = tid & 7;
      const int co = co0 + ch * 8 + j;
      const float s = (red[(0 * 16 + ch) * 8 + j] + red[(1 * 16 + ch) * 8 + j]) +
                      (red[(2 * 16 + ch) * 8 + j] + red[(3 * 16 + ch) * 8 + j]);
      if (co < a.g.Cout) a.dbias_part[(int64_t)blockIdx.z * a.g.Cout + co] = s;
    }
  }
  float *dst = a.part + (int64_t)blockIdx.z * a.g.Cout * NP;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = np0 + wn * 64 + j * 16 + (lane & 15);
    if (col >= NP) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = co0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (row < a.g.Cout) dst[(int64_t)row * NP + col] = acc[i][j][r];
      }
  }
}

// dW[co][ci][tap] (= or +=) sum over splits of part[s][co][tap*Cin + ci].  T lanes of a
// wave share one 4-element output (T = splits fan-in, a power of two <= 64 chosen so
// ~64K threads run): lane l sums splits l, l+T, ... (4 loads in flight), then an xor
// tree over the T lanes — fixed order, deterministic.  Blocks >= nmain reduce the bias
// partials: 64 channels per block, 4 waves over the partial rows, fixed-order combine.
__global__ __launch_bounds__(256) void conv_wgrad_reduce_kernel(const float *__restrict__ part, float *__restrict__ dw,
                                                                int Cout, int Cin, int taps, int splits, int bparts,
                                                                int accumulate, const float *__restrict__ dbias_part,
                                                                float *__restrict__ dbias, WOut wo, int T, int nmain) {
  __shared__ float red[4][64];
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= nmain) {
    const int c = ((int)blockIdx.x - nmain) * 64 + (tid & 63), q = tid >> 6;
    float sb = 0.f;
    if (c < Cout) {
      int k = q;
      for (; k + 12 < bparts; k += 16) {
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = dbias_part[(int64_t)(k + 4 * u) * Cout + c];
#pragma unroll
        for (int u = 0; u < 4; ++u) sb += v[u];
      }
      for (; k < bparts; k += 4) sb += dbias_part[(int64_t)k * Cout + c];
    }
    red[q][tid & 63] = sb;
    __syncthreads();
    if (tid < 64 && c < Cout) {
      const float r = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
      dbias[c] = accumulate ? dbias[c] + r : r;
    }
    return;
  }
  // (the split sums: reduce_jobs.h, shared with the deferred form)
  wgrad_reduce_block(part, dw, Cin, taps, splits, accumulate, wo, T, (int64_t)Cout * taps * Cin, (int)blockIdx.x);
}

// pack fp32 W (element (co, ci, tap) at co*s_co + ci*s_ci + tap*s_tap: any of the
// parameter's memory formats) -> bf16 [Cout][taps][Cin_pad] (fwd, wp) and/or
// [Cin_pad][taps][Cout] (dgrad, wp_t) in one pass; ci >= Cin packs zeros
__global__ __launch_bounds__(256) void conv_pack_kernel(const float *__restrict__ w, int64_t s_co, int64_t s_ci,
                                                        int64_t s_tap, bf16_t *__restrict__ wp,
                                                        bf16_t *__restrict__ wp_t, int Cout, int Cin, int Cin_pad,
                                                        int taps) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // index in the fwd layout
  const int64_t total = (int64_t)Cout * Cin_pad * taps;
  if (i >= total) return;
  const int ci = (int)(i % Cin_pad);
  const int tap = (int)((i / Cin_pad) % taps);
  const int co = (int)(i / ((int64_t)Cin_pad * taps));
  const bf16_t v = f2bf(ci < Cin ? w[co * s_co + ci * s_ci + tap * s_tap] : 0.f);
  if (wp) wp[i] = v;
  if (wp_t) wp_t[((int64_t)ci * taps + tap) * Cout + co] = v;
}

// multi-tensor pack: up to EWVIT_PACK_MAX weights per launch.  A workgroup packs one
// (weight, tap, 64-co x 64-ci) tile: read once, written row-contiguous to the fwd
// layout [co][tap][ci] and, through an LDS transpose, to the bwd_data layout
// [ci][tap][co] (tensor found by a uniform prefix-sum search over tile counts)
struct PackArgs {
  int n;
  int chunk0[EWVIT_PACK_MAX + 1];
  const float *w[EWVIT_PACK_MAX];
  bf16_t *wp[EWVIT_PACK_MAX];
  bf16_t *wpt[EWVIT_PACK_MAX];
  int64_t s_co[EWVIT_PACK_MAX], s_ci[EWVIT_PACK_MAX], s_tap[EWVIT_PACK_MAX];
  int cout[EWVIT_PACK_MAX], cin[EWVIT_PACK_MAX], cin_pad[EWVIT_PACK_MAX], taps[EWVIT_PACK_MAX];
};

__global__ __launch_bounds__(256) void conv_pack_multi_kernel(PackArgs a) {
  __shared__ bf16_t tile[64][66];
  const int blk = blockIdx.x, tid = threadIdx.x;
  int t = 0;
  while (t + 1 < a.n && a.chunk0[t + 1] <= blk) ++t;
  const int Cout = a.cout[t], Cin = a.cin[t], Cin_pad = a.cin_pad[t], taps = a.taps[t];
  const int nco = (Cout + 63) >> 6, nci = (Cin_pad + 63) >> 6;
  const int local = blk - a.chunk0[t];
  const int tap = local / (nco * nci), rem = local - tap * nco * nci;
  const int co0 = (rem / nci) * 64, ci0 = (rem % nci) * 64;
  const float *w = a.w[t];
  bf16_t *wp = a.wp[t], *wpt = a.wpt[t];
  const int64_t sco = a.s_co[t], sci = a.s_ci[t], stap = a.s_tap[t];
  if (sci == 1 && (Cin & 3) == 0 && (Cin_pad & 3) == 0 && (Cout & 3) == 0 && (sco & 3) == 0 && (stap & 3) == 0) {
    // ci-contiguous weights (the 1x1 convs, channels-last 3x3): 4 channels a thread, float4
    // loads, 8-byte stores in both layouts — all 4 loads of a thread in flight
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e4 = tid + 256 * u, r = e4 >> 4, c4 = (e4 & 15) * 4;
      const int co = co0 + r, ci = ci0 + c4;
      v[u] = co < Cout && ci < Cin ? *reinterpret_cast<const float4 *>(w + co * sco + ci + tap * stap)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e4 = tid + 256 * u, r = e4 >> 4, c4 = (e4 & 15) * 4;
      const int co = co0 + r, ci = ci0 + c4;
      const bf16_t b0 = f2bf(v[u].x), b1 = f2bf(v[u].y), b2 = f2bf(v[u].z), b3 = f2bf(v[u].w);
      tile[r][c4] = b0; tile[r][c4 + 1] = b1; tile[r][c4 + 2] = b2; tile[r][c4 + 3] = b3;
      if (wp && co < Cout && ci < Cin_pad) {
        uint2 pk;
        pk.x = (unsigned)b0 | ((unsigned)b1 << 16);
        pk.y = (unsigned)b2 | ((unsigned)b3 << 16);
        *reinterpret_cast<uint2 *>(wp + ((int64_t)co * taps + tap) * Cin_pad + ci) = pk;
      }
    }
    if (!wpt) return;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e4 = tid + 256 * u, r = e4 >> 4, c4 = (e4 & 15) * 4;
      const int ci = ci0 + r, co = co0 + c4;
      if (ci < Cin_pad && co < Cout) {
        uint2 pk;
        pk.x = (unsigned)tile[c4][r] | ((unsigned)tile[c4 + 1][r] << 16);
        pk.y = (unsigned)tile[c4 + 2][r] | ((unsigned)tile[c4 + 3][r] << 16);
        *reinterpret_cast<uint2 *>(wpt + ((int64_t)ci * taps + tap) * Cout + co) = pk;
      }
    }
    return;
  }
#pragma unroll 4
  for (int e = tid; e < 4096; e += 256) {
    const int r = e >> 6, c = e & 63;
    const int co = co0 + r, ci = ci0 + c;
    const bf16_t v = f2bf(co < Cout && ci < Cin ? w[co * sco + ci * sci + tap * stap] : 0.f);
    tile[r][c] = v;
    if (wp && co < Cout && ci < Cin_pad) wp[((int64_t)co * taps + tap) * Cin_pad + ci] = v;
  }
  if (!wpt) return;
  __syncthreads();
#pragma unroll 4
  for (int e = tid; e < 4096; e += 256) {
    const int r = e >> 6, c = e & 63;
    const int ci = ci0 + r, co = co0 + c;
    if (ci < Cin_pad && co < Cout) wpt[((int64_t)ci * taps + tap) * Cout + co] = tile[c][r];
  }
}

// ---------------------------------------------------------------- LDS-DMA kernels
// The same three GEMMs with the operands moved HBM/L2 -> LDS by buffer_load ... lds
// (16 B per lane, no register round trip, no ds_write), for the shapes whose K-tiles
// stay inside one tap and one channel group (fwd/dgrad: KC % 64 == 0; wgrad: Cin %
// 128 == 0 or 1x1).  Out-of-image taps and ragged tile edges are zero-filled by the
// buffer descriptor's range check (the lane's offset is pushed past num_records),
// so there is no per-lane branch around a load.  The DMA writes each wave's 1 KiB
// piece lane-linearly; the XOR swizzle that keeps the fragment reads conflict-free
// is applied to the lane's SOURCE address and undone on the read (the swizzle is an
// involution).  One K-tile is in flight while the previous one is multiplied; grid
// order is remapped so that consecutive tiles (which share input halo rows and, for
// wgrad, the same pixels) run on one XCD and meet in its L2.
// fwd / dgrad: BM x BN_ x 64 tiles, BM/32 waves (BM/64 x 2), NS-deep LDS ring of
// [row][64 k] images (128-B rows); 16-B chunk c of row r is stored at chunk
// c ^ ((r >> 1) & 7): conflict-free ds_read_b128 fragment reads
// DENSE (forward, plain NHWC x, Cin % 8 == 0 and not a multiple of 64: the backbone's 24 /
// 48 / 96-channel inputs, the MWT seperate conv's 16): the K axis is taps x Cin flattened
// ([Cout][taps][Cin] packs are exactly that), so a 64-wide K-tile spans several taps —
// each 16-B chunk of a row is (tap, 8 channels), with its own tap offset and in-image test.
// A lane's chunk index is fixed per row, so it advances by 8 chunks per K-tile: tap +=
// 8 / CC, cc += 8 % CC (CC = Cin / 8).  Zero waste but the last K-tile's tail (A past the
// last tap reads through the OOB offset, B's tail meets only those zeros).
// BST (dgrad): the backward statistics of the BatchNorm before the conv (FwdArgs::bwd) in
// the epilogue — its own instantiation, so the plain dgrad keeps its register budget
template <bool DGRAD, int BM, int BN_, int KS, int NS, int WC = 2, bool DENSE = false, bool BST = false>
__global__ __launch_bounds__(BM / 64 * WC * 64) void conv_glds_kernel(FwdArgs a, int64_t src_bytes, int ntn,
                                                                      int tap_inner, int ntiles) {
  static_assert(!(DENSE && DGRAD), "dense K: forward only");
  static_assert(!BST || DGRAD, "backward statistics: dgrad only");
  constexpr int NW = BM / 64 * WC, BK = 64;      // waves: BM/64 rows x WC columns
  constexpr int WN = BN_ / WC, J = WN / 16;
  constexpr int A_B = BM * BK * 2, B_B = BN_ * BK * 2, STG = A_B + B_B;
  constexpr int PA = BM / 8 / NW, PB = BN_ / 8 / NW;   // 1 KiB pieces per wave per K-tile
  static_assert(PB >= 1, "tile shape");
  // BatchNorm statistics image (fwd, or dgrad with BST), after the ring
  constexpr int RED_B = (DGRAD && !BST) ? 0 : BM / 64 * BN_ * 2 * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[NS * STG + RED_B];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ws = __builtin_amdgcn_readfirstlane(w);   // wave id, provably uniform
  const int wm = ws / WC, wn = ws % WC;
  if ((int)blockIdx.x >= ntiles) return;
  const int K = KS * KS * a.KC;
  const int cbn = (a.KC + BK - 1) / BK;   // ragged KC: the last block's lanes >= KC read zeros
  const bool cls = DGRAD && KS == 3 && a.pc >= 0;
  const int py = a.pc >> 1, px = a.pc & 1;
  const int ntaps = cls ? a.ntap : KS * KS;
  const int CC = a.KC >> 3;                // DENSE: 8-channel chunks per tap
  const int KSP = a.ksplit;                // split K: K-tiles per work item nk / KSP
  const int nk = (DENSE ? (K + BK - 1) / BK : ntaps * cbn) / KSP;
  const int tq = DENSE ? 8 / CC : 0, tr = DENSE ? 8 % CC : 0;   // DENSE: per-K-tile tap / chunk advance
  const int ls = a.g.stride >> 1, smask = a.g.stride - 1;
  const __amdgpu_buffer_rsrc_t rs = mk_rsrc(a.src, src_bytes);
  const __amdgpu_buffer_rsrc_t rw = mk_rsrc(a.wp, (int64_t)a.Ncol * K * 2);
  // (builtin DMAs: hipcc then waits vmcnt(4) ahead of each K-tile's fragment reads, so one
  // K-tile stays in flight whatever NS.  The asm DMAs of the windowed kernels, which leave
  // NS-1 in flight, measured slower here — the step 18.29 -> 18.56 ms on one box,
  // profiles/r05/ab/glds_asm_vs_builtin_ab.log: the backbone's small grids share the CUs with
  // the MWT stream, and deeper DMA queues cost that stream more than they gain)

  // A rows staged by this lane: piece p = w*PA + j covers rows 8p..8p+7.  Every tap's
  // source pixel is the row's base pixel plus a tap offset that is the same for all
  // rows (fwd: +(kh*W + kw); dgrad: -(kh*W + kw), or -((kh/2)*W + kw/2) at stride 2),
  // so a row keeps one byte offset and a mask of the taps that land inside the image
  // (and, for stride-2 dgrad, on the stride lattice); a K-tile adds one scalar.
  //
  // Tile loop: one tile per workgroup, or — with a capped grid (ewvit_set_grid_cap: a
  // branch sharing the GPU with another stream) — a persistent walk over the tiles.  The
  // staging cursor runs ahead of the compute cursor across tile boundaries: the next
  // tile's first K-tiles are in flight while this tile's last ones are multiplied and its
  // epilogue stores, so a walk pays the ring's fill latency once, not once per tile.
  int rb[PA], lc8[PA];
  unsigned vmask[PA];
  int dtap[PA], dcc[PA];  // DENSE: the (tap, chunk) each piece stages next
  uint32_t boff[PB];      // B (packed weights) byte offset of K-tile 0, or OOB
  const int kcr = a.KCr ? a.KCr : a.KC;
  // K-tile cursor: tap, channel block, group index / offset of the block.  With
  // tap_inner the 9 taps of one 64-channel block are consecutive K-tiles, so a block's
  // live input window (its pixels + halo, 64 channels) stays small enough for the
  // XCD's L2 to serve the tap re-reads; otherwise taps are outer.
  int ltap = 0, lcb = 0, lgi = 0, lcin = 0;
  auto setup = [&](int item) {          // the staged tile's row / column offsets
  const int tile = item / KSP;
  const int64_t m0 = (int64_t)(tile / ntn) * BM;
  const int n0 = (tile % ntn) * BN_;
  ltap = 0; lcb = 0; lgi = 0; lcin = 0;
  if (KSP > 1) { lcb = (item % KSP) * nk; lcin = lcb * BK; }   // (1x1, one channel group)
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int p = ws * PA + j, r = p * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((r >> 1) & 7);
    const int64_t m = m0 + r;
    const int64_t mm = m < a.M ? m : 0;
    const int ow = (int)(mm % a.outW);
    const int64_t t = mm / a.outW;
    const int oh = (int)(t % a.outH);
    const int n = (int)(t / a.outH);
    int by, bx;            // base pixel (may lie outside the image)
    unsigned msk = 0;
    if (cls) {
      // class taps: dy pixel (oh + dh, ow + dw), dh = (py + 1 - kh) / 2 in {0, 1} (unrolled:
      // a runtime index into the kernel argument's tapl[] puts the argument on the stack)
#pragma unroll
      for (int lt = 0; lt < 4; ++lt) {
        if (lt >= a.ntap) break;
        const int tp = a.tapl[lt], kh = tp / 3, kw = tp - kh * 3;
        const int sh = oh + ((py + 1 - kh) >> 1), sw = ow + ((px + 1 - kw) >> 1);
        if (m < a.M && sh < a.srcH && sw < a.srcW) msk |= 1u << lt;
      }
    } else
#pragma unroll
    for (int kh = 0; kh < KS; ++kh)
#pragma unroll
      for (int kw = 0; kw < KS; ++kw) {
        int sh, sw;
        bool ok = m < a.M;
        if (!DGRAD) {
          sh = oh * a.g.stride - a.g.pad + kh; sw = ow * a.g.stride - a.g.pad + kw;
        } else {
          const int th = oh + a.g.pad - kh, tw = ow + a.g.pad - kw;
          ok = ok && th >= 0 && tw >= 0 && !((th | tw) & smask);
          sh = th >> ls; sw = tw >> ls;
        }
        ok = ok && (unsigned)sh < (unsigned)a.srcH && (unsigned)sw < (unsigned)a.srcW;
        if (ok) msk |= 1u << (kh * KS + kw);
      }
    if (!DGRAD) { by = oh * a.g.stride - a.g.pad; bx = ow * a.g.stride - a.g.pad; }
    else if (cls) { by = oh; bx = ow; }
    else        { by = (oh + a.g.pad) >> ls;       bx = (ow + a.g.pad) >> ls; }
    const int64_t pix = (int64_t)n * a.srcH * a.srcW + (int64_t)by * a.srcW + bx;
    rb[j] = (int)((pix * a.sgc + (DENSE ? 0 : lc * 8)) * 2);
    vmask[j] = msk;
    lc8[j] = lc * 8;
    if (DENSE) { dtap[j] = lc / CC; dcc[j] = lc - dtap[j] * CC; }
  }
#pragma unroll
  for (int j = 0; j < PB; ++j) {
    const int p = ws * PB + j, r = p * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((r >> 1) & 7);
    const int n = n0 + r;
    boff[j] = n < a.Ncol ? (uint32_t)(((int64_t)n * K + lc * 8) * 2) : OOB;
  }
  };
  int ld = 0;             // K-tiles of the staged tile issued so far
  auto stage = [&](int buf) {
    if constexpr (DENSE) {
      unsigned char *base = smem + buf * STG + ws * PA * 1024;
#pragma unroll
      for (int j = 0; j < PA; ++j) {
        const int tp = dtap[j];
        const int kh = (tp * 11) >> 5, kw = tp - kh * 3;     // tp / 3 for tp < 32 (KS == 3)
        const int dpix = KS == 3 ? kh * a.srcW + kw : 0;
        const bool ok = (tp < KS * KS) & (((vmask[j] >> tp) & 1u) != 0);
        glds16(rs, base + j * 1024, ok ? (uint32_t)(rb[j] + (dpix * a.sgc + dcc[j] * 8) * 2) : OOB);
        dtap[j] += tq;
        dcc[j] += tr;
        if (dcc[j] >= CC) { dcc[j] -= CC; ++dtap[j]; }
      }
      unsigned char *bb = smem + buf * STG + A_B + ws * PB * 1024;
      const uint32_t kb = (uint32_t)(ld * BK * 2);
#pragma unroll
      for (int j = 0; j < PB; ++j) glds16(rw, bb + j * 1024, boff[j] == OOB ? OOB : boff[j] + kb);
      return;
    }
    const int rt = cls ? (ltap == 0 ? a.tapl[0] : ltap == 1 ? a.tapl[1] : ltap == 2 ? a.tapl[2] : a.tapl[3])
                       : ltap;                     // the weight tap
    const int kh = rt / KS, kw = rt - kh * KS;
    int dpix;
    if (!DGRAD) dpix = kh * a.srcW + kw;
    else if (cls) dpix = ((py + 1 - kh) >> 1) * a.srcW + ((px + 1 - kw) >> 1);
    else dpix = -((kh >> ls) * a.srcW + (kw >> ls));
    const int sdelta = (int)(((int64_t)dpix * a.sgc + (int64_t)lgi * a.sgs + lcin) * 2);
    const int tap = ltap, c0 = lcin;
    const uint32_t kb = (uint32_t)((rt * a.KC + lcb * BK) * 2);
    if (tap_inner) {
      if (++ltap == ntaps) {
        ltap = 0; ++lcb;
        lcin += BK;
        if (lcin == a.sgc) { lcin = 0; ++lgi; }
      }
    } else {
      lcin += BK;
      if (lcin == a.sgc) { lcin = 0; ++lgi; }
      if (++lcb == cbn) { lcb = 0; ++ltap; lgi = 0; lcin = 0; }
    }
    unsigned char *base = smem + buf * STG + ws * PA * 1024;
#pragma unroll
    for (int j = 0; j < PA; ++j)
      glds16(rs, base + j * 1024,
                 ((((vmask[j] >> tap) & 1u) != 0) & (c0 + lc8[j] < kcr)) ? (uint32_t)(rb[j] + sdelta) : OOB);
    unsigned char *bb = smem + buf * STG + A_B + ws * PB * 1024;
#pragma unroll
    for (int j = 0; j < PB; ++j) glds16(rw, bb + j * 1024, boff[j] == OOB ? OOB : boff[j] + kb);
  };

  cf32x4 acc[4][J];
  const int fr = lane & 15, fq = lane >> 4;
  auto frag = [&](const unsigned char *img, int r, int ch) -> cbf16x8 {
    return *reinterpret_cast<const cbf16x8 *>(img + r * 128 + 16 * (ch ^ ((r >> 1) & 7)));
  };
  // both 32-deep steps' fragments are read before the MFMAs, so the second step's reads run
  // under the first step's MFMAs
  auto compute = [&](int buf) {
    const unsigned char *As = smem + buf * STG, *Bs = As + A_B;
    cbf16x8 af[BK / 32][4], bfr[BK / 32][J];
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = frag(As, wm * 64 + i * 16 + fr, ks * 4 + fq);
#pragma unroll
      for (int j = 0; j < J; ++j) bfr[ks][j] = frag(Bs, wn * WN + j * 16 + fr, ks * 4 + fq);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j)
          // operands swapped (B first): the lane holds 4 consecutive output COLUMNS of
          // one row, acc[i][j][r] = C[i*16 + (lane&15)][j*16 + 4*(lane>>4) + r], so the
          // epilogue stores 8 B per lane straight from registers (no LDS image)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[ks][j], af[ks][i], acc[i][j], 0, 0, 0);
  };
  // `inflight` counts issued K-tiles not yet multiplied (<= NS-1); the buffer refilled is
  // always the one every wave finished reading before the last barrier
  int ts = blockIdx.x, lbuf = 0, inflight = 0, cur = 0;
  ld = 0;
  setup(xcd_remap(ts, ntiles));
  for (; ld < NS - 1 && ld < nk; ++ld, ++inflight) {
    stage(lbuf);
    lbuf = lbuf + 1 == NS ? 0 : lbuf + 1;
  }
  for (int ti = blockIdx.x; ti < ntiles; ti += gridDim.x) {
  const int item = xcd_remap(ti, ntiles), tile = item / KSP;
  const int64_t m0 = (int64_t)(tile / ntn) * BM;
  const int n0 = (tile % ntn) * BN_;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = cf32x4{0.f, 0.f, 0.f, 0.f};
  int kt = 0;
  for (; ld < nk; ++kt) {     // steady state: refill with this tile's K-tiles
    // K-tile kt landed; the inflight-1 younger ones may stay in flight (the previous
    // tile's epilogue stores, issued after them, only make this wait conservative)
    wait_tile<PA + PB, NS>(inflight - 1);
    stage(lbuf);
    ++ld;
    lbuf = lbuf + 1 == NS ? 0 : lbuf + 1;
    compute(cur);
    cur = cur + 1 == NS ? 0 : cur + 1;
  }
  // this tile is fully issued: the remaining (<= NS-1) iterations refill with the next
  // tile's first K-tiles, so they are in flight during this tile's tail and epilogue
  const bool nxt = ts + (int)gridDim.x < ntiles;
  if (nxt) {
    ts += gridDim.x;
    setup(xcd_remap(ts, ntiles));
  }
  ld = 0;
  for (; kt < nk; ++kt) {
    wait_tile<PA + PB, NS>(inflight - 1);
    if (nxt) {
      stage(lbuf);
      ++ld;
      lbuf = lbuf + 1 == NS ? 0 : lbuf + 1;
    } else {
      --inflight;
    }
    compute(cur);
    cur = cur + 1 == NS ? 0 : cur + 1;
  }
  if (KSP > 1) {
    // split K: the fp32 partial tile, 16 B (4 columns of one row) per lane and row
    float *kp = a.kpart + (int64_t)(item % KSP) * a.M * a.Ncol;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int col = n0 + wn * WN + j * 16 + fq * 4;
      if (col >= a.Ncol) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = m0 + wm * 64 + i * 16 + fr;
        if (row < a.M)
          *reinterpret_cast<float4 *>(kp + row * a.Ncol + col) =
              make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    continue;
  }
  // epilogue: (+ bias) -> bf16, 8-B stores of 4 consecutive channels per lane
  // (Ncol % 8 == 0 and group widths % 32 == 0: a 4-channel run never straddles)
  const bool stats = !DGRAD && a.bn_part != nullptr;
  constexpr bool bstats = BST;
  int64_t opx[4];               // parity-class dgrad: the dx pixel of each of this lane's rows
  if (cls) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = m0 + wm * 64 + i * 16 + fr;
      const int64_t rr = row < a.M ? row : 0;
      const int ow = (int)(rr % a.outW);
      const int64_t t = rr / a.outW;
      const int oh = (int)(t % a.outH);
      const int64_t n = t / a.outH;
      opx[i] = (n * a.dstH + 2 * oh + py) * a.dstW + 2 * ow + px;
    }
  }
  float cs[J][4], cq[J][4];     // this lane's column sums over its 4 rows (BN statistics)
  // BST: the stored bf16 values, kept for the statistics pass after the stores
  uint2 hpk[BST ? J : 1][4];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int col = n0 + wn * WN + j * 16 + fq * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) { cs[j][r] = 0.f; cq[j][r] = 0.f; }
    if (col >= a.Ncol) continue;
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.bias) bv = *reinterpret_cast<const float4 *>(a.bias + col);
    float4 kv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (stats && a.bn_shift) kv = *reinterpret_cast<const float4 *>(a.bn_shift + col);
    const int gi = col / a.ogc;
    bf16_t *ob = a.out + (int64_t)gi * a.ogs + (col - gi * a.ogc);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = m0 + wm * 64 + i * 16 + fr;
      if (row < a.M) {
        const int64_t opix = cls ? opx[i] : row;
        float4 av = bv;
        if (a.addend) {
          const uint2 q = *reinterpret_cast<const uint2 *>(a.addend + (ob - a.out) + opix * a.ogc);
          av.x += __uint_as_float(q.x << 16); av.y += __uint_as_float(q.x & 0xffff0000u);
          av.z += __uint_as_float(q.y << 16); av.w += __uint_as_float(q.y & 0xffff0000u);
        }
        const bf16_t h0 = f2bf(acc[i][j][0] + av.x), h1 = f2bf(acc[i][j][1] + av.y);
        const bf16_t h2 = f2bf(acc[i][j][2] + av.z), h3 = f2bf(acc[i][j][3] + av.w);
        uint2 pk;
        pk.x = (uint32_t)h0 | ((uint32_t)h1 << 16);
        pk.y = (uint32_t)h2 | ((uint32_t)h3 << 16);
        *reinterpret_cast<uint2 *>(ob + opix * a.ogc) = pk;
        if constexpr (BST) hpk[j][i] = pk;
        if (stats) {
          const float d0 = bf2f(h0) - kv.x, d1 = bf2f(h1) - kv.y, d2 = bf2f(h2) - kv.z, d3 = bf2f(h3) - kv.w;
          cs[j][0] += d0; cs[j][1] += d1; cs[j][2] += d2; cs[j][3] += d3;
          cq[j][0] = fmaf(d0, d0, cq[j][0]); cq[j][1] = fmaf(d1, d1, cq[j][1]);
          cq[j][2] = fmaf(d2, d2, cq[j][2]); cq[j][3] = fmaf(d3, d3, cq[j][3]);
        }
      }
    }
  }
  if constexpr (BST) {
    // g = dx * act'(xhat * gamma + beta) (act) or dx * rscale[frame]; sums of g and g * xhat
    // over the stored values, one column block at a time: its 4 BN-input loads and the BN
    // parameters are issued together, so their latencies overlap
    float brs[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = m0 + wm * 64 + i * 16 + fr;
      brs[i] = a.bwd.rscale && row < a.M ? a.bwd.rscale[row / a.bwd.hw] : 1.f;
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int col = n0 + wn * WN + j * 16 + fq * 4;
      if (col >= a.Ncol) continue;
      const int gi = col / a.ogc;
      const bf16_t *xg = a.bwd.x + (int64_t)gi * a.ogs + (col - gi * a.ogc);   // the BN input, dx's layout
      uint2 xq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = m0 + wm * 64 + i * 16 + fr;
        xq[i] = row < a.M ? *reinterpret_cast<const uint2 *>(xg + row * a.ogc) : make_uint2(0u, 0u);
      }
      // statistics: [row group][C] of a row-grouped BN, [channel group][C] = col of a grouped dx;
      // the affine parameters are shared by the groups
      const int64_t sidx = (a.bwd.grows ? m0 / a.bwd.grows * a.ogc : 0) + col;
      const int pidx = col - gi * a.ogc;
      const float4 mu4 = *reinterpret_cast<const float4 *>(a.bwd.mean + sidx);
      const float4 iv4 = *reinterpret_cast<const float4 *>(a.bwd.invstd + sidx);
      const float4 ga4 = a.bwd.gamma ? *reinterpret_cast<const float4 *>(a.bwd.gamma + pidx) : make_float4(1.f, 1.f, 1.f, 1.f);
      const float4 be4 = a.bwd.beta ? *reinterpret_cast<const float4 *>(a.bwd.beta + pidx) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w}, iv[4] = {iv4.x, iv4.y, iv4.z, iv4.w};
      const float ga[4] = {ga4.x, ga4.y, ga4.z, ga4.w}, be[4] = {be4.x, be4.y, be4.z, be4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = m0 + wm * 64 + i * 16 + fr;
        if (row >= a.M) continue;
        const float xv[4] = {__uint_as_float(xq[i].x << 16), __uint_as_float(xq[i].x & 0xffff0000u),
                             __uint_as_float(xq[i].y << 16), __uint_as_float(xq[i].y & 0xffff0000u)};
        const float hv[4] = {__uint_as_float(hpk[j][i].x << 16), __uint_as_float(hpk[j][i].x & 0xffff0000u),
                             __uint_as_float(hpk[j][i].y << 16), __uint_as_float(hpk[j][i].y & 0xffff0000u)};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float xh = (xv[r] - mu[r]) * iv[r];
          const float g = a.bwd.act ? hv[r] * bn_act_grad(a.bwd.act, fmaf(xh, ga[r], be[r])) : hv[r] * brs[i];
          cs[j][r] += g;
          cq[j][r] = fmaf(g, xh, cq[j][r]);
        }
      }
    }
  }
  if (stats || bstats) {
  // BatchNorm partial statistics of this m-tile: the 16 row lanes of each column
  // (DPP row sums), then the BM/64 waves that share a column block through LDS, in order
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      cs[j][r] = row_sum16(cs[j][r]);
      cq[j][r] = row_sum16(cq[j][r]);
    }
  // [BM/64][BN_][2] after the ring (the next tile's K-tiles are landing in it); its
  // previous tile's readers finished before this tile's K-loop barriers
  // (dgrad: no image after the ring — its partials go into ring slot 0 once every wave has
  // finished reading it; an uncapped grid, so no next tile's K-tiles are landing there)
  float *red = reinterpret_cast<float *>(smem + NS * STG);
  if (fr == 0)
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cl = wn * WN + j * 16 + fq * 4 + r;
        red[(wm * BN_ + cl) * 2] = cs[j][r];
        red[(wm * BN_ + cl) * 2 + 1] = cq[j][r];
      }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // no vmcnt drain
  if (tid < BN_) {
    const int col = n0 + tid;
    if (col < a.Ncol) {
      float S = 0.f, Q = 0.f;
#pragma unroll
      for (int q = 0; q < BM / 64; ++q) { S += red[(q * BN_ + tid) * 2]; Q += red[(q * BN_ + tid) * 2 + 1]; }
      const int64_t t = m0 / BM;
      if (DGRAD) {
        // channel group gi of a grouped dx is its own BatchNorm group: rows [gi][m-tile][2 ogc]
        const int gi = col / a.ogc, cl = col - gi * a.ogc;
        float *pr = a.bwd.part + ((int64_t)gi * ((a.M + BM - 1) / BM) + t) * 2 * a.ogc;
        pr[cl] = S;
        pr[a.ogc + cl] = Q;
      } else {
        a.bn_part[t * 2 * a.Ncol + col] = S;
        a.bn_part[t * 2 * a.Ncol + a.Ncol + col] = Q;
      }
      if (!DGRAD && t == 0 && a.bn_shift_out) a.bn_shift_out[col] = a.bn_shift ? a.bn_shift[col] : 0.f;
    }
  }
  }
  }
}

// ---- split-K epilogue (conv_glds_kernel with FwdArgs::ksplit > 1; 1x1, plain layouts): block
// = one bm-row m-tile (the tile the BatchNorm partial rows follow) x 64 columns; thread = 4
// columns x rows r, r + 16, .. of the tile.  It adds the splits' fp32 partials in split order,
// then runs conv_glds_kernel's epilogue once: (+ bias, + addend) -> bf16, and MODE 1 the
// forward statistics sum (y - K), sum (y - K)^2 / MODE 2 the backward statistics (BST: sum g,
// sum g * xhat) of the tile, its 16 row lanes added in order through LDS.
template <int MODE>
__global__ __launch_bounds__(256) void conv_splitk_epi_kernel(FwdArgs a, int bm) {
  __shared__ float red[16][64][2];
  const int tid = threadIdx.x, cq = tid & 15, rl = tid >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * bm;
  const int col = blockIdx.y * 64 + cq * 4;
  const bool cok = col < a.Ncol;
  const int64_t plane = a.M * a.Ncol;
  const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 bv = (cok && a.bias) ? *reinterpret_cast<const float4 *>(a.bias + col) : zero;
  const float4 kv = (MODE == 1 && cok && a.bn_shift) ? *reinterpret_cast<const float4 *>(a.bn_shift + col) : zero;
  float mu[4] = {0.f, 0.f, 0.f, 0.f}, iv[4] = {0.f, 0.f, 0.f, 0.f};
  float ga[4] = {1.f, 1.f, 1.f, 1.f}, be[4] = {0.f, 0.f, 0.f, 0.f};
  if (MODE == 2 && cok) {
    const int64_t sidx = (a.bwd.grows ? m0 / a.bwd.grows * a.ogc : 0) + col;
    const float4 mu4 = *reinterpret_cast<const float4 *>(a.bwd.mean + sidx);
    const float4 iv4 = *reinterpret_cast<const float4 *>(a.bwd.invstd + sidx);
    mu[0] = mu4.x; mu[1] = mu4.y; mu[2] = mu4.z; mu[3] = mu4.w;
    iv[0] = iv4.x; iv[1] = iv4.y; iv[2] = iv4.z; iv[3] = iv4.w;
    if (a.bwd.gamma) {
      const float4 g4 = *reinterpret_cast<const float4 *>(a.bwd.gamma + col);
      ga[0] = g4.x; ga[1] = g4.y; ga[2] = g4.z; ga[3] = g4.w;
    }
    if (a.bwd.beta) {
      const float4 b4 = *reinterpret_cast<const float4 *>(a.bwd.beta + col);
      be[0] = b4.x; be[1] = b4.y; be[2] = b4.z; be[3] = b4.w;
    }
  }
  float cs[4] = {0.f, 0.f, 0.f, 0.f}, cqq[4] = {0.f, 0.f, 0.f, 0.f};
  if (cok) {
    for (int r = rl; r < bm; r += 16) {
      const int64_t row = m0 + r;
      if (row >= a.M) break;
      const float *kp = a.kpart + row * a.Ncol + col;
      float4 t = *reinterpret_cast<const float4 *>(kp);
      for (int sp = 1; sp < a.ksplit; ++sp) {
        const float4 u = *reinterpret_cast<const float4 *>(kp + sp * plane);
        t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
      }
      float4 av = bv;
      if (a.addend) {
        const uint2 q = *reinterpret_cast<const uint2 *>(a.addend + row * a.ogc + col);
        av.x += __uint_as_float(q.x << 16); av.y += __uint_as_float(q.x & 0xffff0000u);
        av.z += __uint_as_float(q.y << 16); av.w += __uint_as_float(q.y & 0xffff0000u);
      }
      const bf16_t h0 = f2bf(t.x + av.x), h1 = f2bf(t.y + av.y), h2 = f2bf(t.z + av.z), h3 = f2bf(t.w + av.w);
      uint2 pk;
      pk.x = (uint32_t)h0 | ((uint32_t)h1 << 16);
      pk.y = (uint32_t)h2 | ((uint32_t)h3 << 16);
      *reinterpret_cast<uint2 *>(a.out + row * a.ogc + col) = pk;
      const float hv[4] = {bf2f(h0), bf2f(h1), bf2f(h2), bf2f(h3)};
      if (MODE == 1) {
        const float kk[4] = {kv.x, kv.y, kv.z, kv.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float d = hv[q] - kk[q];
          cs[q] += d;
          cqq[q] = fmaf(d, d, cqq[q]);
        }
      } else if (MODE == 2) {
        const uint2 xq = *reinterpret_cast<const uint2 *>(a.bwd.x + row * a.ogc + col);
        const float xv[4] = {__uint_as_float(xq.x << 16), __uint_as_float(xq.x & 0xffff0000u),
                             __uint_as_float(xq.y << 16), __uint_as_float(xq.y & 0xffff0000u)};
        const float brs = a.bwd.rscale ? a.bwd.rscale[row / a.bwd.hw] : 1.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float xh = (xv[q] - mu[q]) * iv[q];
          const float g = a.bwd.act ? hv[q] * bn_act_grad(a.bwd.act, fmaf(xh, ga[q], be[q])) : hv[q] * brs;
          cs[q] += g;
          cqq[q] = fmaf(g, xh, cqq[q]);
        }
      }
    }
  }
  if (MODE == 0) return;
#pragma unroll
  for (int q = 0; q < 4; ++q) { red[rl][cq * 4 + q][0] = cs[q]; red[rl][cq * 4 + q][1] = cqq[q]; }
  __syncthreads();
  if (tid < 64) {
    const int c = blockIdx.y * 64 + tid;
    if (c < a.Ncol) {
      float S = 0.f, Q = 0.f;
      for (int q = 0; q < 16; ++q) { S += red[q][tid][0]; Q += red[q][tid][1]; }
      const int64_t t = blockIdx.x;
      if (MODE == 2) {
        float *pr = a.bwd.part + t * 2 * a.ogc;
        pr[c] = S;
        pr[a.ogc + c] = Q;
      } else {
        a.bn_part[t * 2 * a.Ncol + c] = S;
        a.bn_part[t * 2 * a.Ncol + a.Ncol + c] = Q;
        if (t == 0 && a.bn_shift_out) a.bn_shift_out[c] = a.bn_shift ? a.bn_shift[c] : 0.f;
      }
    }
  }
}

// wgrad: C[co][n'] over pixel K-tiles of BK; NS-deep ring of [pixel][128] images of
// 256-B rows, chunk c of row r at c ^ (((r&3)<<2) | ((r>>2)&3)) (read transposed,
// ds_read_b64_tr_b16).  Bias gradient (sum of dy over pixels): the blocks of n'-tile
// t sum the dy image of the K-tiles kt = t (mod n'-tiles), spreading the extra reads.
template <int KS, int BK, int NS, int WJ = 4>
__global__ __launch_bounds__(256) void conv_wgrad_glds_kernel(WgradArgs a, int64_t x_bytes, int ntx, int nty,
                                                              RedJobs rj) {
  constexpr int NB = WJ / 4;         // 128-column x images per stage (n'-tile of 128 * NB)
  constexpr int IMG = BK * 256, STG = (1 + NB) * IMG;
  constexpr int P = BK / 16;        // pieces (4 rows x 256 B) per wave per image
  __shared__ __attribute__((aligned(16))) unsigned char smem[NS * STG];
  // the first rj.nblk workgroups run deferred reductions of earlier weight gradients
  if ((int)blockIdx.x < rj.nblk) {
    run_red_jobs(rj, (int)blockIdx.x, reinterpret_cast<float *>(smem));
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tile = xcd_remap((int)blockIdx.x - rj.nblk, (int)gridDim.x - rj.nblk);
  const int split = tile / (ntx * nty);
  const int tx = tile % ntx, ty = (tile / ntx) % nty;
  const int co0 = ty * 128, np0 = tx * 128 * NB;
  const int NP = KS * KS * a.g.Cin;
  const int64_t mbeg = (int64_t)split * a.mper;
  const int64_t mend = mbeg + a.mper < a.M ? mbeg + a.mper : a.M;
  const int nk = (int)((mend - mbeg + BK - 1) / BK);
  const __amdgpu_buffer_rsrc_t rx = mk_rsrc(a.x, x_bytes);
  const __amdgpu_buffer_rsrc_t rd = mk_rsrc(a.dy, a.M * a.g.Cout * 2);

  // piece p = ws*P + j: rows 4p .. 4p+3; lane -> row 4p + lane/16, stored chunk lane%16.
  // A K-tile's first pixel (n0, oh0, ow0) is tracked in scalars; a row's pixel is that
  // plus r, carried through (ow, oh) with exact multiply-high divisions (r < 64).
  const int ws = __builtin_amdgcn_readfirstlane(w);
  const int wm = ws >> 1, wn = ws & 1;
  int rr[P], aoff[P], tkh[NB * P], tkw[NB * P], bgo[NB * P];
  bool aok[P], bok[NB * P];
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const int p = ws * P + j, r = p * 4 + (lane >> 4);
    const int lc = (lane & 15) ^ (((r & 3) << 2) | ((r >> 2) & 3));
    rr[j] = r;
    aok[j] = co0 + lc * 8 < a.g.Cout;
    aoff[j] = (int)(((mbeg + r) * a.g.Cout + co0 + lc * 8) * 2);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int e = b * P + j;
      const int np = np0 + b * 128 + lc * 8;
      bok[e] = np < NP;
      const int btap = bok[e] ? np / a.g.Cin : 0;
      const int bci = bok[e] ? np - btap * a.g.Cin : 0;
      tkh[e] = btap / KS - a.g.pad;
      tkw[e] = btap % KS - a.g.pad;
      const int gi = bci / a.xgc;
      bgo[e] = (int)(((int64_t)gi * a.xgs + (bci - gi * a.xgc)) * 2);
    }
  }
  // exact floor(x / d) = umulhi(x, ceil(2^32 / d)) for x < 2^32 / d
  const uint32_t magW = (uint32_t)((0x100000000ull + a.g.Wo - 1) / a.g.Wo);
  const uint32_t magH = (uint32_t)((0x100000000ull + a.g.Ho - 1) / a.g.Ho);
  int sn = (int)(mbeg / ((int64_t)a.g.Ho * a.g.Wo));
  int soh = (int)((mbeg / a.g.Wo) % a.g.Ho);
  int sow = (int)(mbeg % a.g.Wo);
  const int xrow = a.xgc * 2;                       // bytes per pixel step
  auto stage = [&](int kt, int buf) {               // kt: the split's K-tile index
    unsigned char *base = smem + buf * STG + ws * P * 1024;
    const int lim = (int)(mend - mbeg) - kt * BK;   // rows r < lim are inside the split
    const int adel = kt * BK * a.g.Cout * 2;
#pragma unroll
    for (int j = 0; j < P; ++j) {
      glds16(rd, base + j * 1024, rr[j] < lim && aok[j] ? (uint32_t)(aoff[j] + adel) : OOB);
      const uint32_t owt = (uint32_t)(sow + rr[j]);
      const uint32_t q = __umulhi(owt, magW);
      const int ow = (int)(owt - q * a.g.Wo);
      const uint32_t oht = (uint32_t)soh + q;
      const uint32_t q2 = __umulhi(oht, magH);
      const int oh = (int)(oht - q2 * a.g.Ho);
      const int n = sn + (int)q2;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int e = b * P + j;
        const int ih = oh * a.g.stride + tkh[e], iw = ow * a.g.stride + tkw[e];
        const bool ok = rr[j] < lim && bok[e] && (unsigned)ih < (unsigned)a.g.H && (unsigned)iw < (unsigned)a.g.W;
        glds16(rx, base + (1 + b) * IMG + j * 1024,
               ok ? (uint32_t)(((n * a.g.H + ih) * a.g.W + iw) * xrow + bgo[e]) : OOB);
      }
    }
    sow += BK;                                      // the next K-tile (scalar)
    while (sow >= a.g.Wo) {
      sow -= a.g.Wo;
      if (++soh == a.g.Ho) { soh = 0; ++sn; }
    }
  };
  auto tr_read = [&](const unsigned char *img, int k0, int c0) -> cs4 {
    const int i = lane & 15, q = i >> 2, p = i & 3;
    const int col = c0 + 4 * p;
    const int off = swz_off(k0 + q, col >> 3) + 2 * (col & 7);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) cs4 *)(img + off));
  };
  const bool do_bias = a.dbias_part != nullptr;
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  cf32x4 acc[4][WJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j) acc[i][j] = cf32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4;
  auto compute = [&](int kt, int buf) {
    const unsigned char *As = smem + buf * STG;
    // wave column wn: 64 columns of the one x image (WJ 4), or a whole image (WJ 8)
    const unsigned char *Bs = As + IMG + (NB > 1 ? wn * IMG : 0);
    const int bc0 = NB > 1 ? 0 : wn * 64;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      cbf16x8 af[4], bfr[WJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const cs4 lo = tr_read(As, ks * 32 + 8 * g, wm * 64 + i * 16);
        const cs4 hi = tr_read(As, ks * 32 + 8 * g + 4, wm * 64 + i * 16);
        af[i] = __builtin_bit_cast(cbf16x8, (__attribute__((ext_vector_type(8))) short){
                                                lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
      }
#pragma unroll
      for (int j = 0; j < WJ; ++j) {
        const cs4 lo = tr_read(Bs, ks * 32 + 8 * g, bc0 + j * 16);
        const cs4 hi = tr_read(Bs, ks * 32 + 8 * g + 4, bc0 + j * 16);
        bfr[j] = __builtin_bit_cast(cbf16x8, (__attribute__((ext_vector_type(8))) short){
                                                 lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < WJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (do_bias && kt % ntx == tx) {
      // thread t of a K-group: rows (t>>4)*(BK/16) .. of its dy image, chunk t & 15 (8 channels)
#pragma unroll
      for (int q = 0; q < BK / 16; ++q) {
        const int r = (tid >> 4) * (BK / 16) + q;
        const uint4 v = *reinterpret_cast<const uint4 *>(As + swz_off(r, tid & 15));
        const unsigned wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bsum[2 * e] += __uint_as_float(wv[e] << 16);
          bsum[2 * e + 1] += __uint_as_float(wv[e] & 0xffff0000u);
        }
      }
    }
  };
  int ld = 0, lbuf = 0;
  for (; ld < NS - 1 && ld < nk; ++ld) {
    stage(ld, lbuf);
    lbuf = lbuf + 1 == NS ? 0 : lbuf + 1;
  }
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    wait_tile<(1 + NB) * P, NS>(nk - 1 - kt);
    if (ld < nk) {
      stage(ld, lbuf);
      ++ld;
      lbuf = lbuf + 1 == NS ? 0 : lbuf + 1;
    }
    compute(kt, cur);
    cur = cur + 1 == NS ? 0 : cur + 1;
  }
  __syncthreads();
  if (do_bias) {
    // threads t, t^16, t^32, t^48 of a wave hold the same 8 channels; then the 4 waves
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bsum[j] = rows_sum4(bsum[j]);
    }
    float *red = reinterpret_cast<float *>(smem);
    if (lane < 16)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[(w * 16 + lane) * 8 + j] = bsum[j];
    __syncthreads();
    if (tid < 128) {
      const int ch = tid >> 3, j = tid & 7;
      const int co = co0 + ch * 8 + j;
      float s = (red[(0 * 16 + ch) * 8 + j] + red[(1 * 16 + ch) * 8 + j]) +
                (red[(2 * 16 + ch) * 8 + j] + red[(3 * 16 + ch) * 8 + j]);
      if (co < a.g.Cout) a.dbias_part[((int64_t)split * ntx + tx) * a.g.Cout + co] = s;
    }
  }
  float *dst = a.part + (int64_t)split * a.g.Cout * NP;
#pragma unroll
  for (int j = 0; j < WJ; ++j) {
    const int col = np0 + wn * 16 * WJ + j * 16 + (lane & 15);
    if (col >= NP) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = co0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (row < a.g.Cout) dst[(int64_t)row * NP + col] = acc[i][j][r];
      }
  }
}

// 1x1 stride-1 weight gradient over a plain NHWC x (the backbone's MBConv expand / project and
// head convs, sfe.py:111-113): dW[co][ci] = sum_m dy[m][co] * x[m][ci] with no pixel map, so a
// staging lane's global offset is one register advanced by a scalar stride per K-tile (lanes
// past Cout / Cin start at OOB and stay there; rows >= M fall past the buffer's end and read
// zeros) — none of the generic kernel's per-piece address math; the DMAs are asm (glds16_asm),
// so hipcc does not drain them before the fragment reads.  128 x 128 output tile, 4 waves
// of 64 x 64, 64-pixel K-tiles in an NS-deep LDS-DMA ring; a K-tile's fragments for both
// 32-pixel steps are read before its MFMAs, so the second step's reads overlap the first
// step's MFMAs.  Leaves [splits][Cout][Cin] slabs (conv_wgrad_reduce_kernel), or dW itself for
// one split.
template <int NS>
__global__ __launch_bounds__(256) void conv_wgrad_1x1_kernel(WgradArgs a, int ntx, int nty, RedJobs rj) {
  constexpr int BK = 64, IMG = BK * 256, STG = 2 * IMG, P = BK / 16;
  __shared__ __attribute__((aligned(16))) unsigned char smem[NS * STG];
  // the first rj.nblk workgroups run deferred reductions of earlier weight gradients
  if ((int)blockIdx.x < rj.nblk) {
    run_red_jobs(rj, (int)blockIdx.x, reinterpret_cast<float *>(smem));
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tile = xcd_remap((int)blockIdx.x - rj.nblk, (int)gridDim.x - rj.nblk);
  const int split = tile / (ntx * nty);
  const int tx = tile % ntx, ty = (tile / ntx) % nty;
  const int co0 = ty * 128, ci0 = tx * 128;
  const int Cout = a.g.Cout, Cin = a.g.Cin;
  const int64_t mbeg = (int64_t)split * a.mper;
  const int64_t mend = mbeg + a.mper < a.M ? mbeg + a.mper : a.M;
  const int nk = (int)((mend - mbeg + BK - 1) / BK);
  const __amdgpu_buffer_rsrc_t rx = mk_rsrc(a.x, a.M * Cin * 2);
  const __amdgpu_buffer_rsrc_t rd = mk_rsrc(a.dy, a.M * Cout * 2);
  const int ws = __builtin_amdgcn_readfirstlane(w);
  const int wm = ws >> 1, wn = ws & 1;
  // piece j of wave ws: rows 16 ws + 4 j + lane / 16, source chunk (lane % 16) ^ swz(row)
  uint32_t aoff[P], boff[P];
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const int r = ws * 16 + 4 * j + (lane >> 4);
    const int lc = (lane & 15) ^ (((r & 3) << 2) | ((r >> 2) & 3));
    aoff[j] = co0 + lc * 8 < Cout ? (uint32_t)(((mbeg + r) * Cout + co0 + lc * 8) * 2) : OOB;
    boff[j] = ci0 + lc * 8 < Cin ? (uint32_t)(((mbeg + r) * Cin + ci0 + lc * 8) * 2) : OOB;
  }
  const uint32_t adel = (uint32_t)(BK * Cout * 2), bdel = (uint32_t)(BK * Cin * 2);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char *)smem + ws * P * 1024;
  auto stage = [&](int buf) __attribute__((always_inline)) {
    const uint32_t base = lds0 + buf * STG;
#pragma unroll
    for (int j = 0; j < P; ++j) {
      glds16_asm(rd, base + j * 1024, aoff[j]);
      glds16_asm(rx, base + IMG + j * 1024, boff[j]);
      aoff[j] += adel;
      boff[j] += bdel;
    }
  };
  auto tr_read = [&](const unsigned char *img, int k0, int c0) __attribute__((always_inline)) -> cs4 {
    const int i = lane & 15, q = i >> 2, p = i & 3;
    const int col = c0 + 4 * p;
    const int off = swz_off(k0 + q, col >> 3) + 2 * (col & 7);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) cs4 *)(img + off));
  };
  cf32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = cf32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4;
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const unsigned char *As = smem + buf * STG, *Bs = As + IMG;
    cbf16x8 af[2][4], bfr[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const cs4 alo = tr_read(As, ks * 32 + 8 * g, wm * 64 + i * 16);
        const cs4 ahi = tr_read(As, ks * 32 + 8 * g + 4, wm * 64 + i * 16);
        af[ks][i] = __builtin_bit_cast(cbf16x8, (__attribute__((ext_vector_type(8))) short){
                                                     alo[0], alo[1], alo[2], alo[3], ahi[0], ahi[1], ahi[2], ahi[3]});
        const cs4 blo = tr_read(Bs, ks * 32 + 8 * g, wn * 64 + i * 16);
        const cs4 bhi = tr_read(Bs, ks * 32 + 8 * g + 4, wn * 64 + i * 16);
        bfr[ks][i] = __builtin_bit_cast(cbf16x8, (__attribute__((ext_vector_type(8))) short){
                                                      blo[0], blo[1], blo[2], blo[3], bhi[0], bhi[1], bhi[2], bhi[3]});
      }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[ks][j], acc[i][j], 0, 0, 0);
  };
  int ld = 0, lbuf = 0;
  for (; ld < NS - 1 && ld < nk; ++ld) {
    stage(lbuf);
    lbuf = lbuf + 1 == NS ? 0 : lbuf + 1;
  }
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    wait_tile<2 * P, NS>(nk - 1 - kt);
    if (ld < nk) {
      stage(lbuf);
      ++ld;
      lbuf = lbuf + 1 == NS ? 0 : lbuf + 1;
    }
    compute(cur);
    cur = cur + 1 == NS ? 0 : cur + 1;
  }
  float *dst = a.part + (int64_t)split * Cout * Cin;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = ci0 + wn * 64 + j * 16 + (lane & 15);
    if (col >= Cin) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = co0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (row < Cout) dst[(int64_t)row * Cin + col] = acc[i][j][r];
      }
  }
}

// Kernel family: 1 (default) the LDS-DMA kernels wherever the shape allows them, the
// register-staged kernels elsewhere; 0 the register-staged kernels everywhere — a test
// switch (ewvit_conv2d_set_glds): they are the fallback of the shapes the LDS-DMA kernels
// refuse, so the tests run every case through both.  (The other tile / ring-depth families
// measured while tuning — 3-deep rings, 256-row tiles everywhere, 64-row tiles for small
// grids, wide 64 x 128 waves, two K-groups per wgrad workgroup — were slower and are gone;
// their numbers are in DESIGN.md §5.)
static int g_glds = 1;
static bool use_glds() { return g_glds != 0; }

// M-tiles of the register-staged grid: all, or (g_grid_cap) at most cap / N-tiles of them
static unsigned capped_mtiles(int64_t M, int ntn) {
  int64_t gx = (M + CBM - 1) / CBM;
  if (g_grid_cap > 0 && gx * ntn > g_grid_cap) gx = g_grid_cap / ntn > 0 ? g_grid_cap / ntn : 1;
  return (unsigned)gx;
}

// ---------------------------------------------------------------- small-channel 3x3
// 3x3 stride-1 convs over few channels (KC = 16 / 24 per tap, <= 64 outputs): stage 1 of the
// backbone (24 -> 24 at 112^2, forward and input gradient) and the MWT seperate conv
// (16 -> 64).  A GEMM tile of 128 pixels re-gathers its 9 taps from L2 per K-tile; here a
// workgroup stages the input rows its TH output rows need ONCE in LDS ([TH+2][W+2][KC] bf16,
// zero halo — no bounds tests in the loop), keeps the packed weights of all taps in
// registers (they are the MFMA A operand: K = 9*KC padded to k-steps of 32, N = Ncol padded
// to 16-wide tiles), and walks 16-pixel groups: per group, KSTEPS ds_read_b128 of the pixel
// operand and NT*KSTEPS v_mfma_f32_16x16x32_bf16.  Operands weights-first, so a lane ends
// with 4 consecutive output channels of one pixel (8-byte stores).  FLIP: the input gradient
// (taps mirrored; weights packed [Cin][taps][Cout]).  Grid: (N * ceil(H/TH)) workgroups,
// walked persistently when the launch is capped.
template <int KC, int NT, bool FLIP>
__global__ __launch_bounds__(256) void conv3x3_small_kernel(FwdArgs a, int TH, int nblk) {
  constexpr int CC = KC / 8, NCH = 9 * CC, KSTEPS = (NCH + 3) / 4, K = 9 * KC;
  extern __shared__ __attribute__((aligned(16))) unsigned char cs_smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int H = a.outH, W = a.outW, Wp = W + 2;
  const int rowb = Wp * KC * 2;                  // bytes per staged row
  // weights (MFMA A operand): lane -> output channel (lane & 15) of each 16-wide tile,
  // k chunk 4*s + (lane >> 4)
  cbf16x8 wf[NT][KSTEPS];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      const int n = t * 16 + (lane & 15), kc = 4 * s + (lane >> 4);
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (n < a.Ncol && kc < NCH) v = *reinterpret_cast<const uint4 *>(a.wp + (int64_t)n * K + kc * 8);
      wf[t][s] = __builtin_bit_cast(cbf16x8, v);
    }
  float bias[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = t * 16 + 4 * (lane >> 4) + i;
      bias[t][i] = (a.bias && n < a.Ncol) ? a.bias[n] : 0.f;
    }
  const int nbh = (H + TH - 1) / TH;
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int img = blk / nbh, r0 = (blk - img * nbh) * TH;
    const int rows = H - r0 < TH ? H - r0 : TH;
    // stage input rows r0-1 .. r0+TH, cols -1 .. W, 16 B (8 channels) per item
    const int items = (TH + 2) * Wp * CC;
    __syncthreads();                             // the previous tile's readers are done
    for (int i = tid; i < items; i += 256) {
      const int c8 = i % CC, px = i / CC;
      const int tr = px / Wp, tc = px - tr * Wp;
      const int ir = r0 - 1 + tr, ic = tc - 1;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if ((unsigned)ir < (unsigned)H && (unsigned)ic < (unsigned)W)
        v = *reinterpret_cast<const uint4 *>(a.src + (((int64_t)img * H + ir) * W + ic) * KC + c8 * 8);
      *reinterpret_cast<uint4 *>(cs_smem + (size_t)tr * rowb + (tc * KC + c8 * 8) * 2) = v;
    }
    __syncthreads();
    const int npx = rows * W, ngr = (npx + 15) / 16;
    for (int gi = w; gi < ngr; gi += 4) {
      const int q = gi * 16 + (lane & 15);
      const int qq = q < npx ? q : npx - 1;
      const int r = qq / W, c = qq - r * W;
      cf32x4 acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = cf32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        const int kc = 4 * s + (lane >> 4);
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (kc < NCH) {
          const int tap = kc / CC, c8 = kc - tap * CC;
          const int kh = tap / 3, kw = tap - kh * 3;
          const int tr = FLIP ? r + 2 - kh : r + kh, tc = FLIP ? c + 2 - kw : c + kw;
          v = *reinterpret_cast<const uint4 *>(cs_smem + (size_t)tr * rowb + (tc * KC + c8 * 8) * 2);
        }
        const cbf16x8 xf = __builtin_bit_cast(cbf16x8, v);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][s], xf, acc[t], 0, 0, 0);
      }
      if (q < npx) {
        bf16_t *o = a.out + (((int64_t)img * H + r0 + r) * W + c) * a.Ncol;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int n = t * 16 + 4 * (lane >> 4);
          if (n < a.Ncol) {
            const uint32_t lo = (uint32_t)f2bf(acc[t][0] + bias[t][0]) | ((uint32_t)f2bf(acc[t][1] + bias[t][1]) << 16);
            const uint32_t hi = (uint32_t)f2bf(acc[t][2] + bias[t][2]) | ((uint32_t)f2bf(acc[t][3] + bias[t][3]) << 16);
            *reinterpret_cast<uint2 *>(o + n) = make_uint2(lo, hi);
          }
        }
      }
    }
  }
}

static bool launch_small(const FwdArgs &a, bool dgrad, hipStream_t s) {
  if (a.g.ks != 3 || a.g.stride != 1 || a.sgs != 0 || a.ogs != 0 || a.sgc != a.KC || a.ogc != a.Ncol ||
      a.KCr || a.addend || a.bn_part || a.pc >= 0 || a.outH != a.srcH || a.outW != a.srcW || a.outW > 256 ||
      a.Ncol % 8)
    return false;
  const int KC = a.KC, NT = (a.Ncol + 15) / 16;
  if (!((KC == 24 && NT <= 2) || (KC == 16 && NT <= 4))) return false;
  const int H = a.outH, W = a.outW;
  // rows per workgroup, LDS <= 64 KB: 4 rows for 24 channels (stage 1: 29 us; 2 / 6 / 8 rows
  // 34 / 31 / 33 us), 8 for 16 (the seperate conv: 119 us; 4 / 6 / 12 rows 129 / 123 / 133 us),
  // tools/small_ab.sh
  const int ldsmax = 64 * 1024;
  const int thmax = KC == 16 ? 8 : 4;
  int TH = thmax;
  while (TH > 1 && (TH + 2) * (W + 2) * KC * 2 > ldsmax) --TH;
  const size_t lds = (size_t)(TH + 2) * (W + 2) * KC * 2;
  const int64_t nblk64 = (int64_t)a.g.N * ((H + TH - 1) / TH);
  if (nblk64 >= (1ll << 31)) return false;
  const int nblk = (int)nblk64;
  const dim3 grid((unsigned)(g_grid_cap > 0 && nblk > g_grid_cap ? g_grid_cap : nblk));
#define EWVIT_SMALL(KC_, NT_)                                                                                     \
  do {                                                                                                          \
    if (dgrad)                                                                                                  \
      hipLaunchKernelGGL((conv3x3_small_kernel<KC_, NT_, true>), grid, dim3(256), lds, s, a, TH, nblk);        \
    else                                                                                                        \
      hipLaunchKernelGGL((conv3x3_small_kernel<KC_, NT_, false>), grid, dim3(256), lds, s, a, TH, nblk);       \
  } while (0)
  if (KC == 24) {
    if (NT == 1) EWVIT_SMALL(24, 1);
    else EWVIT_SMALL(24, 2);
  } else {
    if (NT <= 2) EWVIT_SMALL(16, 2);
    else EWVIT_SMALL(16, 4);
  }
#undef EWVIT_SMALL
  return true;
}

template <bool DGRAD, int KS, int BK, int PF>
static void launch_fwd_v(const FwdArgs &a, hipStream_t s) {
  if (a.Ncol <= 64) {
    dim3 grid(capped_mtiles(a.M, 1), 1);
    hipLaunchKernelGGL((conv_fwd_kernel<DGRAD, 64, KS, BK, PF>), grid, dim3(256), 0, s, a);
  } else {
    const int ntn = (a.Ncol + CBN - 1) / CBN;
    dim3 grid(capped_mtiles(a.M, ntn), (unsigned)ntn);
    hipLaunchKernelGGL((conv_fwd_kernel<DGRAD, 128, KS, BK, PF>), grid, dim3(256), 0, s, a);
  }
}

template <bool DGRAD, int KS>
static void launch_fwd_ks(const FwdArgs &a, hipStream_t s) {
  if (a.KC % 64 == 0 && a.sgc % 64 == 0) launch_fwd_v<DGRAD, KS, 64, 1>(a, s);
  else launch_fwd_v<DGRAD, KS, 32, 1>(a, s);
}

template <bool DGRAD>
static void launch_fwd(const FwdArgs &a, hipStream_t s) {
  if (a.g.ks == 1) launch_fwd_ks<DGRAD, 1>(a, s);
  else launch_fwd_ks<DGRAD, 3>(a, s);
}

// the dense-K forward (conv_glds_kernel<false, ..., DENSE>): 128-row tiles, 8 waves with a
// 2-deep ring for grids of <= 2048 blocks, 4 waves beyond, the 4-deep ring for <= 256
static void launch_glds_dense(const FwdArgs &a, int64_t src_bytes, hipStream_t s) {
  const int bn = 128;
  const int ntn = (a.Ncol + bn - 1) / bn;
  const int64_t nwg = (a.M + 127) / 128 * ntn;
  const int ntiles = (int)nwg;
  const dim3 grid((unsigned)(g_grid_cap > 0 && nwg > g_grid_cap ? g_grid_cap : nwg));
#define EWVIT_GLDS_DENSE(BN__, NS_, WC_)                                                                            \
  do {                                                                                                            \
    if (a.g.ks == 1)                                                                                              \
      hipLaunchKernelGGL((conv_glds_kernel<false, 128, BN__, 1, NS_, WC_, true>), grid, dim3(128 / 64 * WC_ * 64), \
                         0, s, a, src_bytes, ntn, 0, ntiles);                                                     \
    else                                                                                                          \
      hipLaunchKernelGGL((conv_glds_kernel<false, 128, BN__, 3, NS_, WC_, true>), grid, dim3(128 / 64 * WC_ * 64), \
                         0, s, a, src_bytes, ntn, 0, ntiles);                                                     \
  } while (0)
  (void)bn;                                // Ncol > 64: 128-wide column tiles
  // grids up to 4096 blocks take 8 waves (stage 2's 48 -> 192 expands, 3136 blocks: 81 -> 75
  // us); a 3-deep ring for the big grids measured 30-60 % slower
  if (nwg <= 256) EWVIT_GLDS_DENSE(128, 4, 4);
  else if (nwg <= 4096) EWVIT_GLDS_DENSE(128, 2, 4);
  else EWVIT_GLDS_DENSE(128, 2, 2);
#undef EWVIT_GLDS_DENSE
}

// the LDS-DMA fwd/dgrad kernel when every K-tile stays in one tap and one channel
// group and the operands fit 31-bit buffer offsets; false -> register-staged kernel
// Tile of the LDS-DMA fwd / dgrad: 128 rows (256 for a <= 64-column dgrad over > 4096 row tiles:
// the MWT fusion conv's input gradient); grids of < 128 such tiles — the backbone's long-K
// 1x1 convs at 7^2 (stage 6 project forward / expand input gradient: 3136 x 256 x 1536, 50
// tiles, 24 K-tiles each) — take 64-row tiles, and 64-column tiles if still < 128 (4x the
// workgroups).  Any BatchNorm partial rows the kernel leaves follow its row tile.
static int g_small_tiles = 1;
extern "C" int ewvit_conv2d_set_small_tiles(int on) {
  const int prev = g_small_tiles;
  g_small_tiles = on ? 1 : 0;
  return prev;
}
static void glds_tile(const FwdArgs &a, bool dgrad, int &bm, int &bn) {
  bn = a.Ncol <= 32 ? 32 : a.Ncol <= 64 ? 64 : 128;
  const int64_t ntn = (a.Ncol + bn - 1) / bn, mt = (a.M + 127) / 128;
  bm = 128;
  if (dgrad && bn == 64 && mt * ntn > 4096 && !a.bwd.part) { bm = 256; return; }
  if (g_small_tiles && bn >= 64 && mt * ntn < 128) {
    bm = 64;
    if (bn == 128 && (a.M + 63) / 64 * ntn < 128) bn = 64;
  }
}

// split K for the LDS-DMA 1x1 fwd / dgrad (FwdArgs::ksplit): the backbone's long-K 1x1 convs
// over few tiles — stage 6's project forward / expand input gradient (3136 x 256 x 1536: 196
// workgroups of 24 K-tiles), the head conv (K = 1280) — run their K loop serially per workgroup
// on < 256 workgroups.  Split into S ranges (S | K-tiles, >= g_ksplit_min_kt K-tiles each, <= 1024
// work items), fp32 partials in a per-stream scratch buffer, conv_splitk_epi_kernel for the
// epilogue.  OFF by default: measured slower in the step at every setting — S <= 2 / >= 8 K-tiles
// 3725-3729, S <= 2 / >= 4 3710, S <= 4 / >= 8 3708-3713, S <= 8 / >= 4 3665-3679 against
// 3755-3766 frames/s unsplit (same box, profiles/r06/ab/ksplit.log): beside the MWT the step is
// bound by CU-time and memory traffic, which the partials and the epilogue pass add to, not by
// these kernels' latency.  ewvit_conv2d_set_ksplit(1) / EWVIT_CONV_KSPLIT=1: on (tests, A/B).
static int g_ksplit = 0, g_ksplit_max = 2, g_ksplit_min_kt = 8;
extern "C" int ewvit_conv2d_set_ksplit(int on) {
  const int prev = g_ksplit;
  g_ksplit = on ? 1 : 0;
  if (on > 1) { g_ksplit_max = on & 15; g_ksplit_min_kt = on >> 4; }   // tuning: max S | min K-tiles << 4
  return prev;
}
// the split partials' scratch, one buffer per stream (the branches run convs concurrently),
// grown outside stream capture only (nullptr -> the caller runs unsplit); a replaced buffer is
// kept, since kernels queued on the stream may still read it
static float *ksplit_scratch(hipStream_t s, size_t bytes) {
  static std::mutex mu;
  static std::unordered_map<hipStream_t, std::pair<void *, size_t>> bufs;
  std::lock_guard<std::mutex> lk(mu);
  auto &e = bufs[s];
  if (e.second >= bytes) return static_cast<float *>(e.first);
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
  void *p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
  e = {p, bytes};
  return static_cast<float *>(p);
}

template <bool DGRAD>
static bool launch_glds(FwdArgs a, int64_t src_bytes, hipStream_t s, int *bm_out = nullptr) {
  const int64_t K = (int64_t)a.g.ks * a.g.ks * a.KC;
  const bool padded = a.KCr && a.KCr != a.KC;     // plain x, channels padded to 64 per tap
  // ragged: plain (ungrouped) x whose per-tap K is not a multiple of 64 — the last
  // 64-channel block of each tap zero-fills its A lanes >= KC and reads finite weights
  // of the next tap / row (or zeros past the end) for B, which meet only zeros
  // (only while the zero lanes stay <= 20 % of K: K = 48 per tap measured slower than
  // the register-staged kernel, K = 160 -> 3 blocks 17 % faster)
  const bool ragged = !padded && a.KC % 64 != 0;
  // (only with 128-wide column tiles: for Cout <= 64 — stage 1's 24 -> 24 at 112^2, the MWT
  // seperate conv's 16 -> 64, the 96 -> 48 projects — the register-staged kernel measured
  // as fast or faster: 62 vs 64, 166 vs 199, 15 vs 16 us; Cout 96 / 192: 39 -> 32, 106 -> 81,
  // 34 -> 27 us, tools/conv_bench.py)
  if (!DGRAD && ragged && use_glds() && a.Ncol > 64 && a.sgs == 0 && a.sgc == a.KC && a.KC % 8 == 0 &&
      src_bytes < (int64_t)OOB && a.Ncol * K * 2 < (int64_t)OOB && a.M * a.ogc < ((int64_t)1 << 40) &&
      (a.g.ks == 1 || a.g.ks == 3)) {
    launch_glds_dense(a, src_bytes, s);
    return true;
  }
  // a parity-class dgrad, which already skips 3/4 of the taps, takes up to 1/3 zero lanes
  const int kpad = (a.KC + 63) / 64 * 64;
  const bool ragged_ok = a.pc >= 0 ? 2 * kpad <= 3 * a.KC : 5 * kpad <= 6 * a.KC;
  if (ragged && (a.sgs != 0 || a.sgc != a.KC || a.KC % 8 || !ragged_ok))
    return false;
  if (!use_glds() || (!ragged && a.KC % 64) || (padded ? a.sgc != a.KCr : (!ragged && a.sgc % 64)) ||
      src_bytes >= (int64_t)OOB ||
      a.Ncol * K * 2 >= (int64_t)OOB ||
      a.M * a.ogc >= (int64_t)1 << 40)
    return false;
  const int tap_inner = 1;           // the 9 taps of a 64-channel block are consecutive K-tiles
  // <= 32 columns (stage 2's entry-conv input gradient, 24 channels): 32-wide column tiles.
  // A <= 64-column dgrad over > 4096 row tiles (the MWT fusion conv's 56-channel input
  // gradient, 2.4 M pixels): 256-row blocks, 535 -> 505 us.  Stage 2's 48-channel 3x3 dgrad
  // (1568 row tiles) runs faster on 8-wave 128-row blocks (96 -> 75 us, tools/dgrad_ab.sh)
  int BM, bn;
  glds_tile(a, DGRAD, BM, bn);
  const int ntn = (a.Ncol + bn - 1) / bn;
  const bool big = BM == 256;
  if (bm_out) *bm_out = BM;
  const int64_t mt = (a.M + BM - 1) / BM;
  int64_t nwg = mt * ntn;
  if (nwg >= (int64_t)1 << 31) return false;
  int S = 1;
  if (g_ksplit && a.g.ks == 1 && a.pc < 0 && !padded && !ragged && a.sgs == 0 && a.sgc == a.KC && a.ogs == 0 &&
      a.ogc == a.Ncol && !big && nwg < 256) {
    const int nkt = a.KC / 64;
    for (int c = g_ksplit_max; c >= 2; --c)
      if (nkt % c == 0 && nkt / c >= g_ksplit_min_kt && nwg * c <= 1024) { S = c; break; }
    if (S > 1) {
      float *ws = ksplit_scratch(s, (size_t)S * a.M * a.Ncol * sizeof(float));
      if (ws) { a.ksplit = S; a.kpart = ws; nwg *= S; }
      else S = 1;
    }
  }
  const int ntiles = (int)nwg;
  const dim3 grid((unsigned)(g_grid_cap > 0 && nwg > g_grid_cap ? g_grid_cap : nwg));
#define EWVIT_GLDS_FWDW(BM_, BN__, NS_, WC_, BST_)                                                                  \
  do {                                                                                                            \
    if (a.g.ks == 1)                                                                                              \
      hipLaunchKernelGGL((conv_glds_kernel<DGRAD, BM_, BN__, 1, NS_, WC_, false, BST_>), grid,                     \
                         dim3(BM_ / 64 * WC_ * 64), 0, s, a, src_bytes, ntn, tap_inner, ntiles);                  \
    else                                                                                                          \
      hipLaunchKernelGGL((conv_glds_kernel<DGRAD, BM_, BN__, 3, NS_, WC_, false, BST_>), grid,                     \
                         dim3(BM_ / 64 * WC_ * 64), 0, s, a, src_bytes, ntn, tap_inner, ntiles);                  \
  } while (0)
  // Blocks: grids of <= 2048 workgroups (the backbone's 7^2 - 28^2 convs) and every dgrad with
  // 128-wide column tiles (freq_conv's parity-class dgrad 185 -> 162 us, multiscale 834 -> 820)
  // take 8 waves (64 x BN/4 each) — twice the waves per CU to hide the latency of short K
  // loops; big grids keep 4 waves (64 x BN/2 each: fewer LDS reads per MFMA).  Grids of <= 256
  // workgroups (the backbone's long-K 1x1 convs at 7^2 / 14^2: at most one block per CU, so
  // occupancy hides nothing) take 8 waves with a 4-deep ring (3 K-tiles in flight).
  const bool w8 = nwg <= 2048 || (DGRAD && bn == 128);
  const bool sg = nwg <= 256;
  constexpr bool BST = DGRAD;      // (the statistics epilogue is a separate instantiation)
  const bool bst = DGRAD && a.bwd.part && S == 1;   // (split K: the epilogue kernel sums them)
  if (BM == 64) {
    if (bst) {
      if (bn == 64) EWVIT_GLDS_FWDW(64, 64, 4, 4, BST);
      else EWVIT_GLDS_FWDW(64, 128, 4, 4, BST);
    } else if (bn == 64) EWVIT_GLDS_FWDW(64, 64, 4, 4, false);
    else EWVIT_GLDS_FWDW(64, 128, 4, 4, false);
  } else if (bst) {
    // the backward-statistics epilogue: 128-row tiles (the partial rows
    // ewvit_conv2d_bwd_bn_rows promised)
    if (bn == 32) EWVIT_GLDS_FWDW(128, 32, 2, 2, BST);
    else if (bn == 64) {
      if (sg) EWVIT_GLDS_FWDW(128, 64, 4, 4, BST);
      else if (w8) EWVIT_GLDS_FWDW(128, 64, 2, 4, BST);
      else EWVIT_GLDS_FWDW(128, 64, 2, 2, BST);
    } else {
      if (sg) EWVIT_GLDS_FWDW(128, 128, 4, 4, BST);
      else if (w8) EWVIT_GLDS_FWDW(128, 128, 2, 4, BST);
      else EWVIT_GLDS_FWDW(128, 128, 2, 2, BST);
    }
  } else if (bn == 32) EWVIT_GLDS_FWDW(128, 32, 2, 2, false);
  else if (bn == 64) {
    if (big) EWVIT_GLDS_FWDW(256, 64, 2, 2, false);
    else if (sg) EWVIT_GLDS_FWDW(128, 64, 4, 4, false);
    else if (w8) EWVIT_GLDS_FWDW(128, 64, 2, 4, false);
    else EWVIT_GLDS_FWDW(128, 64, 2, 2, false);
  } else {
    if (sg) EWVIT_GLDS_FWDW(128, 128, 4, 4, false);
    else if (w8) EWVIT_GLDS_FWDW(128, 128, 2, 4, false);
    else EWVIT_GLDS_FWDW(128, 128, 2, 2, false);
  }
#undef EWVIT_GLDS_FWDW
  if (S > 1) {
    const dim3 eg((unsigned)mt, (unsigned)((a.Ncol + 63) / 64));
    if (DGRAD && a.bwd.part) hipLaunchKernelGGL(conv_splitk_epi_kernel<2>, eg, dim3(256), 0, s, a, BM);
    else if (!DGRAD && a.bn_part) hipLaunchKernelGGL(conv_splitk_epi_kernel<1>, eg, dim3(256), 0, s, a, BM);
    else hipLaunchKernelGGL(conv_splitk_epi_kernel<0>, eg, dim3(256), 0, s, a, BM);
  }
  return true;
}

static int check_geom(const ConvGeom &g, const char *nm) {
  EWVIT_CHECK_ARG(g.N > 0 && g.H > 0 && g.W > 0 && g.Cin > 0 && g.Cout > 0, "%s: empty shape", nm);
  EWVIT_CHECK_ARG(g.Cin % 8 == 0 && g.Cout % 8 == 0, "%s: Cin=%d Cout=%d must be multiples of 8", nm, g.Cin, g.Cout);
  EWVIT_CHECK_ARG(g.stride == 1 || g.stride == 2, "%s: stride %d", nm, g.stride);
  EWVIT_CHECK_ARG(g.ks == 1 || g.ks == 3, "%s: kernel size %d (1 or 3)", nm, g.ks);
  return 0;
}

// grouped layout (gc, gs) for a tensor of C channels: gc == 0 means plain NHWC
static int check_group(int64_t &gc, int64_t &gs, int64_t C, int64_t pixels, const char *nm, const char *which) {
  if (gc == 0 || gc == C) { gc = C; gs = 0; return 0; }
  EWVIT_CHECK_ARG(gc > 0 && gc % CBK == 0 && C % gc == 0, "%s: %s group width %lld must divide %lld and be a multiple of %d",
                  nm, which, (long long)gc, (long long)C, CBK);
  EWVIT_CHECK_ARG(gs >= pixels * gc, "%s: %s group stride %lld < %lld", nm, which, (long long)gs, (long long)(pixels * gc));
  return 0;
}

static ConvGeom mkg(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ks, int stride) {
  ConvGeom g;
  g.N = (int)N; g.H = (int)H; g.W = (int)W; g.Cin = (int)Cin; g.Cout = (int)Cout; g.stride = stride;
  g.ks = ks; g.pad = ks / 2;
  g.Ho = (int)((H - 1) / stride + 1);
  g.Wo = (int)((W - 1) / stride + 1);
  return g;
}

// ---- deferred weight-gradient reductions (reduce_jobs.h): per-stream FIFO of jobs
static thread_local bool t_defer_next = false;
static std::mutex g_red_mu;
static std::deque<std::pair<hipStream_t, RedJob>> g_red_q;

bool reduce_take_defer() {
  const bool d = t_defer_next;
  t_defer_next = false;
  return d;
}

void reduce_defer(hipStream_t s, const RedJob &j) {
  std::lock_guard<std::mutex> lk(g_red_mu);
  g_red_q.emplace_back(s, j);
}

RedJobs reduce_take_jobs(hipStream_t s) {
  RedJobs r;
  std::lock_guard<std::mutex> lk(g_red_mu);
  int q = 0;
  for (auto it = g_red_q.begin(); it != g_red_q.end() && q < 2;) {
    if (it->first == s) {
      r.j[q] = it->second;
      r.j[q].nblk = red_job_blocks(it->second);
      r.nblk += r.j[q].nblk;
      ++q;
      it = g_red_q.erase(it);
    } else {
      ++it;
    }
  }
  r.nblk = (r.nblk + 7) / 8 * 8;
  return r;
}

// deferred jobs alone (ewvit_reduce_flush): 2 per launch
__global__ __launch_bounds__(256) void red_jobs_kernel(RedJobs rj) {
  __shared__ float red[256];
  run_red_jobs(rj, (int)blockIdx.x, red);
}

}  // namespace ewvit

using namespace ewvit;

// ---- deferred reductions (reduce_jobs.h)
extern "C" int ewvit_reduce_defer_next(int on) {
  t_defer_next = on != 0;
  return 0;
}

extern "C" int ewvit_reduce_pending(void *stream) {
  std::lock_guard<std::mutex> lk(g_red_mu);
  int n = 0;
  for (auto &e : g_red_q)
    if (!stream || e.first == as_stream(stream)) ++n;
  return n;
}

extern "C" int ewvit_reduce_flush(void *stream) {
  hipStream_t s = as_stream(stream);
  for (;;) {
    RedJobs rj = reduce_take_jobs(s);
    if (rj.nblk == 0) return 0;
    hipLaunchKernelGGL(red_jobs_kernel, dim3((unsigned)rj.nblk), dim3(256), 0, s, rj);
    if (int rc = launch_status("reduce_flush")) return rc;
  }
}

extern "C" int ewvit_set_grid_cap(int max_workgroups);
extern "C" int ewvit_conv2d_set_grid_cap(int max_workgroups) { return ewvit_set_grid_cap(max_workgroups); }

extern "C" int ewvit_conv2d_set_glds(int variant) {
  const int prev = g_glds;
  g_glds = variant ? 1 : 0;
  return prev;
}

extern "C" int ewvit_conv2d_pack_weight(const float *w, int64_t s_co, int64_t s_ci, int64_t s_tap, void *wp,
                                        void *wp_t, int64_t Cout, int64_t Cin, int64_t Cin_pad, int ksize,
                                        void *stream) {
  EWVIT_CHECK_ARG(w && (wp || wp_t) && Cout > 0 && Cin > 0 && Cin_pad >= Cin, "conv2d_pack_weight: bad args");
  EWVIT_CHECK_ARG(ksize == 1 || ksize == 3, "conv2d_pack_weight: kernel size %d", ksize);
  const int taps = ksize * ksize;
  const int64_t total = Cout * Cin_pad * taps;
  hipLaunchKernelGGL(conv_pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream), w,
                     s_co, s_ci, s_tap, (bf16_t *)wp, (bf16_t *)wp_t, (int)Cout, (int)Cin, (int)Cin_pad, taps);
  return launch_status("conv2d_pack_weight");
}

extern "C" int ewvit_conv2d_pack_weights(int n, const float *const *w, const int64_t *s_co, const int64_t *s_ci,
                                         const int64_t *s_tap, void *const *wp, void *const *wp_t,
                                         const int64_t *Cout, const int64_t *Cin, const int64_t *Cin_pad,
                                         const int *ksize, void *stream) {
  EWVIT_CHECK_ARG(n >= 0 && n <= EWVIT_PACK_MAX, "conv2d_pack_weights: %d weights (max %d per launch)", n,
                  EWVIT_PACK_MAX);
  if (n == 0) return 0;
  PackArgs a;
  a.n = n;
  int64_t chunks = 0;
  for (int i = 0; i < n; ++i) {
    EWVIT_CHECK_ARG(w[i] && (wp[i] || wp_t[i]) && Cout[i] > 0 && Cin[i] > 0 && Cin_pad[i] >= Cin[i] &&
                        (ksize[i] == 1 || ksize[i] == 3),
                    "conv2d_pack_weights: weight %d", i);
    const int taps = ksize[i] * ksize[i];
    a.chunk0[i] = (int)chunks;
    chunks += (int64_t)taps * ((Cout[i] + 63) / 64) * ((Cin_pad[i] + 63) / 64);
    EWVIT_CHECK_ARG(chunks < ((int64_t)1 << 30), "conv2d_pack_weights: too many elements");
    a.w[i] = w[i]; a.wp[i] = (bf16_t *)wp[i]; a.wpt[i] = (bf16_t *)wp_t[i];
    a.s_co[i] = s_co[i]; a.s_ci[i] = s_ci[i]; a.s_tap[i] = s_tap[i];
    a.cout[i] = (int)Cout[i]; a.cin[i] = (int)Cin[i]; a.cin_pad[i] = (int)Cin_pad[i]; a.taps[i] = taps;
  }
  a.chunk0[n] = (int)chunks;
  hipLaunchKernelGGL(conv_pack_multi_kernel, dim3((unsigned)chunks), dim3(256), 0, as_stream(stream), a);
  return launch_status("conv2d_pack_weights");
}

// rows per BatchNorm partial that ewvit_conv2d_fwd_bn leaves for this shape (the
// LDS-DMA kernel's m-tile), or 0 when the shape takes the register-staged kernel
static FwdArgs fwd_args(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride) {
  FwdArgs a;
  a.g = mkg(N, H, W, Cin, Cout, ksize, stride);
  a.M = (int64_t)a.g.N * a.g.Ho * a.g.Wo; a.Ncol = a.g.Cout; a.KC = a.g.Cin;
  a.srcH = a.g.H; a.srcW = a.g.W; a.outH = a.g.Ho; a.outW = a.g.Wo;
  a.sgc = a.g.Cin; a.sgs = 0; a.ogc = a.g.Cout; a.ogs = 0;
  return a;
}

// (the windowed kernel, convwin.hip, leaves one partial row per 16 x 16 output block)
static int fwd_bn_rows(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride) {
  if (!use_glds() || Cin % 64 || Cout % 8 || Cout > 65536) return 0;
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int64_t K = (int64_t)ksize * ksize * Cin;
  if (2 * N * H * W * Cin >= (int64_t)OOB || Cout * K * 2 >= (int64_t)OOB || N * Ho * Wo * Cout >= (int64_t)1 << 40)
    return 0;
  FwdArgs a = fwd_args(N, H, W, Cin, Cout, ksize, stride);
  a.bn_part = reinterpret_cast<float *>(1);    // (a statistics epilogue)
  if (win_ok(a, false)) return 256;
  int bm, bn;
  glds_tile(a, false, bm, bn);
  return bm;
}

extern "C" int64_t ewvit_conv2d_fwd_bn_rows(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize,
                                           int stride) {
  return fwd_bn_rows(N, H, W, Cin, Cout, ksize, stride);
}

extern "C" int ewvit_conv2d_fwd_bn(const void *x, const void *wp, const float *bias, void *y, int64_t N, int64_t H,
                                   int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride, int64_t x_group_c,
                                   int64_t x_group_stride, const float *bn_shift, float *bn_part,
                                   float *bn_shift_out, void *stream) {
  EWVIT_CHECK_ARG(x && wp && y && bn_part && bn_shift_out, "conv2d_fwd_bn: null pointer");
  ConvGeom g = mkg(N, H, W, Cin, Cout, ksize, stride);
  if (int rc = check_geom(g, "conv2d_fwd_bn")) return rc;
  if (int rc = check_group(x_group_c, x_group_stride, Cin, N * H * W, "conv2d_fwd_bn", "x")) return rc;
  EWVIT_CHECK_ARG(fwd_bn_rows(N, H, W, Cin, Cout, ksize, stride) > 0 && x_group_c % 64 == 0,
                  "conv2d_fwd_bn: shape takes the register-staged kernel (query ewvit_conv2d_fwd_bn_rows)");
  FwdArgs a;
  a.src = (const bf16_t *)x; a.wp = (const bf16_t *)wp; a.bias = bias; a.out = (bf16_t *)y; a.g = g;
  a.M = (int64_t)g.N * g.Ho * g.Wo; a.Ncol = g.Cout; a.KC = g.Cin;
  a.srcH = g.H; a.srcW = g.W; a.outH = g.Ho; a.outW = g.Wo;
  a.sgc = (int)x_group_c; a.sgs = x_group_stride; a.ogc = g.Cout; a.ogs = 0;
  a.bn_shift = bn_shift; a.bn_part = bn_part; a.bn_shift_out = bn_shift_out;
  const int64_t xb = 2 * (x_group_stride ? (Cin / x_group_c - 1) * x_group_stride + N * H * W * x_group_c : N * H * W * Cin);
  if (fwd_bn_rows(N, H, W, Cin, Cout, ksize, stride) == 256)
    EWVIT_CHECK_ARG(launch_win(a, xb, false, as_stream(stream)), "conv2d_fwd_bn: windowed kernel refused the shape");
  else
    EWVIT_CHECK_ARG(launch_glds<false>(a, xb, as_stream(stream)), "conv2d_fwd_bn: LDS-DMA kernel refused the shape");
  return launch_status("conv2d_fwd_bn");
}

// ---- convs reading relu(x * scale + shift): the training BatchNorm + ReLU of x's producer
// applied in the windowed kernels' operand staging (XF; coefficients from ewvit_bn_coef, one
// [2][group channels] block per channel group of x), so the normalised tensor is never written.
// The forward (with the next BatchNorm's statistics) and the weight gradient; the input gradient
// is the plain conv's (it does not read x).  3x3 stride 1 over maps the windowed kernels take.
static WgradArgs wgrad_args(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride);
static bool xf_args(FwdArgs &a, WgradArgs &w, int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize,
                    int stride, int64_t x_group_c, int64_t x_group_stride) {
  if (ksize != 3 || stride != 1 || x_group_c <= 0 || Cin % x_group_c || Cin > 512 || !use_glds()) return false;
  a = fwd_args(N, H, W, Cin, Cout, ksize, stride);
  a.sgc = (int)x_group_c; a.sgs = x_group_stride;
  a.bn_part = reinterpret_cast<float *>(1);
  a.xf = reinterpret_cast<const float *>(1);
  w = wgrad_args(N, H, W, Cin, Cout, ksize, stride);
  w.xgc = (int)x_group_c; w.xgs = x_group_stride;
  const int64_t xb = 2 * (x_group_stride ? (Cin / x_group_c - 1) * x_group_stride + N * H * W * x_group_c : N * H * W * Cin);
  return win_ok(a, false) && xb < (int64_t)OOB && wgrad_win_splits(w, xb) > 0;
}
extern "C" int ewvit_conv2d_xf_ok(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride,
                                  int64_t x_group_c, int64_t x_group_stride) {
  FwdArgs a;
  WgradArgs w;
  return xf_args(a, w, N, H, W, Cin, Cout, ksize, stride, x_group_c, x_group_stride) ? 1 : 0;
}
extern "C" int ewvit_conv2d_fwd_bn_xf(const void *x, const void *wp, const float *bias, void *y, int64_t N, int64_t H,
                                      int64_t W, int64_t Cin, int64_t Cout, int64_t x_group_c, int64_t x_group_stride,
                                      const float *xf, const float *bn_shift, float *bn_part, float *bn_shift_out,
                                      void *stream) {
  EWVIT_CHECK_ARG(x && wp && y && xf && bn_part && bn_shift_out, "conv2d_fwd_bn_xf: null pointer");
  ConvGeom g = mkg(N, H, W, Cin, Cout, 3, 1);
  if (int rc = check_geom(g, "conv2d_fwd_bn_xf")) return rc;
  if (int rc = check_group(x_group_c, x_group_stride, Cin, N * H * W, "conv2d_fwd_bn_xf", "x")) return rc;
  FwdArgs a;
  WgradArgs w;
  EWVIT_CHECK_ARG(xf_args(a, w, N, H, W, Cin, Cout, 3, 1, x_group_c, x_group_stride),
                  "conv2d_fwd_bn_xf: shape not taken by the windowed kernels (query ewvit_conv2d_xf_ok)");
  a.src = (const bf16_t *)x; a.wp = (const bf16_t *)wp; a.bias = bias; a.out = (bf16_t *)y;
  a.bn_shift = bn_shift; a.bn_part = bn_part; a.bn_shift_out = bn_shift_out; a.xf = xf;
  const int64_t xb = 2 * (x_group_stride ? (Cin / x_group_c - 1) * x_group_stride + N * H * W * x_group_c : N * H * W * Cin);
  EWVIT_CHECK_ARG(launch_win(a, xb, false, as_stream(stream)), "conv2d_fwd_bn_xf: windowed kernel refused the shape");
  return launch_status("conv2d_fwd_bn_xf");
}

// input channels per tap the fwd expects its weight pack to have: Cin rounded up to 64
// when Cin % 64 != 0 (Cin % 16 == 0) and the padded LDS-DMA kernel takes the shape
static int64_t fwd_pack_cin(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride) {
  if (Cin % 64 == 0 || Cin % 16 || !use_glds()) return Cin;
  const int64_t Cp = (Cin + 63) / 64 * 64;
  if (4 * Cp > 5 * Cin) return Cin;      // > 25 % zero K (48 -> 64 measured slower): exact-K kernel
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  if (2 * N * H * W * Cin >= (int64_t)OOB || Cout * ksize * ksize * Cp * 2 >= (int64_t)OOB ||
      N * Ho * Wo * Cout >= (int64_t)1 << 40)
    return Cin;
  return Cp;
}

extern "C" int64_t ewvit_conv2d_fwd_pack_cin(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize,
                                            int stride) {
  return fwd_pack_cin(N, H, W, Cin, Cout, ksize, stride);
}

extern "C" int ewvit_conv2d_fwd(const void *x, const void *wp, const float *bias, void *y, int64_t N, int64_t H,
                                int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride, int64_t x_group_c,
                                int64_t x_group_stride, void *stream) {
  EWVIT_CHECK_ARG(x && wp && y, "conv2d_fwd: null pointer");
  ConvGeom g = mkg(N, H, W, Cin, Cout, ksize, stride);
  if (int rc = check_geom(g, "conv2d_fwd")) return rc;
  if (int rc = check_group(x_group_c, x_group_stride, Cin, N * H * W, "conv2d_fwd", "x")) return rc;
  FwdArgs a;
  a.src = (const bf16_t *)x; a.wp = (const bf16_t *)wp; a.bias = bias; a.out = (bf16_t *)y; a.g = g;
  a.M = (int64_t)g.N * g.Ho * g.Wo; a.Ncol = g.Cout; a.KC = g.Cin;
  a.srcH = g.H; a.srcW = g.W; a.outH = g.Ho; a.outW = g.Wo;
  a.sgc = (int)x_group_c; a.sgs = x_group_stride; a.ogc = g.Cout; a.ogs = 0;
  const int64_t xb = 2 * (x_group_stride ? (Cin / x_group_c - 1) * x_group_stride + N * H * W * x_group_c : N * H * W * Cin);
  const int64_t cp = x_group_stride ? Cin : fwd_pack_cin(N, H, W, Cin, Cout, ksize, stride);
  if (cp != Cin) {
    // the weights were packed with cp input channels (ewvit_conv2d_fwd_pack_cin)
    a.KC = (int)cp; a.KCr = (int)Cin;
    EWVIT_CHECK_ARG(launch_glds<false>(a, xb, as_stream(stream)), "conv2d_fwd: padded LDS-DMA kernel refused");
  } else if (!launch_win(a, xb, false, as_stream(stream)) && !launch_small(a, false, as_stream(stream)) &&
             !launch_glds<false>(a, xb, as_stream(stream))) {
    launch_fwd<false>(a, as_stream(stream));
  }
  return launch_status("conv2d_fwd");
}

// stride-2 3x3 dgrad as 4 launches, one per output parity class (py, px), each over
// only its live taps (1, 2, 2 and 4 of the 9); false when the LDS-DMA kernel cannot
// take the class launches (nothing launched)
static bool dgrad_by_parity(FwdArgs a, int64_t src_bytes, hipStream_t s) {
  if (a.g.ks != 3 || a.g.stride != 2 || a.g.pad != 1 || a.ogs != 0 || a.sgs != 0 || !use_glds())
    return false;
  const int H = a.outH, W = a.outW;
  FwdArgs c[4];
  for (int pc = 0; pc < 4; ++pc) {
    const int py = pc >> 1, px = pc & 1;
    c[pc] = a;
    c[pc].pc = pc;
    c[pc].dstH = H; c[pc].dstW = W;
    c[pc].outH = (H - py + 1) / 2; c[pc].outW = (W - px + 1) / 2;
    c[pc].M = (int64_t)a.g.N * c[pc].outH * c[pc].outW;
    int nt = 0;
    for (int kh = 0; kh < 3; ++kh)
      for (int kw = 0; kw < 3; ++kw)
        if (((py + 1 - kh) & 1) == 0 && ((px + 1 - kw) & 1) == 0) c[pc].tapl[nt++] = kh * 3 + kw;
    c[pc].ntap = nt;
  }
  // the KC / layout checks of launch_glds do not depend on the class: probe class 3's
  // shape first so a refusal launches nothing
  int order[4] = {3, 0, 1, 2};
  for (int q = 0; q < 4; ++q) {
    const int pc = order[q];
    if (c[pc].M == 0) continue;
    if (!launch_glds<true>(c[pc], src_bytes, s)) {
      if (q == 0) return false;
      set_error("conv2d_bwd_data: parity class %d refused after class 3 ran", pc);
      return false;
    }
  }
  return true;
}

// 1 when ewvit_conv2d_bwd_data_add can run this shape (the LDS-DMA dgrad kernel)
extern "C" int64_t ewvit_conv2d_bwd_data_add_ok(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize,
                                               int stride) {
  if (!use_glds() || (Cout % 64 && (Cout % 8 || 5 * ((Cout + 63) / 64 * 64) > 6 * Cout)) ||
      Cin % 8 || 2 * N * H * W * Cout >= (int64_t)OOB ||
      Cin * ksize * ksize * Cout * 2 >= (int64_t)OOB)
    return 0;
  (void)stride;
  return 1;
}

// dx = dgrad(dy) + addend (plain NHWC, bf16): the skip connection's gradient of a
// residual block added in the dgrad epilogue of the block's first conv
extern "C" int ewvit_conv2d_bwd_data_add(const void *dy, const void *wp_t, void *dx, const void *addend, int64_t N,
                                         int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride,
                                         void *stream) {
  EWVIT_CHECK_ARG(dy && wp_t && dx && addend, "conv2d_bwd_data_add: null pointer");
  ConvGeom g = mkg(N, H, W, Cin, Cout, ksize, stride);
  if (int rc = check_geom(g, "conv2d_bwd_data_add")) return rc;
  EWVIT_CHECK_ARG(ewvit_conv2d_bwd_data_add_ok(N, H, W, Cin, Cout, ksize, stride),
                  "conv2d_bwd_data_add: shape not supported (query ewvit_conv2d_bwd_data_add_ok)");
  FwdArgs a;
  a.src = (const bf16_t *)dy; a.wp = (const bf16_t *)wp_t; a.bias = nullptr; a.out = (bf16_t *)dx; a.g = g;
  a.M = (int64_t)g.N * g.H * g.W; a.Ncol = g.Cin; a.KC = g.Cout;
  a.srcH = g.Ho; a.srcW = g.Wo; a.outH = g.H; a.outW = g.W;
  a.sgc = g.Cout; a.sgs = 0; a.ogc = g.Cin; a.ogs = 0;
  a.addend = (const bf16_t *)addend;
  const int64_t sb = 2 * N * (int64_t)g.Ho * g.Wo * Cout;
  EWVIT_CHECK_ARG(dgrad_by_parity(a, sb, as_stream(stream)) || launch_glds<true>(a, sb, as_stream(stream)),
                  "conv2d_bwd_data_add: LDS-DMA kernel refused the shape");
  return launch_status("conv2d_bwd_data_add");
}

// partial rows per channel group ewvit_conv2d_bwd_data_bn leaves for this shape (one per 128
// dx rows), or 0 when the shape does not take it: stride 1, the LDS-DMA dgrad
// (ewvit_conv2d_bwd_data_add_ok)
extern "C" int64_t ewvit_conv2d_bwd_bn_rows(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize,
                                           int stride) {
  if (stride != 1 || !ewvit_conv2d_bwd_data_add_ok(N, H, W, Cin, Cout, ksize, stride) ||
      Cin > 65536)
    return 0;
  FwdArgs a = fwd_args(N, H, W, Cin, Cout, ksize, stride);
  a.M = (int64_t)N * H * W; a.Ncol = (int)Cin; a.KC = (int)Cout;
  a.bwd.part = reinterpret_cast<float *>(1);
  int bm, bn;
  glds_tile(a, true, bm, bn);
  return (N * H * W + bm - 1) / bm;
}

// dx = dgrad(dy) (+ addend, when not null; plain dx only) and the backward statistics of the
// BatchNorm whose output was this conv's input (bx: that BN's input, dx's layout, bf16; mean /
// invstd its saved statistics; gamma / beta or null; act 0/1/2; rscale [N] with act 0: the
// drop-path factor per frame of the MBConv tail, or null).  BatchNorm groups: a grouped dx
// (dx_group_c, dx_group_stride: the multiscale conv's level-major input) has one per channel
// group, mean / invstd [groups][group_c]; a plain dx with bn_group_rows > 0 (a multiple of 128
// dividing N*H*W) one per slice of that many rows, mean / invstd [groups][Cin].  part
// [groups][ewvit_conv2d_bwd_bn_rows per channel group or ... / groups per row group][2 C]
// gets per 128-row m-tile (sum g, sum g * xhat) of the bf16-rounded dx; *nrc_out = the partial
// rows per BatchNorm group (what ewvit_bn_bwd_partials is given)
extern "C" int ewvit_conv2d_bwd_data_bn(const void *dy, const void *wp_t, void *dx, const void *addend, int64_t N,
                                        int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride,
                                        int64_t dx_group_c, int64_t dx_group_stride, const void *bx,
                                        const float *mean, const float *invstd, const float *gamma, const float *beta,
                                        int act, const float *rscale, int64_t bn_group_rows, float *part,
                                        int *nrc_out, void *stream) {
  EWVIT_CHECK_ARG(dy && wp_t && dx && bx && mean && invstd && part && nrc_out && act >= 0 && act <= 2 &&
                      !(rscale && act),
                  "conv2d_bwd_data_bn: bad args");
  ConvGeom g = mkg(N, H, W, Cin, Cout, ksize, stride);
  if (int rc = check_geom(g, "conv2d_bwd_data_bn")) return rc;
  if (int rc = check_group(dx_group_c, dx_group_stride, Cin, N * H * W, "conv2d_bwd_data_bn", "dx")) return rc;
  EWVIT_CHECK_ARG(ewvit_conv2d_bwd_bn_rows(N, H, W, Cin, Cout, ksize, stride) > 0,
                  "conv2d_bwd_data_bn: shape not supported (query ewvit_conv2d_bwd_bn_rows)");
  EWVIT_CHECK_ARG(!(addend && dx_group_stride), "conv2d_bwd_data_bn: an addend needs a plain dx");
  EWVIT_CHECK_ARG(bn_group_rows == 0 || (!dx_group_stride && bn_group_rows % 128 == 0 &&
                                         (N * H * W) % bn_group_rows == 0),
                  "conv2d_bwd_data_bn: BatchNorm row groups of %lld rows", (long long)bn_group_rows);
  FwdArgs a;
  a.src = (const bf16_t *)dy; a.wp = (const bf16_t *)wp_t; a.bias = nullptr; a.out = (bf16_t *)dx; a.g = g;
  a.M = (int64_t)g.N * g.H * g.W; a.Ncol = g.Cin; a.KC = g.Cout;
  a.srcH = g.Ho; a.srcW = g.Wo; a.outH = g.H; a.outW = g.W;
  a.sgc = g.Cout; a.sgs = 0; a.ogc = (int)dx_group_c; a.ogs = dx_group_stride;
  a.addend = (const bf16_t *)addend;
  a.bwd.part = part; a.bwd.x = (const bf16_t *)bx; a.bwd.mean = mean; a.bwd.invstd = invstd; a.bwd.gamma = gamma;
  a.bwd.beta = beta; a.bwd.rscale = rscale; a.bwd.act = act; a.bwd.hw = (int)(H * W); a.bwd.grows = bn_group_rows;
  const int64_t sb = 2 * N * (int64_t)g.Ho * g.Wo * Cout;
  int bm = 0;
  EWVIT_CHECK_ARG(launch_glds<true>(a, sb, as_stream(stream), &bm) && bm > 0,
                  "conv2d_bwd_data_bn: LDS-DMA kernel refused the shape");
  const int64_t ntm = (a.M + bm - 1) / bm;
  *nrc_out = (int)(bn_group_rows ? bn_group_rows / bm : ntm);
  return launch_status("conv2d_bwd_data_bn");
}

// the windowed input gradient with the backward statistics of the BatchNorm(+act) whose output
// the conv read (convwin.hip BST): one partial row per 16 x 16 block per channel group, part
// [groups][N*H*W / 256][2 group_c]; BatchNorm groups = dx's channel groups (mean / invstd
// [groups][group_c], gamma / beta [group_c] or null), or — a plain dx (group_c = Cin,
// group_stride 0) with bn_group_rows > 0 — slices of that many rows (whole images; mean / invstd
// [N*H*W / bn_group_rows][Cin]), part [slices][bn_group_rows / 256][2 Cin].
// ewvit_conv2d_bwd_bn_win_rows: N*H*W / 256 (the partial rows per channel group; with row groups
// the total over the slices), 0 when the windowed kernel does not take the shape.
static bool bst_args(FwdArgs &a, int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride,
                     int64_t dx_group_c, int64_t dx_group_stride, int64_t bn_group_rows) {
  if (ksize != 3 || stride != 1 || dx_group_c <= 0 || Cin % dx_group_c) return false;
  a = fwd_args(N, H, W, Cin, Cout, ksize, stride);
  a.M = (int64_t)a.g.N * a.g.H * a.g.W; a.Ncol = a.g.Cin; a.KC = a.g.Cout;
  a.srcH = a.g.Ho; a.srcW = a.g.Wo; a.outH = a.g.H; a.outW = a.g.W;
  a.sgc = a.g.Cout; a.sgs = 0; a.ogc = (int)dx_group_c; a.ogs = dx_group_stride;
  a.bwd.part = reinterpret_cast<float *>(1);
  a.bwd.x = reinterpret_cast<const bf16_t *>(2);
  a.bwd.mean = a.bwd.invstd = reinterpret_cast<const float *>(4);
  if (bn_group_rows < 0 || (bn_group_rows && (dx_group_stride || dx_group_c != Cin))) return false;
  a.bwd.grows = bn_group_rows;
  const int64_t sb = 2 * N * H * W * Cout;
  return sb < (int64_t)OOB && win_ok(a, true);
}
extern "C" int64_t ewvit_conv2d_bwd_bn_win_rows(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize,
                                               int stride, int64_t dx_group_c, int64_t dx_group_stride,
                                               int64_t bn_group_rows) {
  FwdArgs a;
  return bst_args(a, N, H, W, Cin, Cout, ksize, stride, dx_group_c, dx_group_stride, bn_group_rows) ? N * H * W / 256
                                                                                                     : 0;
}
extern "C" int ewvit_conv2d_bwd_data_bn_win(const void *dy, const void *wp_t, void *dx, int64_t N, int64_t H,
                                            int64_t W, int64_t Cin, int64_t Cout, int64_t dx_group_c,
                                            int64_t dx_group_stride, const void *bx, const float *mean,
                                            const float *invstd, const float *gamma, const float *beta, int act,
                                            int64_t bn_group_rows, float *part, void *stream) {
  EWVIT_CHECK_ARG(dy && wp_t && dx && bx && mean && invstd && part && act >= 0 && act <= 2,
                  "conv2d_bwd_data_bn_win: bad args");
  ConvGeom g = mkg(N, H, W, Cin, Cout, 3, 1);
  if (int rc = check_geom(g, "conv2d_bwd_data_bn_win")) return rc;
  if (int rc = check_group(dx_group_c, dx_group_stride, Cin, N * H * W, "conv2d_bwd_data_bn_win", "dx")) return rc;
  FwdArgs a;
  EWVIT_CHECK_ARG(bst_args(a, N, H, W, Cin, Cout, 3, 1, dx_group_c, dx_group_stride, bn_group_rows),
                  "conv2d_bwd_data_bn_win: shape not taken (query ewvit_conv2d_bwd_bn_win_rows)");
  a.src = (const bf16_t *)dy; a.wp = (const bf16_t *)wp_t; a.bias = nullptr; a.out = (bf16_t *)dx;
  a.bwd.part = part; a.bwd.x = (const bf16_t *)bx; a.bwd.mean = mean; a.bwd.invstd = invstd; a.bwd.gamma = gamma;
  a.bwd.beta = beta; a.bwd.rscale = nullptr; a.bwd.act = act; a.bwd.hw = (int)(H * W); a.bwd.grows = bn_group_rows;
  const int64_t sb = 2 * N * H * W * Cout;
  EWVIT_CHECK_ARG(launch_win(a, sb, true, as_stream(stream)), "conv2d_bwd_data_bn_win: windowed kernel refused");
  return launch_status("conv2d_bwd_data_bn_win");
}

extern "C" int ewvit_conv2d_bwd_data(const void *dy, const void *wp_t, void *dx, int64_t N, int64_t H, int64_t W,
                                     int64_t Cin, int64_t Cout, int ksize, int stride, int64_t dx_group_c,
                                     int64_t dx_group_stride, void *stream) {
  EWVIT_CHECK_ARG(dy && wp_t && dx, "conv2d_bwd_data: null pointer");
  ConvGeom g = mkg(N, H, W, Cin, Cout, ksize, stride);
  if (int rc = check_geom(g, "conv2d_bwd_data")) return rc;
  if (int rc = check_group(dx_group_c, dx_group_stride, Cin, N * H * W, "conv2d_bwd_data", "dx")) return rc;
  FwdArgs a;
  a.src = (const bf16_t *)dy; a.wp = (const bf16_t *)wp_t; a.bias = nullptr; a.out = (bf16_t *)dx; a.g = g;
  a.M = (int64_t)g.N * g.H * g.W; a.Ncol = g.Cin; a.KC = g.Cout;
  a.srcH = g.Ho; a.srcW = g.Wo; a.outH = g.H; a.outW = g.W;
  a.sgc = g.Cout; a.sgs = 0; a.ogc = (int)dx_group_c; a.ogs = dx_group_stride;
  const int64_t sb = 2 * N * (int64_t)g.Ho * g.Wo * Cout;
  if (!launch_win(a, sb, true, as_stream(stream)) && !launch_small(a, true, as_stream(stream)) &&
      !dgrad_by_parity(a, sb, as_stream(stream)) && !launch_glds<true>(a, sb, as_stream(stream)))
    launch_fwd<true>(a, as_stream(stream));
  return launch_status("conv2d_bwd_data");
}

// split of the pixel reduction: at most 512 workgroups — the 2 per CU that registers
// and LDS allow, so every split runs in the first (only) round — >= 4 K-tiles of 64
// pixels per split, and f32 partial slabs no larger than 4x the bf16 operands.
// Wide n'-tiles (128 x 256 per block, each wave 64 x 128: a quarter fewer LDS and L2 bytes
// per MFMA; 32 pixels per K-tile, 2-deep ring, 48 KB) for n' >= 2048 over >= 64K pixels
// (multiscale_fusion 384 -> 128, 3x3, 64 x 112^2: 951 -> 850 us; measured slower on
// freq_conv's n' = 1152 and on every backbone 1x1, which keep the 128-column tiles; the
// 64-pixel / 96 KB form ran 1233 us).  ewvit_conv2d_set_wgrad_wide: 4 auto (default), 2 wide
// whenever the shape allows it, 0 never (test switches).
static int g_wgw = 4;
static int wgrad_wide(const ConvGeom &g) {
  const int64_t NP = (int64_t)g.ks * g.ks * g.Cin;
  int v = g_wgw;
  if (v == 4) v = (NP >= 2048 && (int64_t)g.N * g.Ho * g.Wo >= 65536) ? 2 : 0;
  if (!v || NP < 256 || ((NP + 255) / 256 * 256 - NP) * 8 > NP) return 0;
  return 2;
}
static int64_t wgrad_splits(const ConvGeom &g, int wide = 0) {
  const int64_t M = (int64_t)g.N * g.Ho * g.Wo;
  const int64_t NP = (int64_t)g.ks * g.ks * g.Cin;
  const int64_t tn = wide ? 2 * CBN : CBN;
  const int64_t tiles = ((NP + tn - 1) / tn) * ((g.Cout + CBM - 1) / CBM);
  // (fewer, longer splits measured slower: 256 / 128 target workgroups for the backbone's
  // <= 28^2 maps 3231-3233 / 3148 frames/s against 3214-3231 at 512, round 4)
  int64_t s = 512 / tiles;
  if (g_grid_cap > 0 && s * tiles > g_grid_cap) s = g_grid_cap / tiles;
  const int64_t maxs = M / 256;
  if (s > maxs) s = maxs;
  const int64_t cap = 2 * M * ((int64_t)g.Cin + g.Cout) / ((int64_t)g.Cout * NP);
  if (s > cap) s = cap;
  if (s < 1) s = 1;
  return s;
}

// the 1x1 kernel (conv_wgrad_1x1_kernel): plain NHWC x, stride 1, no bias gradient; splits for
// ~g_w1_wg workgroups with >= g_w1_minkt K-tiles of 64 pixels each, slabs <= 4x the operands
// (256 / 8 / 2-deep ring: stage-6 expand 22.2 -> 18.4 us, stage-5 23.7 -> 19.2 us, stage-4
// 26.6 -> 22.7 us against the generic kernel, profiles/r05/ab/wgrad1x1_kernel.log).
// ewvit_conv2d_set_wgrad_1x1 (test / tuning): workgroup target (0 = never), min K-tiles, ring.
static int g_w1_wg = 256, g_w1_minkt = 8, g_w1_ring = 2;
static bool w1x1_ok(const ConvGeom &g, int64_t x_group_stride, bool has_bias, int64_t M) {
  return g_w1_wg > 0 && g.ks == 1 && g.stride == 1 && x_group_stride == 0 && !has_bias &&
         M * g.Cin * 2 < (int64_t)OOB / 2 && M * g.Cout * 2 < (int64_t)OOB / 2;
}
static int64_t w1x1_splits(const ConvGeom &g) {
  const int64_t M = (int64_t)g.N * g.Ho * g.Wo;
  const int64_t tiles = ((g.Cin + CBN - 1) / CBN) * ((g.Cout + CBM - 1) / CBM);
  int64_t s = g_w1_wg / tiles;
  const int64_t maxs = ((M + 63) / 64) / g_w1_minkt;
  if (s > maxs) s = maxs;
  const int64_t cap = 2 * M * ((int64_t)g.Cin + g.Cout) / ((int64_t)g.Cout * g.Cin);
  if (s > cap) s = cap;
  return s < 1 ? 1 : s;
}
// min_ktiles < 1 / ring not 2 or 3 keep the current value (so a caller can move the workgroup
// target alone and restore it without knowing the other two knobs)
extern "C" int ewvit_conv2d_set_wgrad_1x1(int target_wg, int min_ktiles, int ring) {
  const int prev = g_w1_wg;
  g_w1_wg = target_wg;
  if (min_ktiles >= 1) g_w1_minkt = min_ktiles;
  if (ring == 2 || ring == 3) g_w1_ring = ring;
  return prev;
}
// the three knobs: 0 workgroup target, 1 min K-tiles, 2 ring slots
extern "C" int ewvit_conv2d_wgrad_1x1_config(int which) {
  return which == 0 ? g_w1_wg : which == 1 ? g_w1_minkt : g_w1_ring;
}

extern "C" int ewvit_conv2d_set_wgrad_wide(int variant) {
  const int prev = g_wgw;
  g_wgw = variant == 0 || variant == 2 ? variant : 4;
  return prev;
}

static WgradArgs wgrad_args(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride) {
  WgradArgs a;
  a.g = mkg(N, H, W, Cin, Cout, ksize, stride);
  a.M = (int64_t)a.g.N * a.g.Ho * a.g.Wo;
  a.xgc = (int)Cin; a.xgs = 0;
  return a;
}

extern "C" int64_t ewvit_conv2d_bwd_weight_workspace(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout,
                                                     int ksize, int stride) {
  ConvGeom g = mkg(N, H, W, Cin, Cout, ksize, stride);
  // the windowed kernel (convwin.hip): [splits][Cout][9 Cin] slabs + [splits][Cout] bias partials
  const int wsp = wgrad_win_splits(wgrad_args(N, H, W, Cin, Cout, ksize, stride), 2 * N * H * W * Cin);
  const int64_t winb = (int64_t)wsp * Cout * (9 * Cin + 1) * (int64_t)sizeof(float);
  const int64_t ntx = (ksize * ksize * Cin + CBN - 1) / CBN;
  const int64_t narrow = wgrad_splits(g) * Cout * (ksize * ksize * Cin + ntx) * (int64_t)sizeof(float);
  const int wide = wgrad_wide(g);
  int64_t need = narrow > winb ? narrow : winb;
  if (w1x1_ok(g, 0, false, (int64_t)N * H * W)) {
    const int64_t w1 = w1x1_splits(g) * Cout * Cin * (int64_t)sizeof(float);
    if (w1 > need) need = w1;
  }
  if (!wide) return need;
  const int64_t ntw = (ksize * ksize * Cin + 2 * CBN - 1) / (2 * CBN);
  const int64_t wb = wgrad_splits(g, wide) * Cout * (ksize * ksize * Cin + ntw) * (int64_t)sizeof(float);
  return wb > need ? wb : need;
}

extern "C" int ewvit_conv2d_bwd_weight(const void *x, const void *dy, float *dw, float *dbias, int accumulate,
                                       int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize,
                                       int stride, int64_t x_group_c, int64_t x_group_stride, int64_t dw_cin,
                                       int64_t dw_s_co, int64_t dw_s_ci, int64_t dw_s_tap, float *workspace,
                                       void *stream) {
  // (the caller's "defer this reduce" mark is consumed by every call, whatever path it takes)
  const bool defer_mark = reduce_take_defer();
  EWVIT_CHECK_ARG(x && dy && dw && workspace, "conv2d_bwd_weight: null pointer");
  ConvGeom g = mkg(N, H, W, Cin, Cout, ksize, stride);
  if (int rc = check_geom(g, "conv2d_bwd_weight")) return rc;
  if (int rc = check_group(x_group_c, x_group_stride, Cin, N * H * W, "conv2d_bwd_weight", "x")) return rc;
  const int taps = ksize * ksize;
  WgradArgs a;
  a.x = (const bf16_t *)x; a.dy = (const bf16_t *)dy; a.part = workspace; a.g = g;
  a.xgc = (int)x_group_c; a.xgs = x_group_stride;
  a.M = (int64_t)g.N * g.Ho * g.Wo;
  const int64_t xb = 2 * (x_group_stride ? (Cin / x_group_c - 1) * x_group_stride + N * H * W * x_group_c : N * H * W * Cin);
  const bool glds = use_glds() && xb < (int64_t)OOB && a.M * g.Cout * 2 < (int64_t)OOB;
  // the windowed kernel (convwin.hip): 3x3 stride 1 over maps of whole 8 x 16 tiles
  const int wsp = glds ? wgrad_win_splits(a, xb) : 0;
  if (wsp > 0) {
    EWVIT_CHECK_ARG(dw_cin > 0 && dw_cin <= Cin, "conv2d_bwd_weight: dw_cin %lld not in (0, %lld]", (long long)dw_cin,
                    (long long)Cin);
    a.part = workspace;
    a.dbias_part = dbias ? workspace + (int64_t)wsp * g.Cout * taps * g.Cin : nullptr;
    hipStream_t s = as_stream(stream);
    launch_wgrad_win(a, xb, wsp, s);
    if (int rc = launch_status("conv2d_bwd_weight (windowed)")) return rc;
    WOut wo;
    wo.s_co = dw_s_co; wo.s_ci = dw_s_ci; wo.s_tap = dw_s_tap; wo.cin = (int)dw_cin;
    const int64_t n4 = (int64_t)g.Cout * taps * g.Cin / 4;
    int T = 1;
    while (T < 64 && T * 2 <= wsp && n4 * T * 2 <= 65536) T *= 2;
    const int64_t nmain = (n4 * T + 255) / 256;
    const int64_t nbias = dbias ? (g.Cout + 63) / 64 : 0;
    hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3((unsigned)(nmain + nbias)), dim3(256), 0, s, workspace, dw,
                       g.Cout, g.Cin, taps, wsp, wsp, accumulate, a.dbias_part, dbias, wo, T, (int)nmain);
    return launch_status("conv2d_bwd_weight reduce");
  }
  if (glds && w1x1_ok(g, x_group_stride, dbias != nullptr, a.M)) {
    // the 1x1 kernel: K-tile-aligned splits, slabs + the reduce pass (or dW itself, one split)
    EWVIT_CHECK_ARG(dw_cin > 0 && dw_cin <= Cin, "conv2d_bwd_weight: dw_cin %lld not in (0, %lld]", (long long)dw_cin,
                    (long long)Cin);
    const int ntx = (g.Cin + CBN - 1) / CBN, nty = (g.Cout + CBM - 1) / CBM;
    const int64_t sp0 = w1x1_splits(g);
    int64_t mper = (a.M + sp0 - 1) / sp0;
    a.mper = (mper + 63) / 64 * 64;
    const int sp = (int)((a.M + a.mper - 1) / a.mper);
    a.dbias_part = nullptr;
    const bool direct = sp == 1 && !accumulate && dw_cin == Cin && dw_s_ci == 1 && dw_s_co == Cin;
    a.part = direct ? dw : workspace;
    hipStream_t s = as_stream(stream);
    // deferred reductions of earlier weight gradients on this stream ride in front of the tiles
    const RedJobs rj = reduce_take_jobs(s);
    const unsigned nwg = (unsigned)((int64_t)ntx * nty * sp + rj.nblk);
    if (g_w1_ring == 2) hipLaunchKernelGGL(conv_wgrad_1x1_kernel<2>, dim3(nwg), dim3(256), 0, s, a, ntx, nty, rj);
    else hipLaunchKernelGGL(conv_wgrad_1x1_kernel<3>, dim3(nwg), dim3(256), 0, s, a, ntx, nty, rj);
    if (int rc = launch_status("conv2d_bwd_weight (1x1)")) return rc;
    if (direct) return 0;
    WOut wo;
    wo.s_co = dw_s_co; wo.s_ci = dw_s_ci; wo.s_tap = dw_s_tap; wo.cin = (int)dw_cin;
    const int64_t n4 = (int64_t)g.Cout * g.Cin / 4;
    int T = 1;
    while (T < 64 && T * 2 <= sp && n4 * T * 2 <= 65536) T *= 2;
    if (defer_mark) {
      RedJob j;
      j.kind = 1; j.part = workspace; j.dw = dw; j.n = n4 * 4; j.Cin = g.Cin; j.taps = 1; j.splits = sp;
      j.accumulate = accumulate; j.T = T; j.wo = wo;
      reduce_defer(s, j);
      return 0;
    }
    const int64_t nmain = (n4 * T + 255) / 256;
    hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3((unsigned)nmain), dim3(256), 0, s, workspace, dw, g.Cout,
                       g.Cin, 1, sp, 0, accumulate, nullptr, nullptr, wo, T, (int)nmain);
    return launch_status("conv2d_bwd_weight reduce");
  }
  const int wide = glds ? wgrad_wide(g) : 0;
  const int64_t splits = wgrad_splits(g, wide);
  a.dbias_part = dbias ? workspace + splits * g.Cout * taps * (int64_t)g.Cin : nullptr;
  const int tnw = wide ? 2 * CBN : CBN;
  const int ntx = (taps * g.Cin + tnw - 1) / tnw, nty = (g.Cout + CBM - 1) / CBM;
  const int64_t kq = !glds ? CBK : wide ? 32 : 64;  // K-tile depth (pixels)
  int64_t mper = (a.M + splits - 1) / splits;
  mper = (mper + kq - 1) / kq * kq;
  a.mper = mper;
  const int sp = (int)((a.M + mper - 1) / mper);
  // the glds kernel leaves bias partials per (split, n'-tile); the old one per split
  const int bparts = glds ? sp * ntx : sp;
  EWVIT_CHECK_ARG(dw_cin > 0 && dw_cin <= Cin, "conv2d_bwd_weight: dw_cin %lld not in (0, %lld]", (long long)dw_cin,
                  (long long)Cin);
  WOut wo;
  wo.s_co = dw_s_co; wo.s_ci = dw_s_ci; wo.s_tap = dw_s_tap; wo.cin = (int)dw_cin;
  // one split of a 1x1 conv whose dW is [Cout][Cin] row-major: the slab IS dW (and
  // dbias) — no reduce pass
  const bool direct = sp == 1 && taps == 1 && !accumulate && (!dbias || bparts == 1) && dw_cin == Cin &&
                      dw_s_ci == 1 && dw_s_co == Cin;
  if (direct) { a.part = dw; a.dbias_part = dbias; }
  hipStream_t s = as_stream(stream);
  if (glds) {
    // deferred reductions of earlier weight gradients on this stream ride in front of the tiles
    const RedJobs rj = reduce_take_jobs(s);
    const unsigned nwg = (unsigned)((int64_t)ntx * nty * sp + rj.nblk);
#define EWVIT_GLDS_WG(BK_, NS_, WJ_)                                                                        \
  do {                                                                                                    \
    if (ksize == 1) hipLaunchKernelGGL((conv_wgrad_glds_kernel<1, BK_, NS_, WJ_>), dim3(nwg), dim3(256), 0, s, a, xb, ntx, nty, rj); \
    else hipLaunchKernelGGL((conv_wgrad_glds_kernel<3, BK_, NS_, WJ_>), dim3(nwg), dim3(256), 0, s, a, xb, ntx, nty, rj);            \
  } while (0)
    if (wide) EWVIT_GLDS_WG(32, 2, 8);
    else EWVIT_GLDS_WG(64, 2, 4);
#undef EWVIT_GLDS_WG
  } else {
    dim3 grid((unsigned)ntx, (unsigned)nty, (unsigned)sp);
    if (ksize == 1) hipLaunchKernelGGL(conv_wgrad_kernel<1>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(conv_wgrad_kernel<3>, grid, dim3(256), 0, s, a);
  }
  if (int rc = launch_status("conv2d_bwd_weight")) return rc;
  if (direct) return 0;
  const int64_t n4 = (int64_t)g.Cout * taps * g.Cin / 4;
  int T = 1;                       // split lanes per output: ~64K threads, <= splits, <= 64
  while (T < 64 && T * 2 <= sp && n4 * T * 2 <= 65536) T *= 2;
  if (defer_mark && glds && !dbias) {
    RedJob j;
    j.kind = 1; j.part = workspace; j.dw = dw; j.n = n4 * 4; j.Cin = g.Cin; j.taps = taps; j.splits = sp;
    j.accumulate = accumulate; j.T = T; j.wo = wo;
    reduce_defer(s, j);
    return 0;
  }
  const int64_t nmain = (n4 * T + 255) / 256;
  const int64_t nbias = dbias ? (g.Cout + 63) / 64 : 0;
  hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3((unsigned)(nmain + nbias)), dim3(256), 0, s, workspace, dw,
                     g.Cout, g.Cin, taps, sp, bparts, accumulate, a.dbias_part, dbias, wo, T, (int)nmain);
  return launch_status("conv2d_bwd_weight reduce");
}

// dW (+ db) of the conv over relu(x * scale + shift) (see ewvit_conv2d_fwd_bn_xf): the windowed
// kernel with the transform in its x staging, then the split reduction; same workspace as
// ewvit_conv2d_bwd_weight
extern "C" int ewvit_conv2d_bwd_weight_xf(const void *x, const void *dy, float *dw, float *dbias, int accumulate,
                                          int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout,
                                          int64_t x_group_c, int64_t x_group_stride, const float *xf, int64_t dw_cin,
                                          int64_t dw_s_co, int64_t dw_s_ci, int64_t dw_s_tap, float *workspace,
                                          void *stream) {
  EWVIT_CHECK_ARG(x && dy && dw && xf && workspace, "conv2d_bwd_weight_xf: null pointer");
  ConvGeom g = mkg(N, H, W, Cin, Cout, 3, 1);
  if (int rc = check_geom(g, "conv2d_bwd_weight_xf")) return rc;
  if (int rc = check_group(x_group_c, x_group_stride, Cin, N * H * W, "conv2d_bwd_weight_xf", "x")) return rc;
  FwdArgs fa;
  WgradArgs a;
  EWVIT_CHECK_ARG(xf_args(fa, a, N, H, W, Cin, Cout, 3, 1, x_group_c, x_group_stride),
                  "conv2d_bwd_weight_xf: shape not taken by the windowed kernels (query ewvit_conv2d_xf_ok)");
  EWVIT_CHECK_ARG(dw_cin > 0 && dw_cin <= Cin, "conv2d_bwd_weight_xf: dw_cin %lld not in (0, %lld]", (long long)dw_cin,
                  (long long)Cin);
  a.x = (const bf16_t *)x; a.dy = (const bf16_t *)dy; a.xf = xf;
  const int64_t xb = 2 * (x_group_stride ? (Cin / x_group_c - 1) * x_group_stride + N * H * W * x_group_c : N * H * W * Cin);
  const int wsp = wgrad_win_splits(a, xb);
  const int taps = 9;
  a.part = workspace;
  a.dbias_part = dbias ? workspace + (int64_t)wsp * g.Cout * taps * g.Cin : nullptr;
  hipStream_t s = as_stream(stream);
  launch_wgrad_win(a, xb, wsp, s);
  if (int rc = launch_status("conv2d_bwd_weight_xf (windowed)")) return rc;
  WOut wo;
  wo.s_co = dw_s_co; wo.s_ci = dw_s_ci; wo.s_tap = dw_s_tap; wo.cin = (int)dw_cin;
  const int64_t n4 = (int64_t)g.Cout * taps * g.Cin / 4;
  int T = 1;
  while (T < 64 && T * 2 <= wsp && n4 * T * 2 <= 65536) T *= 2;
  const int64_t nmain = (n4 * T + 255) / 256;
  const int64_t nbias = dbias ? (g.Cout + 63) / 64 : 0;
  hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3((unsigned)(nmain + nbias)), dim3(256), 0, s, workspace, dw,
                     g.Cout, g.Cin, taps, wsp, wsp, accumulate, a.dbias_part, dbias, wo, T, (int)nmain);
  return launch_status("conv2d_bwd_weight_xf reduce");
}
