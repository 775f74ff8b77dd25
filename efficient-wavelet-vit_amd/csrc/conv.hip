// 3x3 convolution as an MFMA implicit GEMM, channels-last bf16 (gfx950).
//
// The MWT conv stack of network/mwt.py:23-72 — hf_conv['fusion'] (Cin 54 -> padded
// 64, 112^2, all 3 levels batched), multiscale_fusion (384 -> 128, 112^2),
// freq_conv (128 -> 128, stride 2) and freq_pool's conv (stride 2) — holds 74 % of
// the model's FLOPs (SURVEY §8 note 3).  Three kernels:
//
//   fwd    y[m, co]  = sum_{tap, ci} x[pix(m, tap), ci] * W[co, ci, tap]   (+ bias)
//   dgrad  dx[m, ci] = sum_{tap, co} dy[pix^T(m, tap), co] * W[co, ci, tap]
//          (same kernel: A gathers dy through the transposed pixel map, B = W packed
//           [ci][tap][co]; stride 2 handled by the parity test of pix^T)
//   wgrad  dW[co, tap, ci] = sum_m dy[m, co] * x[pix(m, tap), ci]   (split over m)
//
// GEMM tile 128x128x32, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4
// v_mfma_f32_16x16x32_bf16 tiles, fp32 accumulate.  Operands are staged
// global -> registers -> LDS with the next K-tile's loads in flight during the
// current tile's MFMAs.  fwd/dgrad images are [row][k] (k contiguous, 16-B rows
// chunks, padded rows) read with ds_read_b128; wgrad's operands both have the
// reduction (pixel) index outermost in HBM, so they are staged as natural
// [k][row] images (256-B rows, XOR-swizzled 16-B chunks) and read as MFMA
// fragments with ds_read_b64_tr_b16 (the gfx950 transposing LDS read).
#include "common.h"

namespace ewvit {

typedef __attribute__((ext_vector_type(8))) __bf16 cbf16x8;
typedef __attribute__((ext_vector_type(4))) float cf32x4;
typedef __attribute__((ext_vector_type(4))) short cs4;

constexpr int CBM = 128, CBN = 128, CBK = 32;
constexpr int CLD = CBK + 8;  // padded [row][k] image row (80 B)

struct ConvGeom {
  int N, H, W, Cin;      // x (fwd) / dx (dgrad) grid
  int Ho, Wo, Cout;      // y / dy grid
  int stride;
};

// ---------------------------------------------------------------- fwd / dgrad
// A(m, k): m = pixel of the OUTPUT grid of this GEMM (y for fwd, dx for dgrad),
// k = tap * KC + c (KC = Cin for fwd, Cout for dgrad).  B(k, n) = Wp[n][k].
struct FwdArgs {
  const bf16_t *src;     // gathered operand: x (fwd) or dy (dgrad), NHWC
  const bf16_t *wp;      // packed weights [Ncol][9][KC]
  const float *bias;     // [Ncol] or null
  bf16_t *out;           // [M][Ncol] NHWC
  ConvGeom g;
  int64_t M;
  int Ncol, KC;          // GEMM N and per-tap K
  int srcH, srcW;        // spatial size of `src`
  int outH, outW;        // spatial size of the GEMM's output grid
};

template <bool DGRAD>
__device__ __forceinline__ bool src_pixel(const FwdArgs &a, int oh, int ow, int tap, int &sh, int &sw) {
  const int kh = tap / 3, kw = tap % 3;
  if (!DGRAD) {
    sh = oh * a.g.stride - 1 + kh;
    sw = ow * a.g.stride - 1 + kw;
  } else {
    // dx pixel (oh, ow) receives dy[(oh + 1 - kh)/s, (ow + 1 - kw)/s] when divisible
    const int th = oh + 1 - kh, tw = ow + 1 - kw;
    if (th < 0 || tw < 0) return false;
    if (a.g.stride == 2 && ((th | tw) & 1)) return false;
    sh = th / a.g.stride;
    sw = tw / a.g.stride;
  }
  return sh >= 0 && sh < a.srcH && sw >= 0 && sw < a.srcW;
}

template <bool DGRAD, int BN_>
__global__ __launch_bounds__(256) void conv3x3_fwd_kernel(FwdArgs a) {
  constexpr int WN = BN_ / 2, J = WN / 16;  // per-wave columns, 16-wide MFMA tiles
  __shared__ __attribute__((aligned(16))) bf16_t As[2][CBM][CLD];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][BN_][CLD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int64_t m0 = (int64_t)blockIdx.x * CBM;
  const int n0 = blockIdx.y * BN_;
  const int K = 9 * a.KC;
  const int nk = (K + CBK - 1) / CBK;

  // each thread stages 2 A vectors and 2 B vectors (8 bf16 each) per K-tile
  int arow[2], ach[2];
  int an[2], aoh[2], aow[2];
  bool avalid[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int v = tid + 256 * u;
    arow[u] = v >> 2;
    ach[u] = (v & 3) * 8;
    const int64_t m = m0 + arow[u];
    avalid[u] = m < a.M;
    const int64_t mm = avalid[u] ? m : 0;
    aow[u] = (int)(mm % a.outW);
    const int64_t t = mm / a.outW;
    aoh[u] = (int)(t % a.outH);
    an[u] = (int)(t / a.outH);
  }
  uint4 ra[2], rb[2];
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = kt * CBK + ach[u];
      uint4 va = make_uint4(0u, 0u, 0u, 0u);
      if (avalid[u] && k < K) {
        const int tap = k / a.KC, c = k % a.KC;
        int sh, sw;
        if (src_pixel<DGRAD>(a, aoh[u], aow[u], tap, sh, sw))
          va = *reinterpret_cast<const uint4 *>(a.src + (((int64_t)an[u] * a.srcH + sh) * a.srcW + sw) * a.KC + c);
      }
      ra[u] = va;
      const int n = n0 + arow[u];  // B rows use the same (row, chunk) split
      uint4 vb = make_uint4(0u, 0u, 0u, 0u);
      if ((BN_ == 128 || u == 0) && n < a.Ncol && k < K) vb = *reinterpret_cast<const uint4 *>(a.wp + (int64_t)n * K + k);
      rb[u] = vb;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      *reinterpret_cast<uint4 *>(&As[buf][arow[u]][ach[u]]) = ra[u];
      if (BN_ == 128 || u == 0) *reinterpret_cast<uint4 *>(&Bs[buf][arow[u]][ach[u]]) = rb[u];
    }
  };

  cf32x4 acc[4][J];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = cf32x4{0.f, 0.f, 0.f, 0.f};

  load_tile(0);
  store_tile(0);
  __syncthreads();
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) load_tile(kt + 1);
    cbf16x8 af[4], bfr[J];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const cbf16x8 *>(&As[cur][wm * 64 + i * 16 + fr][fk]);
#pragma unroll
    for (int j = 0; j < J; ++j) bfr[j] = *reinterpret_cast<const cbf16x8 *>(&Bs[cur][wn * WN + j * 16 + fr][fk]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < J; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (more) store_tile(cur ^ 1);
    __syncthreads();
  }
  // epilogue: C/D map col = lane&15, row = (lane>>4)*4 + r
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int col = n0 + wn * WN + j * 16 + (lane & 15);
    if (col >= a.Ncol) continue;
    const float b = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (row < a.M) a.out[row * a.Ncol + col] = f2bf(acc[i][j][r] + b);
      }
  }
}

// ---------------------------------------------------------------- wgrad
// C[co][n'] with n' = tap*Cin + ci, reduction over output pixels m.
// A(co, m) = dy[m][co]   -> image Ast[m][co]  (rows of 128 co = 256 B)
// B(m, n') = x[pix(m,tap)][ci] -> image Bst[m][n'] (rows of 128 n' = 256 B)
// 16-B chunk ch of row r lives at 256*r + 16*(ch ^ swz(r)),
// swz(r) = ((r&3)<<2) | ((r>>2)&3)  (T10 image (b): conflict-free tr reads).
struct WgradArgs {
  const bf16_t *x;       // [N, H, W, Cin]
  const bf16_t *dy;      // [N, Ho, Wo, Cout]
  float *part;           // [splits][Cout][9*Cin]
  float *dbias_part;     // [splits][Cout] partial bias gradients (sum of dy), or null
  ConvGeom g;
  int64_t M;             // N*Ho*Wo
  int64_t mper;          // pixels per split (multiple of 32)
};

__device__ __forceinline__ int swz_off(int r, int ch) {
  return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3)));
}

__global__ __launch_bounds__(256) void conv3x3_wgrad_kernel(WgradArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2][2][CBK * 256];  // [buf][A/B][32 rows x 256 B]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int co0 = blockIdx.y * CBM;
  const int np0 = blockIdx.x * CBN;
  const int NP = 9 * a.g.Cin;
  const int64_t mbeg = (int64_t)blockIdx.z * a.mper;
  const int64_t mend = mbeg + a.mper < a.M ? mbeg + a.mper : a.M;
  const int nk = (int)((mend - mbeg + CBK - 1) / CBK);

  // staging: 32 rows x 16 chunks per operand = 512 vectors -> 2 per thread
  // vector v: row = v >> 4, chunk = v & 15
  uint4 ra[2], rb[2];
  int vrow[2], vch[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int v = tid + 256 * u;
    vrow[u] = v >> 4;
    vch[u] = v & 15;
  }
  // the B chunk's (tap, ci) is fixed per thread
  int btap[2], bci[2];
  bool bok[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int np = np0 + vch[u] * 8;
    bok[u] = np < NP;
    btap[u] = bok[u] ? np / a.g.Cin : 0;
    bci[u] = bok[u] ? np % a.g.Cin : 0;
  }
  const int bkh = 0, bkw = 0;
  (void)bkh; (void)bkw;
  int tkh[2], tkw[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) { tkh[u] = btap[u] / 3; tkw[u] = btap[u] % 3; }
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
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t m = mbeg + (int64_t)kt * CBK + vrow[u];
      uint4 va = make_uint4(0u, 0u, 0u, 0u), vb = va;
      if (m < mend) {
        const int co = co0 + vch[u] * 8;
        if (co < a.g.Cout) va = *reinterpret_cast<const uint4 *>(a.dy + m * a.g.Cout + co);
        if (bok[u]) {
          const int ih = poh[u] * a.g.stride - 1 + tkh[u], iw = pow_[u] * a.g.stride - 1 + tkw[u];
          if (ih >= 0 && ih < a.g.H && iw >= 0 && iw < a.g.W)
            vb = *reinterpret_cast<const uint4 *>(a.x + (((int64_t)pn[u] * a.g.H + ih) * a.g.W + iw) * a.g.Cin + bci[u]);
        }
      }
      ra[u] = va;
      rb[u] = vb;
      pow_[u] += CBK;
      while (pow_[u] >= a.g.Wo) {
        pow_[u] -= a.g.Wo;
        if (++poh[u] == a.g.Ho) { poh[u] = 0; ++pn[u]; }
      }
    }
  };
  auto bias_acc = [&]() {
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
  auto store_tile = [&](int buf) {
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

  if (nk > 0) {
    load_tile(0);
    if (do_bias) bias_acc();
    store_tile(0);
  }
  __syncthreads();
  const int g = lane >> 4;  // k rows 8g .. 8g+7 of the 32-row tile
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      load_tile(kt + 1);
      if (do_bias) bias_acc();
    }
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
    if (more) store_tile(cur ^ 1);
    __syncthreads();
  }
  if (do_bias) {
    // threads with equal (tid & 15) hold the same 8 channels: lanes l, l^16, l^32, l^48
    // in a wave, then the 4 waves through LDS (the staging buffers are free now)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bsum[j] += __shfl_xor(bsum[j], 16, 64);
      bsum[j] += __shfl_xor(bsum[j], 32, 64);
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

// dW[co][ci][kh][kw] (= or +=) sum over splits of part[s][co][tap*Cin + ci]
__global__ __launch_bounds__(256) void conv3x3_wgrad_reduce_kernel(const float *__restrict__ part, float *__restrict__ dw,
                                                                  int Cout, int Cin, int splits, int accumulate,
                                                                  const float *__restrict__ dbias_part,
                                                                  float *__restrict__ dbias) {
  const int64_t NP = 9 * (int64_t)Cin;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // index in part layout
  if (dbias && i < Cout) {
    float sb = 0.f;
    for (int k = 0; k < splits; ++k) sb += dbias_part[(int64_t)k * Cout + i];
    dbias[i] = accumulate ? dbias[i] + sb : sb;
  }
  if (i >= (int64_t)Cout * NP) return;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += part[(int64_t)k * Cout * NP + i];
  const int co = (int)(i / NP);
  const int np = (int)(i % NP);
  const int tap = np / Cin, ci = np % Cin;
  const int64_t o = ((int64_t)co * Cin + ci) * 9 + tap;
  dw[o] = accumulate ? dw[o] + s : s;
}

// pack fp32 W [Cout][Cin][3][3] -> bf16 [Cout][9][Cin] (fwd) or [Cin][9][Cout] (dgrad)
__global__ __launch_bounds__(256) void conv3x3_pack_kernel(const float *__restrict__ w, bf16_t *__restrict__ wp,
                                                          int Cout, int Cin, int Cin_pad, int transposed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)Cout * Cin_pad * 9;
  if (i >= total) return;
  // i enumerates the packed layout
  int co, ci, tap;
  if (!transposed) {            // [Cout][9][Cin_pad]
    ci = (int)(i % Cin_pad);
    tap = (int)((i / Cin_pad) % 9);
    co = (int)(i / ((int64_t)Cin_pad * 9));
  } else {                      // [Cin_pad][9][Cout]
    co = (int)(i % Cout);
    tap = (int)((i / Cout) % 9);
    ci = (int)(i / ((int64_t)Cout * 9));
  }
  const float v = ci < Cin ? w[((int64_t)co * Cin + ci) * 9 + tap] : 0.f;
  wp[i] = f2bf(v);
}

// Ncol <= 64 (the fusion conv's input gradient: 56 channels) uses the 128x64 tile
template <bool DGRAD>
static void launch_fwd(const FwdArgs &a, hipStream_t s) {
  if (a.Ncol <= 64) {
    dim3 grid((unsigned)((a.M + CBM - 1) / CBM), 1);
    hipLaunchKernelGGL((conv3x3_fwd_kernel<DGRAD, 64>), grid, dim3(256), 0, s, a);
  } else {
    dim3 grid((unsigned)((a.M + CBM - 1) / CBM), (unsigned)((a.Ncol + CBN - 1) / CBN));
    hipLaunchKernelGGL((conv3x3_fwd_kernel<DGRAD, 128>), grid, dim3(256), 0, s, a);
  }
}

static int check_geom(const ConvGeom &g, const char *nm) {
  EWVIT_CHECK_ARG(g.N > 0 && g.H > 0 && g.W > 0 && g.Cin > 0 && g.Cout > 0, "%s: empty shape", nm);
  EWVIT_CHECK_ARG(g.Cin % 8 == 0 && g.Cout % 8 == 0, "%s: Cin=%d Cout=%d must be multiples of 8", nm, g.Cin, g.Cout);
  EWVIT_CHECK_ARG(g.stride == 1 || g.stride == 2, "%s: stride %d", nm, g.stride);
  EWVIT_CHECK_ARG(g.Ho == (g.H - 1) / g.stride + 1 && g.Wo == (g.W - 1) / g.stride + 1, "%s: output size", nm);
  return 0;
}

static ConvGeom mkg(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int stride) {
  ConvGeom g;
  g.N = (int)N; g.H = (int)H; g.W = (int)W; g.Cin = (int)Cin; g.Cout = (int)Cout; g.stride = stride;
  g.Ho = (int)((H - 1) / stride + 1);
  g.Wo = (int)((W - 1) / stride + 1);
  return g;
}

}  // namespace ewvit

using namespace ewvit;

extern "C" int ewvit_conv3x3_pack_weight(const float *w, void *wp, int64_t Cout, int64_t Cin, int64_t Cin_pad,
                                         int transposed, void *stream) {
  EWVIT_CHECK_ARG(w && wp && Cout > 0 && Cin > 0 && Cin_pad >= Cin, "conv3x3_pack_weight: bad args");
  const int64_t total = Cout * Cin_pad * 9;
  hipLaunchKernelGGL(conv3x3_pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream), w,
                     (bf16_t *)wp, (int)Cout, (int)Cin, (int)Cin_pad, transposed);
  return launch_status("conv3x3_pack_weight");
}

extern "C" int ewvit_conv3x3_fwd(const void *x, const void *wp, const float *bias, void *y, int64_t N, int64_t H,
                                 int64_t W, int64_t Cin, int64_t Cout, int stride, void *stream) {
  EWVIT_CHECK_ARG(x && wp && y, "conv3x3_fwd: null pointer");
  ConvGeom g = mkg(N, H, W, Cin, Cout, stride);
  if (int rc = check_geom(g, "conv3x3_fwd")) return rc;
  FwdArgs a;
  a.src = (const bf16_t *)x; a.wp = (const bf16_t *)wp; a.bias = bias; a.out = (bf16_t *)y; a.g = g;
  a.M = (int64_t)g.N * g.Ho * g.Wo; a.Ncol = g.Cout; a.KC = g.Cin;
  a.srcH = g.H; a.srcW = g.W; a.outH = g.Ho; a.outW = g.Wo;
  launch_fwd<false>(a, as_stream(stream));
  return launch_status("conv3x3_fwd");
}

extern "C" int ewvit_conv3x3_bwd_data(const void *dy, const void *wp_t, void *dx, int64_t N, int64_t H, int64_t W,
                                      int64_t Cin, int64_t Cout, int stride, void *stream) {
  EWVIT_CHECK_ARG(dy && wp_t && dx, "conv3x3_bwd_data: null pointer");
  ConvGeom g = mkg(N, H, W, Cin, Cout, stride);
  if (int rc = check_geom(g, "conv3x3_bwd_data")) return rc;
  FwdArgs a;
  a.src = (const bf16_t *)dy; a.wp = (const bf16_t *)wp_t; a.bias = nullptr; a.out = (bf16_t *)dx; a.g = g;
  a.M = (int64_t)g.N * g.H * g.W; a.Ncol = g.Cin; a.KC = g.Cout;
  a.srcH = g.Ho; a.srcW = g.Wo; a.outH = g.H; a.outW = g.W;
  launch_fwd<true>(a, as_stream(stream));
  return launch_status("conv3x3_bwd_data");
}

static int64_t wgrad_splits(const ConvGeom &g) {
  const int64_t M = (int64_t)g.N * g.Ho * g.Wo;
  const int64_t tiles = ((9 * (int64_t)g.Cin + CBN - 1) / CBN) * ((g.Cout + CBM - 1) / CBM);
  int64_t s = (512 + tiles - 1) / tiles;          // aim at >= 512 workgroups
  const int64_t maxs = (M + 32 * CBK - 1) / (32 * CBK);  // >= 32 K-tiles per split
  if (s > maxs) s = maxs;
  if (s < 1) s = 1;
  return s;
}

extern "C" int64_t ewvit_conv3x3_bwd_weight_workspace(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout,
                                                      int stride) {
  ConvGeom g = mkg(N, H, W, Cin, Cout, stride);
  return wgrad_splits(g) * Cout * (9 * Cin + 1) * (int64_t)sizeof(float);
}

extern "C" int ewvit_conv3x3_bwd_weight(const void *x, const void *dy, float *dw, float *dbias, int accumulate,
                                        int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int stride,
                                        float *workspace, void *stream) {
  EWVIT_CHECK_ARG(x && dy && dw && workspace, "conv3x3_bwd_weight: null pointer");
  ConvGeom g = mkg(N, H, W, Cin, Cout, stride);
  if (int rc = check_geom(g, "conv3x3_bwd_weight")) return rc;
  WgradArgs a;
  a.x = (const bf16_t *)x; a.dy = (const bf16_t *)dy; a.part = workspace; a.g = g;
  a.dbias_part = dbias ? workspace + wgrad_splits(g) * g.Cout * 9 * (int64_t)g.Cin : nullptr;
  a.M = (int64_t)g.N * g.Ho * g.Wo;
  const int64_t splits = wgrad_splits(g);
  int64_t mper = (a.M + splits - 1) / splits;
  mper = (mper + CBK - 1) / CBK * CBK;
  a.mper = mper;
  const int sp = (int)((a.M + mper - 1) / mper);
  dim3 grid((unsigned)((9 * g.Cin + CBN - 1) / CBN), (unsigned)((g.Cout + CBM - 1) / CBM), (unsigned)sp);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(conv3x3_wgrad_kernel, grid, dim3(256), 0, s, a);
  if (int rc = launch_status("conv3x3_bwd_weight")) return rc;
  const int64_t n = (int64_t)g.Cout * 9 * g.Cin;
  hipLaunchKernelGGL(conv3x3_wgrad_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, workspace, dw,
                     g.Cout, g.Cin, sp, accumulate, a.dbias_part, dbias);
  return launch_status("conv3x3_bwd_weight reduce");
}
