// bf16 MFMA GEMM with fused epilogues (gfx950).
//
// C[m,n] = epi(alpha * sum_k A(m,k) B(k,n)), fp32 accumulation on
// v_mfma_f32_16x16x32_bf16.  Serves every projection of the hot path: the ViT
// to_qkv/to_out/FeedForward (network/sfe.py:29-55), the cross-attention
// to_q/to_kv/to_out (network/dama.py:25-31), patch_to_embedding
// (sfe.py:127,155; K = 62720 -> split-K) and all their backward products
// (dX = dY W needs B n-contiguous, dW = dY^T X needs A m-contiguous).
//
// Tile 64x64x32, 256 threads = 4 waves in 2x2, each wave 32x32 = 2x2 MFMA
// 16x16 tiles; LDS images are [row][k] (k contiguous, padded by 8 bf16) so each
// lane's A/B fragment (8 consecutive k) is one ds_read_b128.  Global->LDS
// staging is double-buffered through registers: the next K-tile's loads are in
// flight while the current one feeds the MFMAs.  Operands may be f32 (converted
// to bf16 while staging: the fp32 master weights are consumed without a cast
// kernel) or bf16.
//
// gemm_mx8_kernel: the same contract with MXFP8 operands (mx8.h: e4m3 elements, one E8M0
// scale per 32 consecutive K elements, quantized from the f32 / bf16 operands while staging)
// on v_mfma_scale_f32_16x16x128_f8f6f4 — BASELINE configs[4]'s fp8 token GEMMs.
#include <type_traits>

#include "common.h"
#include "mx8.h"

namespace ewvit {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int GBM = 64, GBN = 64, GBK = 32, GPAD = 8, GLD = GBK + GPAD;
constexpr int MBK = 128, MLD = MBK + 4;   // MX K-tile and its fp32 LDS image row (floats)

struct GemmArgs {
  const void *A; int64_t lda_m, lda_k;
  const void *B; int64_t ldb_k, ldb_n;
  void *C; int64_t ldc;
  int64_t M, N, K;
  float alpha, beta;
  const float *bias;
  int act;
  void *aux;
  float drop_p;
  uint64_t seed;
  const int64_t *seed_off;
  const void *resid; int resid_dtype; int64_t ldr;
  int c_dtype;
  int64_t kper;  // K per split
  float *ws;     // split-K slabs [splitk][M][N]
};

// Load 8 consecutive elements (along the contiguous dim) starting at flat
// index `base`; `n_ok` of them are in range (rest zero).
template <int DT, bool VEC>
__device__ __forceinline__ void load8(const void *p, int64_t base, int n_ok, float (&v)[8]) {
  if (VEC && n_ok == 8) {
    if (DT == EWVIT_F32) {
      const float4 *q = reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(p) + base);
      const float4 a = q[0], b = q[1];
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
      v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
      const uint4 q = *reinterpret_cast<const uint4 *>(reinterpret_cast<const bf16_t *>(p) + base);
      const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (i < n_ok) ? Elem<DT>::load(p, base + i) : 0.f;
  }
}

__device__ __forceinline__ float epilogue(const GemmArgs &g, int64_t row, int64_t col, float acc) {
  float v = g.alpha * acc;
  if (g.bias) v += g.bias[col];
  if (g.act == 1) {
    if (g.aux) reinterpret_cast<bf16_t *>(g.aux)[row * g.ldc + col] = f2bf(v);
    v = gelu_erf(v);
  } else if (g.act == 2) {
    if (g.aux) reinterpret_cast<bf16_t *>(g.aux)[row * g.ldc + col] = f2bf(v);
    v = v > 0.f ? v : 0.f;
  } else if (g.act == 3) {
    v *= gelu_erf_grad(bf2f(reinterpret_cast<const bf16_t *>(g.aux)[row * g.ldc + col]));
  }
  if (g.drop_p > 0.f) {
    const float u = uniform01(step_seed(g.seed, g.seed_off), (uint64_t)(row * g.N + col));
    v = (u >= g.drop_p) ? v * (1.0f / (1.0f - g.drop_p)) : 0.f;
  }
  if (g.resid) v += load_dt(g.resid, row * g.ldr + col, g.resid_dtype);
  if (g.beta != 0.f) v += g.beta * reinterpret_cast<const float *>(g.C)[row * g.ldc + col];
  return v;
}

__device__ __forceinline__ void store_c(const GemmArgs &g, int64_t row, int64_t col, float v) {
  if (g.c_dtype == EWVIT_F32)
    reinterpret_cast<float *>(g.C)[row * g.ldc + col] = v;
  else
    reinterpret_cast<bf16_t *>(g.C)[row * g.ldc + col] = f2bf(v);
}

// Stage one 64x32 operand tile into registers.  ROWS = the M (or N) index,
// K the reduction index.  KCONTIG: element (r,k) at base + r*ld_r + k.
// otherwise at base + r + k*ld_k (r contiguous).
template <int DT, bool KCONTIG, bool VEC>
struct Stager {
  float v[8];
  int r, k;  // first element coordinates inside the tile
  __device__ __forceinline__ void load(const void *p, int64_t ld_r, int64_t ld_k, int64_t r0,
                                       int64_t R, int64_t k0, int64_t kend, int tid) {
    if (KCONTIG) {
      r = tid >> 2; k = (tid & 3) * 8;
      const int64_t gr = r0 + r, gk = k0 + k;
      int n_ok = 0;
      if (gr < R) n_ok = (int)(kend - gk > 8 ? 8 : (kend - gk > 0 ? kend - gk : 0));
      load8<DT, VEC>(p, gr * ld_r + gk, n_ok, v);
    } else {
      k = tid >> 3; r = (tid & 7) * 8;
      const int64_t gr = r0 + r, gk = k0 + k;
      int n_ok = 0;
      if (gk < kend) n_ok = (int)(R - gr > 8 ? 8 : (R - gr > 0 ? R - gr : 0));
      load8<DT, VEC>(p, gr + gk * ld_k, n_ok, v);
    }
  }
  // the MX kernel's source image for block quantization, in the operand's own dtype (exact):
  // fp32 for an fp32 operand, bf16 for a bf16 one (no rounding while staging)
  template <typename T>
  __device__ __forceinline__ void store_img(T (*lds)[MLD], int k_off) {
    if (KCONTIG) {
#pragma unroll
      for (int i = 0; i < 8; ++i) lds[r][k_off + k + i] = (T)v[i];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) lds[r + i][k_off + k] = (T)v[i];
    }
  }
  // MX (KCONTIG only): this thread's 8 values of 32-element block p of row r, quantized with
  // the block's scale — the block is this row's 4 adjacent lanes (k = 0, 8, 16, 24 of it), so
  // their maxima meet by two xor shuffles; lane 0 of the four stores the E8M0 byte
  template <int LDQ>
  __device__ __forceinline__ void store_mx(uint8_t (*img)[LDQ], uint8_t (*sc)[4], int p) {
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) m = fmaxf(m, fabsf(v[i]));
    m = fmaxf(m, __shfl_xor(m, 1, 64));
    m = fmaxf(m, __shfl_xor(m, 2, 64));
    const int e = mx_exp(m);
    const float s = mx_inv_scale(e);
    unsigned w[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int q = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * h] * s, v[4 * h + 1] * s, 0, false);
      q = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * h + 2] * s, v[4 * h + 3] * s, q, true);
      w[h] = (unsigned)q;
    }
    *reinterpret_cast<uint2 *>(&img[r][p * 32 + k]) = make_uint2(w[0], w[1]);
    if ((threadIdx.x & 3) == 0) sc[r][p] = (uint8_t)e;
  }
  __device__ __forceinline__ void store(bf16_t (*lds)[GLD]) {
    if (KCONTIG) {
      __attribute__((aligned(16))) bf16_t t[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) t[i] = f2bf(v[i]);
      *reinterpret_cast<uint4 *>(&lds[r][k]) = *reinterpret_cast<const uint4 *>(t);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) lds[r + i][k] = f2bf(v[i]);
    }
  }
};

template <int ADT, int BDT, bool AK, bool BK, bool AV, bool BV>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) bf16_t As[2][GBM][GLD];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][GBN][GLD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int64_t m0 = (int64_t)blockIdx.y * GBM, n0 = (int64_t)blockIdx.x * GBN;
  const int64_t kbeg = (int64_t)blockIdx.z * g.kper;
  const int64_t kend = (kbeg + g.kper < g.K) ? kbeg + g.kper : g.K;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Stager<ADT, AK, AV> sa;
  Stager<BDT, BK, BV> sb;
  const int nk = (int)((kend - kbeg + GBK - 1) / GBK);
  if (nk > 0) {
    sa.load(g.A, AK ? g.lda_m : 0, AK ? 0 : g.lda_k, m0, g.M, kbeg, kend, tid);
    sb.load(g.B, BK ? g.ldb_n : 0, BK ? 0 : g.ldb_k, n0, g.N, kbeg, kend, tid);
    sa.store(As[0]);
    sb.store(Bs[0]);
  }
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      const int64_t k0 = kbeg + (int64_t)(kt + 1) * GBK;
      sa.load(g.A, AK ? g.lda_m : 0, AK ? 0 : g.lda_k, m0, g.M, k0, kend, tid);
      sb.load(g.B, BK ? g.ldb_n : 0, BK ? 0 : g.ldb_k, n0, g.N, k0, kend, tid);
    }
    bf16x8 af[2], bfr[2];
    const int fr = lane & 15, fk = (lane >> 4) * 8;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      af[i] = *reinterpret_cast<const bf16x8 *>(&As[cur][wm * 32 + i * 16 + fr][fk]);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8 *>(&Bs[cur][wn * 32 + j * 16 + fr][fk]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (more) {
      sa.store(As[cur ^ 1]);
      sb.store(Bs[cur ^ 1]);
    }
    __syncthreads();
    cur ^= 1;
  }

  // C/D map of 16x16x32: col = lane&15, row = (lane>>4)*4 + r
  const bool split = gridDim.z > 1;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int64_t col = n0 + wn * 32 + j * 16 + (lane & 15);
        if (row < g.M && col < g.N) {
          if (split)
            g.ws[((int64_t)blockIdx.z * g.M + row) * g.N + col] = acc[i][j][r];
          else
            store_c(g, row, col, epilogue(g, row, col, acc[i][j][r]));
        }
      }
}

// MXFP8 GEMM: 64 x 64 output tile, 128-wide K-tiles.  An operand stored K-contiguous is
// quantized in registers as it is staged (a 32-element block is the Stager's 4 adjacent lanes of
// one row: two xor shuffles) straight into its e4m3 image; an operand stored the other way (the
// backward products' dY^T / X) is staged as fp32 in LDS first and each of the 256 threads then
// quantizes one 32-element block of it (row t / 4, block t % 4) — every block once, any layout.
// The e4m3 images alternate per K-tile, so one or two barriers per K-tile order the phases (the
// fp32 images are rewritten only after every wave quantized them; an e4m3 image only after every
// wave passed the next K-tile's first barrier, i.e. finished its MFMAs).  The 4 waves (2 x 2,
// 32 x 32 each) read their fragments from the images (two 16-B runs per lane, mx8.h's lane map)
// and run one v_mfma_scale_f32_16x16x128_f8f6f4 per 16 x 16 tile; the next K-tile's global
// loads are in flight meanwhile.  Rows / K past the matrix are zero.  The MFMA applies both
// block scales, so the epilogue sees the descaled product.
constexpr int Q8LD = MBK + 16;          // e4m3 image row (bytes): conflict-free 16-B fragment reads
template <int ADT, int BDT, bool AK, bool BK, bool AV, bool BV>
__global__ __launch_bounds__(256) void gemm_mx8_kernel(GemmArgs g) {
  // source images (non-K-contiguous operands only) in the operand's dtype; e4m3 images doubled
  // for a K-contiguous operand (written in the staging phase, which may run while a slower wave
  // still reads the previous K-tile's image), single for the others (written after the barrier
  // every wave reaches only after its MFMAs)
  using AT = typename std::conditional<ADT == EWVIT_BF16, __bf16, float>::type;
  using BT = typename std::conditional<BDT == EWVIT_BF16, __bf16, float>::type;
  constexpr int NQA = AK ? 2 : 1, NQB = BK ? 2 : 1;
  __shared__ __attribute__((aligned(16))) AT As[AK ? 1 : GBM][MLD];
  __shared__ __attribute__((aligned(16))) BT Bs[BK ? 1 : GBN][MLD];
  __shared__ __attribute__((aligned(16))) uint8_t Aq[NQA][GBM][Q8LD];
  __shared__ __attribute__((aligned(16))) uint8_t Bq[NQB][GBN][Q8LD];
  __shared__ uint8_t Asc[NQA][GBM][4], Bsc[NQB][GBN][4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int64_t m0 = (int64_t)blockIdx.y * GBM, n0 = (int64_t)blockIdx.x * GBN;
  const int64_t kbeg = (int64_t)blockIdx.z * g.kper;
  const int64_t kend = (kbeg + g.kper < g.K) ? kbeg + g.kper : g.K;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  Stager<ADT, AK, AV> sa[4];
  Stager<BDT, BK, BV> sb[4];
  const int nk = (int)((kend - kbeg + MBK - 1) / MBK);
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      sa[p].load(g.A, AK ? g.lda_m : 0, AK ? 0 : g.lda_k, m0, g.M, k0 + p * GBK, kend, tid);
      sb[p].load(g.B, BK ? g.ldb_n : 0, BK ? 0 : g.ldb_k, n0, g.N, k0 + p * GBK, kend, tid);
    }
  };
  // one 32-element block of an fp32 image row -> its e4m3 bytes and scale
  auto quant = [&](const auto (*src)[MLD], uint8_t (*dst)[Q8LD], uint8_t (*sc)[4]) {
    const int row = tid >> 2, blk = tid & 3;
    float v[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) v[q] = (float)src[row][blk * 32 + q];
    int d[8];
    sc[row][blk] = (uint8_t)mx_quant_block(v, d);
    uint4 *o = reinterpret_cast<uint4 *>(&dst[row][blk * 32]);
    o[0] = make_uint4(d[0], d[1], d[2], d[3]);
    o[1] = make_uint4(d[4], d[5], d[6], d[7]);
  };
  auto frag = [&](const uint8_t (*img)[Q8LD], const uint8_t (*sc)[4], int row) {
    MxFrag f;
    const uint4 x = *reinterpret_cast<const uint4 *>(&img[row][mx_k0(lane)]);
    const uint4 y = *reinterpret_cast<const uint4 *>(&img[row][mx_k1(lane)]);
    f.d[0] = (int)x.x; f.d[1] = (int)x.y; f.d[2] = (int)x.z; f.d[3] = (int)x.w;
    f.d[4] = (int)y.x; f.d[5] = (int)y.y; f.d[6] = (int)y.z; f.d[7] = (int)y.w;
    f.sc = sc[row][lane >> 4];
    return f;
  };
  if (nk > 0) load(kbeg);
  const int r = lane & 15;
  for (int kt = 0; kt < nk; ++kt) {
    const int ba = AK ? kt & 1 : 0, bb = BK ? kt & 1 : 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if constexpr (AK) sa[p].store_mx(Aq[ba], Asc[ba], p);
      else sa[p].store_img(As, p * GBK);
      if constexpr (BK) sb[p].store_mx(Bq[bb], Bsc[bb], p);
      else sb[p].store_img(Bs, p * GBK);
    }
    __syncthreads();
    if (kt + 1 < nk) load(kbeg + (int64_t)(kt + 1) * MBK);
    if constexpr (!AK || !BK) {
      if constexpr (!AK) quant(As, Aq[0], Asc[0]);
      if constexpr (!BK) quant(Bs, Bq[0], Bsc[0]);
      __syncthreads();
    }
    MxFrag af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = frag(Aq[ba], Asc[ba], wm * 32 + i * 16 + r);
#pragma unroll
    for (int j = 0; j < 2; ++j) bfr[j] = frag(Bq[bb], Bsc[bb], wn * 32 + j * 16 + r);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mx_mma(af[i], bfr[j], acc[i][j]);
  }

  const bool split = gridDim.z > 1;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + q;
        const int64_t col = n0 + wn * 32 + j * 16 + (lane & 15);
        if (row < g.M && col < g.N) {
          if (split)
            g.ws[((int64_t)blockIdx.z * g.M + row) * g.N + col] = acc[i][j][q];
          else
            store_c(g, row, col, epilogue(g, row, col, acc[i][j][q]));
        }
      }
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs g, int splitk) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= g.M * g.N) return;
  const int64_t row = idx / g.N, col = idx % g.N;
  float s = 0.f;
  for (int z = 0; z < splitk; ++z) s += g.ws[(int64_t)z * g.M * g.N + idx];
  store_c(g, row, col, epilogue(g, row, col, s));
}

__global__ __launch_bounds__(256) void colsum_kernel(const void *X, int dt, int64_t ldx, int64_t M,
                                                     int64_t N, float *out, int accumulate) {
  // one thread per column, 4 row-groups per block reduced through LDS
  __shared__ float part[4][64];
  const int64_t col = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int grp = threadIdx.x >> 6;
  float s = 0.f;
  if (col < N)
    for (int64_t m = grp; m < M; m += 4) s += load_dt(X, m * ldx + col, dt);
  part[grp][threadIdx.x & 63] = s;
  __syncthreads();
  if (grp == 0 && col < N) {
    const float t = part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x];
    out[col] = accumulate ? out[col] + t : t;
  }
}

__global__ __launch_bounds__(256) void dropout_bwd_kernel(void *g, int dt, int64_t rows, int64_t cols,
                                                          int64_t ldg, float p, uint64_t seed,
                                                          const int64_t *seed_off) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * cols) return;
  const int64_t r = idx / cols, c = idx % cols;
  const float u = uniform01(step_seed(seed, seed_off), (uint64_t)idx);
  const int64_t o = r * ldg + c;
  const float v = load_dt(g, o, dt);
  store_dt(g, o, u >= p ? v * (1.0f / (1.0f - p)) : 0.f, dt);
}

// g_pre = dy * keep(seed)/(1-p) * act'(aux): the backward of the GEMM epilogue
__global__ __launch_bounds__(256) void act_bwd_kernel(const void *dy, int dydt, int64_t lddy,
                                                      const bf16_t *aux, int act, float p, uint64_t seed,
                                                      const int64_t *seed_off,
                                                      void *out, int odt, int64_t M, int64_t N) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  const int64_t r = idx / N, c = idx % N;
  float v = load_dt(dy, r * lddy + c, dydt);
  if (p > 0.f) v = uniform01(step_seed(seed, seed_off), (uint64_t)idx) >= p ? v * (1.0f / (1.0f - p)) : 0.f;
  if (act == 1) v *= gelu_erf_grad(bf2f(aux[idx]));
  else if (act == 2) v = bf2f(aux[idx]) > 0.f ? v : 0.f;
  store_dt(out, idx, v, odt);
}

template <int ADT, int BDT, bool AK, bool BK>
static void launch_typed(const GemmArgs &g, bool av, bool bv, bool q8, dim3 grid, hipStream_t s) {
  dim3 block(256);
  if (q8) {
    if (av && bv) hipLaunchKernelGGL((gemm_mx8_kernel<ADT, BDT, AK, BK, true, true>), grid, block, 0, s, g);
    else if (av) hipLaunchKernelGGL((gemm_mx8_kernel<ADT, BDT, AK, BK, true, false>), grid, block, 0, s, g);
    else if (bv) hipLaunchKernelGGL((gemm_mx8_kernel<ADT, BDT, AK, BK, false, true>), grid, block, 0, s, g);
    else hipLaunchKernelGGL((gemm_mx8_kernel<ADT, BDT, AK, BK, false, false>), grid, block, 0, s, g);
    return;
  }
  if (av && bv) hipLaunchKernelGGL((gemm_kernel<ADT, BDT, AK, BK, true, true>), grid, block, 0, s, g);
  else if (av) hipLaunchKernelGGL((gemm_kernel<ADT, BDT, AK, BK, true, false>), grid, block, 0, s, g);
  else if (bv) hipLaunchKernelGGL((gemm_kernel<ADT, BDT, AK, BK, false, true>), grid, block, 0, s, g);
  else hipLaunchKernelGGL((gemm_kernel<ADT, BDT, AK, BK, false, false>), grid, block, 0, s, g);
}

template <int ADT, int BDT>
static void launch_layout(const GemmArgs &g, bool ak, bool bk, bool av, bool bv, bool q8, dim3 grid,
                          hipStream_t s) {
  if (ak && bk) launch_typed<ADT, BDT, true, true>(g, av, bv, q8, grid, s);
  else if (ak) launch_typed<ADT, BDT, true, false>(g, av, bv, q8, grid, s);
  else if (bk) launch_typed<ADT, BDT, false, true>(g, av, bv, q8, grid, s);
  else launch_typed<ADT, BDT, false, false>(g, av, bv, q8, grid, s);
}

// 8 consecutive elements along the contiguous dim can be one 16/32-B load iff
// the base and every row start are aligned.
static bool vec_ok(const void *p, int dt, int64_t ld_other) {
  const int64_t esz = dt == EWVIT_F32 ? 4 : 2;
  const int64_t align = dt == EWVIT_F32 ? 16 : 16;
  return ((uintptr_t)p % align == 0) && ((ld_other * esz) % align == 0);
}

}  // namespace ewvit

using namespace ewvit;

static int gemm_impl(const void *A, int a_dtype, int64_t lda_m, int64_t lda_k, const void *B,
                     int b_dtype, int64_t ldb_k, int64_t ldb_n, void *C, int c_dtype,
                     int64_t ldc, int64_t M, int64_t N, int64_t K, float alpha, float beta,
                     const float *bias, int act, void *aux, float drop_p, uint64_t seed,
                     const int64_t *seed_offset, const void *resid, int resid_dtype, int64_t ldr, int splitk,
                     float *workspace, bool q8, void *stream) {
  EWVIT_CHECK_ARG(A && B && C, "gemm: null operand");
  EWVIT_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "gemm: negative size");
  EWVIT_CHECK_ARG(dtype_ok(a_dtype) && dtype_ok(b_dtype) && dtype_ok(c_dtype), "gemm: bad dtype");
  EWVIT_CHECK_ARG(lda_m == 1 || lda_k == 1, "gemm: A needs a unit stride (lda_m=%lld lda_k=%lld)",
                  (long long)lda_m, (long long)lda_k);
  EWVIT_CHECK_ARG(ldb_k == 1 || ldb_n == 1, "gemm: B needs a unit stride");
  EWVIT_CHECK_ARG(act >= 0 && act <= 3, "gemm: act=%d", act);
  EWVIT_CHECK_ARG(act != 3 || aux, "gemm: act 3 needs aux (pre-activation)");
  EWVIT_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f, "gemm: drop_p=%f", (double)drop_p);
  EWVIT_CHECK_ARG(beta == 0.f || c_dtype == EWVIT_F32, "gemm: beta needs f32 C");
  EWVIT_CHECK_ARG(!resid || dtype_ok(resid_dtype), "gemm: bad resid dtype");
  EWVIT_CHECK_ARG(splitk >= 1 && splitk <= 256, "gemm: splitk=%d", splitk);
  EWVIT_CHECK_ARG(splitk == 1 || workspace, "gemm: split-K needs a workspace");
  if (M == 0 || N == 0) return 0;
  GemmArgs g;
  g.A = A; g.lda_m = lda_m; g.lda_k = lda_k;
  g.B = B; g.ldb_k = ldb_k; g.ldb_n = ldb_n;
  g.C = C; g.ldc = ldc; g.M = M; g.N = N; g.K = K;
  g.alpha = alpha; g.beta = beta; g.bias = bias; g.act = act; g.aux = aux;
  g.drop_p = drop_p; g.seed = seed; g.seed_off = seed_offset; g.resid = resid; g.resid_dtype = resid_dtype; g.ldr = ldr;
  g.c_dtype = c_dtype; g.ws = workspace;
  // K per split, a multiple of the K tile (128 for the MX kernel)
  const int kt = q8 ? MBK : GBK;
  int64_t kper = (K + splitk - 1) / splitk;
  kper = ((kper + kt - 1) / kt) * kt;
  if (kper == 0) kper = kt;
  int sk = (int)((K + kper - 1) / kper);
  if (sk < 1) sk = 1;
  g.kper = kper;
  const bool ak = (lda_k == 1), bk = (ldb_k == 1);
  const bool av = vec_ok(A, a_dtype, ak ? lda_m : lda_k);
  const bool bv = vec_ok(B, b_dtype, bk ? ldb_n : ldb_k);
  dim3 grid((unsigned)((N + GBN - 1) / GBN), (unsigned)((M + GBM - 1) / GBM), (unsigned)sk);
  EWVIT_CHECK_ARG(grid.y <= 65535, "gemm: M too large");
  hipStream_t s = as_stream(stream);
  if (a_dtype == EWVIT_BF16 && b_dtype == EWVIT_BF16) launch_layout<EWVIT_BF16, EWVIT_BF16>(g, ak, bk, av, bv, q8, grid, s);
  else if (a_dtype == EWVIT_BF16) launch_layout<EWVIT_BF16, EWVIT_F32>(g, ak, bk, av, bv, q8, grid, s);
  else if (b_dtype == EWVIT_BF16) launch_layout<EWVIT_F32, EWVIT_BF16>(g, ak, bk, av, bv, q8, grid, s);
  else launch_layout<EWVIT_F32, EWVIT_F32>(g, ak, bk, av, bv, q8, grid, s);
  int rc = launch_status(q8 ? "gemm_mx8" : "gemm");
  if (rc || sk == 1) return rc;
  const int64_t total = M * N;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, g, sk);
  return launch_status("gemm splitk reduce");
}

extern "C" int ewvit_gemm(const void *A, int a_dtype, int64_t lda_m, int64_t lda_k, const void *B,
                          int b_dtype, int64_t ldb_k, int64_t ldb_n, void *C, int c_dtype,
                          int64_t ldc, int64_t M, int64_t N, int64_t K, float alpha, float beta,
                          const float *bias, int act, void *aux, float drop_p, uint64_t seed,
                          const int64_t *seed_offset, const void *resid, int resid_dtype, int64_t ldr, int splitk,
                          float *workspace, void *stream) {
  return gemm_impl(A, a_dtype, lda_m, lda_k, B, b_dtype, ldb_k, ldb_n, C, c_dtype, ldc, M, N, K, alpha, beta, bias,
                   act, aux, drop_p, seed, seed_offset, resid, resid_dtype, ldr, splitk, workspace, false, stream);
}

extern "C" int ewvit_gemm_mx8(const void *A, int a_dtype, int64_t lda_m, int64_t lda_k, const void *B,
                              int b_dtype, int64_t ldb_k, int64_t ldb_n, void *C, int c_dtype,
                              int64_t ldc, int64_t M, int64_t N, int64_t K, float alpha, float beta,
                              const float *bias, int act, void *aux, float drop_p, uint64_t seed,
                              const int64_t *seed_offset, const void *resid, int resid_dtype, int64_t ldr,
                              int splitk, float *workspace, void *stream) {
  return gemm_impl(A, a_dtype, lda_m, lda_k, B, b_dtype, ldb_k, ldb_n, C, c_dtype, ldc, M, N, K, alpha, beta, bias,
                   act, aux, drop_p, seed, seed_offset, resid, resid_dtype, ldr, splitk, workspace, true, stream);
}

extern "C" int ewvit_colsum(const void *X, int x_dtype, int64_t ldx, int64_t M, int64_t N,
                            float *out, int accumulate, void *stream) {
  EWVIT_CHECK_ARG(X && out, "colsum: null pointer");
  EWVIT_CHECK_ARG(dtype_ok(x_dtype) && M >= 0 && N >= 0, "colsum: bad args");
  if (N == 0) return 0;
  hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)((N + 63) / 64)), dim3(256), 0, as_stream(stream),
                     X, x_dtype, ldx, M, N, out, accumulate);
  return launch_status("colsum");
}

extern "C" int ewvit_dropout_bwd(void *g, int g_dtype, int64_t rows, int64_t cols, int64_t ldg,
                                 float p, uint64_t seed, const int64_t *seed_offset, void *stream) {
  EWVIT_CHECK_ARG(g && dtype_ok(g_dtype) && p >= 0.f && p < 1.f, "dropout_bwd: bad args");
  const int64_t total = rows * cols;
  if (total == 0 || p == 0.f) return 0;
  hipLaunchKernelGGL(dropout_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     as_stream(stream), g, g_dtype, rows, cols, ldg, p, seed, seed_offset);
  return launch_status("dropout_bwd");
}

extern "C" int ewvit_act_bwd(const void *dy, int dy_dtype, int64_t lddy, const void *aux, int act,
                             float drop_p, uint64_t seed, const int64_t *seed_offset, void *out,
                             int out_dtype, int64_t M,
                             int64_t N, void *stream) {
  EWVIT_CHECK_ARG(dy && out && dtype_ok(dy_dtype) && dtype_ok(out_dtype), "act_bwd: bad args");
  EWVIT_CHECK_ARG(act >= 0 && act <= 2 && (act == 0 || aux), "act_bwd: act=%d needs aux", act);
  EWVIT_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f, "act_bwd: drop_p");
  const int64_t total = M * N;
  if (total == 0) return 0;
  hipLaunchKernelGGL(act_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     as_stream(stream), dy, dy_dtype, lddy, (const bf16_t *)aux, act, drop_p, seed,
                     seed_offset, out, out_dtype, M, N);
  return launch_status("act_bwd");
}
