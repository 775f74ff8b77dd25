// The DAMA frame head on one workgroup (gfx950): everything of DAMA._process_frame after its
// two branches (reference network/dama.py:143-169) —
//   * BidirectionalCrossTransformer, depth 2 (dama.py:56-78, 116-122): per layer
//     s = s + CA_s(LN(s), f); f = f + CA_f(LN(f), s) with CrossAttention (dama.py:15-53):
//     kv_include_self, 4 heads of 32, to_q / to_kv without bias, to_out + Dropout(0.1);
//   * fusion_gate (dama.py:124-128, 152-153): Conv3x3(256 -> 128, pad 1) on the 1x1 map —
//     only the centre tap meets data — + BatchNorm2d (batch statistics over the chunk's
//     frames in training) + ReLU;
//   * gate_net (dama.py:105-113, 156-157): Linear(256 -> 64) + ReLU + Dropout(0.1) +
//     Linear(64 -> 3) + Softmax;
//   * the 3-way weighted sum (dama.py:159-163).
// The token streams are one token per frame (the 1x1 maps of both branches), so the whole
// head is [N <= 64, 128] matrices against 0.3 M parameters: ~90 small launches in the
// module-by-module form, here
//   ewvit_head_fwd        one workgroup: the forward, saving what the backward needs;
//   ewvit_head_bwd_data   one workgroup: the gradients of every activation, back to the two
//                         branch inputs, and the BatchNorm affine gradients;
//   ewvit_head_bwd_weight a grid: every weight / bias gradient as fp32 dot products over the
//                         frames (the fusion-gate conv's 8 dead taps written as zeros).
// GEMMs on v_mfma_f32_16x16x32_bf16 (bf16 operands, fp32 accumulation, as the module path's
// ewvit_gemm rounds them): the activation operand staged in LDS, the fp32 master weights
// loaded straight to registers and rounded (each weight element read once per workgroup).
// Per-row statistics (LayerNorm, softmax, attention) and every accumulation in fp32.
// Intermediates live in a caller workspace (L2-resident at this size; visible to the
// workgroup's own later phases across __syncthreads()).
#include "common.h"

namespace ewvit {

typedef ewvit_head_ca HeadCA;
typedef ewvit_head_params HeadParams;

constexpr int HD = 128;           // dama dim
constexpr int HN = 64;            // frames per chunk, at most (pos_embedding rows)
constexpr int HKP = 256 + 8;      // LDS row pitch (bf16) of the GEMM activation operand
constexpr int HSITE = 1 << 20;    // dropout counter stride between sites

typedef __attribute__((ext_vector_type(8))) __bf16 hbf16x8;
typedef __attribute__((ext_vector_type(4))) float hf32x4;

// ---- workspace layout (floats); N <= 64 rows each.  Pointers are computed from the base (no
// arrays of pointers: a runtime block index would put such an array in scratch memory).
constexpr int64_t W_BLK = HN * HD + 2 * HN + HN * HD + HN * 512 + HN * 8 + HN * HD;   // per attention block
constexpr int64_t W_BLK0 = 6 * HN * HD;
constexpr int64_t W_FUS0 = W_BLK0 + 4 * W_BLK;
constexpr int64_t W_BBLK = HN * HD + HN * HD + HN * 512 + HN * HD;                    // per block, backward
constexpr int64_t W_BBLK0 = W_FUS0 + HN * HD + 2 * HD + HN * HD + HN * 64 + HN * 4;
constexpr int64_t W_TAIL0 = W_BBLK0 + 4 * W_BBLK;
constexpr int64_t W_TOTAL = W_TAIL0 + HN * HD + HN * 64 + HN * 4 + 2 * HN * HD + HN * 256 + HN * 256 + HD * 256;

struct HeadWs {
  float *b;
  // states s0 (copy), f0 (copy), s1, f1, s2, f2   [N][128]
  __device__ float *st(int i) const { return b + (int64_t)i * HN * HD; }
  // per attention block: LayerNorm output [N][128], its mean / rstd [N], to_q [N][128], to_kv of
  // (self, context) [N][2][256], softmax weights [N][4][2], attention output [N][128]
  __device__ float *xn(int i) const { return b + W_BLK0 + i * W_BLK; }
  __device__ float *mu(int i) const { return xn(i) + HN * HD; }
  __device__ float *rs(int i) const { return mu(i) + HN; }
  __device__ float *q(int i) const { return rs(i) + HN; }
  __device__ float *kv(int i) const { return q(i) + HN * HD; }
  __device__ float *at(int i) const { return kv(i) + HN * 512; }
  __device__ float *o(int i) const { return at(i) + HN * 8; }
  __device__ float *yfg() const { return b + W_FUS0; }            // fusion conv out, pre-BN [N][128]
  __device__ float *bnm() const { return yfg() + HN * HD; }       // BatchNorm mean [128]
  __device__ float *bni() const { return bnm() + HD; }            // and invstd [128]
  __device__ float *fus() const { return bni() + HD; }            // ReLU(BN(yfg)) [N][128]
  __device__ float *h1() const { return fus() + HN * HD; }        // gate first layer, pre-act [N][64]
  __device__ float *gw() const { return h1() + HN * 64; }         // softmax gate [N][4] (3 used)
  // backward, per block: d LayerNorm output, d q, d kv, d to_out pre-dropout output
  __device__ float *dxn(int i) const { return b + W_BBLK0 + i * W_BBLK; }
  __device__ float *dq(int i) const { return dxn(i) + HN * HD; }
  __device__ float *dkv(int i) const { return dq(i) + HN * HD; }
  __device__ float *dpre(int i) const { return dkv(i) + HN * 512; }
  __device__ float *dy() const { return b + W_TAIL0; }            // d fusion conv out [N][128]
  __device__ float *dh1() const { return dy() + HN * HD; }        // d gate pre-activation [N][64]
  __device__ float *dz2() const { return dh1() + HN * 64; }       // d gate logits [N][4]
  __device__ float *ds(int i) const { return dz2() + HN * 4 + (int64_t)i * HN * HD; }  // state grads s, f
  __device__ float *dcat() const { return ds(0) + 2 * HN * HD; }  // d concat [N][256]
  __device__ float *tmp() const { return dcat() + HN * 256; }     // scratch [N][256]
  __device__ float *wc() const { return tmp() + HN * 256; }       // fusion centre tap, re-laid [128*256]
};

__host__ __device__ inline int64_t head_ws_floats() { return W_TOTAL; }

__device__ inline HeadWs head_ws(float *b) { return HeadWs{b}; }

// attention blocks in forward order: 0 = layer 0 s, 1 = layer 0 f, 2 = layer 1 s, 3 = layer 1 f
// block i reads state x = st[xin(i)] and context ctx = st[cin(i)], writes st[xout(i)]
__device__ __forceinline__ int h_xin(int i) { return (i >> 1) * 2 + (i & 1); }        // s0 f0 s1 f1
__device__ __forceinline__ int h_xout(int i) { return (i >> 1) * 2 + 2 + (i & 1); }   // s1 f1 s2 f2
__device__ __forceinline__ int h_cin(int i) { return (i & 1) ? (i >> 1) * 2 + 2 : (i >> 1) * 2 + 1; }  // f0 s1 f1 s2

__device__ __forceinline__ float h_drop(const HeadParams &p, int site, int n, int c, float prob) {
  if (prob <= 0.f) return 1.f;
  const float u = uniform01(step_seed(p.seed, p.seed_off), (uint64_t)site * HSITE + (uint64_t)n * 256 + c);
  return u >= prob ? 1.f / (1.f - prob) : 0.f;
}

// C[n][col] (n < 64, ldc) = sum_k A[n][k] B(k, col) for the workgroup: A bf16 in LDS (pitch
// HKP, rows >= N zero), B from the fp32 weight W: TRANS = false: B(k, col) = W[col * ldw + k]
// (nn.Linear forward, k contiguous); TRANS = true: B(k, col) = W[k * ldw + col] (input
// gradient).  NOUT columns split over the 4 waves (NOUT / 4 each, multiples of 16); every
// B fragment of the wave is loaded before the MFMAs.
template <int NOUT, int K, bool TRANS>
__device__ __forceinline__ void h_gemm(const bf16_t *A, const float *W, int64_t ldw, float *C, int ldc, int N) {
  constexpr int NW = NOUT / 4, NT = NW / 16, KS = K / 32;
  static_assert(NW % 16 == 0 && K % 32 == 0, "h_gemm shape");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = w * NW;
  hbf16x8 bfr[NT][KS];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int col = c0 + j * 16 + (lane & 15), k0 = s * 32 + (lane >> 4) * 8;
      float v[8];
      if (!TRANS) {
        const float4 a = *reinterpret_cast<const float4 *>(W + (int64_t)col * ldw + k0);
        const float4 b = *reinterpret_cast<const float4 *>(W + (int64_t)col * ldw + k0 + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = W[(int64_t)(k0 + e) * ldw + col];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) bfr[j][s][e] = (__bf16)v[e];
    }
  hf32x4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = hf32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    hbf16x8 af[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      af[i] = *reinterpret_cast<const hbf16x8 *>(A + (i * 16 + (lane & 15)) * HKP + s * 32 + (lane >> 4) * 8);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j][s], acc[i][j], 0, 0, 0);
  }
  // C/D map: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i * 16 + (lane >> 4) * 4 + r;
        if (row < N) C[row * ldc + c0 + j * 16 + (lane & 15)] = acc[i][j][r];
      }
}

// A (LDS, bf16) rows n < 64, cols [0, ncol): src[n * lds + c] (fp32) for n < N, 0 beyond
__device__ __forceinline__ void h_stage(bf16_t *A, int acol, const float *src, int lds, int ncol, int N) {
  for (int e = threadIdx.x; e < HN * ncol; e += 256) {
    const int n = e / ncol, c = e - n * ncol;
    A[n * HKP + acol + c] = n < N ? f2bf(src[n * lds + c]) : (bf16_t)0;
  }
}

// LayerNorm of the rows of x (fp32 [N][128]) -> xn (fp32, ws) and A (bf16 LDS); one wave per
// row, lane = 2 columns; two-pass statistics, biased variance, eps inside the rsqrt (torch)
__device__ void h_layernorm(const float *x, const float *g, const float *b, float eps, float *xn, float *mu,
                            float *rs, bf16_t *A, int N) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int n = w; n < HN; n += 4) {
    if (n >= N) {
      A[n * HKP + lane] = 0; A[n * HKP + lane + 64] = 0;
      continue;
    }
    const float v0 = x[n * HD + lane], v1 = x[n * HD + lane + 64];
    const float m = wave_sum(v0 + v1) * (1.f / HD);
    const float d0 = v0 - m, d1 = v1 - m;
    const float r = rsqrtf(wave_sum(d0 * d0 + d1 * d1) * (1.f / HD) + eps);
    const float y0 = d0 * r * g[lane] + b[lane], y1 = d1 * r * g[lane + 64] + b[lane + 64];
    xn[n * HD + lane] = y0; xn[n * HD + lane + 64] = y1;
    A[n * HKP + lane] = f2bf(y0); A[n * HKP + lane + 64] = f2bf(y1);
    if (lane == 0) { mu[n] = m; rs[n] = r; }
  }
}

extern __shared__ __attribute__((aligned(16))) unsigned char h_smem[];

__global__ __launch_bounds__(256) void head_fwd_kernel(HeadParams p, const float *s0, const float *f0, float *ws_base,
                                                       float *fused_out, float *s_out, float *f_out, int N) {
  bf16_t *A = reinterpret_cast<bf16_t *>(h_smem);                     // [64][HKP]
  float *red = reinterpret_cast<float *>(h_smem + HN * HKP * 2);      // [4][256]
  HeadWs ws = head_ws(ws_base);
  const int tid = threadIdx.x;
  const float scale = 0.17677669529663687f;                           // 32^-0.5 (dama.py:30)
  for (int e = tid; e < N * HD; e += 256) { ws.st(0)[e] = s0[e]; ws.st(1)[e] = f0[e]; }
  __syncthreads();
  for (int i = 0; i < 4; ++i) {
    const HeadCA &ca = p.ca[i];
    const float *x = ws.st(h_xin(i)), *ctx = ws.st(h_cin(i));
    h_layernorm(x, ca.ln_w, ca.ln_b, p.ln_eps, ws.xn(i), ws.mu(i), ws.rs(i), A, N);
    __syncthreads();
    // to_q (dama.py:43) and to_kv of the self token (kv_include_self: the NORMALISED x, :38-39)
    h_gemm<128, 128, false>(A, ca.wq, HD, ws.q(i), HD, N);
    h_gemm<256, 128, false>(A, ca.wkv, HD, ws.kv(i), 512, N);
    __syncthreads();
    h_stage(A, 0, ctx, HD, HD, N);
    __syncthreads();
    h_gemm<256, 128, false>(A, ca.wkv, HD, ws.kv(i) + 256, 512, N);   // the context token
    __syncthreads();
    // attention: one thread per (frame, head); 1 query x 2 keys
    {
      const int n = tid >> 2, h = tid & 3;
      if (n < N) {
        const float *q = ws.q(i) + n * HD + h * 32, *k0 = ws.kv(i) + n * 512 + h * 32, *k1 = k0 + 256;
        float d0 = 0.f, d1 = 0.f;
#pragma unroll 8
        for (int d = 0; d < 32; ++d) { d0 = fmaf(q[d], k0[d], d0); d1 = fmaf(q[d], k1[d], d1); }
        d0 *= scale; d1 *= scale;
        const float m = fmaxf(d0, d1);
        const float e0 = __expf(d0 - m), e1 = __expf(d1 - m);
        const float inv = 1.f / (e0 + e1);
        const float a0 = e0 * inv, a1 = e1 * inv;
        ws.at(i)[n * 8 + h * 2] = a0; ws.at(i)[n * 8 + h * 2 + 1] = a1;
        const float *v0 = k0 + 128, *v1 = k1 + 128;
        float *o = ws.o(i) + n * HD + h * 32;
#pragma unroll 8
        for (int d = 0; d < 32; ++d) {
          const float v = a0 * v0[d] + a1 * v1[d];
          o[d] = v;
          A[n * HKP + h * 32 + d] = f2bf(v);
        }
      } else {
        for (int d = 0; d < 32; ++d) A[n * HKP + h * 32 + d] = 0;
      }
    }
    __syncthreads();
    // to_out + bias, dropout, residual (dama.py:50-53, 71-76): the output projection into the
    // red-free tail of the workspace row, then x_new = x + drop(out)
    float *xnew = ws.st(h_xout(i));
    h_gemm<128, 128, false>(A, ca.wo, HD, xnew, HD, N);
    __syncthreads();
    for (int e = tid; e < N * HD; e += 256) {
      const int n = e >> 7, c = e & 127;
      xnew[e] = x[e] + (xnew[e] + ca.bo[c]) * h_drop(p, i, n, c, p.p_ca);
    }
    __syncthreads();
  }
  // concat = [s2, f2] (dama.py:151) as the A operand of the fusion conv and the gate
  const float *s2 = ws.st(4), *f2 = ws.st(5);
  h_stage(A, 0, s2, HD, HD, N);
  h_stage(A, HD, f2, HD, HD, N);
  __syncthreads();
  // fusion_gate centre tap: W_c[o][i] = wfg[o * fg_so + i * fg_si + 4 * fg_tap]
  {
    // the 256 x 128 centre-tap matrix is strided: stage it in the transposed form h_gemm reads
    // (TRANS: B(k, col) = W[k * ldw + col])
    float *wc = ws.wc();                          // [256][128]
    for (int e = tid; e < 256 * HD; e += 256) {
      const int k = e >> 7, o = e & 127;
      wc[e] = p.wfg[(int64_t)o * p.fg_so + (int64_t)k * p.fg_si + 4 * p.fg_tap];
    }
    __syncthreads();
    h_gemm<128, 256, true>(A, wc, HD, ws.yfg(), HD, N);
  }
  h_gemm<64, 256, false>(A, p.g1w, 256, ws.h1(), 64, N);
  __syncthreads();
  // BatchNorm over the frames (training: batch statistics, running-stat update; eval: running)
  if (tid < HD) {
    const int c = tid;
    float m, iv;
    if (p.training) {
      float s = 0.f;
      for (int n = 0; n < N; ++n) s += ws.yfg()[n * HD + c] + p.bfg[c];
      m = s / (float)N;
      float q = 0.f;
      for (int n = 0; n < N; ++n) { const float d = ws.yfg()[n * HD + c] + p.bfg[c] - m; q = fmaf(d, d, q); }
      const float var = q / (float)N;
      iv = rsqrtf(var + p.bn_eps);
      const float unb = N > 1 ? q / (float)(N - 1) : var;
      p.bn_rm[c] = (1.f - p.bn_mom) * p.bn_rm[c] + p.bn_mom * m;
      p.bn_rv[c] = (1.f - p.bn_mom) * p.bn_rv[c] + p.bn_mom * unb;
    } else {
      m = p.bn_rm[c];
      iv = rsqrtf(p.bn_rv[c] + p.bn_eps);
    }
    ws.bnm()[c] = m; ws.bni()[c] = iv;
  }
  if (tid == 0 && p.training && p.bn_nbt) p.bn_nbt[0] += 1;
  __syncthreads();
  for (int e = tid; e < N * HD; e += 256) {
    const int c = e & 127;
    const float z = (ws.yfg()[e] + p.bfg[c] - ws.bnm()[c]) * ws.bni()[c] * p.bn_w[c] + p.bn_b[c];
    ws.fus()[e] = z > 0.f ? z : 0.f;
  }
  // gate_net second layer + softmax (dama.py:105-113): one thread per frame
  if (tid < N) {
    const int n = tid;
    float z[3] = {p.g2b[0], p.g2b[1], p.g2b[2]};
    for (int j = 0; j < 64; ++j) {
      const float h = ws.h1()[n * 64 + j] + p.g1b[j];
      const float hd = (h > 0.f ? h : 0.f) * h_drop(p, 4, n, j, p.p_gate);
#pragma unroll
      for (int o = 0; o < 3; ++o) z[o] = fmaf(hd, p.g2w[o * 64 + j], z[o]);
    }
    const float m = fmaxf(z[0], fmaxf(z[1], z[2]));
    const float e0 = __expf(z[0] - m), e1 = __expf(z[1] - m), e2 = __expf(z[2] - m);
    const float inv = 1.f / (e0 + e1 + e2);
    ws.gw()[n * 4] = e0 * inv; ws.gw()[n * 4 + 1] = e1 * inv; ws.gw()[n * 4 + 2] = e2 * inv;
  }
  __syncthreads();
  for (int e = tid; e < N * HD; e += 256) {
    const int n = e >> 7;
    const float *g = ws.gw() + n * 4;
    fused_out[e] = g[0] * s2[e] + g[1] * f2[e] + g[2] * ws.fus()[e];
    s_out[e] = s2[e];
    f_out[e] = f2[e];
  }
  (void)red;
}

// ---------------------------------------------------------------- backward, activations
// LayerNorm backward of block i's pre-norm into dx (+=): dxh = dxn * gamma,
// dx = rs * (dxh - mean(dxh) - xhat * mean(dxh * xhat))
__device__ void h_ln_bwd(const HeadCA &ca, const HeadWs &ws, int i, const float *x, float *dx, int N) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int n = w; n < N; n += 4) {
    const float m = ws.mu(i)[n], r = ws.rs(i)[n];
    float xh[2], g[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int c = lane + 64 * t;
      xh[t] = (x[n * HD + c] - m) * r;
      g[t] = ws.dxn(i)[n * HD + c] * ca.ln_w[c];
    }
    const float a = wave_sum(g[0] + g[1]) * (1.f / HD);
    const float b = wave_sum(g[0] * xh[0] + g[1] * xh[1]) * (1.f / HD);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int c = lane + 64 * t;
      dx[n * HD + c] += r * (g[t] - a - xh[t] * b);
    }
  }
}

__global__ __launch_bounds__(256) void head_bwd_data_kernel(HeadParams p, float *ws_base, const float *g_fused,
                                                            const float *g_s, const float *g_f, float *ds0,
                                                            float *df0, float *dbn_w, float *dbn_b, int N) {
  bf16_t *A = reinterpret_cast<bf16_t *>(h_smem);
  HeadWs ws = head_ws(ws_base);
  const int tid = threadIdx.x;
  const float scale = 0.17677669529663687f;
  const float *s2 = ws.st(4), *f2 = ws.st(5);
  float *dS = ws.ds(0), *dF = ws.ds(1);
  // weighted sum and the gate (dama.py:156-163)
  for (int e = tid; e < N * HD; e += 256) {
    const int n = e >> 7;
    const float *g = ws.gw() + n * 4;
    const float gf = g_fused[e];
    dS[e] = g_s[e] + g[0] * gf;
    dF[e] = g_f[e] + g[1] * gf;
  }
  if (tid < N) {
    const int n = tid;
    float dg[3] = {0.f, 0.f, 0.f};
    for (int c = 0; c < HD; ++c) {
      const float gf = g_fused[n * HD + c];
      dg[0] = fmaf(gf, s2[n * HD + c], dg[0]);
      dg[1] = fmaf(gf, f2[n * HD + c], dg[1]);
      dg[2] = fmaf(gf, ws.fus()[n * HD + c], dg[2]);
    }
    const float *g = ws.gw() + n * 4;
    const float dot = g[0] * dg[0] + g[1] * dg[1] + g[2] * dg[2];
#pragma unroll
    for (int o = 0; o < 3; ++o) ws.dz2()[n * 4 + o] = g[o] * (dg[o] - dot);
    ws.dz2()[n * 4 + 3] = 0.f;
  }
  __syncthreads();
  // gate_net: d h1 (pre-activation) = (dz2 W2) * drop * relu'
  for (int e = tid; e < N * 64; e += 256) {
    const int n = e >> 6, j = e & 63;
    const float h = ws.h1()[e] + p.g1b[j];
    float d = 0.f;
#pragma unroll
    for (int o = 0; o < 3; ++o) d = fmaf(ws.dz2()[n * 4 + o], p.g2w[o * 64 + j], d);
    ws.dh1()[e] = h > 0.f ? d * h_drop(p, 4, n, j, p.p_gate) : 0.f;
  }
  // fusion BatchNorm + ReLU backward (batch statistics over the frames)
  if (tid < HD) {
    const int c = tid;
    const float m = ws.bnm()[c], iv = ws.bni()[c], gam = p.bn_w[c];
    float sg = 0.f, sgx = 0.f;
    for (int n = 0; n < N; ++n) {
      const float gr = ws.fus()[n * HD + c] > 0.f ? g_fused[n * HD + c] * ws.gw()[n * 4 + 2] : 0.f;
      const float xh = (ws.yfg()[n * HD + c] + p.bfg[c] - m) * iv;
      sg += gr;
      sgx = fmaf(gr, xh, sgx);
    }
    if (dbn_w) dbn_w[c] = sgx;
    if (dbn_b) dbn_b[c] = sg;
    const float a = sg / (float)N, b = sgx / (float)N;
    for (int n = 0; n < N; ++n) {
      const float gr = ws.fus()[n * HD + c] > 0.f ? g_fused[n * HD + c] * ws.gw()[n * 4 + 2] : 0.f;
      const float xh = (ws.yfg()[n * HD + c] + p.bfg[c] - m) * iv;
      ws.dy()[n * HD + c] = p.training ? gam * iv * (gr - a - xh * b) : gam * iv * gr;
    }
  }
  __syncthreads();
  // d concat = dy Wc + dh1 W1: two GEMMs into dcat (the second adds)
  h_stage(A, 0, ws.dy(), HD, HD, N);
  __syncthreads();
  {
    float *wc = ws.wc();                   // centre tap [128][256] (o, i)
    for (int e = tid; e < HD * 256; e += 256) {
      const int o = e >> 8, k = e & 255;
      wc[e] = p.wfg[(int64_t)o * p.fg_so + (int64_t)k * p.fg_si + 4 * p.fg_tap];
    }
    __syncthreads();
    h_gemm<256, 128, true>(A, wc, 256, ws.dcat(), 256, N);
  }
  __syncthreads();
  h_stage(A, 0, ws.dh1(), 64, 64, N);
  __syncthreads();
  {
    float *t = ws.tmp();                   // dh1 W1 [N][256]
    h_gemm<256, 64, true>(A, p.g1w, 256, t, 256, N);
    __syncthreads();
    for (int e = tid; e < N * 256; e += 256) ws.dcat()[e] += t[e];
  }
  __syncthreads();
  for (int e = tid; e < N * HD; e += 256) {
    const int n = e >> 7, c = e & 127;
    dS[e] += ws.dcat()[n * 256 + c];
    dF[e] += ws.dcat()[n * 256 + HD + c];
  }
  __syncthreads();
  // the attention blocks in reverse (3: layer 1 f, 2: layer 1 s, 1: layer 0 f, 0: layer 0 s)
  for (int i = 3; i >= 0; --i) {
    const HeadCA &ca = p.ca[i];
    float *dX = (i & 1) ? dF : dS;        // the block's own stream: grad of x_new, becomes grad of x
    float *dC = (i & 1) ? dS : dF;        // the context stream
    const float *x = ws.st(h_xin(i));
    // to_out backward: dpre = dX * drop; d o = dpre Wo
    for (int e = tid; e < N * HD; e += 256) {
      const int n = e >> 7, c = e & 127;
      const float d = dX[e] * h_drop(p, i, n, c, p.p_ca);
      ws.dpre(i)[e] = d;
      A[n * HKP + c] = f2bf(d);
    }
    for (int e = N * HD + tid; e < HN * HD; e += 256) A[(e >> 7) * HKP + (e & 127)] = 0;
    __syncthreads();
    float *dO = ws.dxn(i);                // scratch: d o, then overwritten by d xn below
    h_gemm<128, 128, true>(A, ca.wo, HD, dO, HD, N);
    __syncthreads();
    // attention backward, one thread per (frame, head)
    {
      const int n = tid >> 2, h = tid & 3;
      if (n < N) {
        const float *q = ws.q(i) + n * HD + h * 32, *k0 = ws.kv(i) + n * 512 + h * 32, *k1 = k0 + 256;
        const float *v0 = k0 + 128, *v1 = k1 + 128, *dout = dO + n * HD + h * 32;
        const float a0 = ws.at(i)[n * 8 + h * 2], a1 = ws.at(i)[n * 8 + h * 2 + 1];
        float da0 = 0.f, da1 = 0.f;
#pragma unroll 8
        for (int d = 0; d < 32; ++d) { da0 = fmaf(dout[d], v0[d], da0); da1 = fmaf(dout[d], v1[d], da1); }
        const float dot = a0 * da0 + a1 * da1;
        const float dl0 = a0 * (da0 - dot) * scale, dl1 = a1 * (da1 - dot) * scale;
        float *dq = ws.dq(i) + n * HD + h * 32, *dk0 = ws.dkv(i) + n * 512 + h * 32, *dk1 = dk0 + 256;
#pragma unroll 8
        for (int d = 0; d < 32; ++d) {
          dq[d] = dl0 * k0[d] + dl1 * k1[d];
          dk0[d] = dl0 * q[d];
          dk1[d] = dl1 * q[d];
          dk0[128 + d] = a0 * dout[d];
          dk1[128 + d] = a1 * dout[d];
        }
      }
    }
    __syncthreads();
    // d xn = dq Wq + dkv_self Wkv;  d ctx += dkv_ctx Wkv
    h_stage(A, 0, ws.dq(i), HD, HD, N);
    __syncthreads();
    float *dxn = ws.dxn(i);
    h_gemm<128, 128, true>(A, ca.wq, HD, dxn, HD, N);
    __syncthreads();
    h_stage(A, 0, ws.dkv(i), 512, 256, N);
    __syncthreads();
    float *t = ws.tmp();
    h_gemm<128, 256, true>(A, ca.wkv, HD, t, HD, N);
    __syncthreads();
    for (int e = tid; e < N * HD; e += 256) dxn[e] += t[e];
    h_stage(A, 0, ws.dkv(i) + 256, 512, 256, N);
    __syncthreads();
    h_gemm<128, 256, true>(A, ca.wkv, HD, t, HD, N);
    __syncthreads();
    for (int e = tid; e < N * HD; e += 256) dC[e] += t[e];
    // LayerNorm backward into the own stream (which already holds the residual's gradient)
    h_ln_bwd(ca, ws, i, x, dX, N);
    __syncthreads();
  }
  for (int e = tid; e < N * HD; e += 256) { ds0[e] = dS[e]; df0[e] = dF[e]; }
}

// ---------------------------------------------------------------- backward, weights
// One thread per output element: dW[o][k] = sum_rows D[row][o] X[row][k] (fp32, fixed row
// order), db[o] = sum_rows D[row][o].  Jobs, in grid order:
//   per attention block i: Wq [128][128], Wkv [256][128] (rows: both tokens), Wo [128][128],
//     bo [128], LayerNorm gamma / beta [128];
//   fusion conv [128][256][3][3] (the 8 non-centre taps: 0), its bias; gate W1 [64][256], b1,
//   W2 [3][64], b2.
struct HeadGrads {
  float *wq[4], *wkv[4], *wo[4], *bo[4], *lnw[4], *lnb[4];
  float *wfg; int64_t fg_so, fg_si, fg_tap;
  float *bfg, *g1w, *g1b, *g2w, *g2b;
};

__global__ __launch_bounds__(256) void head_bwd_weight_kernel(HeadParams p, const float *ws_base, HeadGrads g, int N) {
  HeadWs ws = head_ws(const_cast<float *>(ws_base));
  int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (int i = 0; i < 4; ++i) {
    if (t < HD * HD) {                                   // Wq: dq^T xn
      const int o = (int)(t >> 7), k = (int)(t & 127);
      float s = 0.f;
      for (int n = 0; n < N; ++n) s = fmaf(ws.dq(i)[n * HD + o], ws.xn(i)[n * HD + k], s);
      g.wq[i][t] = s;
      return;
    }
    t -= HD * HD;
    if (t < 256 * HD) {                                  // Wkv: sum over both tokens
      const int o = (int)(t >> 7), k = (int)(t & 127);
      const float *ctx = ws.st(h_cin(i));
      float s = 0.f;
      for (int n = 0; n < N; ++n) {
        s = fmaf(ws.dkv(i)[n * 512 + o], ws.xn(i)[n * HD + k], s);
        s = fmaf(ws.dkv(i)[n * 512 + 256 + o], ctx[n * HD + k], s);
      }
      g.wkv[i][t] = s;
      return;
    }
    t -= 256 * HD;
    if (t < HD * HD) {                                   // Wo: dpre^T o
      const int o = (int)(t >> 7), k = (int)(t & 127);
      float s = 0.f;
      for (int n = 0; n < N; ++n) s = fmaf(ws.dpre(i)[n * HD + o], ws.o(i)[n * HD + k], s);
      g.wo[i][t] = s;
      return;
    }
    t -= HD * HD;
    if (t < 3 * HD) {                                    // bo, LayerNorm gamma, beta
      const int which = (int)(t >> 7), c = (int)(t & 127);
      float s = 0.f;
      if (which == 0) {
        for (int n = 0; n < N; ++n) s += ws.dpre(i)[n * HD + c];
        g.bo[i][c] = s;
      } else {
        const float *x = ws.st(h_xin(i));
        for (int n = 0; n < N; ++n) {
          const float d = ws.dxn(i)[n * HD + c];
          s = which == 1 ? fmaf(d, (x[n * HD + c] - ws.mu(i)[n]) * ws.rs(i)[n], s) : s + d;
        }
        (which == 1 ? g.lnw[i] : g.lnb[i])[c] = s;
      }
      return;
    }
    t -= 3 * HD;
  }
  if (t < HD * 256 * 9) {                                // fusion conv: centre tap = dy^T concat
    const int o = (int)(t / (256 * 9)), r = (int)(t - (int64_t)o * 256 * 9), k = r / 9, tap = r - k * 9;
    float s = 0.f;
    if (tap == 4) {
      const float *src = k < HD ? ws.st(4) + k : ws.st(5) + (k - HD);
      for (int n = 0; n < N; ++n) s = fmaf(ws.dy()[n * HD + o], src[n * HD], s);
    }
    g.wfg[(int64_t)o * g.fg_so + (int64_t)k * g.fg_si + tap * g.fg_tap] = s;
    return;
  }
  t -= HD * 256 * 9;
  if (t < HD) {
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += ws.dy()[n * HD + t];
    g.bfg[t] = s;
    return;
  }
  t -= HD;
  if (t < 64 * 256) {                                    // gate W1: dh1^T concat
    const int o = (int)(t >> 8), k = (int)(t & 255);
    const float *src = k < HD ? ws.st(4) + k : ws.st(5) + (k - HD);
    float s = 0.f;
    for (int n = 0; n < N; ++n) s = fmaf(ws.dh1()[n * 64 + o], src[n * HD], s);
    g.g1w[t] = s;
    return;
  }
  t -= 64 * 256;
  if (t < 64) {
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += ws.dh1()[n * 64 + t];
    g.g1b[t] = s;
    return;
  }
  t -= 64;
  if (t < 3 * 64) {                                      // gate W2: dz2^T dropout(relu(h1))
    const int o = (int)(t >> 6), j = (int)(t & 63);
    float s = 0.f;
    for (int n = 0; n < N; ++n) {
      const float h = ws.h1()[n * 64 + j] + p.g1b[j];
      const float hd = (h > 0.f ? h : 0.f) * h_drop(p, 4, n, j, p.p_gate);
      s = fmaf(ws.dz2()[n * 4 + o], hd, s);
    }
    g.g2w[t] = s;
    return;
  }
  t -= 3 * 64;
  if (t < 3) {
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += ws.dz2()[n * 4 + t];
    g.g2b[t] = s;
  }
}

constexpr int64_t head_wgrad_threads() {
  return 4 * (HD * HD + 256 * HD + HD * HD + 3 * HD) + HD * 256 * 9 + HD + 64 * 256 + 64 + 3 * 64 + 3;
}

}  // namespace ewvit

using namespace ewvit;

static int head_check(const HeadParams &p, int N, const char *nm) {
  EWVIT_CHECK_ARG(N >= 1 && N <= HN, "%s: %d frames per chunk (1..%d)", nm, N, HN);
  for (int i = 0; i < 4; ++i)
    EWVIT_CHECK_ARG(p.ca[i].ln_w && p.ca[i].ln_b && p.ca[i].wq && p.ca[i].wkv && p.ca[i].wo && p.ca[i].bo,
                    "%s: attention block %d: null parameter", nm, i);
  EWVIT_CHECK_ARG(p.wfg && p.bfg && p.bn_w && p.bn_b && p.bn_rm && p.bn_rv && p.g1w && p.g1b && p.g2w && p.g2b,
                  "%s: null parameter", nm);
  EWVIT_CHECK_ARG(p.p_ca >= 0.f && p.p_ca < 1.f && p.p_gate >= 0.f && p.p_gate < 1.f, "%s: dropout", nm);
  return 0;
}

static size_t head_lds() { return (size_t)HN * HKP * 2 + 4 * 256 * sizeof(float); }

extern "C" int64_t ewvit_head_workspace(void) { return head_ws_floats() * (int64_t)sizeof(float); }

extern "C" int ewvit_head_fwd(const HeadParams *params, const float *s0, const float *f0, int N, float *workspace,
                              float *fused, float *s_out, float *f_out, void *stream) {
  EWVIT_CHECK_ARG(params && s0 && f0 && workspace && fused && s_out && f_out, "head_fwd: null pointer");
  if (int rc = head_check(*params, N, "head_fwd")) return rc;
  hipLaunchKernelGGL(head_fwd_kernel, dim3(1), dim3(256), head_lds(), as_stream(stream), *params, s0, f0, workspace,
                     fused, s_out, f_out, N);
  return launch_status("head_fwd");
}

extern "C" int ewvit_head_bwd(const HeadParams *params, const float *workspace, int N, const float *g_fused,
                              const float *g_s, const float *g_f, float *ds0, float *df0, float *const *wq,
                              float *const *wkv, float *const *wo, float *const *bo, float *const *lnw,
                              float *const *lnb, float *wfg, int64_t fg_so, int64_t fg_si, int64_t fg_tap, float *bfg,
                              float *bn_w, float *bn_b, float *g1w, float *g1b, float *g2w, float *g2b, void *stream) {
  EWVIT_CHECK_ARG(params && workspace && g_fused && g_s && g_f && ds0 && df0 && wq && wkv && wo && bo && lnw && lnb &&
                      wfg && bfg && bn_w && bn_b && g1w && g1b && g2w && g2b,
                  "head_bwd: null pointer");
  if (int rc = head_check(*params, N, "head_bwd")) return rc;
  HeadGrads g;
  for (int i = 0; i < 4; ++i) {
    EWVIT_CHECK_ARG(wq[i] && wkv[i] && wo[i] && bo[i] && lnw[i] && lnb[i], "head_bwd: block %d: null gradient", i);
    g.wq[i] = wq[i]; g.wkv[i] = wkv[i]; g.wo[i] = wo[i]; g.bo[i] = bo[i]; g.lnw[i] = lnw[i]; g.lnb[i] = lnb[i];
  }
  g.wfg = wfg; g.fg_so = fg_so; g.fg_si = fg_si; g.fg_tap = fg_tap;
  g.bfg = bfg; g.g1w = g1w; g.g1b = g1b; g.g2w = g2w; g.g2b = g2b;
  hipStream_t s = as_stream(stream);
  float *ws = const_cast<float *>(workspace);
  hipLaunchKernelGGL(head_bwd_data_kernel, dim3(1), dim3(256), head_lds(), s, *params, ws, g_fused, g_s, g_f, ds0,
                     df0, bn_w, bn_b, N);
  if (int rc = launch_status("head_bwd data")) return rc;
  const int64_t nt = head_wgrad_threads();
  hipLaunchKernelGGL(head_bwd_weight_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, *params, workspace, g,
                     N);
  return launch_status("head_bwd weight");
}
