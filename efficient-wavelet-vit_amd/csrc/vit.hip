// One pre-norm ViT encoder layer of the spatial branch (gfx950), forward and backward —
// reference network/sfe.py:72-85 (Transformer), 20-27 (PreNorm), 42-70 (Attention), 29-40
// (FeedForward):
//   x1 = x0 + Dropout(to_out(Attention(LN1(x0))))
//   x2 = x1 + W2 GELU(W1 LN2(x1) + b1) + b2
// at the hot path's shape: dim 512, 8 heads of 64, mlp 2048, 2 tokens per frame (CLS + the
// single 7x7 patch), R = 2 x frames <= 128 rows, row 2b + i = token i of frame b.
//
// The module path issues 11 forward launches per layer (LayerNorm, to_qkv + split-K reduce,
// attention, to_out + reduce, LayerNorm, Linear1 + reduce, Linear2 + reduce) and ~25 backward.
// Every GEMM here is [128 rows] x [<= 2048] x [<= 2048] against fp32 master weights: a few
// MFLOP and a few MB of weight reads, so each launch is latency: the fusion below cuts the
// launches, not the bytes.
//   forward   F1 vit_ln_gemm_kernel<0>   LN1 (statistics per workgroup, its 64 rows) + to_qkv;
//                                        LN1 output written transposed for the weight gradient
//             F2 vit_attn_proj_kernel     softmax of the 2x2 scores per (frame, head) + to_out
//                                        with the attention output formed in the A fragments,
//                                        bias, dropout, residual
//             F3 vit_ln_gemm_kernel<1>   LN2 + Linear1 + bias + GELU (pre-activation kept)
//             F4 ewvit_gemm (split-K)     Linear2 + bias + residual (K = 2048 split over 256
//                                        workgroups; a column-block kernel reading all of h
//                                        per workgroup ran 32 us)
//   backward  B1 vit_mlp2_bwd_kernel      dh = g W2 (rounded like the module path's bf16 dh),
//                                        g1 = dh GELU'(pre), db1; g transposed, db2
//             B2 vit_mlp1_bwd_kernel      dLN2 = g1 W1 | dW2 = g^T h | dW1 = g1^T LN2
//             B3 vit_ln2_bwd_attn_kernel  LN2 backward + residual (dx1), to_out's dropout,
//                                        d(attention out) = g_o Wo per head, attention
//                                        backward | dx1, g_o transposed, dbo, dLN2 affine
//             B4 vit_qkv_bwd_kernel       dLN1 = dqkv Wqkv | dWqkv = dqkv^T LN1 | dWo = g_o^T o
//             B5 vit_ln1_bwd_kernel       LN1 backward + residual (dx0), dLN1 affine
// GEMM fragments: v_mfma_f32_16x16x32_bf16, bf16 operands rounded from the fp32 masters /
// activations exactly where the module path's ewvit_gemm rounds them, fp32 accumulation.
// Weight gradients reduce over the rows (K = rows): their operands are the activations /
// gradients stored transposed ([feature][128 rows] bf16, zero past R), written by the kernel
// that produces them (the MFMA output layout gives a lane 4 consecutive rows of one column).
// Forward / input-gradient GEMMs read their A fragments straight from global memory (L2) and
// their B fragments from the fp32 weights (forward) or from an LDS image of the weight slice
// transposed to k-contiguous bf16 (input gradients reduce over the weight's output index).
#include "common.h"
#include "mx8.h"

namespace ewvit {

constexpr int VD = 512, VQ = 1536, VF = 2048, VH = 8, VDH = 64, VRP = 128;
constexpr float VSCALE = 0.125f;   // dim_head^-0.5 (sfe.py:50)
constexpr int VF4_SPLIT = 16;      // K splits of Linear2 (ewvit_gemm, K = 2048: 16 x 128)

typedef ewvit_vit_layer VitP;
typedef ewvit_vit_grads VitG;
typedef __attribute__((ext_vector_type(8))) __bf16 vb8;
typedef __attribute__((ext_vector_type(4))) float vf4;

__device__ __forceinline__ vf4 mma(vb8 a, vb8 b, vf4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ vb8 pack8(const float *v) {
  vb8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (__bf16)v[e];
  return r;
}
__device__ __forceinline__ void ld8f(const float *p, float *v) {
  const float4 a = *reinterpret_cast<const float4 *>(p), b = *reinterpret_cast<const float4 *>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ vb8 ld8b(const bf16_t *p) { return *reinterpret_cast<const vb8 *>(p); }
__device__ __forceinline__ void unpack8(vb8 b, float *v) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (float)b[e];
}
__device__ __forceinline__ vb8 zero8() {
  vb8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (__bf16)0.f;
  return r;
}
__device__ __forceinline__ float rbf(float v) { return bf2f(f2bf(v)); }
// rows >= R are loaded from row R - 1 (in bounds) and masked after the load: a load under a
// per-lane branch gets its own block and waits, so the epilogues' loads would run one by one
__device__ __forceinline__ int rclamp(int r, int R) { return r < R ? r : R - 1; }
__device__ __forceinline__ float keep_scale(float p, uint64_t sd, uint64_t idx) {
  return uniform01(sd, idx) >= p ? 1.0f / (1.0f - p) : 0.f;
}

// ---------------------------------------------------------------- saved state / scratch
struct VitSaved {
  float *mu1, *rs1, *mu2, *rs2, *p, *x1;
  bf16_t *qkv, *aux, *h, *ln1T, *oT, *ln2T, *hT;
  float *ws2;                       // Linear2's split-K slabs (forward only)
};
struct VitScratch {
  bf16_t *gT, *g1, *g1T, *goT, *dqkv, *dqkvT;
  float *dln2, *dx1, *dln1;
  float *rp2, *rp1;                 // LN backward row partials [32 column blocks][128 rows][2]
  float *db1p;                      // Linear1 bias gradient per row half [2][2048]
};
// The layer's four weights in bf16, packed once per step by ewvit_vit_pack (fp32 masters read
// once): each as W [out][in] (forward B fragments, k = in contiguous) and W^T [in][out] (input
// gradient B fragments, k = out contiguous).  Element offsets within a layer's block:
constexpr int64_t PK_QKV = 0, PK_QKVT = PK_QKV + (int64_t)VQ * VD, PK_O = PK_QKVT + (int64_t)VQ * VD,
                  PK_OT = PK_O + (int64_t)VD * VD, PK_1 = PK_OT + (int64_t)VD * VD, PK_1T = PK_1 + (int64_t)VF * VD,
                  PK_2 = PK_1T + (int64_t)VF * VD, PK_2T = PK_2 + (int64_t)VF * VD, PK_LAYER = PK_2T + (int64_t)VF * VD;
__host__ __device__ inline int64_t al256(int64_t b) { return (b + 255) / 256 * 256; }
// MXFP8 pack (ewvit_vit_pack_mx, configs[4]): the same eight operand images as e4m3 bytes, each
// row followed (in a separate array) by its E8M0 scales, one per 32 consecutive elements along
// the row (the GEMM's K): W [out][in] + S [out][in / 32], W^T [in][out] + S^T [in][out / 32].
// Byte offsets within a layer's block, image m = 0..7 (qkv, qkvT, o, oT, 1, 1T, 2, 2T):
struct MxW {
  const uint8_t *d, *s;
  int K;
  __device__ __forceinline__ const uint8_t *row(int r) const { return d + (int64_t)r * K; }
  __device__ __forceinline__ const uint8_t *srow(int r) const { return s + (int64_t)r * (K / 32); }
};
__host__ __device__ inline void mx_dims(int m, int &rows, int &cols) {
  const int R[8] = {VQ, VD, VD, VD, VF, VD, VD, VF}, C[8] = {VD, VQ, VD, VD, VD, VF, VF, VD};
  rows = R[m];
  cols = C[m];
}
__host__ __device__ inline int64_t mx_off(int m) {     // data at mx_off(m), scales right after
  int64_t o = 0;
  for (int i = 0; i < m; ++i) {
    int r, c;
    mx_dims(i, r, c);
    o += al256((int64_t)r * c) + al256((int64_t)r * (c / 32));
  }
  return o;
}
__device__ __forceinline__ MxW mx_image(const void *packed, int m) {
  int r, c;
  mx_dims(m, r, c);
  const uint8_t *b = reinterpret_cast<const uint8_t *>(packed) + mx_off(m);
  return MxW{b, b + al256((int64_t)r * c), c};
}
template <class F> __host__ __device__ inline int64_t saved_layout(F f) {
  int64_t o = 0;
  auto put = [&](int idx, int64_t bytes) { f(idx, o); o += al256(bytes); };
  put(0, 4 * VRP); put(1, 4 * VRP); put(2, 4 * VRP); put(3, 4 * VRP);
  put(4, 4 * VRP * VH * 2); put(5, 4 * VRP * VD);
  put(6, 2 * VRP * VQ); put(7, 2 * VRP * VF); put(8, 2 * VRP * VF);
  put(9, 2 * VD * VRP); put(10, 2 * VD * VRP); put(11, 2 * VD * VRP); put(12, 2 * VF * VRP);
  put(13, 4 * VF4_SPLIT * VRP * VD);
  return o;
}
template <class F> __host__ __device__ inline int64_t scratch_layout(F f) {
  int64_t o = 0;
  auto put = [&](int idx, int64_t bytes) { f(idx, o); o += al256(bytes); };
  put(0, 2 * VD * VRP); put(1, 2 * VRP * VF); put(2, 2 * VF * VRP); put(3, 2 * VD * VRP);
  put(4, 2 * VRP * VQ); put(5, 2 * VQ * VRP);
  put(6, 4 * VRP * VD); put(7, 4 * VRP * VD); put(8, 4 * VRP * VD);
  put(9, 4 * 32 * VRP * 2); put(10, 4 * 32 * VRP * 2); put(11, 4 * 2 * VF);
  return o;
}
inline VitSaved vit_saved(void *base) {
  VitSaved s;
  char *b = reinterpret_cast<char *>(base);
  saved_layout([&](int i, int64_t o) {
    void *q = b + o;
    switch (i) {
      case 0: s.mu1 = (float *)q; break;
      case 1: s.rs1 = (float *)q; break;
      case 2: s.mu2 = (float *)q; break;
      case 3: s.rs2 = (float *)q; break;
      case 4: s.p = (float *)q; break;
      case 5: s.x1 = (float *)q; break;
      case 6: s.qkv = (bf16_t *)q; break;
      case 7: s.aux = (bf16_t *)q; break;
      case 8: s.h = (bf16_t *)q; break;
      case 9: s.ln1T = (bf16_t *)q; break;
      case 10: s.oT = (bf16_t *)q; break;
      case 11: s.ln2T = (bf16_t *)q; break;
      case 12: s.hT = (bf16_t *)q; break;
      default: s.ws2 = (float *)q; break;
    }
  });
  return s;
}
inline VitScratch vit_scratch(void *base) {
  VitScratch s;
  char *b = reinterpret_cast<char *>(base);
  scratch_layout([&](int i, int64_t o) {
    void *q = b + o;
    switch (i) {
      case 0: s.gT = (bf16_t *)q; break;
      case 1: s.g1 = (bf16_t *)q; break;
      case 2: s.g1T = (bf16_t *)q; break;
      case 3: s.goT = (bf16_t *)q; break;
      case 4: s.dqkv = (bf16_t *)q; break;
      case 5: s.dqkvT = (bf16_t *)q; break;
      case 6: s.dln2 = (float *)q; break;
      case 7: s.dx1 = (float *)q; break;
      case 8: s.dln1 = (float *)q; break;
      case 9: s.rp2 = (float *)q; break;
      case 10: s.rp1 = (float *)q; break;
      default: s.db1p = (float *)q; break;
    }
  });
  return s;
}

// ---------------------------------------------------------------- shared pieces
// LayerNorm statistics of rows w, w + nw, ... (< 128; rows >= R get 0 / 0): a wave per row,
// 8 contiguous columns per lane; two-pass mean / centred variance, biased, eps inside the
// rsqrt (torch's formula, layernorm.hip's)
template <int NW, int NROWS = VRP>
__device__ __forceinline__ void ln_stats_rows(const float *x, int R, float eps, float *smu, float *srs, int w,
                                              int lane, int r0 = 0) {
  constexpr int NR = NROWS / NW;        // rows of this wave: r0 + w, r0 + w + NW, ... (all loads in flight)
  float v[NR][8];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int r = r0 + w + i * NW;
    ld8f(x + (int64_t)rclamp(r, R) * VD + lane * 8, v[i]);
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int r = r0 + w + i * NW;
    float mu = 0.f, rs = 0.f;
    if (r < R) {
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[i][e];
      mu = wave_sum(s) / (float)VD;
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) q += (v[i][e] - mu) * (v[i][e] - mu);
      rs = rsqrtf(wave_sum(q) / (float)VD + eps);
    }
    if (lane == 0) { smu[r] = mu; srs[r] = rs; }
  }
}

// A 64 x 64 block of a weight gradient out[r][c] = sum_k AT[r][k] BT[c][k] over the 128 rows
// k (zero past R in both operands); wave w of 4 takes the 32 x 32 quadrant (w >> 1, w & 1)
// MX: both operands block-quantized along the 128 rows in registers (4 blocks of 32 rows)
template <bool MX>
__device__ __forceinline__ void wgrad_block(const bf16_t *AT, const bf16_t *BT, float *out, int64_t ldo, int r0,
                                            int c0, int w, int lane) {
  const int li = lane & 15, lq = lane >> 4;
  const int rb = r0 + (w >> 1) * 32, cb = c0 + (w & 1) * 32;
  if constexpr (MX) {
    MxFrag fa[2], fb[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float va[32], vb[32];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int k = (hh ? mx_k1(lane) : mx_k0(lane)) + 8 * q;
          unpack8(ld8b(AT + (int64_t)(rb + t * 16 + li) * VRP + k), va + hh * 16 + q * 8);
          unpack8(ld8b(BT + (int64_t)(cb + t * 16 + li) * VRP + k), vb + hh * 16 + q * 8);
        }
      fa[t] = mx_quant(va);
      fb[t] = mx_quant(vb);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const vf4 acc = mx_mma(fa[i], fb[j], vf4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int e = 0; e < 4; ++e) out[(int64_t)(rb + i * 16 + lq * 4 + e) * ldo + cb + j * 16 + li] = acc[e];
      }
    return;
  }
  vb8 a[4][2], b[4][2];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      a[s][t] = ld8b(AT + (int64_t)(rb + t * 16 + li) * VRP + s * 32 + lq * 8);
      b[s][t] = ld8b(BT + (int64_t)(cb + t * 16 + li) * VRP + s * 32 + lq * 8);
    }
  vf4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = vf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mma(a[s][i], b[s][j], acc[i][j]);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) out[(int64_t)(rb + i * 16 + lq * 4 + e) * ldo + cb + j * 16 + li] = acc[i][j][e];
}

// ---------------------------------------------------------------- F1 / F3: LN + GEMM
// MODE 0: qkv = LN1(x0) Wqkv^T (48 column blocks of 32); MODE 1: pre = LN2(x1) W1^T + b1,
// aux = pre, h = GELU(pre) (64 column blocks).  Workgroup (column block cb, row half rh):
// 64 rows, so a workgroup reads half of the A rows (the workgroups are latency / per-CU
// bandwidth bound: 48-64 workgroups reading all 128 rows ran 26-30 us).  512 threads: wave
// (rg = w & 1, kq = w >> 1) owns rows 32 rg .. + 32 of the half and the K quarter kq (4 k-steps,
// one batch of loads); the quarters meet in LDS in a fixed order.
template <int MODE, bool MX>
__global__ __launch_bounds__(512) void vit_ln_gemm_kernel(VitP p, int R, const float *xin, VitSaved s) {
  __shared__ float smu[VRP], srs[VRP];
  __shared__ vf4 red[3][2][2][2][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int cb = blockIdx.x >> 1, rh = blockIdx.x & 1, rbase = rh * 64;
  const float *gw = MODE ? p.ln2_w : p.ln1_w, *gb = MODE ? p.ln2_b : p.ln1_b;
  const bf16_t *W = reinterpret_cast<const bf16_t *>(p.packed) + (MODE ? PK_1 : PK_QKV);
  ln_stats_rows<8, 64>(xin, R, p.ln_eps, smu, srs, w, lane, rbase);
  __syncthreads();
  if (cb == 0 && tid < 64) {
    (MODE ? s.mu2 : s.mu1)[rbase + tid] = smu[rbase + tid];
    (MODE ? s.rs2 : s.rs1)[rbase + tid] = srs[rbase + tid];
  }
  if (cb < 32 && tid < 128) {
    // the LN output transposed, [k][128 rows] bf16: 16 columns k per column block, 8 rows a thread
    bf16_t *lnT = MODE ? s.ln2T : s.ln1T;
    const int k = cb * 16 + (tid >> 3), r0 = rbase + (tid & 7) * 8;
    const float g = gw[k], bb = gb[k];
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int r = r0 + e;
      const float xv = (xin[(int64_t)rclamp(r, R) * VD + k] - smu[r]) * srs[r] * g + bb;
      v[e] = r < R ? xv : 0.f;
    }
    *reinterpret_cast<vb8 *>(lnT + (int64_t)k * VRP + r0) = pack8(v);
  }
  const int rg = w & 1, kq = w >> 1, li = lane & 15, lq = lane >> 4;
  const int c0 = cb * 32;
  int row[2];
  float mu[2], rs[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    row[t] = rbase + rg * 32 + t * 16 + li;
    mu[t] = smu[row[t]];
    rs[t] = srs[row[t]];
  }
  vf4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = vf4{0.f, 0.f, 0.f, 0.f};
  if constexpr (MX) {
    // the wave's K quarter is one 128-wide MX step: LN output quantized from fp32 in registers
    const MxW W8 = mx_image(p.packed, MODE ? 4 : 0);
    MxFrag af[2], bf[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float v[32];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int k = kq * 128 + (hh ? mx_k1(lane) : mx_k0(lane)) + 8 * q;
          float g8[8], b8[8], x8[8];
          ld8f(gw + k, g8);
          ld8f(gb + k, b8);
          ld8f(xin + (int64_t)rclamp(row[t], R) * VD + k, x8);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            v[hh * 16 + q * 8 + e] = row[t] < R ? (x8[e] - mu[t]) * rs[t] * g8[e] + b8[e] : 0.f;
        }
      af[t] = mx_quant(v);
      const int n = c0 + t * 16 + li;
      bf[t] = mx_load(W8.row(n), kq * 128, W8.srow(n));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mx_mma(af[i], bf[j], acc[i][j]);
  } else {
    vb8 af[4][2], bf[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = kq * 128 + u * 32 + lq * 8;
      float g8[8], b8[8];
      ld8f(gw + k, g8);
      ld8f(gb + k, b8);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        float v[8];
        ld8f(xin + (int64_t)rclamp(row[t], R) * VD + k, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = row[t] < R ? (v[e] - mu[t]) * rs[t] * g8[e] + b8[e] : 0.f;
        af[u][t] = pack8(v);
        bf[u][t] = ld8b(W + (int64_t)(c0 + t * 16 + li) * VD + k);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mma(af[u][i], bf[u][j], acc[i][j]);
  }
  if (kq > 0)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) red[kq - 1][rg][i][j][lane] = acc[i][j];
  __syncthreads();
  if (kq > 0) return;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const vf4 a = red[0][rg][i][j][lane], b = red[1][rg][i][j][lane], c = red[2][rg][i][j][lane];
      const int col = c0 + j * 16 + li;
      const int rb = rbase + rg * 32 + i * 16 + lq * 4;
      float v4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v4[e] = ((acc[i][j][e] + a[e]) + b[e]) + c[e];
      if (MODE == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (rb + e < R) s.qkv[(int64_t)(rb + e) * VQ + col] = f2bf(v4[e]);
      } else {
        const float bias = p.b1[col];
        float hv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float pre = v4[e] + bias;
          hv[e] = rb + e < R ? gelu_erf(pre) : 0.f;
          if (rb + e < R) {
            s.aux[(int64_t)(rb + e) * VF + col] = f2bf(pre);
            s.h[(int64_t)(rb + e) * VF + col] = f2bf(hv[e]);
          }
        }
        uint2 pk;
        pk.x = (unsigned)f2bf(hv[0]) | ((unsigned)f2bf(hv[1]) << 16);
        pk.y = (unsigned)f2bf(hv[2]) | ((unsigned)f2bf(hv[3]) << 16);
        *reinterpret_cast<uint2 *>(s.hT + (int64_t)col * VRP + rb) = pk;
      }
    }
}

// ---------------------------------------------------------------- F2: attention + to_out
// Workgroup (column block cb of 32 outputs, row half rh = 32 frames), 512 threads.  The
// workgroup forms the softmax weights of its frames' (frame, head) pairs — 4 dot products of 64
// per pair — in LDS; the attention output o[r][k] = p[r][h][0] v[2f][k] + p[r][h][1] v[2f+1][k]
// (f = r / 2, h = k / 64) is formed in the A fragments; column block cb also writes o
// transposed for its 32 columns and the half's rows.  Waves (rg = w & 1, kq = w >> 1) as F1.
template <bool MX>
__global__ __launch_bounds__(512) void vit_attn_proj_kernel(VitP p, int R, const float *x0, VitSaved s) {
  __shared__ float sp[VRP][VH][2];
  __shared__ vf4 red[3][2][2][2][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int cb = blockIdx.x >> 1, rh = blockIdx.x & 1, rbase = rh * 64;
  const int B = R >> 1;
  if (tid < 256) {
    // thread = (frame b of the half, head h): the 4 dot products of 64 of the frame's 2x2 scores
    const int b = rh * 32 + (tid >> 3), h = tid & 7, bc = b < B ? b : B - 1;
    float s00 = 0.f, s01 = 0.f, s10 = 0.f, s11 = 0.f;
    {
      const bf16_t *q0p = s.qkv + (int64_t)(2 * bc) * VQ + h * VDH, *q1p = q0p + VQ;
      vb8 a0[8], a1[8], c0[8], c1[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a0[u] = ld8b(q0p + u * 8);
        a1[u] = ld8b(q1p + u * 8);
        c0[u] = ld8b(q0p + VD + u * 8);
        c1[u] = ld8b(q1p + VD + u * 8);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float q0[8], q1[8], k0[8], k1[8];
        unpack8(a0[u], q0);
        unpack8(a1[u], q1);
        unpack8(c0[u], k0);
        unpack8(c1[u], k1);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s00 += q0[e] * k0[e];
          s01 += q0[e] * k1[e];
          s10 += q1[e] * k0[e];
          s11 += q1[e] * k1[e];
        }
      }
    }
    const float sc[2][2] = {{s00 * VSCALE, s01 * VSCALE}, {s10 * VSCALE, s11 * VSCALE}};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float p0 = 0.f, p1 = 0.f;
      if (b < B) {
        const float mx = fmaxf(sc[i][0], sc[i][1]);
        const float e0 = __expf(sc[i][0] - mx), e1 = __expf(sc[i][1] - mx);
        const float inv = 1.0f / (e0 + e1);
        p0 = e0 * inv;
        p1 = e1 * inv;
      }
      sp[2 * b + i][h][0] = p0;
      sp[2 * b + i][h][1] = p1;
    }
  }
  __syncthreads();
  if (cb == 0)
    for (int i = rbase * VH * 2 + tid; i < (rbase + 64) * VH * 2 && i < R * VH * 2; i += 512) s.p[i] = (&sp[0][0][0])[i];
  if (tid < 256) {
    // o transposed: columns k = 32 cb + (tid >> 3), rows rbase + 8 (tid & 7) .. + 8
    const int k = cb * 32 + (tid >> 3), r0 = rbase + (tid & 7) * 8, h = k >> 6;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int r = r0 + e, f = rclamp(r, R) >> 1;
      float o = sp[r][h][0] * bf2f(s.qkv[(int64_t)(2 * f) * VQ + 2 * VD + k]);
      o += sp[r][h][1] * bf2f(s.qkv[(int64_t)(2 * f + 1) * VQ + 2 * VD + k]);
      v[e] = r < R ? o : 0.f;
    }
    *reinterpret_cast<vb8 *>(s.oT + (int64_t)k * VRP + r0) = pack8(v);
  }
  const int rg = w & 1, kq = w >> 1, li = lane & 15, lq = lane >> 4;
  const int c0 = cb * 32;
  vf4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = vf4{0.f, 0.f, 0.f, 0.f};
  if constexpr (MX) {
    const MxW W8 = mx_image(p.packed, 2);
    MxFrag af[2], bf[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int r = rbase + rg * 32 + t * 16 + li, f = rclamp(r, R) >> 1;
      float v[32];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int k = kq * 128 + (hh ? mx_k1(lane) : mx_k0(lane)) + 8 * q, h = k >> 6;
          float v0[8], v1[8];
          unpack8(ld8b(s.qkv + (int64_t)(2 * f) * VQ + 2 * VD + k), v0);
          unpack8(ld8b(s.qkv + (int64_t)(2 * f + 1) * VQ + 2 * VD + k), v1);
          const float p0 = sp[r][h][0], p1 = sp[r][h][1];      // 0 past R
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float o = p0 * v0[e];
            o += p1 * v1[e];
            v[hh * 16 + q * 8 + e] = o;
          }
        }
      af[t] = mx_quant(v);
      const int n = c0 + t * 16 + li;
      bf[t] = mx_load(W8.row(n), kq * 128, W8.srow(n));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mx_mma(af[i], bf[j], acc[i][j]);
  } else {
    vb8 af[4][2], bf[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = kq * 128 + u * 32 + lq * 8, h = k >> 6;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int r = rbase + rg * 32 + t * 16 + li, f = rclamp(r, R) >> 1;
        float v0[8], v1[8], o[8];
        unpack8(ld8b(s.qkv + (int64_t)(2 * f) * VQ + 2 * VD + k), v0);
        unpack8(ld8b(s.qkv + (int64_t)(2 * f + 1) * VQ + 2 * VD + k), v1);
        const float p0 = sp[r][h][0], p1 = sp[r][h][1];      // 0 past R
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          o[e] = p0 * v0[e];
          o[e] += p1 * v1[e];
        }
        af[u][t] = pack8(o);
        bf[u][t] = ld8b(reinterpret_cast<const bf16_t *>(p.packed) + PK_O + (int64_t)(c0 + t * 16 + li) * VD + k);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mma(af[u][i], bf[u][j], acc[i][j]);
  }
  if (kq > 0)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) red[kq - 1][rg][i][j][lane] = acc[i][j];
  __syncthreads();
  if (kq > 0) return;
  const uint64_t sd = step_seed(p.seed, p.seed_off);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const vf4 a = red[0][rg][i][j][lane], b = red[1][rg][i][j][lane], c = red[2][rg][i][j][lane];
      const int col = c0 + j * 16 + li;
      const float bias = p.bo[col];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = rbase + rg * 32 + i * 16 + lq * 4 + e;
        const float res = x0[(int64_t)rclamp(r, R) * VD + col];
        float v = (((acc[i][j][e] + a[e]) + b[e]) + c[e]) + bias;
        if (p.drop_p > 0.f) v = uniform01(sd, (uint64_t)(r * VD + col)) >= p.drop_p ? v * (1.0f / (1.0f - p.drop_p)) : 0.f;
        v += res;
        if (r < R) s.x1[(int64_t)r * VD + col] = v;
      }
    }
}

// ---------------------------------------------------------------- B1: Linear2 / GELU backward
// 64 workgroups of 32 hidden columns J, 512 threads (rg, kh as F1).  dh[:, J] = g W2[:, J]
// (K = 512 over W2's output index: W2[:, J] staged transposed in LDS), rounded to bf16 like the
// module path's dh, g1 = dh GELU'(pre) -> g1 (bf16), g1^T, db1[J].  Side job of workgroup b:
// g's columns 8 b .. + 8 transposed (gT) and their sums (db2).
template <bool MX>
__global__ __launch_bounds__(512) void vit_mlp2_bwd_kernel(VitP p, VitG G, int R, const float *g, VitSaved s,
                                                           VitScratch z) {
  __shared__ vf4 red[3][2][2][2][64];
  __shared__ float sg[VRP][9];
  __shared__ float scol[2][32];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int jb = blockIdx.x >> 1, rh = blockIdx.x & 1, rbase = rh * 64;
  const int J0 = jb * 32;
  const bf16_t *wT = reinterpret_cast<const bf16_t *>(p.packed) + PK_2T;    // W2^T [2048][512]
  if (rh == 0) {
    // side job: g's columns 8 jb .. + 8 transposed (gT) and their sums (db2)
    if (tid < VRP) {
      const int r = tid;
      float v[8];
      ld8f(g + (int64_t)rclamp(r, R) * VD + jb * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = r < R ? v[e] : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sg[r][e] = v[e];
        z.gT[(int64_t)(jb * 8 + e) * VRP + r] = f2bf(v[e]);
      }
    }
    __syncthreads();
    if (tid < 8) {
      float a = 0.f;
      for (int r = 0; r < R; ++r) a += sg[r][tid];
      G.b2[jb * 8 + tid] = a;
    }
  }
  const int rg = w & 1, kq = w >> 1, li = lane & 15, lq = lane >> 4;
  vf4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = vf4{0.f, 0.f, 0.f, 0.f};
  if constexpr (MX) {
    const MxW W8 = mx_image(p.packed, 7);         // W2^T [2048][512]
    MxFrag af[2], bf[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int r = rbase + rg * 32 + t * 16 + li;
      float v[32];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int k = kq * 128 + (hh ? mx_k1(lane) : mx_k0(lane)) + 8 * q;
          ld8f(g + (int64_t)rclamp(r, R) * VD + k, v + hh * 16 + q * 8);
        }
      if (r >= R)
#pragma unroll
        for (int e = 0; e < 32; ++e) v[e] = 0.f;
      af[t] = mx_quant(v);
      const int n = J0 + t * 16 + li;
      bf[t] = mx_load(W8.row(n), kq * 128, W8.srow(n));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mx_mma(af[i], bf[j], acc[i][j]);
  } else {
    vb8 af[4][2], bf[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = kq * 128 + u * 32 + lq * 8;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int r = rbase + rg * 32 + t * 16 + li;
        float v[8];
        ld8f(g + (int64_t)rclamp(r, R) * VD + k, v);
        af[u][t] = pack8(v);
        if (r >= R) af[u][t] = zero8();
        bf[u][t] = ld8b(wT + (int64_t)(J0 + t * 16 + li) * VD + k);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mma(af[u][i], bf[u][j], acc[i][j]);
  }
  if (kq > 0)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) red[kq - 1][rg][i][j][lane] = acc[i][j];
  __syncthreads();
  if (kq == 0) {
    float cs[2] = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const vf4 ra = red[0][rg][i][j][lane], rb2 = red[1][rg][i][j][lane], rc = red[2][rg][i][j][lane];
        const int col = J0 + j * 16 + li;
        const int rb = rbase + rg * 32 + i * 16 + lq * 4;
        float gv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = rb + e;
          const float a = bf2f(s.aux[(int64_t)rclamp(r, R) * VF + col]);
          const float dh = rbf(((acc[i][j][e] + ra[e]) + rb2[e]) + rc[e]);
          gv[e] = r < R ? dh * gelu_erf_grad(a) : 0.f;
          if (r < R) z.g1[(int64_t)r * VF + col] = f2bf(gv[e]);
          cs[j] += gv[e];
        }
        uint2 pk;
        pk.x = (unsigned)f2bf(gv[0]) | ((unsigned)f2bf(gv[1]) << 16);
        pk.y = (unsigned)f2bf(gv[2]) | ((unsigned)f2bf(gv[3]) << 16);
        *reinterpret_cast<uint2 *>(z.g1T + (int64_t)col * VRP + rb) = pk;
      }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float v = rows_sum4(cs[j]);
      if (lq == 0) scol[rg][j * 16 + li] = v;
    }
  }
  __syncthreads();
  // this row half's Linear1 bias-gradient partial (B2 adds the halves)
  if (tid < 32) z.db1p[rh * VF + J0 + tid] = scol[0][tid] + scol[1][tid];
}

// An input-gradient block out[rows 32 rq .. + 32][I0 .. I0 + 16] = A[rows][K] (bf16, row stride
// K) x BT[I0 .. + 16][K]^T (bf16 k-contiguous weight image), 4 waves = 4 K quarters added in LDS
// in a fixed order (fp32 out, row stride 512)
// ... and, for the LayerNorm whose output gradient it is, the block's row partials of the LN
// backward sums over its 16 columns: rpart[I0 / 16][row] = (sum gamma d, sum gamma d xhat)
// with xhat from X, mu, rs (the consumer adds the 32 column blocks in order)
// MX: A block-quantized in registers, B from the MXFP8 image BT8 of the same weight
template <int K, bool MX>
__device__ __forceinline__ void dgrad_block(const bf16_t *A, const bf16_t *BT, const MxW &BT8, float *out, int R,
                                            int I0, int rq, int w, int lane, vf4 *red, const float *X,
                                            const float *mu, const float *rs, const float *gamma, float *rpart) {
  constexpr int KQ = K / 4, NS = KQ / 32;
  const int li = lane & 15, lq = lane >> 4;
  vf4 acc[2];
  acc[0] = acc[1] = vf4{0.f, 0.f, 0.f, 0.f};
  if constexpr (MX) {
#pragma unroll 1
    for (int sb = 0; sb < NS; sb += 4) {
      const int kb = w * KQ + sb * 32;
      MxFrag af[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int r = rq * 32 + t * 16 + li;
        float v[32];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int q = 0; q < 2; ++q)
            unpack8(ld8b(A + (int64_t)rclamp(r, R) * K + kb + (hh ? mx_k1(lane) : mx_k0(lane)) + 8 * q),
                    v + hh * 16 + q * 8);
        if (r >= R)
#pragma unroll
          for (int e = 0; e < 32; ++e) v[e] = 0.f;
        af[t] = mx_quant(v);
      }
      const MxFrag bf = mx_load(BT8.row(I0 + li), kb, BT8.srow(I0 + li));
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = mx_mma(af[t], bf, acc[t]);
    }
  } else {
#pragma unroll 1
    for (int sb = 0; sb < NS; sb += 4) {
      vb8 af[4][2], bf[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = w * KQ + (sb + u) * 32 + lq * 8;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int r = rq * 32 + t * 16 + li;
          af[u][t] = ld8b(A + (int64_t)rclamp(r, R) * K + k);
          if (r >= R) af[u][t] = zero8();
        }
        bf[u] = ld8b(BT + (int64_t)(I0 + li) * K + k);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[t] = mma(af[u][t], bf[u], acc[t]);
    }
  }
  if (w > 0)
#pragma unroll
    for (int t = 0; t < 2; ++t) red[((w - 1) * 2 + t) * 64 + lane] = acc[t];
  __syncthreads();
  if (w > 0) return;
  const float gm = gamma[I0 + li];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const vf4 a = red[(0 * 2 + t) * 64 + lane], b = red[(1 * 2 + t) * 64 + lane], c = red[(2 * 2 + t) * 64 + lane];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = rq * 32 + t * 16 + lq * 4 + e, rr = rclamp(r, R);
      const float d = ((acc[t][e] + a[e]) + b[e]) + c[e];
      const float xh = (X[(int64_t)rr * VD + I0 + li] - mu[rr]) * rs[rr];
      if (r < R) out[(int64_t)r * VD + I0 + li] = d;
      const float ga = row_sum16(r < R ? gm * d : 0.f), gb = row_sum16(r < R ? gm * d * xh : 0.f);
      if (li == 0) {
        rpart[((I0 >> 4) * VRP + r) * 2] = ga;
        rpart[((I0 >> 4) * VRP + r) * 2 + 1] = gb;
      }
    }
  }
}

// the LN backward row sums from the producers' 32 column-block partials, added in order
__device__ __forceinline__ void lnb_rows_parts(const float *rpart, float *sa, float *sb, int tid) {
  if (tid < VRP) {
    float a = 0.f, b = 0.f;
#pragma unroll 8
    for (int q = 0; q < 32; ++q) {
      a += rpart[(q * VRP + tid) * 2];
      b += rpart[(q * VRP + tid) * 2 + 1];
    }
    sa[tid] = a / (float)VD;
    sb[tid] = b / (float)VD;
  }
}

// ---------------------------------------------------------------- B2: Linear1 backward, dW2, dW1
// 256 threads.  Workgroups 0..127: dLN2 = g1 W1 in (16 columns, 32 rows) blocks (W1^T from the
// packed image; 4 waves = 4 K quarters of 512, added in LDS); 128..383: dW2 = g^T h in 64 x 64
// blocks; 384..639: dW1 = g1^T LN2.
template <bool MX>
__global__ __launch_bounds__(256) void vit_mlp1_bwd_kernel(VitP p, VitG G, int R, VitSaved s, VitScratch z) {
  __shared__ vf4 red[3 * 2 * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int blk = blockIdx.x;
  if (blk >= 128 + 512) {
    // Linear1 bias gradient: the two row halves' partials added
    const int j = (blk - 640) * 256 + threadIdx.x;
    G.b1[j] = z.db1p[j] + z.db1p[VF + j];
    return;
  }
  if (blk >= 128 + 256) {
    const int q = blk - 384;
    wgrad_block<MX>(z.g1T, s.ln2T, G.w1, VD, (q >> 3) * 64, (q & 7) * 64, w, lane);
    return;
  }
  if (blk >= 128) {
    const int q = blk - 128;
    wgrad_block<MX>(z.gT, s.hT, G.w2, VF, (q >> 5) * 64, (q & 31) * 64, w, lane);
    return;
  }
  // input gradient: workgroup (16-column block, row quarter)
  const MxW W8 = MX ? mx_image(p.packed, 5) : MxW{nullptr, nullptr, 0};
  dgrad_block<VF, MX>(z.g1, reinterpret_cast<const bf16_t *>(p.packed) + PK_1T, W8, z.dln2, R, (blk >> 2) * 16,
                      blk & 3, w, lane, red, s.x1, s.mu2, s.rs2, p.ln2_w, z.rp2);
}

// ---------------------------------------------------------------- LayerNorm backward pieces
// columns c0 .. c0 + 32, 512 threads (column tid & 31, rows 8 (tid >> 5) .. + 8):
// dX = resid + rstd (gamma dY - ma - xhat mb) -> dXout [R][512] f32; the affine gradients
// (sum dY xhat, sum dY) and, with a dropout (to_out), g_o = dX keep / (1 - p) transposed into
// goT and its column sums (to_out's bias gradient)
__device__ __forceinline__ void lnb_cols(const float *dY, const float *X, const float *gamma, const float *mu,
                                         const float *rs, const float *resid, int R, const float *sa,
                                         const float *sb, int c0, float *dXout, float *dgamma, float *dbeta,
                                         bool drop, float dp, uint64_t sd, bf16_t *goT, float *dbo, float *part,
                                         int tid) {
  const int c = c0 + (tid & 31), rg = tid >> 5;
  const float gm = gamma[c];
  float pg = 0.f, pb = 0.f, po = 0.f, gov[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int r = rg * 8 + e, rr = rclamp(r, R);
    const float dv = dY[(int64_t)rr * VD + c], xv = X[(int64_t)rr * VD + c], res = resid[(int64_t)rr * VD + c];
    gov[e] = 0.f;
    if (r < R) {
      const float xh = (xv - mu[r]) * rs[r];
      const float dx = rs[r] * (gm * dv - sa[r] - xh * sb[r]) + res;
      dXout[(int64_t)r * VD + c] = dx;
      pg += dv * xh;
      pb += dv;
      if (drop) {
        gov[e] = dp > 0.f ? dx * keep_scale(dp, sd, (uint64_t)(r * VD + c)) : dx;
        po += gov[e];
      }
    }
  }
  if (drop) *reinterpret_cast<vb8 *>(goT + (int64_t)c * VRP + rg * 8) = pack8(gov);
  part[(0 * 16 + rg) * 32 + (tid & 31)] = pg;
  part[(1 * 16 + rg) * 32 + (tid & 31)] = pb;
  part[(2 * 16 + rg) * 32 + (tid & 31)] = po;
  __syncthreads();
  if (tid < 32) {
    float a = 0.f, b = 0.f, o = 0.f;
    for (int q = 0; q < 16; ++q) {
      a += part[(0 * 16 + q) * 32 + tid];
      b += part[(1 * 16 + q) * 32 + tid];
      o += part[(2 * 16 + q) * 32 + tid];
    }
    dgamma[c0 + tid] = a;
    dbeta[c0 + tid] = b;
    if (drop) dbo[c0 + tid] = o;
  }
}

// ---------------------------------------------------------------- B3: LN2 backward + attention
// 512 threads.  Every workgroup takes the per-row LN2 backward sums.  Workgroups 0..31 = (head h,
// row quarter q of 32 rows = 16 frames): d(attention out)[rows, head h] = g_o Wo^T[head h] with
// g_o = (g + LN2 backward) keep / (1 - p) formed in the A fragments, the 8 waves taking K slices
// of 64 (added in LDS in a fixed order), rounded to bf16 like the module path's; then the
// attention backward of the head over the 16 two-token frames -> dqkv (bf16) and dqkv^T.
// Workgroups 32..47: 32 columns each of dx1, g_o^T, the to_out bias and the LN2 affine gradients.
// MX: the 8 waves as 4 K slices of 128 (one MX step each) x 2 column halves of the head
template <bool MX>
__global__ __launch_bounds__(512) void vit_ln2_bwd_attn_kernel(VitP p, VitG G, int R, const float *g, VitSaved s,
                                                               VitScratch z) {
  __shared__ vf4 red[8][2][4][64];                 // 64 KB: the waves' K-slice partials
  __shared__ float sdo[32][68];
  __shared__ float sa[VRP], sbm[VRP];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  lnb_rows_parts(z.rp2, sa, sbm, tid);
  __syncthreads();
  const uint64_t sd = step_seed(p.seed, p.seed_off);
  if (blockIdx.x >= 4 * VH) {
    lnb_cols(z.dln2, s.x1, p.ln2_w, s.mu2, s.rs2, g, R, sa, sbm, (blockIdx.x - 4 * VH) * 32, z.dx1, G.ln2_w,
             G.ln2_b, true, p.drop_p, sd, z.goT, G.bo, reinterpret_cast<float *>(&red[0][0][0][0]), tid);
    return;
  }
  const int h = blockIdx.x >> 2, q = blockIdx.x & 3;
  const bf16_t *wT = reinterpret_cast<const bf16_t *>(p.packed) + PK_OT;    // Wo^T [512][512]
  const int li = lane & 15, lq = lane >> 4;
  int row[2];
  float mu[2], rs[2], ma[2], mb[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    row[t] = q * 32 + t * 16 + li;
    mu[t] = s.mu2[rclamp(row[t], R)];
    rs[t] = s.rs2[rclamp(row[t], R)];
    ma[t] = sa[row[t]];
    mb[t] = sbm[row[t]];
  }
  constexpr int NSL = MX ? 4 : 8;                  // K slices added in the reduction below
  if constexpr (MX) {
    const MxW W8 = mx_image(p.packed, 3);          // Wo^T [512][512]
    const int ks = w & 3, ch = w >> 2;
    MxFrag af[2], bf[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int r = row[t], rr = rclamp(r, R);
      float v[32];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int k = ks * 128 + (hh ? mx_k1(lane) : mx_k0(lane)) + 8 * q;
          float gm[8], d[8], x[8], gg[8];
          ld8f(p.ln2_w + k, gm);
          ld8f(z.dln2 + (int64_t)rr * VD + k, d);
          ld8f(s.x1 + (int64_t)rr * VD + k, x);
          ld8f(g + (int64_t)rr * VD + k, gg);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float xh = (x[e] - mu[t]) * rs[t];
            float dx = rs[t] * (gm[e] * d[e] - ma[t] - xh * mb[t]) + gg[e];
            if (p.drop_p > 0.f) dx *= keep_scale(p.drop_p, sd, (uint64_t)(r * VD + k + e));
            v[hh * 16 + q * 8 + e] = r < R ? dx : 0.f;
          }
        }
      af[t] = mx_quant(v);
    }
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int n = h * VDH + (ch * 2 + jj) * 16 + li;
      bf[jj] = mx_load(W8.row(n), ks * 128, W8.srow(n));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) red[ks][i][ch * 2 + jj][lane] = mx_mma(af[i], bf[jj], vf4{0.f, 0.f, 0.f, 0.f});
  } else {
  vf4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = vf4{0.f, 0.f, 0.f, 0.f};
  {
    vb8 af[2][2], bf[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = w * 64 + u * 32 + lq * 8;
      float gm[8];
      ld8f(p.ln2_w + k, gm);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int r = row[t], rr = rclamp(r, R);
        float d[8], x[8], gg[8], v[8];
        ld8f(z.dln2 + (int64_t)rr * VD + k, d);
        ld8f(s.x1 + (int64_t)rr * VD + k, x);
        ld8f(g + (int64_t)rr * VD + k, gg);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xh = (x[e] - mu[t]) * rs[t];
          float dx = rs[t] * (gm[e] * d[e] - ma[t] - xh * mb[t]) + gg[e];
          if (p.drop_p > 0.f) dx *= keep_scale(p.drop_p, sd, (uint64_t)(r * VD + k + e));
          v[e] = r < R ? dx : 0.f;
        }
        af[u][t] = pack8(v);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[u][j] = ld8b(wT + (int64_t)(h * VDH + j * 16 + li) * VD + k);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mma(af[u][i], bf[u][j], acc[i][j]);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) red[w][i][j][lane] = acc[i][j];
  }
  __syncthreads();
  if (tid < 2 * 4 * 64) {
    // the K slices added in order; thread (i, j, lane) of the 32 x 64 block
    const int i = tid >> 8, j = (tid >> 6) & 3, l = tid & 63;
    vf4 a = red[0][i][j][l];
#pragma unroll
    for (int k = 1; k < NSL; ++k) {
      const vf4 b = red[k][i][j][l];
      a = vf4{a[0] + b[0], a[1] + b[1], a[2] + b[2], a[3] + b[3]};
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) sdo[i * 16 + (l >> 4) * 4 + e][j * 16 + (l & 15)] = rbf(a[e]);
  }
  __syncthreads();
  if (tid >= 128) return;
  // attention backward of head h: 8 lanes per frame (8 head dims each), the quarter's 16 frames
  const int fl = tid >> 3, f = q * 16 + fl, d0 = (tid & 7) * 8, B = R >> 1;
  const int fc = f < B ? f : B - 1;
  float qv[2][8], kk[2][8], vv[2][8], dO[2][8];
  float pr[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t rb = (int64_t)(2 * fc + i) * VQ + h * VDH + d0;
    unpack8(ld8b(s.qkv + rb), qv[i]);
    unpack8(ld8b(s.qkv + rb + VD), kk[i]);
    unpack8(ld8b(s.qkv + rb + 2 * VD), vv[i]);
#pragma unroll
    for (int e = 0; e < 8; ++e) dO[i][e] = f < B ? sdo[2 * fl + i][d0 + e] : 0.f;
    pr[i][0] = f < B ? s.p[((2 * fc + i) * VH + h) * 2] : 0.f;
    pr[i][1] = f < B ? s.p[((2 * fc + i) * VH + h) * 2 + 1] : 0.f;
  }
  float dp[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float a = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) a += dO[i][e] * vv[j][e];
#pragma unroll
      for (int m = 1; m < 8; m <<= 1) a += __shfl_xor(a, m, 64);
      dp[i][j] = a;
    }
  float dq[2][8], dk[2][8], dv[2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) { dq[i][e] = dk[i][e] = dv[i][e] = 0.f; }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float dot = pr[i][0] * dp[i][0] + pr[i][1] * dp[i][1];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float ds = pr[i][j] * (dp[i][j] - dot) * VSCALE;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dq[i][e] += ds * kk[j][e];
        dk[j][e] += ds * qv[i][e];
        dv[j][e] += pr[i][j] * dO[i][e];
      }
    }
  }
  // dqkv rows 2f, 2f + 1 (bf16) and dqkv^T [col][rows 2f, 2f + 1] (0 past R)
#pragma unroll
  for (int part = 0; part < 3; ++part) {
    const float(*src)[8] = part == 0 ? dq : part == 1 ? dk : dv;
    const int cb = part * VD + h * VDH + d0;
    if (f < B)
#pragma unroll
      for (int i = 0; i < 2; ++i) *reinterpret_cast<vb8 *>(z.dqkv + (int64_t)(2 * f + i) * VQ + cb) = pack8(src[i]);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const unsigned pk = (unsigned)f2bf(src[0][e]) | ((unsigned)f2bf(src[1][e]) << 16);
      *reinterpret_cast<unsigned *>(z.dqkvT + (int64_t)(cb + e) * VRP + 2 * f) = pk;
    }
  }
}

// ---------------------------------------------------------------- B4: to_qkv backward, dWqkv, dWo
// 256 threads.  Workgroups 0..127: dLN1 = dqkv Wqkv in (16 columns, 32 rows) blocks (4 waves = K
// quarters of 384, added in LDS); 128..319: dWqkv = dqkv^T LN1; 320..383: dWo = g_o^T o.
template <bool MX>
__global__ __launch_bounds__(256) void vit_qkv_bwd_kernel(VitP p, VitG G, int R, const float *x0, VitSaved s,
                                                          VitScratch z) {
  __shared__ vf4 red[3 * 2 * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int blk = blockIdx.x;
  if (blk >= 128 + 192) {
    const int q = blk - 320;
    wgrad_block<MX>(z.goT, s.oT, G.wo, VD, (q >> 3) * 64, (q & 7) * 64, w, lane);
    return;
  }
  if (blk >= 128) {
    const int q = blk - 128;
    wgrad_block<MX>(z.dqkvT, s.ln1T, G.wqkv, VD, (q >> 3) * 64, (q & 7) * 64, w, lane);
    return;
  }
  // input gradient: workgroup (16-column block, row quarter)
  const MxW W8 = MX ? mx_image(p.packed, 1) : MxW{nullptr, nullptr, 0};
  dgrad_block<VQ, MX>(z.dqkv, reinterpret_cast<const bf16_t *>(p.packed) + PK_QKVT, W8, z.dln1, R, (blk >> 2) * 16,
                      blk & 3, w, lane, red, x0, s.mu1, s.rs1, p.ln1_w, z.rp1);
}

// ---------------------------------------------------------------- B5: LN1 backward + residual
// 16 workgroups of 32 columns, 512 threads: dx0 = dx1 + LN1 backward(dLN1), dLN1 affine.
__global__ __launch_bounds__(512) void vit_ln1_bwd_kernel(VitP p, VitG G, int R, const float *x0, VitSaved s,
                                                          VitScratch z, float *dx0) {
  __shared__ float sa[VRP], sbm[VRP], part[3 * 16 * 32];
  const int tid = threadIdx.x;
  lnb_rows_parts(z.rp1, sa, sbm, tid);
  __syncthreads();
  lnb_cols(z.dln1, x0, p.ln1_w, s.mu1, s.rs1, z.dx1, R, sa, sbm, blockIdx.x * 32, dx0, G.ln1_w, G.ln1_b, false,
           0.f, 0, nullptr, nullptr, part, tid);
}


// ---------------------------------------------------------------- token embedding (sfe.py:155-160)
// tok[b][0] = drop(cls + pos[b]), tok[b][1] = drop(y[b] + pos[b]) (pos_embedding[0:B] broadcast
// over the 2 tokens); dropout keep(seed, (b * 2 + i) * 512 + c).  One thread per 4 columns.
__global__ __launch_bounds__(256) void vit_embed_fwd_kernel(const float *y, const float *cls, const float *pos, int B,
                                                            float dp, uint64_t seed, const int64_t *seed_off,
                                                            float *tok) {
  const int i = blockIdx.x * 256 + threadIdx.x;          // (b, token, column quad)
  if (i >= B * 2 * (VD / 4)) return;
  const int c = (i % (VD / 4)) * 4, t = (i / (VD / 4)) & 1, b = i / (2 * (VD / 4));
  const float4 src = *reinterpret_cast<const float4 *>((t ? y + (int64_t)b * VD : cls) + c);
  const float4 pe = *reinterpret_cast<const float4 *>(pos + (int64_t)b * VD + c);
  float v[4] = {src.x + pe.x, src.y + pe.y, src.z + pe.z, src.w + pe.w};
  if (dp > 0.f) {
    const uint64_t sd = step_seed(seed, seed_off);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] *= keep_scale(dp, sd, (uint64_t)((b * 2 + t) * VD + c + e));
  }
  *reinterpret_cast<float4 *>(tok + ((int64_t)b * 2 + t) * VD + c) = make_float4(v[0], v[1], v[2], v[3]);
}
// d y[b] = m dtok[b][1], d pos[b] = m dtok[b][0] + m dtok[b][1] (rows >= B: 0, up to npos <= 64),
// d cls = sum_b m dtok[b][0] (fixed order).  8 workgroups of 64 columns; thread (column,
// frame group q) takes frames q, q + 8, ... with all loads in flight.
__global__ __launch_bounds__(512) void vit_embed_bwd_kernel(const float *dtok, int B, int npos, float dp, uint64_t seed,
                                                            const int64_t *seed_off, float *dy, float *dcls,
                                                            float *dpos) {
  __shared__ float part[8][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), q = threadIdx.x >> 6;
  const uint64_t sd = step_seed(seed, seed_off);
  float g0[8], g1[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int b = q + 8 * u;
    g0[u] = b < B ? dtok[((int64_t)b * 2) * VD + c] : 0.f;
    g1[u] = b < B ? dtok[((int64_t)b * 2 + 1) * VD + c] : 0.f;
  }
  float acc = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int b = q + 8 * u;
    if (b < B) {
      if (dp > 0.f) {
        g0[u] *= keep_scale(dp, sd, (uint64_t)((b * 2) * VD + c));
        g1[u] *= keep_scale(dp, sd, (uint64_t)((b * 2 + 1) * VD + c));
      }
      dy[(int64_t)b * VD + c] = g1[u];
      acc += g0[u];
    }
    if (b < npos) dpos[(int64_t)b * VD + c] = g0[u] + g1[u];
  }
  part[q][threadIdx.x & 63] = acc;
  __syncthreads();
  if (q == 0) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) a += part[k][threadIdx.x];
    dcls[c] = a;
  }
}

// ---------------------------------------------------------------- weight pack (once per step)
// a workgroup per 64 x 64 tile of one weight: fp32 [out][in] -> bf16 [out][in] and [in][out]
struct VitPackSrc { const float *w[4 * EWVIT_VIT_PACK_MAX]; };
__global__ __launch_bounds__(256) void vit_pack_kernel(VitPackSrc src, int nlayers, bf16_t *packed) {
  __shared__ float tile[64][65];
  // tiles per layer: qkv 24 x 8, o 8 x 8, w1 32 x 8, w2 8 x 32
  constexpr int T0 = 24 * 8, T1 = T0 + 64, T2 = T1 + 256, TL = T2 + 256;
  const int layer = blockIdx.x / TL, t = blockIdx.x % TL;
  int m, tr, tc, rows, cols;
  int64_t off, offT;
  if (t < T0) { m = 0; tr = t / 8; tc = t % 8; rows = VQ; cols = VD; off = PK_QKV; offT = PK_QKVT; }
  else if (t < T1) { m = 1; tr = (t - T0) / 8; tc = (t - T0) % 8; rows = VD; cols = VD; off = PK_O; offT = PK_OT; }
  else if (t < T2) { m = 2; tr = (t - T1) / 8; tc = (t - T1) % 8; rows = VF; cols = VD; off = PK_1; offT = PK_1T; }
  else { m = 3; tr = (t - T2) / 32; tc = (t - T2) % 32; rows = VD; cols = VF; off = PK_2; offT = PK_2T; }
  const float *W = src.w[layer * 4 + m];
  bf16_t *dst = packed + (int64_t)layer * PK_LAYER;
  const int tid = threadIdx.x, r0 = tr * 64, c0 = tc * 64;
  float4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = tid + u * 256, r = i >> 4, q = i & 15;
    v[u] = *reinterpret_cast<const float4 *>(W + (int64_t)(r0 + r) * cols + c0 + 4 * q);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = tid + u * 256, r = i >> 4, q = i & 15;
    tile[r][4 * q] = v[u].x; tile[r][4 * q + 1] = v[u].y; tile[r][4 * q + 2] = v[u].z; tile[r][4 * q + 3] = v[u].w;
    uint2 pk;
    pk.x = (unsigned)f2bf(v[u].x) | ((unsigned)f2bf(v[u].y) << 16);
    pk.y = (unsigned)f2bf(v[u].z) | ((unsigned)f2bf(v[u].w) << 16);
    *reinterpret_cast<uint2 *>(dst + off + (int64_t)(r0 + r) * cols + c0 + 4 * q) = pk;
  }
  __syncthreads();
  // transposed: row c (of W^T) = column c of W, 64 rows r per tile
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = tid + u * 256, c = i >> 4, q = i & 15;
    uint2 pk;
    pk.x = (unsigned)f2bf(tile[4 * q][c]) | ((unsigned)f2bf(tile[4 * q + 1][c]) << 16);
    pk.y = (unsigned)f2bf(tile[4 * q + 2][c]) | ((unsigned)f2bf(tile[4 * q + 3][c]) << 16);
    *reinterpret_cast<uint2 *>(dst + offT + (int64_t)(c0 + c) * rows + r0 + 4 * q) = pk;
  }
  (void)rows;
}

// MXFP8 pack: the same 64 x 64 tiles; threads 0..127 quantize the tile's 64 rows x 2 blocks of
// W (blocks along in), threads 128..255 its 64 columns x 2 blocks of W^T (blocks along out),
// straight from the fp32 masters (one rounding)
__global__ __launch_bounds__(256) void vit_pack_mx_kernel(VitPackSrc src, int nlayers, uint8_t *packed) {
  __shared__ float tile[64][65];
  constexpr int T0 = 24 * 8, T1 = T0 + 64, T2 = T1 + 256, TL = T2 + 256;
  const int layer = blockIdx.x / TL, t = blockIdx.x % TL;
  int m, tr, tc;
  if (t < T0) { m = 0; tr = t / 8; tc = t % 8; }
  else if (t < T1) { m = 1; tr = (t - T0) / 8; tc = (t - T0) % 8; }
  else if (t < T2) { m = 2; tr = (t - T1) / 8; tc = (t - T1) % 8; }
  else { m = 3; tr = (t - T2) / 32; tc = (t - T2) % 32; }
  int rows, cols;
  mx_dims(2 * m, rows, cols);
  const float *W = src.w[layer * 4 + m];
  uint8_t *base = packed + (int64_t)layer * mx_off(8);
  const int tid = threadIdx.x, r0 = tr * 64, c0 = tc * 64;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = tid + u * 256, r = i >> 4, q = i & 15;
    const float4 v = *reinterpret_cast<const float4 *>(W + (int64_t)(r0 + r) * cols + c0 + 4 * q);
    tile[r][4 * q] = v.x; tile[r][4 * q + 1] = v.y; tile[r][4 * q + 2] = v.z; tile[r][4 * q + 3] = v.w;
  }
  __syncthreads();
  const int tr_ = tid & 127, hb = tr_ & 1, x = tr_ >> 1;
  float v[32];
  int d[8];
  uint8_t *dst, *sdst;
  if (tid < 128) {          // W row r0 + x, in-columns c0 + 32 hb ..
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = tile[x][32 * hb + j];
    uint8_t *img = base + mx_off(2 * m);
    dst = img + (int64_t)(r0 + x) * cols + c0 + 32 * hb;
    sdst = img + al256((int64_t)rows * cols) + (int64_t)(r0 + x) * (cols / 32) + c0 / 32 + hb;
  } else {                  // W^T row c0 + x (= W column), out-rows r0 + 32 hb ..
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = tile[32 * hb + j][x];
    uint8_t *img = base + mx_off(2 * m + 1);
    dst = img + (int64_t)(c0 + x) * rows + r0 + 32 * hb;
    sdst = img + al256((int64_t)cols * rows) + (int64_t)(c0 + x) * (rows / 32) + r0 / 32 + hb;
  }
  const int e = mx_quant_block(v, d);
  *reinterpret_cast<uint4 *>(dst) = make_uint4(d[0], d[1], d[2], d[3]);
  *reinterpret_cast<uint4 *>(dst + 16) = make_uint4(d[4], d[5], d[6], d[7]);
  *sdst = (uint8_t)e;
}

}  // namespace ewvit

using namespace ewvit;

extern "C" int64_t ewvit_vit_layer_workspace(int which) {
  if (which == 3) return mx_off(8);
  if (which == 2) return PK_LAYER * 2;
  return which == 0 ? saved_layout([](int, int64_t) {}) : scratch_layout([](int, int64_t) {});
}

extern "C" int ewvit_vit_pack(const ewvit_vit_layer *layers, int n, void *packed, void *stream) {
  EWVIT_CHECK_ARG(layers && packed && n >= 1 && n <= EWVIT_VIT_PACK_MAX, "vit_pack: n=%d", n);
  VitPackSrc src;
  for (int i = 0; i < n; ++i) {
    EWVIT_CHECK_ARG(layers[i].wqkv && layers[i].wo && layers[i].w1 && layers[i].w2, "vit_pack: null weight");
    src.w[4 * i] = layers[i].wqkv;
    src.w[4 * i + 1] = layers[i].wo;
    src.w[4 * i + 2] = layers[i].w1;
    src.w[4 * i + 3] = layers[i].w2;
  }
  hipLaunchKernelGGL(vit_pack_kernel, dim3(n * (24 * 8 + 64 + 256 + 256)), dim3(256), 0, as_stream(stream), src, n,
                     (bf16_t *)packed);
  return launch_status("vit_pack");
}

extern "C" int ewvit_vit_pack_mx(const ewvit_vit_layer *layers, int n, void *packed, void *stream) {
  EWVIT_CHECK_ARG(layers && packed && n >= 1 && n <= EWVIT_VIT_PACK_MAX, "vit_pack_mx: n=%d", n);
  VitPackSrc src;
  for (int i = 0; i < n; ++i) {
    EWVIT_CHECK_ARG(layers[i].wqkv && layers[i].wo && layers[i].w1 && layers[i].w2, "vit_pack_mx: null weight");
    src.w[4 * i] = layers[i].wqkv;
    src.w[4 * i + 1] = layers[i].wo;
    src.w[4 * i + 2] = layers[i].w1;
    src.w[4 * i + 3] = layers[i].w2;
  }
  hipLaunchKernelGGL(vit_pack_mx_kernel, dim3(n * (24 * 8 + 64 + 256 + 256)), dim3(256), 0, as_stream(stream), src,
                     n, (uint8_t *)packed);
  return launch_status("vit_pack_mx");
}

static int vit_check(const ewvit_vit_layer *p, int R) {
  EWVIT_CHECK_ARG(p && p->ln1_w && p->ln1_b && p->wqkv && p->wo && p->bo && p->ln2_w && p->ln2_b && p->w1 && p->b1 &&
                      p->w2 && p->b2,
                  "vit_layer: null parameter");
  EWVIT_CHECK_ARG(R >= 2 && R <= VRP && R % 2 == 0, "vit_layer: R=%d rows (2 tokens per frame, <= %d)", R, VRP);
  EWVIT_CHECK_ARG(p->drop_p >= 0.f && p->drop_p < 1.f, "vit_layer: drop_p=%f", (double)p->drop_p);
  EWVIT_CHECK_ARG(p->packed, "vit_layer: no packed weights (ewvit_vit_pack)");
  return 0;
}

extern "C" int ewvit_vit_layer_fwd(const ewvit_vit_layer *p, int R, const float *x0, void *saved, float *x2,
                                   void *stream) {
  if (int rc = vit_check(p, R)) return rc;
  EWVIT_CHECK_ARG(x0 && saved && x2, "vit_layer_fwd: null pointer");
  const VitSaved s = vit_saved(saved);
  hipStream_t st = as_stream(stream);
  if (p->mx) {
    hipLaunchKernelGGL((vit_ln_gemm_kernel<0, true>), dim3(2 * VQ / 32), dim3(512), 0, st, *p, R, x0, s);
    hipLaunchKernelGGL(vit_attn_proj_kernel<true>, dim3(2 * VD / 32), dim3(512), 0, st, *p, R, x0, s);
    hipLaunchKernelGGL((vit_ln_gemm_kernel<1, true>), dim3(2 * VF / 32), dim3(512), 0, st, *p, R, (const float *)s.x1, s);
    if (int rc = launch_status("vit_layer_fwd")) return rc;
    // Linear2 on the MXFP8 split-K GEMM (W2 block-quantized from the fp32 master as it is
    // staged: the same e4m3 values and scales as the pack's image 6)
    return ewvit_gemm_mx8(s.h, EWVIT_BF16, VF, 1, p->w2, EWVIT_F32, 1, VF, x2, EWVIT_F32, VD, R, VD, VF, 1.f, 0.f,
                          p->b2, 0, nullptr, 0.f, 0, nullptr, s.x1, EWVIT_F32, VD, VF4_SPLIT, s.ws2, stream);
  }
  hipLaunchKernelGGL((vit_ln_gemm_kernel<0, false>), dim3(2 * VQ / 32), dim3(512), 0, st, *p, R, x0, s);
  hipLaunchKernelGGL(vit_attn_proj_kernel<false>, dim3(2 * VD / 32), dim3(512), 0, st, *p, R, x0, s);
  hipLaunchKernelGGL((vit_ln_gemm_kernel<1, false>), dim3(2 * VF / 32), dim3(512), 0, st, *p, R, (const float *)s.x1, s);
  if (int rc = launch_status("vit_layer_fwd")) return rc;
  // Linear2 + bias + residual: K = 2048 against 128 rows wants its K split over many
  // workgroups (one workgroup per column block reading all of h measured 32 us): the split-K
  // MFMA GEMM with the packed bf16 W2, its reduce adding b2 and x1
  return ewvit_gemm(s.h, EWVIT_BF16, VF, 1, reinterpret_cast<const bf16_t *>(p->packed) + PK_2, EWVIT_BF16, 1, VF,
                    x2, EWVIT_F32, VD, R, VD, VF, 1.f, 0.f, p->b2, 0, nullptr, 0.f, 0, nullptr, s.x1, EWVIT_F32, VD,
                    VF4_SPLIT, s.ws2, stream);
}

extern "C" int ewvit_vit_layer_bwd(const ewvit_vit_layer *p, int R, const float *x0, const void *saved,
                                   const float *g, void *scratch, float *dx0, const ewvit_vit_grads *G,
                                   void *stream) {
  if (int rc = vit_check(p, R)) return rc;
  EWVIT_CHECK_ARG(x0 && saved && g && scratch && dx0 && G, "vit_layer_bwd: null pointer");
  EWVIT_CHECK_ARG(G->ln1_w && G->ln1_b && G->wqkv && G->wo && G->bo && G->ln2_w && G->ln2_b && G->w1 && G->b1 &&
                      G->w2 && G->b2,
                  "vit_layer_bwd: null gradient");
  const VitSaved s = vit_saved(const_cast<void *>(saved));
  const VitScratch z = vit_scratch(scratch);
  hipStream_t st = as_stream(stream);
  if (p->mx) {
    hipLaunchKernelGGL(vit_mlp2_bwd_kernel<true>, dim3(2 * VF / 32), dim3(512), 0, st, *p, *G, R, g, s, z);
    hipLaunchKernelGGL(vit_mlp1_bwd_kernel<true>, dim3(128 + 256 + 256 + VF / 256), dim3(256), 0, st, *p, *G, R, s, z);
    hipLaunchKernelGGL(vit_ln2_bwd_attn_kernel<true>, dim3(4 * VH + 16), dim3(512), 0, st, *p, *G, R, g, s, z);
    hipLaunchKernelGGL(vit_qkv_bwd_kernel<true>, dim3(128 + 192 + 64), dim3(256), 0, st, *p, *G, R, x0, s, z);
  } else {
    hipLaunchKernelGGL(vit_mlp2_bwd_kernel<false>, dim3(2 * VF / 32), dim3(512), 0, st, *p, *G, R, g, s, z);
    hipLaunchKernelGGL(vit_mlp1_bwd_kernel<false>, dim3(128 + 256 + 256 + VF / 256), dim3(256), 0, st, *p, *G, R, s, z);
    hipLaunchKernelGGL(vit_ln2_bwd_attn_kernel<false>, dim3(4 * VH + 16), dim3(512), 0, st, *p, *G, R, g, s, z);
    hipLaunchKernelGGL(vit_qkv_bwd_kernel<false>, dim3(128 + 192 + 64), dim3(256), 0, st, *p, *G, R, x0, s, z);
  }
  hipLaunchKernelGGL(vit_ln1_bwd_kernel, dim3(VD / 32), dim3(512), 0, st, *p, *G, R, x0, s, z, dx0);
  return launch_status("vit_layer_bwd");
}

extern "C" int ewvit_vit_embed_fwd(const float *y, const float *cls, const float *pos, int B, int npos, float drop_p,
                                   uint64_t seed, const int64_t *seed_off, float *tok, void *stream) {
  EWVIT_CHECK_ARG(y && cls && pos && tok && B >= 1 && npos >= B && drop_p >= 0.f && drop_p < 1.f,
                  "vit_embed_fwd: bad args (B %d, npos %d: pos_embedding needs a row per frame)", B, npos);
  const int n = B * 2 * (VD / 4);
  hipLaunchKernelGGL(vit_embed_fwd_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), y, cls, pos, B, drop_p,
                     seed, seed_off, tok);
  return launch_status("vit_embed_fwd");
}

extern "C" int ewvit_vit_embed_bwd(const float *dtok, int B, int npos, float drop_p, uint64_t seed,
                                   const int64_t *seed_off, float *dy, float *dcls, float *dpos, void *stream) {
  EWVIT_CHECK_ARG(dtok && dy && dcls && dpos && B >= 1 && npos >= B && npos <= 64 && drop_p >= 0.f && drop_p < 1.f,
                  "vit_embed_bwd: bad args");
  hipLaunchKernelGGL(vit_embed_bwd_kernel, dim3(VD / 64), dim3(512), 0, as_stream(stream), dtok, B, npos, drop_p, seed,
                     seed_off, dy, dcls, dpos);
  return launch_status("vit_embed_bwd");
}

// ---------------------------------------------------------------- tall-K, few-row GEMM
// C[M][N] = A[M][K] (bf16, row stride lda) x W[N][K]^T (fp32 master, rounded to bf16 as
// ewvit_gemm rounds it) + bias, M <= 64, N % 256 == 0, K % 256 == 0 — the patch_to_embedding
// forward (sfe.py:155: 64 frames x 62720 x 512, 128 MB of fp32 weight).  The generic split-K
// GEMM tiles it 64 x 64 and reads the 8 MB activation 8 times (54 us isolated, 69 us in the
// step); here a workgroup owns a 256-wide K slice and 256 columns (each W element read once, the
// K slice of A once per wave from L2) and leaves a fp32 partial; the reduce adds the slices in
// a fixed order with the bias.
namespace ewvit {
__global__ __launch_bounds__(256) void tallk_part_kernel(const bf16_t *A, int64_t lda, const float *W, int64_t K,
                                                         int M, int N, float *part) {
  const int s = blockIdx.x, ch = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int64_t k0 = (int64_t)s * 256;
  const int c0 = ch * 256 + w * 64;
  vf4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = vf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int sb = 0; sb < 8; sb += 2) {
    vb8 af[2][4], bf[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t k = k0 + (sb + u) * 32 + lq * 8;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int r = t * 16 + li;
        af[u][t] = ld8b(A + (int64_t)rclamp(r, M) * lda + k);
        if (r >= M) af[u][t] = zero8();
        float v[8];
        ld8f(W + (int64_t)(c0 + t * 16 + li) * K + k, v);
        bf[u][t] = pack8(v);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mma(af[u][i], bf[u][j], acc[i][j]);
  }
  float *dst = part + (int64_t)s * 64 * N;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[(int64_t)(i * 16 + lq * 4 + e) * N + c0 + j * 16 + li] = acc[i][j][e];
}

// out[r][c] = bias[c] + sum_s part[s][r][c]: a workgroup per 64 outputs of one row, 4 slice
// quarters per output (8 loads in flight per thread), quarters added in order in LDS
__global__ __launch_bounds__(256) void tallk_reduce_kernel(const float *part, int S, int M, int N, const float *bias,
                                                           float *C, int64_t ldc) {
  __shared__ float red[4][64];
  const int o = blockIdx.x * 64 + (threadIdx.x & 63), q = threadIdx.x >> 6;
  const int r = o / N, c = o % N;
  const int sq = (S + 3) / 4, s0 = q * sq, s1 = s0 + sq < S ? s0 + sq : S;
  float a = 0.f;
  int sidx = s0;
  for (; sidx + 8 <= s1; sidx += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[((int64_t)(sidx + u) * 64 + r) * N + c];
#pragma unroll
    for (int u = 0; u < 8; ++u) a += v[u];
  }
  for (; sidx < s1; ++sidx) a += part[((int64_t)sidx * 64 + r) * N + c];
  red[q][threadIdx.x & 63] = a;
  __syncthreads();
  if (q == 0 && r < M) {
    const int l = threadIdx.x;
    C[(int64_t)r * ldc + c] = (((red[0][l] + red[1][l]) + red[2][l]) + red[3][l]) + (bias ? bias[c] : 0.f);
  }
}
}  // namespace ewvit

extern "C" int64_t ewvit_gemm_tallk_workspace(int64_t M, int64_t N, int64_t K) {
  return (K / 256) * 64 * N * (int64_t)sizeof(float);
}

extern "C" int ewvit_gemm_tallk(const void *A, int64_t lda, const float *W, const float *bias, float *C, int64_t ldc,
                                int64_t M, int64_t N, int64_t K, float *workspace, void *stream) {
  EWVIT_CHECK_ARG(A && W && C && workspace, "gemm_tallk: null pointer");
  EWVIT_CHECK_ARG(M >= 1 && M <= 64 && N % 256 == 0 && K % 256 == 0 && K / 256 <= 65535 && lda % 8 == 0 &&
                      lda >= K && ldc >= N,
                  "gemm_tallk: M=%lld N=%lld K=%lld outside its shape class", (long long)M, (long long)N,
                  (long long)K);
  hipStream_t st = as_stream(stream);
  const int S = (int)(K / 256);
  hipLaunchKernelGGL(tallk_part_kernel, dim3((unsigned)S, (unsigned)(N / 256)), dim3(256), 0, st, (const bf16_t *)A, lda,
                     W, K, (int)M, (int)N, workspace);
  if (int rc = launch_status("gemm_tallk")) return rc;
  hipLaunchKernelGGL(tallk_reduce_kernel, dim3((unsigned)(64 * N / 64)), dim3(256), 0, st, workspace, S, (int)M, (int)N,
                     bias, C, ldc);
  return launch_status("gemm_tallk reduce");
}
