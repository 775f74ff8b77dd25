// The DAMA frame head (gfx950): everything of DAMA._process_frame after its two branches
// (reference network/dama.py:143-169) —
//   * BidirectionalCrossTransformer, depth 2 (dama.py:56-78, 116-122): per layer
//     s = s + CA_s(LN(s), f); f = f + CA_f(LN(f), s) with CrossAttention (dama.py:15-53):
//     kv_include_self, 4 heads of 32, to_q / to_kv without bias, to_out + Dropout(0.1);
//   * fusion_gate (dama.py:124-128, 152-153): Conv3x3(256 -> 128, pad 1) on the 1x1 map —
//     only the centre tap meets data — + BatchNorm2d (batch statistics over the chunk's
//     frames in training) + ReLU;
//   * gate_net (dama.py:105-113, 156-157): Linear(256 -> 64) + ReLU + Dropout(0.1) +
//     Linear(64 -> 3) + Softmax;
//   * the 3-way weighted sum (dama.py:159-163).
// The token streams are one token per frame (the 1x1 maps of both branches), so the head is
// [N <= 64, 128] matrices against 0.3 M parameters: ~90 small launches in the module-by-module
// form.  Every frame is independent up to the fusion BatchNorm, so the work splits as
//   forward   head_fwd_rows_kernel   one workgroup per FG frames: the 4 attention blocks, the
//                                    fusion conv and the gate's first layer, activations held
//                                    in LDS, what the backward needs written to the workspace;
//             head_fwd_tail_kernel   one workgroup: the BatchNorm over the frames (running
//                                    statistics), ReLU, the gate's second layer + softmax and
//                                    the weighted sum;
//   backward  head_bwd_tail_kernel   one workgroup: weighted sum, gate and BatchNorm backward
//                                    (the affine gradients);
//             head_bwd_rows_kernel   one workgroup per FG frames: the fusion conv / gate input
//                                    gradients and the attention blocks in reverse, back to the
//                                    two branch inputs;
//             head_bwd_weight_kernel a grid: every weight / bias gradient as fp32 dot products
//                                    over the frames (the fusion conv's 8 dead taps written 0).
// GEMMs on v_mfma_f32_16x16x32_bf16 (bf16 operands, fp32 accumulation, as the module path's
// ewvit_gemm rounds them): a workgroup's 16 frame rows are one MFMA row tile; its 8 waves take
// the 16-column output tiles of a phase, each loading the B fragments of two tiles straight
// from the fp32 master weights (rounded in registers) before their MFMAs.  Per-row statistics
// (LayerNorm, softmax, attention) and every accumulation in fp32.
#include "common.h"
#include "mx8.h"

namespace ewvit {

typedef ewvit_head_ca HeadCA;
typedef ewvit_head_params HeadParams;

constexpr int HD = 128;           // dama dim
constexpr int HN = 64;            // frames per chunk, at most (pos_embedding rows)
constexpr int FG = 16;            // frames per workgroup of the per-frame kernels (one row tile)
constexpr int HT = 512;           // threads per workgroup (8 waves)
constexpr int HKP = 256 + 8;      // LDS row pitch (bf16) of an activation operand, K <= 256
constexpr int HKC = 384 + 8;      // ... K <= 384
constexpr int HSITE = 1 << 20;    // dropout counter stride between sites
constexpr float HSCALE = 0.17677669529663687f;   // 32^-0.5 (dama.py:30)

typedef __attribute__((ext_vector_type(8))) __bf16 hbf16x8;
typedef __attribute__((ext_vector_type(4))) float hf32x4;

// ---- workspace layout (floats); rows are frames n < HN.  Pointers are computed from the base
// (no arrays of pointers: a runtime block index would put such an array in scratch memory).
constexpr int64_t W_BLK = HN * HD + 2 * HN + HN * HD + HN * 512 + HN * 8 + HN * HD;   // per attention block
constexpr int64_t W_BLK0 = 6 * HN * HD;
constexpr int64_t W_FUS0 = W_BLK0 + 4 * W_BLK;
constexpr int64_t W_BBLK = HN * HD + HN * HD + HN * 512 + HN * HD;                    // per block, backward
constexpr int64_t W_BBLK0 = W_FUS0 + HN * HD + 2 * HD + HN * HD + HN * 64 + HN * 4;
constexpr int64_t W_TAIL0 = W_BBLK0 + 4 * W_BBLK;
constexpr int64_t W_TOTAL = W_TAIL0 + HN * HD + HN * 64 + HN * 4 + 2 * HN * HD + HD * 256 + 256;   // + 128 trace stamps

struct HeadWs {
  float *b;
  // states s0, f0, s1, f1, s2, f2   [N][128]
  __device__ float *st(int i) const { return b + (int64_t)i * HN * HD; }
  // per attention block: LayerNorm output [N][128], its mean / rstd [N], to_q [N][128], to_kv of
  // (self, context) [N][2][256] (k: 0..127, v: 128..255), softmax weights [N][4][2], attention
  // output [N][128]
  __device__ float *xn(int i) const { return b + W_BLK0 + i * W_BLK; }
  __device__ float *mu(int i) const { return xn(i) + HN * HD; }
  __device__ float *rs(int i) const { return mu(i) + HN; }
  __device__ float *q(int i) const { return rs(i) + HN; }
  __device__ float *kv(int i) const { return q(i) + HN * HD; }
  __device__ float *at(int i) const { return kv(i) + HN * 512; }
  __device__ float *o(int i) const { return at(i) + HN * 8; }
  __device__ float *yfg() const { return b + W_FUS0; }            // fusion conv out, no bias [N][128]
  __device__ float *bnm() const { return yfg() + HN * HD; }       // BatchNorm mean [128]
  __device__ float *bni() const { return bnm() + HD; }            // and invstd [128]
  __device__ float *fus() const { return bni() + HD; }            // ReLU(BN(yfg + bias)) [N][128]
  __device__ float *h1() const { return fus() + HN * HD; }        // gate first layer, no bias [N][64]
  __device__ float *gw() const { return h1() + HN * 64; }         // softmax gate [N][4] (3 used)
  // backward, per block: d LayerNorm output, d q, d kv, d to_out pre-dropout output
  __device__ float *dxn(int i) const { return b + W_BBLK0 + i * W_BBLK; }
  __device__ float *dq(int i) const { return dxn(i) + HN * HD; }
  __device__ float *dkv(int i) const { return dq(i) + HN * HD; }
  __device__ float *dpre(int i) const { return dkv(i) + HN * 512; }
  __device__ float *dy() const { return b + W_TAIL0; }            // d fusion conv out [N][128]
  __device__ float *dh1() const { return dy() + HN * HD; }        // d gate pre-activation [N][64]
  __device__ float *dz2() const { return dh1() + HN * 64; }       // d gate logits [N][4]
  __device__ float *ds(int i) const { return dz2() + HN * 4 + (int64_t)i * HN * HD; }  // d s2, d f2
  __device__ float *wc() const { return ds(2); }                  // (unused; kept for the layout)
};

__host__ __device__ inline int64_t head_ws_floats() { return W_TOTAL; }
// EWVIT_HEAD_TRACE builds: workgroup 0's phase boundaries as wall-clock stamps (100 MHz) in the
// workspace's last 128 slots — fwd rows 0.., fwd tail 32.., bwd tail 48.., bwd rows 64..
#ifdef EWVIT_HEAD_TRACE
#define HTR(k)                                                                                        \
  do {                                                                                                \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                                          \
      reinterpret_cast<uint64_t *>(ws_base + W_TOTAL - 256)[(k)] = wall_clock64();                    \
  } while (0)
#else
#define HTR(k) do { (void)(k); } while (0)
#endif
__device__ inline HeadWs head_ws(float *b) { return HeadWs{b}; }

// The rows kernels' weights as bf16, packed once per call by ewvit_head_fwd (head_pack_kernel):
// per attention block i, to_q / to_kv / to_out in their own layout (forward B fragments, k
// contiguous) and transposed (backward B fragments: the input gradient reduces over the
// weight's output index); the gate's first layer and the fusion conv's centre tap transposed.
// The fp32 masters round to the same bf16 values the fragment loaders produced from them.
constexpr int64_t HP_Q = 0, HP_KV = HP_Q + HD * HD, HP_O = HP_KV + 2 * HD * HD, HP_QT = HP_O + HD * HD,
                  HP_KVT = HP_QT + HD * HD, HP_OT = HP_KVT + 2 * HD * HD, HP_BLK = HP_OT + HD * HD;
constexpr int64_t HP_G1T = 4 * HP_BLK, HP_WCT = HP_G1T + 256 * 64, HP_TOTAL = HP_WCT + 256 * HD;
__device__ __forceinline__ hbf16x8 h_ld8(const bf16_t *p) { return *reinterpret_cast<const hbf16x8 *>(p); }

// attention blocks in forward order: 0 = layer 0 s, 1 = layer 0 f, 2 = layer 1 s, 3 = layer 1 f
// block i reads state x = st[xin(i)] and context ctx = st[cin(i)], writes st[xout(i)]
__device__ __forceinline__ int h_xin(int i) { return (i >> 1) * 2 + (i & 1); }        // s0 f0 s1 f1
__device__ __forceinline__ int h_xout(int i) { return (i >> 1) * 2 + 2 + (i & 1); }   // s1 f1 s2 f2
__device__ __forceinline__ int h_cin(int i) { return (i & 1) ? (i >> 1) * 2 + 2 : (i >> 1) * 2 + 1; }  // f0 s1 f1 s2

// sd: the launch's effective seed, step_seed(p.seed, p.seed_off), read once per kernel
__device__ __forceinline__ float h_drop(uint64_t sd, int site, int n, int c, float prob) {
  if (prob <= 0.f) return 1.f;
  const float u = uniform01(sd, (uint64_t)site * HSITE + (uint64_t)n * 256 + c);
  return u >= prob ? 1.f / (1.f - prob) : 0.f;
}

__device__ __forceinline__ hbf16x8 h_pack8(const float *v) {
  hbf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (__bf16)v[e];
  return r;
}
// B fragment from a weight with k contiguous (nn.Linear forward: W[col][k])
__device__ __forceinline__ hbf16x8 h_frag_rowk(const float *w) {
  const float4 a = *reinterpret_cast<const float4 *>(w), b = *reinterpret_cast<const float4 *>(w + 4);
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return h_pack8(v);
}
// ... with k strided (input gradient: B(k, col) = W[k * ld + col])
__device__ __forceinline__ hbf16x8 h_frag_colk(const float *w, int64_t ld) {
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = w[e * ld];
  return h_pack8(v);
}

// raw workgroup barrier: this wave's LDS traffic retired (lgkmcnt), its global loads left in
// flight (the fence of __syncthreads() would drain them with vmcnt(0)); the phases of the
// per-frame kernels exchange data through LDS only
__device__ __forceinline__ void h_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// 16-row GEMM tiles.  A phase's output is split into 16-column tiles; tile t = w + 8u goes to
// wave w.  g16_load issues the B fragments (frag(t, s, c, k0): column c of the tile, k = k0 ..
// k0 + 7, the first nk(t) 32-wide k-steps) — a phase EARLY, so their L2 latency overlaps the
// LDS-only work in between; g16_mma multiplies them with the tiles' activations A (LDS bf16
// rows 0..15, pitch ap) and hands every output element to epi(t, row, c, v).
template <int NU, int KS, class NkF, class FragF>
__device__ __forceinline__ void g16_load(hbf16x8 (&b)[NU][KS], int ntiles, NkF nk, FragF frag) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, kq = (lane >> 4) * 8;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int t = w + 8 * u;
    if (t < ntiles) {
      const int n = nk(t);
#pragma unroll
      for (int s = 0; s < KS; ++s)
        if (s < n) b[u][s] = frag(t, s, c, s * 32 + kq);
    }
  }
}
template <int NU, int KS, class NkF, class AF, class EpiF>
__device__ __forceinline__ void g16_mma(const hbf16x8 (&b)[NU][KS], int ntiles, NkF nk, AF afn, EpiF epi) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, kq = (lane >> 4) * 8;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int t = w + 8 * u;
    if (t >= ntiles) break;
    const int n = nk(t);
    const bf16_t *A;
    int ap;
    afn(t, A, ap);
    hf32x4 acc = hf32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s)
      if (s < n) {
        const hbf16x8 af = *reinterpret_cast<const hbf16x8 *>(A + c * ap + s * 32 + kq);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, b[u][s], acc, 0, 0, 0);
      }
    // C/D map: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
    for (int r = 0; r < 4; ++r) epi(t, (lane >> 4) * 4 + r, c, acc[r]);
    __builtin_amdgcn_sched_barrier(0);   // one tile's operands live at a time (register budget)
  }
}

// MXFP8 forms (configs[4]): the attention blocks' weights from the MX pack (one 128-wide K step
// per MxFrag), the activations block-quantized from their bf16 LDS rows in registers
// (mx_quant).  Image m of block i: 0 Wq [128][128], 1 Wq^T, 2 Wkv [256][128], 3 Wkv^T [128][256],
// 4 Wo, 5 Wo^T — each e4m3 [rows][cols] + E8M0 [rows][cols / 32] (blocks along the row, the K of
// the GEMM that reads it).
__host__ __device__ inline void hmx_dims(int m, int &rows, int &cols) {
  rows = m == 2 ? 2 * HD : HD;
  cols = m == 3 ? 2 * HD : HD;
}
__host__ __device__ inline int64_t hmx_img(int m) {
  int64_t o = 0;
  for (int j = 0; j < m; ++j) {
    int r, c;
    hmx_dims(j, r, c);
    o += (int64_t)r * c + (int64_t)r * (c / 32);
  }
  return o;
}
constexpr int64_t HMX_BLK = 4 * HD * HD + 4 * HD * (HD / 32) + 2 * (2 * HD * HD + 2 * HD * (HD / 32));
struct HMxW {
  const uint8_t *d, *s;
  int K;
  __device__ __forceinline__ MxFrag frag(int row, int kstep) const {
    return mx_load(d + (int64_t)row * K, kstep, s + (int64_t)row * (K / 32));
  }
};
__device__ __forceinline__ HMxW hmx(const void *pk, int blk, int m) {
  int r, c;
  hmx_dims(m, r, c);
  const uint8_t *b = reinterpret_cast<const uint8_t *>(pk) + blk * HMX_BLK + hmx_img(m);
  return HMxW{b, b + (int64_t)r * c, c};
}
template <int NU, int KS, class NkF, class FragF>
__device__ __forceinline__ void g16_load_mx(MxFrag (&b)[NU][KS], int ntiles, NkF nk, FragF frag) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int t = w + 8 * u;
    if (t < ntiles) {
      const int n = nk(t);
#pragma unroll
      for (int s = 0; s < KS; ++s)
        if (s < n) b[u][s] = frag(t, s, c);
    }
  }
}
// A rows 0..15 of the tile from LDS (bf16, pitch ap), block-quantized per 128-wide K step
template <int NU, int KS, class NkF, class AF, class EpiF>
__device__ __forceinline__ void g16_mma_mx(const MxFrag (&b)[NU][KS], int ntiles, NkF nk, AF afn, EpiF epi) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int t = w + 8 * u;
    if (t >= ntiles) break;
    const int n = nk(t);
    const bf16_t *A;
    int ap;
    afn(t, A, ap);
    hf32x4 acc = hf32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s)
      if (s < n) {
        float v[32];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const hbf16x8 x = *reinterpret_cast<const hbf16x8 *>(A + c * ap + s * 128 + (hh ? mx_k1(lane) : mx_k0(lane)) + 8 * q);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[hh * 16 + q * 8 + e] = (float)x[e];
          }
        acc = mx_mma(mx_quant(v), b[u][s], acc);
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) epi(t, (lane >> 4) * 4 + r, c, acc[r]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

extern __shared__ __attribute__((aligned(16))) unsigned char h_smem[];

// ---------------------------------------------------------------- forward, per frame group
// A phase issues all of its weight fragments before its MFMAs (one L2 round trip per phase);
// between them the phases touch LDS only (the small parameter vectors are staged there), so no
// other global load waits behind the fragments.
template <bool MX>
__global__ __launch_bounds__(HT) void head_fwd_rows_kernel(HeadParams p, const float *s0, const float *f0,
                                                           float *ws_base, float *s_out, float *f_out, int N) {
  int trk = 0;
  HTR(trk++);
  const uint64_t sd = step_seed(p.seed, p.seed_off);
  float *st = reinterpret_cast<float *>(h_smem);                 // [6][FG][HD]
  float *qs = st + 6 * FG * HD;                                  // [FG][HD]
  float *kvs = qs + FG * HD;                                     // [FG][2][256]
  bf16_t *A1 = reinterpret_cast<bf16_t *>(kvs + FG * 512);       // [FG][HKP]
  bf16_t *A2 = A1 + FG * HKP;                                    // [FG][HKP]
  float *vec = reinterpret_cast<float *>(A2 + FG * HKP);         // [4][3][HD]: LN gamma, beta, to_out bias
  const HeadWs ws{ws_base};
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g0 = blockIdx.x * FG, nr = N - g0 < FG ? N - g0 : FG;
  int bi = 0;                                                    // the block the fragment loaders read
  auto nk4 = [](int) { return 4; };
  // to_q (8 tiles) and to_kv of the self token and of the context token (16 + 16 tiles)
  const bf16_t *pk = reinterpret_cast<const bf16_t *>(p.packed);
  auto frag_qkv = [&](int t, int s, int c, int k0) {
    const bf16_t *wr = t < 8 ? pk + bi * HP_BLK + HP_Q + (int64_t)(t * 16 + c) * HD
                             : pk + bi * HP_BLK + HP_KV + (int64_t)((t < 24 ? t - 8 : t - 24) * 16 + c) * HD;
    return h_ld8(wr + k0);
  };
  auto frag_o = [&](int t, int s, int c, int k0) { return h_ld8(pk + bi * HP_BLK + HP_O + (int64_t)(t * 16 + c) * HD + k0); };
  hbf16x8 bA[5][4], bO[1][4];
  MxFrag mA[5][1], mO[1][1];
  auto nk1 = [](int) { return 1; };
  auto mfrag_qkv = [&](int t, int, int c) {
    return t < 8 ? hmx(p.packed_mx, bi, 0).frag(t * 16 + c, 0) : hmx(p.packed_mx, bi, 2).frag((t < 24 ? t - 8 : t - 24) * 16 + c, 0);
  };
  auto mfrag_o = [&](int t, int, int c) { return hmx(p.packed_mx, bi, 4).frag(t * 16 + c, 0); };
  for (int e = tid; e < 4 * 3 * HD; e += HT) {
    const int i = e / (3 * HD), j = (e / HD) % 3, c = e % HD;
    vec[e] = (j == 0 ? p.ca[i].ln_w : j == 1 ? p.ca[i].ln_b : p.ca[i].bo)[c];
  }
#pragma unroll
  for (int j = 0; j < FG * HD / HT; ++j) {
    const int e = tid + j * HT, r = e >> 7;
    const int64_t gi = (int64_t)g0 * HD + (r < nr ? e : 0);     // clamped: the loads issue together
    const float a = s0[gi], b = f0[gi];
    st[e] = r < nr ? a : 0.f;
    st[FG * HD + e] = r < nr ? b : 0.f;
    if (r < nr) { ws.st(0)[gi] = a; ws.st(1)[gi] = b; }
  }
  h_bar();
    HTR(trk++);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float *lnw = vec + i * 3 * HD, *lnb = lnw + HD, *bo = lnb + HD;
    const float *x = st + h_xin(i) * FG * HD, *ctx = st + h_cin(i) * FG * HD;
    // LayerNorm (two-pass, biased variance, eps inside the rsqrt as torch): one wave per row
    for (int r = w; r < FG; r += 8) {
      const float v0 = x[r * HD + lane], v1 = x[r * HD + lane + 64];
      const float m = wave_sum(v0 + v1) * (1.f / HD);
      const float d0 = v0 - m, d1 = v1 - m;
      const float rs = rsqrtf(wave_sum(d0 * d0 + d1 * d1) * (1.f / HD) + p.ln_eps);
      const float y0 = d0 * rs * lnw[lane] + lnb[lane];
      const float y1 = d1 * rs * lnw[lane + 64] + lnb[lane + 64];
      A1[r * HKP + lane] = f2bf(y0);
      A1[r * HKP + lane + 64] = f2bf(y1);
      if (r < nr) {
        const int64_t n = g0 + r;
        ws.xn(i)[n * HD + lane] = y0;
        ws.xn(i)[n * HD + lane + 64] = y1;
        if (lane == 0) { ws.mu(i)[n] = m; ws.rs(i)[n] = rs; }
      }
    }
    for (int e = tid; e < FG * HD; e += HT) A2[(e >> 7) * HKP + (e & 127)] = f2bf(ctx[e]);
    bi = i;
    auto epi_qkv = [&](int t, int row, int c, float v) {
          const int64_t n = g0 + row;
          if (t < 8) {
            const int col = t * 16 + c;
            qs[row * HD + col] = v;
            if (row < nr) ws.q(i)[n * HD + col] = v;
          } else {
            const int tok = t >= 24, col = (t - (tok ? 24 : 8)) * 16 + c;
            kvs[row * 512 + tok * 256 + col] = v;
            if (row < nr) ws.kv(i)[n * 512 + tok * 256 + col] = v;
          }
        };
    auto afn_qkv = [&](int t, const bf16_t *&A, int &ap) { A = t < 24 ? A1 : A2; ap = HKP; };
    if constexpr (MX) {
      g16_load_mx(mA, 40, nk1, mfrag_qkv);
      h_bar();
      HTR(trk++);
      g16_mma_mx(mA, 40, nk1, afn_qkv, epi_qkv);
    } else {
      g16_load(bA, 40, nk4, frag_qkv);
      h_bar();
      HTR(trk++);
      g16_mma(bA, 40, nk4, afn_qkv, epi_qkv);
    }
    h_bar();
    HTR(trk++);
    // attention: 1 query x 2 keys per (frame, head); 4 lanes per pair, 8 dims each
    if (tid < FG * 16) {
      const int n = tid >> 4, h = (tid >> 2) & 3, d0 = h * 32 + (tid & 3) * 8;
      const float *q = qs + n * HD + d0, *k0 = kvs + n * 512 + d0, *k1 = k0 + 256;
      float e0 = 0.f, e1 = 0.f;
#pragma unroll
      for (int d = 0; d < 8; ++d) { e0 = fmaf(q[d], k0[d], e0); e1 = fmaf(q[d], k1[d], e1); }
      e0 += __shfl_xor(e0, 1); e0 += __shfl_xor(e0, 2);
      e1 += __shfl_xor(e1, 1); e1 += __shfl_xor(e1, 2);
      e0 *= HSCALE; e1 *= HSCALE;
      const float m = fmaxf(e0, e1);
      const float x0 = __expf(e0 - m), x1 = __expf(e1 - m);
      const float inv = 1.f / (x0 + x1);
      const float a0 = x0 * inv, a1 = x1 * inv;
      const bool live = n < nr;
      const int64_t gn = g0 + n;
      if (live && (tid & 3) == 0) { ws.at(i)[gn * 8 + h * 2] = a0; ws.at(i)[gn * 8 + h * 2 + 1] = a1; }
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        const float v = a0 * k0[128 + d] + a1 * k1[128 + d];
        A1[n * HKP + d0 + d] = f2bf(v);
        if (live) ws.o(i)[gn * HD + d0 + d] = v;
      }
    }
    if constexpr (MX) g16_load_mx(mO, 8, nk1, mfrag_o);
    else g16_load(bO, 8, nk4, frag_o);
    h_bar();
    HTR(trk++);
    // to_out + bias, dropout, residual (dama.py:50-53, 71-76)
    float *xnew = st + h_xout(i) * FG * HD;
    auto afn_o = [&](int t, const bf16_t *&A, int &ap) { A = A1; ap = HKP; };
    auto epi_o = [&](int t, int row, int c, float v) {
          const int col = t * 16 + c;
          const int64_t n = g0 + row;
          const float y = x[row * HD + col] + (v + bo[col]) * h_drop(sd, i, (int)n, col, p.p_ca);
          xnew[row * HD + col] = y;
          if (row < nr) ws.st(h_xout(i))[n * HD + col] = y;
        };
    if constexpr (MX) g16_mma_mx(mO, 8, nk1, afn_o, epi_o);
    else g16_mma(bO, 8, nk4, afn_o, epi_o);
    h_bar();
    HTR(trk++);
  }
  const float *s2 = st + 4 * FG * HD, *f2 = st + 5 * FG * HD;
  for (int e = tid; e < FG * HD; e += HT) {
    if ((e >> 7) >= nr) continue;
    s_out[(int64_t)g0 * HD + e] = s2[e];
    f_out[(int64_t)g0 * HD + e] = f2[e];
  }
  HTR(trk++);
}

// ---------------------------------------------------------------- forward, fusion conv + gate input
// fusion_gate centre tap W_c[o][k] = wfg[o * fg_so + k * fg_si + 4 * fg_tap] (8 column tiles) and
// the gate's first layer W1 [64][256] (4 tiles) over concat = [s2, f2] (dama.py:151), K = 256:
// one wave per (16 frames, 16 output columns), so the strided centre-tap reads spread over 32+
// CUs (the backward reads the tap transposed from the head pack, head_pack_kernel).
__global__ __launch_bounds__(64) void head_fwd_fuse_kernel(HeadParams p, float *ws_base, int N) {
  const HeadWs ws{ws_base};
  const int t = blockIdx.x % 12, gq = blockIdx.x / 12;
  const int lane = threadIdx.x, c = lane & 15, kq = (lane >> 4) * 8;
  const int n = gq * 16 + c;
  const int64_t nc = n < N ? n : 0;
  hbf16x8 af[8], bf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int k0 = s * 32 + kq;
    const float *src = (k0 < HD ? ws.st(4) + k0 : ws.st(5) + (k0 - HD)) + nc * HD;
    const float4 u = *reinterpret_cast<const float4 *>(src), v = *reinterpret_cast<const float4 *>(src + 4);
    const float m = n < N ? 1.f : 0.f;
    const float a[8] = {u.x * m, u.y * m, u.z * m, u.w * m, v.x * m, v.y * m, v.z * m, v.w * m};
    af[s] = h_pack8(a);
    if (t < 8) {
      const int o = t * 16 + c;
      float w[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) w[e] = p.wfg[(int64_t)o * p.fg_so + (int64_t)(k0 + e) * p.fg_si + 4 * p.fg_tap];
      bf[s] = h_pack8(w);
    } else {
      bf[s] = h_frag_rowk(p.g1w + (int64_t)((t - 8) * 16 + c) * 256 + k0);
    }
  }
  hf32x4 acc = hf32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s], bf[s], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = gq * 16 + (lane >> 4) * 4 + r;
    if (row >= N) continue;
    if (t < 8) ws.yfg()[(int64_t)row * HD + t * 16 + c] = acc[r];
    else ws.h1()[(int64_t)row * 64 + (t - 8) * 16 + c] = acc[r];
  }
}

// ---------------------------------------------------------------- forward, the frame-coupled tail
// thread (c = tid & 127, part = tid >> 7): frames n = part, part + 4, ...
__global__ __launch_bounds__(HT) void head_fwd_tail_kernel(HeadParams p, float *ws_base, float *fused_out, int N) {
  int trk = 32;
  HTR(trk++);
  const uint64_t sd = step_seed(p.seed, p.seed_off);
  float *fus = reinterpret_cast<float *>(h_smem);     // [HN][HD]
  float *h1 = fus + HN * HD;                         // [HN][64]  ReLU(h1 + b1) * dropout
  float *z = h1 + HN * 64;                           // [HN][4]
  float *red = z + HN * 4;                           // [4][HD]
  float *stat = red + 4 * HD;                        // mean [HD], invstd [HD]
  float *w2 = stat + 2 * HD;                         // gate W2 [3][64]
  const HeadWs ws{ws_base};
  const int tid = threadIdx.x, c = tid & 127, part = tid >> 7;
  if (tid < 3 * 64) w2[tid] = p.g2w[tid];
  constexpr int PN = HN / 4;
  float y[PN];
  const float bc = p.bfg[c];
#pragma unroll
  for (int j = 0; j < PN; ++j) {
    const int n = part + 4 * j;
    y[j] = n < N ? ws.yfg()[(int64_t)n * HD + c] + bc : 0.f;
  }
  if (p.training) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < PN; ++j) s += y[j];
    red[part * HD + c] = s;
    __syncthreads();
    HTR(trk++);
    const float m = ((red[c] + red[HD + c]) + (red[2 * HD + c] + red[3 * HD + c])) / (float)N;
    __syncthreads();
    HTR(trk++);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < PN; ++j)
      if (part + 4 * j < N) { const float d = y[j] - m; q = fmaf(d, d, q); }
    red[part * HD + c] = q;
    __syncthreads();
    HTR(trk++);
    if (part == 0) {
      const float qq = (red[c] + red[HD + c]) + (red[2 * HD + c] + red[3 * HD + c]);
      const float var = qq / (float)N;
      const float unb = N > 1 ? qq / (float)(N - 1) : var;
      stat[c] = m;
      stat[HD + c] = rsqrtf(var + p.bn_eps);
      p.bn_rm[c] = (1.f - p.bn_mom) * p.bn_rm[c] + p.bn_mom * m;
      p.bn_rv[c] = (1.f - p.bn_mom) * p.bn_rv[c] + p.bn_mom * unb;
      if (c == 0 && p.bn_nbt) p.bn_nbt[0] += 1;
    }
  } else if (part == 0) {
    stat[c] = p.bn_rm[c];
    stat[HD + c] = rsqrtf(p.bn_rv[c] + p.bn_eps);
  }
#pragma unroll
  for (int u = 0; u < HN * 64 / HT; ++u) {
    const int e = tid + u * HT, n = e >> 6, j = e & 63;
    const float h = ws.h1()[e < N * 64 ? e : 0] + p.g1b[j];
    if (e < N * 64) h1[e] = (h > 0.f ? h : 0.f) * h_drop(sd, 4, n, j, p.p_gate);
  }
  __syncthreads();
    HTR(trk++);
  const float m = stat[c], iv = stat[HD + c], gm = p.bn_w[c], bt = p.bn_b[c];
  if (part == 0) { ws.bnm()[c] = m; ws.bni()[c] = iv; }
#pragma unroll
  for (int j = 0; j < PN; ++j) {
    const int n = part + 4 * j;
    if (n < N) {
      const float v = (y[j] - m) * iv * gm + bt;
      const float r = v > 0.f ? v : 0.f;
      fus[n * HD + c] = r;
      ws.fus()[(int64_t)n * HD + c] = r;
    }
  }
  // gate_net second layer (dama.py:105-113): thread (n, o)
  if (tid < N * 4) {
    const int n = tid >> 2, o = tid & 3;
    if (o < 3) {
      float a = p.g2b[o];
#pragma unroll 8
      for (int j = 0; j < 64; ++j) a = fmaf(h1[n * 64 + j], w2[o * 64 + j], a);
      z[n * 4 + o] = a;
    }
  }
  __syncthreads();
    HTR(trk++);
  if (tid < N) {
    const int n = tid;
    const float z0 = z[n * 4], z1 = z[n * 4 + 1], z2 = z[n * 4 + 2];
    const float mx = fmaxf(z0, fmaxf(z1, z2));
    const float e0 = __expf(z0 - mx), e1 = __expf(z1 - mx), e2 = __expf(z2 - mx);
    const float inv = 1.f / (e0 + e1 + e2);
    z[n * 4] = e0 * inv; z[n * 4 + 1] = e1 * inv; z[n * 4 + 2] = e2 * inv;
    float *g = ws.gw() + n * 4;
    g[0] = e0 * inv; g[1] = e1 * inv; g[2] = e2 * inv; g[3] = 0.f;
  }
  __syncthreads();
    HTR(trk++);
  const float *s2 = ws.st(4), *f2 = ws.st(5);
#pragma unroll
  for (int u = 0; u < HN * HD / HT; ++u) {
    const int e = tid + u * HT, n = e >> 7, ec = e < N * HD ? e : 0;
    const float a = s2[ec], b = f2[ec];
    if (e < N * HD) fused_out[e] = z[n * 4] * a + z[n * 4 + 1] * b + z[n * 4 + 2] * fus[e];
  }
  HTR(trk++);
}

// ---------------------------------------------------------------- backward, the frame-coupled tail
__global__ __launch_bounds__(HT) void head_bwd_tail_kernel(HeadParams p, float *ws_base, const float *g_fused,
                                                           const float *g_s, const float *g_f, float *dbn_w,
                                                           float *dbn_b, int N) {
  int trk = 48;
  HTR(trk++);
  const uint64_t sd = step_seed(p.seed, p.seed_off);
  float *gws = reinterpret_cast<float *>(h_smem);    // [HN][4]
  float *dz = gws + HN * 4;                          // [HN][4]
  float *red = dz + HN * 4;                          // [4][2][HD]
  const HeadWs ws{ws_base};
  const int tid = threadIdx.x;
  for (int e = tid; e < N * 4; e += HT) gws[e] = ws.gw()[e];
  __syncthreads();
    HTR(trk++);
  const float *s2 = ws.st(4), *f2 = ws.st(5), *fu = ws.fus();
  // weighted sum (dama.py:159-163): the state gradients' direct part
#pragma unroll
  for (int u = 0; u < HN * HD / HT; ++u) {
    const int e = tid + u * HT, n = e >> 7, ec = e < N * HD ? e : 0;
    const float gf = g_fused[ec], gs = g_s[ec], gr = g_f[ec];
    if (e < N * HD) {
      ws.ds(0)[e] = gs + gws[n * 4] * gf;
      ws.ds(1)[e] = gr + gws[n * 4 + 1] * gf;
    }
  }
  // d gate weights -> softmax backward: thread (n, part of 16 channels), 8 lanes per frame
  {
    const int n = tid >> 3, pc = (tid & 7) * 16;
    float d0 = 0.f, d1 = 0.f, d2 = 0.f;
    if (n < N) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int64_t e = (int64_t)n * HD + pc + k;
        const float gf = g_fused[e];
        d0 = fmaf(gf, s2[e], d0); d1 = fmaf(gf, f2[e], d1); d2 = fmaf(gf, fu[e], d2);
      }
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
      d0 += __shfl_xor(d0, o); d1 += __shfl_xor(d1, o); d2 += __shfl_xor(d2, o);
    }
    if (n < N && (tid & 7) == 0) {
      const float *g = gws + n * 4;
      const float dot = g[0] * d0 + g[1] * d1 + g[2] * d2;
      const float z0 = g[0] * (d0 - dot), z1 = g[1] * (d1 - dot), z2 = g[2] * (d2 - dot);
      dz[n * 4] = z0; dz[n * 4 + 1] = z1; dz[n * 4 + 2] = z2;
      float *o = ws.dz2() + n * 4;
      o[0] = z0; o[1] = z1; o[2] = z2; o[3] = 0.f;
    }
  }
  __syncthreads();
    HTR(trk++);
  // gate_net: d h1 (pre-activation) = (dz2 W2) * dropout * relu'
#pragma unroll
  for (int u = 0; u < HN * 64 / HT; ++u) {
    const int e = tid + u * HT, n = e >> 6, j = e & 63;
    if (e >= N * 64) break;
    const float h = ws.h1()[e] + p.g1b[j];
    float d = 0.f;
#pragma unroll
    for (int o = 0; o < 3; ++o) d = fmaf(dz[n * 4 + o], p.g2w[o * 64 + j], d);
    ws.dh1()[e] = h > 0.f ? d * h_drop(sd, 4, n, j, p.p_gate) : 0.f;
  }
  // fusion BatchNorm + ReLU backward (batch statistics over the frames)
  const int c = tid & 127, part = tid >> 7;
  constexpr int PN = HN / 4;
  const float m = ws.bnm()[c], iv = ws.bni()[c], gam = p.bn_w[c], bc = p.bfg[c];
  float gr[PN], xh[PN], sg = 0.f, sgx = 0.f;
#pragma unroll
  for (int j = 0; j < PN; ++j) {
    const int n = part + 4 * j;
    gr[j] = 0.f; xh[j] = 0.f;
    if (n < N) {
      const int64_t e = (int64_t)n * HD + c;
      gr[j] = fu[e] > 0.f ? g_fused[e] * gws[n * 4 + 2] : 0.f;
      xh[j] = (ws.yfg()[e] + bc - m) * iv;
      sg += gr[j];
      sgx = fmaf(gr[j], xh[j], sgx);
    }
  }
  red[part * 2 * HD + c] = sg;
  red[part * 2 * HD + HD + c] = sgx;
  __syncthreads();
    HTR(trk++);
  const float SG = (red[c] + red[2 * HD + c]) + (red[4 * HD + c] + red[6 * HD + c]);
  const float SGX = (red[HD + c] + red[3 * HD + c]) + (red[5 * HD + c] + red[7 * HD + c]);
  if (part == 0) {
    if (dbn_w) dbn_w[c] = SGX;
    if (dbn_b) dbn_b[c] = SG;
  }
  const float a = SG / (float)N, b = SGX / (float)N;
#pragma unroll
  for (int j = 0; j < PN; ++j) {
    const int n = part + 4 * j;
    if (n < N)
      ws.dy()[(int64_t)n * HD + c] = p.training ? gam * iv * (gr[j] - a - xh[j] * b) : gam * iv * gr[j];
  }
  HTR(trk++);
}

// ---------------------------------------------------------------- backward, per frame group
// As in the forward, a phase issues its weight fragments before its MFMAs and the phases in
// between touch LDS only; a block's attention / LayerNorm operands (global) are loaded at its
// start, ahead of its first fragments.
template <bool MX>
__global__ __launch_bounds__(HT) void head_bwd_rows_kernel(HeadParams p, float *ws_base, float *ds0, float *df0,
                                                           int N) {
  int trk = 64;
  HTR(trk++);
  const uint64_t sd = step_seed(p.seed, p.seed_off);
  float *dS = reinterpret_cast<float *>(h_smem);     // [FG][HD]
  float *dF = dS + FG * HD;                          // [FG][HD]
  float *dO = dF + FG * HD;                          // [FG][HD]
  float *dxs = dO + FG * HD;                         // [FG][HD]
  bf16_t *Ac = reinterpret_cast<bf16_t *>(dxs + FG * HD);   // [FG][HKC]
  bf16_t *A3 = Ac + FG * HKC;                               // [FG][HKP]
  float *lnw = reinterpret_cast<float *>(A3 + FG * HKP);    // [4][HD] LayerNorm gamma
  const HeadWs ws{ws_base};
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g0 = blockIdx.x * FG, nr = N - g0 < FG ? N - g0 : FG;
  int bi = 3;
  auto nk4 = [](int) { return 4; };
  auto nk6 = [](int) { return 6; };
  auto nkx = [](int t) { return t < 8 ? 12 : 8; };
  // d concat = dy Wc + dh1 W1 (K = 128 + 64): 16 tiles of concat columns
  const bf16_t *pk = reinterpret_cast<const bf16_t *>(p.packed);
  auto frag_c = [&](int t, int s, int c, int k0) {
    const int col = t * 16 + c;
    if (s < 4) return h_ld8(pk + HP_WCT + (int64_t)col * HD + k0);           // Wc^T [256][128]
    return h_ld8(pk + HP_G1T + (int64_t)col * 64 + (k0 - HD));                // W1^T [256][64]
  };
  auto frag_o = [&](int t, int s, int c, int k0) {
    return h_ld8(pk + bi * HP_BLK + HP_OT + (int64_t)(t * 16 + c) * HD + k0);
  };
  // d xn = [dq | dkv_self] [Wq ; Wkv] (8 tiles, K = 384); d ctx = dkv_ctx Wkv (8 tiles, K = 256)
  auto frag_x = [&](int t, int s, int c, int k0) {
    const int col = (t & 7) * 16 + c;
    if (t < 8 && s < 4) return h_ld8(pk + bi * HP_BLK + HP_QT + (int64_t)col * HD + k0);
    const int kk = t < 8 ? k0 - HD : k0;
    return h_ld8(pk + bi * HP_BLK + HP_KVT + (int64_t)col * (2 * HD) + kk);
  };
  hbf16x8 bC[2][6], bO[1][4], bX[2][12];
  MxFrag mO[1][1], mX[2][3];
  auto nk1 = [](int) { return 1; };
  auto nkxm = [](int t) { return t < 8 ? 3 : 2; };
  auto mfrag_o = [&](int t, int, int c) { return hmx(p.packed_mx, bi, 5).frag(t * 16 + c, 0); };
  auto mfrag_x = [&](int t, int s, int c) {
    const int col = (t & 7) * 16 + c;
    if (t < 8 && s == 0) return hmx(p.packed_mx, bi, 1).frag(col, 0);
    return hmx(p.packed_mx, bi, 3).frag(col, (t < 8 ? s - 1 : s) * 128);
  };
  for (int e = tid; e < 4 * HD; e += HT) lnw[e] = p.ca[e >> 7].ln_w[e & 127];
#pragma unroll
  for (int u = 0; u < FG * HD / HT; ++u) {
    const int e = tid + u * HT, r = e >> 7, c = e & 127;
    const int64_t gi = (int64_t)g0 * HD + (r < nr ? e : 0);     // clamped: the loads issue together
    const float a = ws.ds(0)[gi], b = ws.ds(1)[gi], d = ws.dy()[gi];
    dS[e] = r < nr ? a : 0.f;
    dF[e] = r < nr ? b : 0.f;
    Ac[r * HKC + c] = f2bf(r < nr ? d : 0.f);
  }
#pragma unroll
  for (int u = 0; u < FG * 64 / HT; ++u) {
    const int e = tid + u * HT, r = e >> 6, j = e & 63;
    const float d = ws.dh1()[(int64_t)(g0 + (r < nr ? r : 0)) * 64 + j];
    Ac[r * HKC + HD + j] = f2bf(r < nr ? d : 0.f);
  }
  g16_load(bC, 16, nk6, frag_c);
  h_bar();
    HTR(trk++);
  g16_mma(
      bC, 16, nk6, [&](int t, const bf16_t *&A, int &ap) { A = Ac; ap = HKC; },
      [&](int t, int row, int c, float v) {
        const int col = t * 16 + c;
        if (col < HD) dS[row * HD + col] += v;
        else dF[row * HD + col - HD] += v;
      });
  h_bar();
    HTR(trk++);
  // the attention blocks in reverse (3: layer 1 f, 2: layer 1 s, 1: layer 0 f, 0: layer 0 s)
  const int an = tid >> 4, ah = (tid >> 2) & 3, ad0 = ah * 32 + (tid & 3) * 8;   // attention lane roles
  const bool alive = tid < FG * 16 && an < nr;
  const int64_t agn = g0 + (alive ? an : 0);
#pragma unroll
  for (int i = 3; i >= 0; --i) {
    float *dX = (i & 1) ? dF : dS;        // the block's own stream: grad of x_new, becomes grad of x
    float *dC = (i & 1) ? dS : dF;        // the context stream
    // this block's attention operands and LayerNorm rows, issued first
    float qv[8], kv0[8], kv1[8], vv0[8], vv1[8], a0 = 0.f, a1 = 0.f;
    if (alive) {
      const float *q = ws.q(i) + agn * HD + ad0, *k0 = ws.kv(i) + agn * 512 + ad0, *k1 = k0 + 256;
#pragma unroll
      for (int d = 0; d < 8; ++d) { qv[d] = q[d]; kv0[d] = k0[d]; kv1[d] = k1[d]; vv0[d] = k0[128 + d]; vv1[d] = k1[128 + d]; }
      a0 = ws.at(i)[agn * 8 + ah * 2];
      a1 = ws.at(i)[agn * 8 + ah * 2 + 1];
    } else {
#pragma unroll
      for (int d = 0; d < 8; ++d) { qv[d] = 0.f; kv0[d] = 0.f; kv1[d] = 0.f; vv0[d] = 0.f; vv1[d] = 0.f; }
    }
    float lx[2][2], lm[2], lr[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = w + 8 * u;
      const int64_t n = g0 + (r < nr ? r : 0);
      const float *x = ws.st(h_xin(i)) + n * HD;
      lx[u][0] = x[lane]; lx[u][1] = x[lane + 64];
      lm[u] = ws.mu(i)[n]; lr[u] = ws.rs(i)[n];
    }
    // to_out backward: dpre = dX * dropout; d o = dpre Wo
    for (int e = tid; e < FG * HD; e += HT) {
      const int r = e >> 7, c = e & 127;
      const float d = dX[e] * h_drop(sd, i, g0 + r, c, p.p_ca);
      Ac[r * HKC + c] = f2bf(d);
      if (r < nr) ws.dpre(i)[(int64_t)g0 * HD + e] = d;
    }
    bi = i;
    if constexpr (MX) g16_load_mx(mO, 8, nk1, mfrag_o);
    else g16_load(bO, 8, nk4, frag_o);
    h_bar();
    HTR(trk++);
    auto afn_c = [&](int t, const bf16_t *&A, int &ap) { A = Ac; ap = HKC; };
    auto epi_do = [&](int t, int row, int c, float v) { dO[row * HD + t * 16 + c] = v; };
    if constexpr (MX) g16_mma_mx(mO, 8, nk1, afn_c, epi_do);
    else g16_mma(bO, 8, nk4, afn_c, epi_do);
    h_bar();
    HTR(trk++);
    // attention backward: 4 lanes per (frame, head), 8 dims each
    if (tid < FG * 16) {
      float dov[8];
#pragma unroll
      for (int d = 0; d < 8; ++d) dov[d] = dO[an * HD + ad0 + d];
      float da0 = 0.f, da1 = 0.f;
#pragma unroll
      for (int d = 0; d < 8; ++d) { da0 = fmaf(dov[d], vv0[d], da0); da1 = fmaf(dov[d], vv1[d], da1); }
      da0 += __shfl_xor(da0, 1); da0 += __shfl_xor(da0, 2);
      da1 += __shfl_xor(da1, 1); da1 += __shfl_xor(da1, 2);
      const float dot = a0 * da0 + a1 * da1;
      const float dl0 = a0 * (da0 - dot) * HSCALE, dl1 = a1 * (da1 - dot) * HSCALE;
      float *wq_ = ws.dq(i) + agn * HD + ad0, *wk0 = ws.dkv(i) + agn * 512 + ad0, *wk1 = wk0 + 256;
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        const float dq = dl0 * kv0[d] + dl1 * kv1[d];
        const float dk0 = dl0 * qv[d], dk1 = dl1 * qv[d];
        const float dv0 = a0 * dov[d], dv1 = a1 * dov[d];
        // [dq | dk_self | dv_self] (K = 384, against [Wq ; Wkv]) and [dk_ctx | dv_ctx] (K = 256)
        Ac[an * HKC + ad0 + d] = f2bf(dq);
        Ac[an * HKC + HD + ad0 + d] = f2bf(dk0);
        Ac[an * HKC + 2 * HD + ad0 + d] = f2bf(dv0);
        A3[an * HKP + ad0 + d] = f2bf(dk1);
        A3[an * HKP + HD + ad0 + d] = f2bf(dv1);
        if (alive) {
          wq_[d] = dq; wk0[d] = dk0; wk0[128 + d] = dv0; wk1[d] = dk1; wk1[128 + d] = dv1;
        }
      }
    }
    if constexpr (MX) g16_load_mx(mX, 16, nkxm, mfrag_x);
    else g16_load(bX, 16, nkx, frag_x);
    h_bar();
    HTR(trk++);
    auto afn_x = [&](int t, const bf16_t *&A, int &ap) {
          if (t < 8) { A = Ac; ap = HKC; } else { A = A3; ap = HKP; }
        };
    auto epi_x = [&](int t, int row, int c, float v) {
          const int col = (t & 7) * 16 + c;
          if (t < 8) {
            dxs[row * HD + col] = v;
            if (row < nr) ws.dxn(i)[(int64_t)(g0 + row) * HD + col] = v;
          } else {
            dC[row * HD + col] += v;
          }
        };
    if constexpr (MX) g16_mma_mx(mX, 16, nkxm, afn_x, epi_x);
    else g16_mma(bX, 16, nkx, afn_x, epi_x);
    h_bar();
    HTR(trk++);
    // LayerNorm backward into the own stream (which already holds the residual's gradient):
    // dxh = dxn * gamma, dx += rs * (dxh - mean(dxh) - xhat * mean(dxh * xhat))
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = w + 8 * u;
      if (r >= nr) break;
      float xh[2], g[2];
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int c = lane + 64 * v;
        xh[v] = (lx[u][v] - lm[u]) * lr[u];
        g[v] = dxs[r * HD + c] * lnw[i * HD + c];
      }
      const float a = wave_sum(g[0] + g[1]) * (1.f / HD);
      const float b = wave_sum(g[0] * xh[0] + g[1] * xh[1]) * (1.f / HD);
#pragma unroll
      for (int v = 0; v < 2; ++v) dX[r * HD + lane + 64 * v] += lr[u] * (g[v] - a - xh[v] * b);
    }
    h_bar();
    HTR(trk++);
  }
  for (int e = tid; e < FG * HD; e += HT) {
    if ((e >> 7) >= nr) continue;
    ds0[(int64_t)g0 * HD + e] = dS[e];
    df0[(int64_t)g0 * HD + e] = dF[e];
  }
  HTR(trk++);
}

// ---------------------------------------------------------------- backward, weights
// dW[o][k] = sum_frames D[n][o] X[n][k] as 16 x 16 MFMA tiles over the frames (K = 64 frames, two
// 32-frame k-steps; bf16 operands and fp32 accumulation as the module path's weight GEMMs),
// one wave per tile, 4 waves per workgroup:
//   per attention block i (256 tiles): Wq [128][128] = dq^T xn; Wkv [256][128] = dkv_self^T xn
//     + dkv_ctx^T ctx (four k-steps: both tokens); Wo [128][128] = dpre^T o;
//   the fusion conv's centre tap [128][256] = dy^T concat (128 tiles); gate W1 [64][256] =
//   dh1^T concat (64 tiles).
// Then the vectors (one quad of lanes per output, the frames split over the quad): bo, the
// LayerNorm gamma / beta, the fusion bias, b1, W2 [3][64] (dz2^T dropout(relu(h1 + b1))), b2; and
// the fusion conv's 8 dead taps, written as zeros.
struct HeadGrads {
  float *wq[4], *wkv[4], *wo[4], *bo[4], *lnw[4], *lnb[4];
  float *wfg; int64_t fg_so, fg_si, fg_tap;
  float *bfg, *g1w, *g1b, *g2w, *g2b;
};

constexpr int HW_TILES = 4 * 256 + 128 + 64;
constexpr int HW_TBLK = HW_TILES / 4;                       // workgroups of MFMA tiles
constexpr int HW_VEC = 4 * 3 * HD + HD + 64 + 3 * 64 + 3;   // vector outputs
constexpr int HW_VBLK = (HW_VEC + 63) / 64;                 // 64 outputs (quads) per workgroup
constexpr int64_t HW_DEAD = (int64_t)HD * 256 * 8;          // dead-tap zeros
constexpr int HW_DBLK = (int)((HW_DEAD + 255) / 256);

template <bool MX>
__global__ __launch_bounds__(256) void head_bwd_weight_kernel(HeadParams p, const float *ws_base, HeadGrads g, int N) {
  const uint64_t sd = step_seed(p.seed, p.seed_off);
  const HeadWs ws{const_cast<float *>(ws_base)};
  const int tid = threadIdx.x, lane = tid & 63;
  int blk = blockIdx.x;
  if (blk < HW_TBLK) {
    const int T = blk * 4 + (tid >> 6);
    // operands: D rows n (ld, column offset of o), X rows n (ld, column offset of k); a second
    // pair for the context token of Wkv; the output with its row stride
    const float *D0, *X0, *D1 = nullptr, *X1 = nullptr;
    int ldd, ldx, o0, k0;
    float *out;
    int64_t ldo, kstr = 1;
    if (T < 1024) {
      const int i = T >> 8, r = T & 255;
      if (r < 64) {
        D0 = ws.dq(i); ldd = HD; X0 = ws.xn(i); ldx = HD;
        o0 = (r >> 3) * 16; k0 = (r & 7) * 16; out = g.wq[i]; ldo = HD;
      } else if (r < 192) {
        const int rr = r - 64;
        D0 = ws.dkv(i); D1 = ws.dkv(i) + 256; ldd = 512; X0 = ws.xn(i); X1 = ws.st(h_cin(i)); ldx = HD;
        o0 = (rr >> 3) * 16; k0 = (rr & 7) * 16; out = g.wkv[i]; ldo = HD;
      } else {
        const int rr = r - 192;
        D0 = ws.dpre(i); ldd = HD; X0 = ws.o(i); ldx = HD;
        o0 = (rr >> 3) * 16; k0 = (rr & 7) * 16; out = g.wo[i]; ldo = HD;
      }
    } else if (T < 1024 + 128) {
      const int rr = T - 1024;
      D0 = ws.dy(); ldd = HD; o0 = (rr >> 4) * 16; k0 = (rr & 15) * 16;
      X0 = k0 < HD ? ws.st(4) + k0 : ws.st(5) + (k0 - HD); ldx = HD;
      out = g.wfg + 4 * g.fg_tap; ldo = g.fg_so; kstr = g.fg_si;
    } else {
      const int rr = T - 1024 - 128;
      D0 = ws.dh1(); ldd = 64; o0 = (rr >> 4) * 16; k0 = (rr & 15) * 16;
      X0 = k0 < HD ? ws.st(4) + k0 : ws.st(5) + (k0 - HD); ldx = HD;
      out = g.g1w; ldo = 256;
    }
    const bool xoff = T < 1024;         // X0 indexed with + k0 (the concat tiles point at their block)
    const int c = lane & 15, kq = (lane >> 4) * 8;
    auto dfrag = [&](const float *D, int s) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int n = s * 32 + kq + e;
        v[e] = n < N ? D[(int64_t)n * ldd + o0 + c] : 0.f;
      }
      return h_pack8(v);
    };
    auto xfrag = [&](const float *X, int s) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int n = s * 32 + kq + e;
        v[e] = n < N ? X[(int64_t)n * ldx + (xoff ? k0 : 0) + c] : 0.f;
      }
      return h_pack8(v);
    };
    const bool two = D1 != nullptr;
    if (MX && T < 1024) {
      // one 128-wide MX step over the frames: K = frames of the self token (k < 64) and, for
      // Wkv, of the context token (k >= 64); zero past N
      float va[32], vb[32];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int k = (hh ? mx_k1(lane) : mx_k0(lane)) + e, n = k & 63;
          const bool ok = n < N && (k < 64 || two);
          const float *D = k < 64 ? D0 : D1, *X = k < 64 ? X0 : X1;
          va[hh * 16 + e] = ok ? D[(int64_t)n * ldd + o0 + c] : 0.f;
          vb[hh * 16 + e] = ok ? X[(int64_t)n * ldx + k0 + c] : 0.f;
        }
      const hf32x4 acc = mx_mma(mx_quant(va), mx_quant(vb), hf32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(int64_t)(o0 + (lane >> 4) * 4 + r) * ldo + (int64_t)(k0 + c) * kstr] = acc[r];
      return;
    }
    const hbf16x8 a0 = dfrag(D0, 0), a1 = dfrag(D0, 1), b0 = xfrag(X0, 0), b1 = xfrag(X0, 1);
    hbf16x8 a2 = {}, a3 = {}, b2 = {}, b3 = {};
    if (two) { a2 = dfrag(D1, 0); a3 = dfrag(D1, 1); b2 = xfrag(X1, 0); b3 = xfrag(X1, 1); }
    hf32x4 acc = hf32x4{0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc, 0, 0, 0);
    if (two) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b2, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a3, b3, acc, 0, 0, 0);
    }
    // C[o0 + (lane >> 4) * 4 + r][k0 + c]
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(int64_t)(o0 + (lane >> 4) * 4 + r) * ldo + (int64_t)(k0 + c) * kstr] = acc[r];
    return;
  }
  blk -= HW_TBLK;
  if (blk < HW_VBLK) {
    // one quad per output: frames n = q, q + 4, ...
    int t = blk * 64 + (tid >> 2);
    const int q = tid & 3;
    float s = 0.f, *dst = nullptr;
    if (t < 4 * 3 * HD) {
      const int i = t / (3 * HD), which = (t / HD) % 3, cc = t % HD;
      if (which == 0) {
        for (int n = q; n < N; n += 4) s += ws.dpre(i)[n * HD + cc];
        dst = g.bo[i] + cc;
      } else {
        const float *x = ws.st(h_xin(i));
        for (int n = q; n < N; n += 4) {
          const float d = ws.dxn(i)[n * HD + cc];
          s = which == 1 ? fmaf(d, (x[n * HD + cc] - ws.mu(i)[n]) * ws.rs(i)[n], s) : s + d;
        }
        dst = (which == 1 ? g.lnw[i] : g.lnb[i]) + cc;
      }
    } else if ((t -= 4 * 3 * HD) < HD) {
      for (int n = q; n < N; n += 4) s += ws.dy()[n * HD + t];
      dst = g.bfg + t;
    } else if ((t -= HD) < 64) {
      for (int n = q; n < N; n += 4) s += ws.dh1()[n * 64 + t];
      dst = g.g1b + t;
    } else if ((t -= 64) < 3 * 64) {
      const int o = t >> 6, j = t & 63;
      for (int n = q; n < N; n += 4) {
        const float h = ws.h1()[n * 64 + j] + p.g1b[j];
        const float hd = (h > 0.f ? h : 0.f) * h_drop(sd, 4, n, j, p.p_gate);
        s = fmaf(ws.dz2()[n * 4 + o], hd, s);
      }
      dst = g.g2w + t;
    } else if ((t -= 3 * 64) < 3) {
      for (int n = q; n < N; n += 4) s += ws.dz2()[n * 4 + t];
      dst = g.g2b + t;
    }
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    if (dst && q == 0) *dst = s;
    return;
  }
  blk -= HW_VBLK;
  // the fusion conv's non-centre taps: no input pixel ever meets them (1x1 map, pad 1)
  const int64_t t = (int64_t)blk * 256 + tid;
  if (t < HW_DEAD) {
    const int o = (int)(t / (256 * 8)), r = (int)(t - (int64_t)o * 256 * 8), k = r >> 3, d = r & 7;
    const int tap = d < 4 ? d : d + 1;
    g.wfg[(int64_t)o * g.fg_so + (int64_t)k * g.fg_si + tap * g.fg_tap] = 0.f;
  }
}

// one thread per source element: the 4 blocks' to_q / to_kv / to_out (both layouts), the gate's
// first layer and the fusion conv's centre tap transposed
__global__ __launch_bounds__(256) void head_pack_kernel(HeadParams p, bf16_t *pk) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  constexpr int64_t PER = 4 * HD * HD;                 // wq + wkv + wo elements of one block
  if (i < 4 * PER) {
    const int b = (int)(i / PER);
    const int64_t e = i - b * PER;
    const HeadCA &ca = p.ca[b];
    bf16_t *blk = pk + b * HP_BLK;
    if (e < HD * HD) {                                  // wq [o][k]
      const int o = (int)(e / HD), k = (int)(e % HD);
      const bf16_t v = f2bf(ca.wq[e]);
      blk[HP_Q + e] = v;
      blk[HP_QT + (int64_t)k * HD + o] = v;
    } else if (e < 3 * HD * HD) {                       // wkv [o][k], o < 256
      const int64_t f = e - HD * HD;
      const int o = (int)(f / HD), k = (int)(f % HD);
      const bf16_t v = f2bf(ca.wkv[f]);
      blk[HP_KV + f] = v;
      blk[HP_KVT + (int64_t)k * (2 * HD) + o] = v;
    } else {                                            // wo [o][k]
      const int64_t f = e - 3 * HD * HD;
      const int o = (int)(f / HD), k = (int)(f % HD);
      const bf16_t v = f2bf(ca.wo[f]);
      blk[HP_O + f] = v;
      blk[HP_OT + (int64_t)k * HD + o] = v;
    }
    return;
  }
  const int64_t j = i - 4 * PER;
  if (j < 64 * 256) {                                   // g1w [o = 64][k = 256] -> [k][o]
    const int o = (int)(j / 256), k = (int)(j % 256);
    pk[HP_G1T + (int64_t)k * 64 + o] = f2bf(p.g1w[j]);
    return;
  }
  const int64_t m = j - 64 * 256;
  if (m < (int64_t)HD * 256) {                          // centre tap Wc[o = 128][k = 256] -> [k][o]
    const int o = (int)(m / 256), k = (int)(m % 256);
    pk[HP_WCT + (int64_t)k * HD + o] = f2bf(p.wfg[o * p.fg_so + k * p.fg_si + 4 * p.fg_tap]);
  }
}

// MXFP8 pack of the attention blocks' weights: one thread per 32-element block of an image
// (4 blocks x (Wq, Wq^T, Wkv, Wkv^T, Wo, Wo^T)), straight from the fp32 masters
constexpr int HMX_NB = HD * 4 * 4 + 2 * HD * 4 + HD * 8;    // 32-element blocks per attention block
__global__ __launch_bounds__(256) void head_pack_mx_kernel(HeadParams p, uint8_t *pk) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 4 * HMX_NB) return;
  const int b = i / HMX_NB;
  int j = i - b * HMX_NB;
  // image m, its row and block within the row
  int m = 0;
  for (; m < 6; ++m) {
    int r, c;
    hmx_dims(m, r, c);
    if (j < r * (c / 32)) break;
    j -= r * (c / 32);
  }
  int rows, cols;
  hmx_dims(m, rows, cols);
  const int row = j / (cols / 32), kb = j % (cols / 32);
  const HeadCA &ca = p.ca[b];
  const float *W = m < 2 ? ca.wq : m < 4 ? ca.wkv : ca.wo;    // [out][in = 128]
  const bool tr = m & 1;
  float v[32];
#pragma unroll
  for (int e = 0; e < 32; ++e) {
    const int k = kb * 32 + e;
    v[e] = tr ? W[(int64_t)k * HD + row] : W[(int64_t)row * HD + k];
  }
  int d[8];
  const int ex = mx_quant_block(v, d);
  uint8_t *img = pk + b * HMX_BLK + hmx_img(m);
  uint8_t *dst = img + (int64_t)row * cols + kb * 32;
  *reinterpret_cast<uint4 *>(dst) = make_uint4(d[0], d[1], d[2], d[3]);
  *reinterpret_cast<uint4 *>(dst + 16) = make_uint4(d[4], d[5], d[6], d[7]);
  img[(int64_t)rows * cols + (int64_t)row * (cols / 32) + kb] = (uint8_t)ex;
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

constexpr size_t HL_FWD_ROWS = (size_t)(6 * FG * HD + FG * HD + FG * 512) * 4 + 2 * (size_t)FG * HKP * 2 + 4 * 3 * HD * 4;
constexpr size_t HL_FWD_TAIL = (size_t)(HN * HD + HN * 64 + HN * 4 + 4 * HD + 2 * HD + 3 * 64) * 4;
constexpr size_t HL_BWD_TAIL = (size_t)(HN * 4 + HN * 4 + 8 * HD) * 4;
constexpr size_t HL_BWD_ROWS = (size_t)4 * FG * HD * 4 + (size_t)FG * HKC * 2 + (size_t)FG * HKP * 2 + 4 * HD * 4;
static_assert(HL_FWD_ROWS <= 160 * 1024 && HL_BWD_ROWS <= 64 * 1024 && HL_FWD_TAIL <= 64 * 1024, "head LDS");
static unsigned head_groups(int N) { return (unsigned)((N + FG - 1) / FG); }

extern "C" int64_t ewvit_head_workspace(void) { return head_ws_floats() * (int64_t)sizeof(float); }
extern "C" int64_t ewvit_head_pack_bytes(void) { return HP_TOTAL * (int64_t)sizeof(bf16_t); }
extern "C" int64_t ewvit_head_pack_bytes_mx(void) { return 4 * HMX_BLK; }

extern "C" int ewvit_head_fwd(const HeadParams *params, const float *s0, const float *f0, int N, float *workspace,
                              float *fused, float *s_out, float *f_out, void *stream) {
  EWVIT_CHECK_ARG(params && s0 && f0 && workspace && fused && s_out && f_out, "head_fwd: null pointer");
  if (int rc = head_check(*params, N, "head_fwd")) return rc;
  static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void *>(head_fwd_rows_kernel<false>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)HL_FWD_ROWS) == hipSuccess &&
                           hipFuncSetAttribute(reinterpret_cast<const void *>(head_fwd_rows_kernel<true>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)HL_FWD_ROWS) == hipSuccess;
  (void)attr;
  EWVIT_CHECK_ARG(params->packed, "head_fwd: no pack buffer (ewvit_head_pack_bytes)");
  hipStream_t s = as_stream(stream);
  constexpr int64_t npk = 4 * 4 * HD * HD + 64 * 256 + HD * 256;
  hipLaunchKernelGGL(head_pack_kernel, dim3((unsigned)((npk + 255) / 256)), dim3(256), 0, s, *params,
                     (bf16_t *)params->packed);
  if (int rc = launch_status("head_fwd pack")) return rc;
  if (params->packed_mx) {
    hipLaunchKernelGGL(head_pack_mx_kernel, dim3((4 * HMX_NB + 255) / 256), dim3(256), 0, s, *params,
                       (uint8_t *)params->packed_mx);
    hipLaunchKernelGGL(head_fwd_rows_kernel<true>, dim3(head_groups(N)), dim3(HT), HL_FWD_ROWS, s, *params, s0, f0,
                       workspace, s_out, f_out, N);
  } else {
    hipLaunchKernelGGL(head_fwd_rows_kernel<false>, dim3(head_groups(N)), dim3(HT), HL_FWD_ROWS, s, *params, s0, f0,
                       workspace, s_out, f_out, N);
  }
  if (int rc = launch_status("head_fwd rows")) return rc;
  hipLaunchKernelGGL(head_fwd_fuse_kernel, dim3(12 * head_groups(N)), dim3(64), 0, s, *params, workspace, N);
  if (int rc = launch_status("head_fwd fuse")) return rc;
  hipLaunchKernelGGL(head_fwd_tail_kernel, dim3(1), dim3(HT), HL_FWD_TAIL, s, *params, workspace, fused, N);
  return launch_status("head_fwd tail");
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
  hipLaunchKernelGGL(head_bwd_tail_kernel, dim3(1), dim3(HT), HL_BWD_TAIL, s, *params, ws, g_fused, g_s, g_f, bn_w,
                     bn_b, N);
  if (int rc = launch_status("head_bwd tail")) return rc;
  if (params->packed_mx) {
    hipLaunchKernelGGL(head_bwd_rows_kernel<true>, dim3(head_groups(N)), dim3(HT), HL_BWD_ROWS, s, *params, ws, ds0,
                       df0, N);
    if (int rc = launch_status("head_bwd rows")) return rc;
    hipLaunchKernelGGL(head_bwd_weight_kernel<true>, dim3(HW_TBLK + HW_VBLK + HW_DBLK), dim3(256), 0, s, *params,
                       workspace, g, N);
  } else {
    hipLaunchKernelGGL(head_bwd_rows_kernel<false>, dim3(head_groups(N)), dim3(HT), HL_BWD_ROWS, s, *params, ws, ds0,
                       df0, N);
    if (int rc = launch_status("head_bwd rows")) return rc;
    hipLaunchKernelGGL(head_bwd_weight_kernel<false>, dim3(HW_TBLK + HW_VBLK + HW_DBLK), dim3(256), 0, s, *params,
                       workspace, g, N);
  }
  return launch_status("head_bwd weight");
}
