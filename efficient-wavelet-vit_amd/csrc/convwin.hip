// Windowed 3x3 stride-1 convolution (fwd and input gradient) for the MWT's big maps
// (gfx950).
//
// Callers: the MWT conv stack of network/mwt.py:60-72,112-114 — multiscale_fusion
// (384 -> 128 over the level-major fusion outputs, 64 x 112^2) and its input
// gradient (128 -> 384), hf_conv['fusion'] forward (64 -> 128 over 192 x 112^2).  The
// generic implicit-GEMM kernel (conv.hip conv_glds_kernel) stages every K-tile's
// A operand as 128 gathered pixel rows — each input pixel crosses L2 -> LDS nine
// times, once per tap — and runs a 2-deep ring with a full vmcnt drain + barrier per
// K-tile, the structure whose ceiling is ~0.9 PF/s (cdna_hip_programming.md
// "The step-3 structure's ~900 TF ceiling").
//
// Here a workgroup owns a 16 x 16-pixel output block x 128 output channels and walks
// the K axis as (64-channel block, tap) — the same K order as conv_glds_kernel's
// tap_inner walk, and the same MFMA operand order, so results are bit-identical:
//
//   * A: the block's 18 x 18-pixel input window of one 64-channel block is staged
//     ONCE into LDS (41 LDS-DMA pieces of 8 pixels x 128 B); the nine taps read it at
//     a per-tap pixel offset.  Window pixel p keeps 16-B chunk c at c ^ (p & 7): for
//     any offset, the 16 consecutive pixels of an MFMA fragment read conflict-free
//     with ds_read_b128 (brute-forced over all window offsets).  Two window buffers:
//     the next channel block's (or the next tile's) window lands during taps 0-5 of
//     the current one.
//   * B: the packed weights, one 128 x 64 K-tile per tap, in a 4-slot LDS ring; each
//     K-tile is issued 4 K-tiles ahead.
//   * One raw s_barrier per K-tile behind a COUNTED s_waitcnt vmcnt(N): the K-tile
//     after the one being multiplied must have landed, two more stay in flight
//     across the barrier (N is exact per tap position, epilogue stores included).
//     The fragments of K-tile i+1 are read into registers while K-tile i's MFMAs
//     run (register double buffer), so no wave stalls on LDS latency after the
//     barrier.  All LDS lives in one __shared__ array; the epilogue's bias / BN
//     shift come from LDS, so no ordinary global load ever waits on the DMA queue
//     (cdna_hip_programming.md "Projection GEMM at M = 256" item 4 traps).
//   * 8 waves (4 row groups = 4 image rows each x 2 column halves), 64 x 64 per wave,
//     one workgroup per CU, persistent over the tiles (XCD-aware order: a spatial
//     block's column tiles and its neighbours run on one XCD).
//   * Epilogue straight from the MFMA registers (8-B buffer stores of 4 channels),
//     optional bias and the BatchNorm statistics of the rounded output per 16 x 16
//     block (one partial row per block).
#include "conv_common.h"

#include <type_traits>

namespace ewvit {

int g_win = 1;
// The windowed kernels request the CU's whole 160 KB of LDS (dynamic padding after their static
// arrays), so no workgroup of the other stream co-resides on a CU one of them holds: config 2
// 3627 -> 3636-3646 frames/s (same box, profiles/r05/ab/lds_pad.log).  EWVIT_LDS_PAD=0 /
// ewvit_conv2d_set_lds_pad(0): their own footprint.
int g_lds_pad = 1;
// the non-temporal hint on the windowed kernels' activation-window DMAs (the windows stream
// through once per tile; the hint keeps them from displacing the concurrent backbone's L2 lines):
// config 2 +0.26 / +0.34 / +0.63 % in three interleaved same-box rounds and +0.7 / +0.5 % on
// another box (profiles/r06/ab/win_nt*.log).  Only under a grid cap, i.e. beside the other
// stream: the MWT alone (config 4, uncapped) re-reads the window halos through L2 and lost 3.7 %
// with the hint (1497 against 1554 frames/s, profiles/r06/ab/win_nt_config4.log).
// A mask: 1 the fwd / dgrad windows, 2 the wgrad dy tiles, 4 the wgrad x windows (default 7);
// EWVIT_WIN_NT / ewvit_conv2d_set_win_nt(mask), 0 = off everywhere
int g_win_nt = 7;
template <typename K>
static size_t lds_pad(K kern, size_t stat) {
  if (!g_lds_pad || stat >= 160 * 1024) return 0;
  const size_t d = 160 * 1024 - stat;
  (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)d);
  return d;
}

namespace {
constexpr int WT = 16;                    // output block side (pixels)
constexpr int WW = WT + 2;                // window side
constexpr int WPIX = WW * WW;             // 324 window pixels
constexpr int WPIECES = (WPIX + 7) / 8;   // 41 LDS-DMA pieces of 8 pixels x 128 B
constexpr int WIN_B = WPIECES * 1024;
constexpr int NSLOT = 3;                  // weight ring slots (K-tiles): 9 taps = 3 rounds, so a
                                          // tap's slot is T % 3 in every unit (immediate offsets)
constexpr int SLOT_B = 128 * 128;         // 128 columns x 64 k, bf16
constexpr int VEC_N = 512;                // bias / BN shift entries (Ncol <= 512 with either)
constexpr int VEC0 = NSLOT * SLOT_B;      // bias [512] + BN shift [512] floats
constexpr int RED0 = VEC0 + 2 * VEC_N * 4; // BN statistics partials [4 row groups][128 cols][2]
constexpr int WIN0 = RED0 + 4096;         // [ring][vec][stats][window 0][window 1][xf][sink]
constexpr int XF0 = WIN0 + 2 * WIN_B;     // fwd: input-transform coefficients [groups][2][sgc] (KC <= 512);
                                          // dgrad: BatchNorm backward table (BST_N, BST_G below)
constexpr int BST_N = 768;                // BST: mean / invstd entries (Ncol, or groups x Ncol)
constexpr int BST_G = 256;                // BST: gamma / beta entries (the group width ogc)
static_assert((2 * BST_N + 2 * BST_G) * 4 <= 8192, "BST table exceeds the XF0 region");
constexpr int SINK0 = XF0 + 8192;         // 1 KB target of the window slots past the last piece
constexpr int SMEM_B = SINK0 + 1024;      // 147,456 B: one workgroup per CU
}  // namespace

// all LDS-DMA pieces except the N youngest landed, LDS reads drained, workgroup barrier
template <int N> __device__ __forceinline__ void win_sync() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

typedef __attribute__((ext_vector_type(2))) unsigned int cu32x2;
__device__ __forceinline__ void bstore64(__amdgpu_buffer_rsrc_t r, uint2 v, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b64(cu32x2{v.x, v.y}, r, off, 0, 0);
}
// ... with the non-temporal hint (aux 2 = nt on gfx950) when `nt` (uniform): the MWT's output maps
__device__ __forceinline__ void bstore64(__amdgpu_buffer_rsrc_t r, uint2 v, uint32_t off, bool nt) {
  if (nt) __builtin_amdgcn_raw_buffer_store_b64(cu32x2{v.x, v.y}, r, off, 0, 2);
  else __builtin_amdgcn_raw_buffer_store_b64(cu32x2{v.x, v.y}, r, off, 0, 0);
}
__device__ __forceinline__ void bstore32(__amdgpu_buffer_rsrc_t r, float v, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}

// LDS-DMA through inline asm (conv_common.h glds16_asm): with the builtin, hipcc waits vmcnt(0)
// before every ds_read_b64_tr_b16 of the weight-gradient loop and after any branch between the
// DMA and the reads, draining the loads that should stay in flight.

// one unit = (tile, 64-channel block): 9 K-tiles, one per tap
struct WinUnit {
  int n0;        // first output column of the tile
  int kb;        // byte offset of the channel block inside a packed weight row
  uint32_t wsrc; // byte offset of window pixel (0, 0) and the channel block in src (may wrap: only used with valid pixels)
  int oh0, ow0;  // window pixel (0, 0) = image pixel (oh0 - 1, ow0 - 1)
  int img;       // image
  int part;      // BatchNorm partial row (spatial block index)
  int last;      // last channel block of the tile
  int ok;        // the unit exists
  int xo;        // XF: the channel block's first scale in the coefficient table (its shift at + sgc)
};

// XF (fwd only): the window is staged raw, then each wave rewrites the pieces it staged as
// relu(x * scale + shift) of the pixel's channel group (FwdArgs::xf; bit-identical to the
// BatchNorm apply pass the transform replaces), zero outside the image — at taps 6 and 7 of the
// unit before (its pieces landed by then; tap 8's barrier publishes them), in the prologue for
// the first unit.
// BST (dgrad only): the backward statistics of the BatchNorm(+act) whose output this conv read
// (FwdArgs::bwd, common.h BnBwdStats: x = that BN's input in dx's layout, mean / invstd per
// column, gamma / beta per group channel): per 16 x 16 block and column, sum g and sum g * xhat
// over the bf16-rounded dx, g = dx * act'(xhat * gamma + beta) — what ewvit_bn_bwd_partials
// finalises.  The block's BN-input values are loaded at tap 5 of its last channel block (asm,
// counted in the waits of taps 6, 7; OOB for other units), so the epilogue never waits on them.
// KS (dgrad, 64 output columns: hf_conv['fusion']'s input gradient, 128 -> 64): a tile is the
// block's 256 pixels x 64 columns and the two waves of a row group split each K-tile's 64 k
// between them (wn = the k32 half) — the same 64 x 64 wave tile, so the same LDS bytes per
// MFMA as the 128-column form, over a 64 x 64 weight K-tile (8 KB slots).  At a tile's end
// each wave hands the partner the two accumulator rows the partner stores (8 KB per wave,
// through the 24 KB the smaller ring leaves and the just-consumed window buffer) and adds the
// partner's half of its own two rows: the k-halves summed half 0 + half 1 in fp32, then rounded
// once as before (not bit-identical to the generic kernel's k order; within its rounding).
template <bool DGRAD, bool STATS, bool XF = false, bool BST = false, bool KS = false>
__global__ __launch_bounds__(512) void conv_win_kernel(FwdArgs a, int64_t src_bytes, int64_t out_bytes, int ntn,
                                                       int ntiles, int ncb) {
  static_assert(!KS || (DGRAD && !STATS && !XF), "k-split: plain / BST dgrad only");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_B];
  const int tid = threadIdx.x, lane = tid & 63;
  const int ws = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave 0..7
  const int wm = ws >> 1, wn = ws & 1;                        // rows wm*64.., cols wn*64.. (KS: k half wn)
  constexpr int SLB = KS ? 8192 : SLOT_B;                     // ring slot bytes
  constexpr int BPW = KS ? 1 : 2;                             // weight pieces per wave per K-tile
  constexpr int NCT = KS ? 64 : 128;                          // columns per tile
  const int fr = lane & 15, fq = lane >> 4;
  const int G = gridDim.x;
  const int ntb = ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / G + 1 : 0;
  const int nu = ntb * ncb;                 // units this workgroup walks
  if (nu == 0) return;
  const int H = a.outH, W = a.outW;         // == srcH, srcW (stride 1)
  const int nbx = W / WT, nbl = (H / WT) * nbx;
  const int K = 9 * a.KC;
  const ci32x4 rs = mk_rsrc4(a.src, src_bytes);
  const ci32x4 rw = mk_rsrc4(a.wp, (int64_t)a.Ncol * K * 2);
  const __amdgpu_buffer_rsrc_t ro = mk_rsrc(a.out, out_bytes);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char *)smem;

  if (STATS && blockIdx.x == 0 && a.bn_shift_out)
    for (int c = tid; c < a.Ncol; c += 512) a.bn_shift_out[c] = a.bn_shift ? a.bn_shift[c] : 0.f;
  // bias / BN shift (Ncol <= 512 when either is used) in LDS, staged before any DMA; the
  // epilogue reads them by inline asm (a compiler-visible LDS read there could be preceded by
  // a vmcnt(0) drain of the DMA queue)
  float *vec = reinterpret_cast<float *>(smem + VEC0);
  const bool has_bias = a.bias != nullptr;   // (Ncol may exceed VEC_N without bias / statistics)
  if (a.bias || STATS)
    for (int c = tid; c < a.Ncol && c < VEC_N; c += 512) {
      vec[c] = a.bias ? a.bias[c] : 0.f;
      vec[VEC_N + c] = (STATS && a.bn_shift) ? a.bn_shift[c] : 0.f;
    }
  if constexpr (XF) {
    float *xt = reinterpret_cast<float *>(smem + XF0);
    for (int c = tid; c < 2 * a.KC; c += 512) xt[c] = a.xf[c];
  }
  // BST table (XF0): mean / invstd per column [BST_N] each (row groups — a plain dx whose
  // BatchNorm keeps statistics per slice of grows rows, whole images — [groups][Ncol]), then
  // gamma / beta per group channel [256] each (shared by the channel groups)
  const int bgi = (BST && a.bwd.grows) ? (int)(a.bwd.grows / ((int64_t)a.outH * a.outW)) : 0;   // images per group
  if constexpr (BST) {
    float *bt = reinterpret_cast<float *>(smem + XF0);
    const int nst = a.bwd.grows ? (int)(a.M / a.bwd.grows) * a.Ncol : a.Ncol;
    for (int c = tid; c < nst; c += 512) {
      bt[c] = a.bwd.mean[c];
      bt[BST_N + c] = a.bwd.invstd[c];
    }
    for (int c = tid; c < a.ogc; c += 512) {
      bt[2 * BST_N + c] = a.bwd.gamma ? a.bwd.gamma[c] : 1.f;
      bt[2 * BST_N + BST_G + c] = a.bwd.beta ? a.bwd.beta[c] : 0.f;
    }
  }
  __syncthreads();

  auto unit = [&](int u) -> WinUnit {
    WinUnit d;
    d.ok = u < nu;
    const int uu = d.ok ? u : nu - 1;
    const int k = uu / ncb, cb = uu - k * ncb;
    const int tile = xcd_remap((int)blockIdx.x + k * G, ntiles);
    const int jn = tile % ntn, s = tile / ntn;
    d.img = s / nbl;
    const int r = s - d.img * nbl;
    const int by = r / nbx;
    d.oh0 = by * WT;
    d.ow0 = (r - by * nbx) * WT;
    d.part = s;
    d.n0 = jn * NCT;
    d.kb = cb * 128;                     // 64 channels x 2 B
    d.last = cb == ncb - 1;
    const int c = cb * 64, gi = c / a.sgc;
    const int64_t pix = ((int64_t)d.img * H + (d.oh0 - 1)) * W + (d.ow0 - 1);
    d.wsrc = (uint32_t)((pix * a.sgc + (int64_t)gi * a.sgs + (c - gi * a.sgc)) * 2);
    d.xo = gi * 2 * a.sgc + (c - gi * a.sgc);
    return d;
  };

  // this lane's B rows (pieces 2ws, 2ws+1: rows 8p + lane/8) — byte offsets in a packed
  // weight row for column tile 0, chunk-swizzled
  uint32_t brow[BPW];
#pragma unroll
  for (int j = 0; j < BPW; ++j) {
    const int r = (BPW * ws + j) * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((r >> 1) & 7);
    brow[j] = (uint32_t)((r * K + lc * 8) * 2);
  }
  // B(K-tile of unit d, weight tap rt) -> ring slot
  auto issue_b = [&](const WinUnit &d, int rt, int slot) {
    const uint32_t dst = lds0 + slot * SLB + ws * (BPW * 1024);
    const uint32_t base = (uint32_t)((d.n0 * K + rt * a.KC) * 2 + d.kb);
#pragma unroll
    for (int j = 0; j < BPW; ++j) glds16_asm(rw, dst + j * 1024, d.ok ? base + brow[j] : OOB);
  };
  // window piece q (8 pixels) of unit d into window buffer wb.  The lane's pixel is q * 8 +
  // lane / 8 and its source chunk (lane & 7) ^ (pixel & 7) — loop-invariant (q * 8 keeps
  // pixel & 7); the pixel's row / column are recomputed per issue with 24-bit multiplies (the
  // empty asm keeps hipcc from hoisting the six sets out of the loop into spilled registers)
  const int wlc16 = ((lane & 7) ^ ((lane >> 3) & 7)) * 16;
  const uint32_t sgc2 = (uint32_t)a.sgc * 2;
  auto issue_w = [&](const WinUnit &d, int q, int wb) {
    int pl = lane >> 3;
    asm volatile("" : "+v"(pl));
    const uint32_t p = (uint32_t)(q * 8 + pl);
    const uint32_t wr = __umul24(p, 3641u) >> 16;          // p / 18 for p < 328
    const uint32_t wc = p - __umul24(wr, (uint32_t)WW);
    const int ih = d.oh0 - 1 + (int)wr, iw = d.ow0 - 1 + (int)wc;
    const bool ok = d.ok & (p < (uint32_t)WPIX) & ((unsigned)ih < (unsigned)H) & ((unsigned)iw < (unsigned)W);
    const uint32_t off = d.wsrc + __umul24(__umul24(wr, (uint32_t)W) + wc, sgc2) + (uint32_t)wlc16;
    // (slots past the last piece load zeros into the sink, so every wave issues the same count)
    glds16_asm(rs, q < WPIECES ? lds0 + WIN0 + wb * WIN_B + q * 1024 : lds0 + SINK0, ok ? off : OOB, a.nt != 0);
  };
  // XF: this wave's pieces of unit d's window (buffer wb) -> relu(x * scale + shift), zero
  // outside the image.  The lane's pixel is 8 q + lane / 8 and its chunk (lane & 7) ^ (lane / 8)
  // for every piece, so its 8 channels' coefficients are one pair of table rows per unit.
  auto xform = [&](const WinUnit &d, int wb, int half) __attribute__((always_inline)) {
    const int lc = (lane & 7) ^ ((lane >> 3) & 7);
    const float *xt = reinterpret_cast<const float *>(smem + XF0) + d.xo + lc * 8;
    float sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { sc[e] = xt[e]; sh[e] = xt[a.sgc + e]; }
    int pl = lane >> 3;
    asm volatile("" : "+v"(pl));
    // three of the wave's six pieces (half 0 | 1), one after another (batching the reads costs
    // registers this loop does not have: spills); slots past the last piece skip
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int kk = half * 3 + k;
      const int q = ((kk >> 1) * 8 + ws) * 2 + (kk & 1);
      if (q >= WPIECES) continue;
      const uint32_t p = (uint32_t)(q * 8 + pl);
      const uint32_t wr = __umul24(p, 3641u) >> 16;
      const uint32_t wc = p - __umul24(wr, (uint32_t)WW);
      const int ih = d.oh0 - 1 + (int)wr, iw = d.ow0 - 1 + (int)wc;
      const bool ok = d.ok & (p < (uint32_t)WPIX) & ((unsigned)ih < (unsigned)H) & ((unsigned)iw < (unsigned)W);
      uint4 *ptr = reinterpret_cast<uint4 *>(smem + WIN0 + wb * WIN_B + q * 1024 + lane * 16);
      const uint4 v = *ptr;
      const unsigned wv[4] = {v.x, v.y, v.z, v.w};
      unsigned o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float z0 = fmaf(__uint_as_float(wv[e] << 16), sc[2 * e], sh[2 * e]);
        const float z1 = fmaf(__uint_as_float(wv[e] & 0xffff0000u), sc[2 * e + 1], sh[2 * e + 1]);
        o[e] = (unsigned)f2bf(z0 > 0.f ? z0 : 0.f) | ((unsigned)f2bf(z1 > 0.f ? z1 : 0.f) << 16);
      }
      *ptr = ok ? make_uint4(o[0], o[1], o[2], o[3]) : make_uint4(0u, 0u, 0u, 0u);
    }
  };

  // fragment addresses, no VALU in the loop.  A: window pixel p = p0 + c, p0 = (wm*4)*18 + fr,
  // c = i*18 + tap offset (compile-time); chunk ch at ch ^ (p & 7) and p & 7 = (fr + c) & 7
  // (72 = 0 mod 8), so a lane's address is atab[buffer][c & 7] + c * 128 (the k32 half 1 =
  // chunks + 4: atab[(c + 4) & 7]).  B: ring row wn*64 + j*16 + fr, chunk ch at ch ^ ((fr >> 1)
  // & 7) for every j; slot / j / half in the immediate.
  uint32_t atab[2][8];
  {
    const int p0 = wm * 4 * WW + fr;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 8; ++r)
        atab[b][r] = lds0 + WIN0 + b * WIN_B + (uint32_t)(p0 * 128 + 16 * ((fq | (KS ? 4 * wn : 0)) ^ ((fr + r) & 7)));
  }
  const uint32_t bfo = lds0 + (uint32_t)(((KS ? 0 : wn * 64) + fr) * 128 + 16 * ((fq | (KS ? 4 * wn : 0)) ^ ((fr >> 1) & 7)));
  typedef __attribute__((address_space(3))) const cbf16x8 lds_frag;
  auto ldsr = [&](uint32_t addr) -> cbf16x8 { return *reinterpret_cast<lds_frag *>((uintptr_t)addr); };
  cbf16x8 fa[2][4], fb[2][4];
  // fragments of the K-tile (window buffer WB, tap RT, ring slot SL) into xa / xb
  auto read_frags = [&](auto WBc, auto RTc, auto SLc, cbf16x8 (&xa)[2][4], cbf16x8 (&xb)[2][4]) {
    constexpr int WB = decltype(WBc)::value, RT = decltype(RTc)::value, SL = decltype(SLc)::value;
    constexpr int kh = RT / 3, kw = RT % 3;
    constexpr int woff = DGRAD ? (2 - kh) * WW + (2 - kw) : kh * WW + kw;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = i * WW + woff;
      xa[0][i] = ldsr(atab[WB][c & 7] + c * 128);
      if constexpr (!KS) xa[1][i] = ldsr(atab[WB][(c + 4) & 7] + c * 128);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      xb[0][j] = ldsr(bfo + SL * SLB + j * 2048);
      if constexpr (!KS) xb[1][j] = ldsr((bfo ^ 64) + SL * SLB + j * 2048);
    }
  };

  cf32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = cf32x4{0.f, 0.f, 0.f, 0.f};

  // BST: this lane's BN-input values at its 16 epilogue positions of unit d (zeros, no traffic,
  // unless d ends its tile)
  // KS: a wave stores rows ER0 .. ER0 + NER - 1 of its row group, all 64 columns
  constexpr int NER = KS ? 2 : 4;
  const int ER0 = KS ? 2 * wn : 0;
  const int ECOL = KS ? 0 : wn * 64;
  uint2 xq[4][NER];
  const __amdgpu_buffer_rsrc_t rbx = mk_rsrc(BST ? (const void *)a.bwd.x : (const void *)a.out, out_bytes);
  auto issue_x = [&](const WinUnit &d) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = d.n0 + ECOL + j * 16 + fq * 4;
      const int gi = col / a.ogc;
      const int64_t cbase = (int64_t)gi * a.ogs + (col - gi * a.ogc);
#pragma unroll
      for (int i = 0; i < NER; ++i) {
        const int64_t pix = ((int64_t)d.img * H + d.oh0 + wm * 4 + ER0 + i) * W + d.ow0 + fr;
        const uint32_t off = d.last ? (uint32_t)((pix * a.ogc + cbase) * 2) : OOB;
        if (EWVIT_MWT_NT && a.nt) asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen nt" : "=v"(xq[j][i]) : "v"(off), "s"(rbx) : "memory");
        else asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(xq[j][i]) : "v"(off), "s"(rbx) : "memory");
      }
    }
  };

  // tile epilogue: (+ bias) -> bf16, 16 stores per wave; STATS: one more store per wave
  auto epilogue = [&](const WinUnit &d, int wb) __attribute__((always_inline)) {
    float cs[4][4], cq[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cl = ECOL + j * 16 + fq * 4;             // column in the tile
      const int col = d.n0 + cl;
      float4 bv, kv;
      {
        const uint32_t va = lds0 + VEC0 + (uint32_t)col * 4;
        if (has_bias) asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(bv) : "v"(va) : "memory");
        else bv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (STATS) asm volatile("ds_read_b128 %0, %1 offset:2048\n\ts_waitcnt lgkmcnt(0)" : "=v"(kv) : "v"(va) : "memory");
        else kv = make_float4(0.f, 0.f, 0.f, 0.f);
        __builtin_amdgcn_sched_barrier(0);
      }
      const int gi = col / a.ogc;
      const int64_t cbase = (int64_t)gi * a.ogs + (col - gi * a.ogc);
#pragma unroll
      for (int r = 0; r < 4; ++r) { cs[j][r] = 0.f; cq[j][r] = 0.f; }
      float bmu[4], biv[4], bga[4], bbe[4];
      if constexpr (BST) {
        const float *bt = reinterpret_cast<const float *>(smem + XF0);
        const int so = (bgi ? d.img / bgi * a.Ncol : 0) + col;     // the row group's statistics
        const int cg = col - gi * a.ogc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          bmu[r] = bt[so + r]; biv[r] = bt[BST_N + so + r];
          bga[r] = bt[2 * BST_N + cg + r]; bbe[r] = bt[2 * BST_N + BST_G + cg + r];
        }
      }
#pragma unroll
      for (int i = 0; i < NER; ++i) {
        // (KS: the exchange left the wave's rows ER0, ER0 + 1 in acc[0], acc[1])
        const int64_t pix = ((int64_t)d.img * H + d.oh0 + wm * 4 + ER0 + i) * W + d.ow0 + fr;
        const bf16_t h0 = f2bf(acc[i][j][0] + bv.x), h1 = f2bf(acc[i][j][1] + bv.y);
        const bf16_t h2 = f2bf(acc[i][j][2] + bv.z), h3 = f2bf(acc[i][j][3] + bv.w);
        uint2 pk;
        pk.x = (uint32_t)h0 | ((uint32_t)h1 << 16);
        pk.y = (uint32_t)h2 | ((uint32_t)h3 << 16);
        bstore64(ro, pk, (uint32_t)((pix * a.ogc + cbase) * 2), EWVIT_MWT_NT && a.nt != 0);
        if constexpr (BST) {
          const float hv[4] = {bf2f(h0), bf2f(h1), bf2f(h2), bf2f(h3)};
          const float xv[4] = {__uint_as_float(xq[j][i].x << 16), __uint_as_float(xq[j][i].x & 0xffff0000u),
                               __uint_as_float(xq[j][i].y << 16), __uint_as_float(xq[j][i].y & 0xffff0000u)};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float xh = (xv[r] - bmu[r]) * biv[r];
            const float gg = a.bwd.act ? hv[r] * bn_act_grad(a.bwd.act, fmaf(xh, bga[r], bbe[r])) : hv[r];
            cs[j][r] += gg;
            cq[j][r] = fmaf(gg, xh, cq[j][r]);
          }
        }
        if (STATS) {
          const float d0 = bf2f(h0) - kv.x, d1 = bf2f(h1) - kv.y, d2 = bf2f(h2) - kv.z, d3 = bf2f(h3) - kv.w;
          cs[j][0] += d0; cs[j][1] += d1; cs[j][2] += d2; cs[j][3] += d3;
          cq[j][0] = fmaf(d0, d0, cq[j][0]); cq[j][1] = fmaf(d1, d1, cq[j][1]);
          cq[j][2] = fmaf(d2, d2, cq[j][2]); cq[j][3] = fmaf(d3, d3, cq[j][3]);
        }
        acc[i][j] = cf32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    if constexpr (STATS || BST) {
      // the 16 row lanes of each column (DPP) here; the 4 row-group waves' partials are
      // summed after the NEXT K-tile's barrier (stats_flush), so this epilogue has no barrier
      // of its own and the MFMAs of the next unit start right away
      float *red = reinterpret_cast<float *>(smem + RED0);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float S = row_sum16(cs[j][r]), Q = row_sum16(cq[j][r]);
          if (fr == 0) {
            // KS: [8 waves][64 columns]; else [4 row groups][128 columns]
            const int cl = ECOL + j * 16 + fq * 4 + r;
            const int ro = KS ? ws * 64 : wm * 128;
            red[(ro + cl) * 2] = S;
            red[(ro + cl) * 2 + 1] = Q;
          }
        }
    }
    (void)wb;
  };
  // the BN partial row of the tile whose epilogue ran last: one store per wave (threads
  // 256-511 store the same value to the same address), after a barrier that every wave
  // passed with its partials written (lgkmcnt(0))
  int pend_part = 0, pend_n0 = 0;
  const __amdgpu_buffer_rsrc_t rp = mk_rsrc(a.bn_part, (int64_t)OOB);
  const int ncol = a.Ncol;
  const __amdgpu_buffer_rsrc_t rq = mk_rsrc(BST ? a.bwd.part : a.bn_part, (int64_t)OOB);
  const int nblk = (int)(a.M / (WT * WT));
  auto stats_flush = [&]() __attribute__((always_inline)) {
    const float *red = reinterpret_cast<const float *>(smem + RED0);
    const int v = tid & 255, cl = (v >> 1) & (NCT - 1), w = v & 1;
    float t;
    if constexpr (KS) {
      // the 8 waves' partials of the 64 columns (threads v >= 128 store out of range: every
      // wave issues the one store the counted waits expect)
      t = ((red[(0 * 64 + cl) * 2 + w] + red[(1 * 64 + cl) * 2 + w]) +
           (red[(2 * 64 + cl) * 2 + w] + red[(3 * 64 + cl) * 2 + w])) +
          ((red[(4 * 64 + cl) * 2 + w] + red[(5 * 64 + cl) * 2 + w]) +
           (red[(6 * 64 + cl) * 2 + w] + red[(7 * 64 + cl) * 2 + w]));
    } else {
      t = (red[(0 * 128 + cl) * 2 + w] + red[(1 * 128 + cl) * 2 + w]) +
          (red[(2 * 128 + cl) * 2 + w] + red[(3 * 128 + cl) * 2 + w]);
    }
    if constexpr (BST) {
      // [channel group][block][2 group channels]
      const int gi = pend_n0 / a.ogc;
      const uint32_t off = (uint32_t)((((int64_t)gi * nblk + pend_part) * 2 * a.ogc + w * a.ogc + pend_n0 - gi * a.ogc + cl) * 4);
      bstore32(rq, t, (KS && v >= 128) ? OOB : off);
    } else {
      bstore32(rp, t, (uint32_t)((pend_part * 2 * ncol + w * ncol + pend_n0 + cl) * 4));
    }
  };
  // KS: the k-halves of the tile's accumulators meet.  Wave ws writes the two rows its partner
  // (ws ^ 1) stores — wn 0 sends rows 2, 3, wn 1 rows 0, 1 — to its 8 KB block (blocks 0-2 in
  // the ring's unused upper 24 KB, 3-7 in window buffer WB: consumed by this unit's last reads,
  // refilled only after the next unit's first barrier), then adds the partner's block into the
  // rows it keeps, left in acc[0], acc[1].
  auto exchange = [&](int wb) __attribute__((always_inline)) {
    auto blk = [&](int w) -> float4 * {
      return reinterpret_cast<float4 *>(w < 3 ? smem + 3 * 8192 + w * 8192 : smem + WIN0 + wb * WIN_B + (w - 3) * 8192);
    };
    float4 *mine = blk(ws), *theirs = blk(ws ^ 1);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const cf32x4 v = wn ? acc[ii][j] : acc[2 + ii][j];
        mine[(ii * 4 + j) * 64 + lane] = make_float4(v[0], v[1], v[2], v[3]);
      }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 p = theirs[(ii * 4 + j) * 64 + lane];
        const cf32x4 k = wn ? acc[2 + ii][j] : acc[ii][j];
        acc[ii][j] = cf32x4{k[0] + p.x, k[1] + p.y, k[2] + p.z, k[3] + p.w};
        acc[2 + ii][j] = cf32x4{0.f, 0.f, 0.f, 0.f};
      }
  };
  constexpr int ST = 4 * NER;                // output stores of one epilogue per wave
  constexpr int SS = (STATS || BST) ? 1 : 0; // the statistics store (at the next unit's tap 0)
  constexpr int XL = BST ? 4 * NER : 0;      // BST: BN-input loads issued at tap 5

  // window pieces of the next unit: 2 per wave at taps 0-2 (48 slots for 41 pieces; the extra
  // slots repeat piece 40), so a unit's window has landed long before its first read
  constexpr int WPT = 2;
  auto wpiece = [&](int T, int jj) { return (T * 8 + ws) * WPT + jj; };

  // ---- prologue: unit 0's window (all pieces), K-tiles 0..2 of unit 0
  WinUnit cu = unit(0), nx = unit(1);
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int jj = 0; jj < WPT; ++jj) issue_w(cu, wpiece(t, jj), 0);
#pragma unroll
  for (int t = 0; t < 3; ++t) issue_b(cu, t, t);
  win_sync<2 * BPW>();                      // window 0 and K-tile 0 landed (B 1, 2 in flight)
  if constexpr (XF) {
    xform(cu, 0, 0);
    xform(cu, 0, 1);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  read_frags(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{},
             fa, fb);
  bool prev_st = false;                     // the previous unit ended a tile (its stores are in flight)

  // one unit (window buffer WB): 9 K-tiles.  K-tile i: wait for K-tile i+1 (and its
  // window), issue the next unit's window pieces (taps 0-2) and K-tile i+3 into slot i % 3,
  // read K-tile i+1's fragments, multiply K-tile i
  auto unit_body = [&](auto WBc) {
    constexpr int WB = decltype(WBc)::value;
    auto step = [&](auto TT) {
      constexpr int T = decltype(TT)::value;
      // (the address tables re-enter every step: else hipcc hoists every (tap, i) address sum
      // out of the loop into registers it then spills)
#pragma unroll
      for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(atab[0][r]), "+v"(atab[1][r]));
      // vector-memory ops younger than K-tile i+1's pieces (issued at i-2): iteration i-1's
      // window pieces + weight K-tile, and the previous unit's epilogue stores (tap 8) for
      // T = 0, 1
      // (+ the output stores of the previous unit's tap 8 for T = 0, 1 and its statistics
      // store, issued at this unit's tap 0, for T = 1, 2)
      constexpr int NB = BPW + (((T + 8) % 9) < 3 ? WPT : 0) + ((T == 6 || T == 7) ? XL : 0);
      constexpr int X = (T <= 1 ? ST : 0) + ((T == 1 || T == 2) ? SS : 0);
      if constexpr (X > 0) {
        if (prev_st) win_sync<NB + X>();
        else win_sync<NB>();
      } else {
        win_sync<NB>();
      }
      if constexpr (T < 3) {
#pragma unroll
        for (int jj = 0; jj < WPT; ++jj) issue_w(nx, wpiece(T, jj), WB ^ 1);
      }
      if constexpr (T + 3 < 9) issue_b(cu, T + 3, T % 3);
      else issue_b(nx, T + 3 - 9, T % 3);
      if constexpr ((STATS || BST) && T == 0) {
        if (prev_st) stats_flush();
      }
      if constexpr (BST && T == 5) issue_x(cu);
      if constexpr (BST && T == 8) {
        // (landed: older than the K-tile this step waited for; the empty asm keeps their
        // uses below the wait)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(xq[j][i]));
      }
      cbf16x8 na[2][4], nb[2][4];
      if constexpr (T + 1 < 9)
        read_frags(std::integral_constant<int, WB>{}, std::integral_constant<int, T + 1>{},
                   std::integral_constant<int, (T + 1) % 3>{}, na, nb);
      else
        read_frags(std::integral_constant<int, WB ^ 1>{}, std::integral_constant<int, 0>{},
                   std::integral_constant<int, 0>{}, na, nb);
#pragma unroll
      for (int ks = 0; ks < (KS ? 1 : 2); ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ks][j], fa[ks][i], acc[i][j], 0, 0, 0);
      if constexpr (XF && (T == 6 || T == 7)) xform(nx, WB ^ 1, T - 6);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int q = 0; q < 4; ++q) { fa[ks][q] = na[ks][q]; fb[ks][q] = nb[ks][q]; }
      if constexpr (T == 8) {
        prev_st = cu.last;
        if (cu.last) {
          if constexpr (KS) exchange(WB);
          epilogue(cu, WB);
          pend_part = cu.part;
          pend_n0 = cu.n0;
        }
      }
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 3>{});
    step(std::integral_constant<int, 4>{});
    step(std::integral_constant<int, 5>{});
    step(std::integral_constant<int, 6>{});
    step(std::integral_constant<int, 7>{});
    step(std::integral_constant<int, 8>{});
  };
  for (int u = 0; u < nu; u += 2) {
    unit_body(std::integral_constant<int, 0>{});
    cu = nx;
    nx = unit(u + 2);
    if (u + 1 >= nu) break;
    unit_body(std::integral_constant<int, 1>{});
    cu = nx;
    nx = unit(u + 3);
  }
  if constexpr (STATS || BST) {             // the last tile's statistics
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    stats_flush();
  }
  // no LDS-DMA may land after the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// the k-split form: a plain 64-column input gradient
static bool win_ks(const FwdArgs &a, bool dgrad) {
  return dgrad && a.Ncol == 64 && a.ogc == 64 && !a.ogs && !a.bias;
}

bool win_ok(const FwdArgs &a, bool dgrad) {
  if (!g_win || a.g.ks != 3 || a.g.stride != 1 || a.g.pad != 1 || a.pc >= 0 || a.addend) return false;
  if (a.bwd.part && (!dgrad || a.bwd.rscale || !a.bwd.x || !a.bwd.mean || !a.bwd.invstd || a.Ncol > BST_N ||
                     a.ogc > BST_G)) return false;
  // BatchNorm row groups of whole images, their statistics table in LDS
  if (a.bwd.part && a.bwd.grows &&
      (a.ogs || a.bwd.grows % ((int64_t)a.outH * a.outW) || a.M % a.bwd.grows || (a.M / a.bwd.grows) * a.Ncol > BST_N))
    return false;
  const bool ks = win_ks(a, dgrad);
  // (the transform and the BST epilogue measured slower at config 4's 768-channel multiscale conv:
  // 1445 frames/s unfolded, 1391-1396 folded, 1413-1420 folded without BST — two column tiles
  // transform every window twice; profiles/r05/ab/fold_config4_768.log)
  if (a.xf && (dgrad || a.KC > 512)) return false;
  if (a.bwd.part && !a.bwd.grows && a.Ncol > 512) return false;
  if (dgrad && a.bn_part) return false;
  if (a.outH != a.srcH || a.outW != a.srcW || a.outH % WT || a.outW % WT) return false;
  if (a.KC % 64 || a.sgc % 64 || (a.KCr && a.KCr != a.KC)) return false;
  if (!ks && (a.Ncol % 128 || a.ogc % 128)) return false;
  if ((a.bias || a.bn_part) && a.Ncol > VEC_N) return false;
  if (a.M != (int64_t)a.g.N * a.outH * a.outW) return false;
  const int64_t K = 9LL * a.KC;
  if (a.Ncol * K * 2 >= (int64_t)OOB) return false;
  const int64_t ob = 2 * (a.ogs ? (a.Ncol / a.ogc - 1) * a.ogs + a.M * a.ogc : a.M * a.Ncol);
  if (ob >= (int64_t)OOB) return false;
  const int64_t nt = a.M / (WT * WT) * (ks ? 1 : a.Ncol / 128);
  return nt < (1 << 30);
}

static int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

// ---------------------------------------------------------------- weight gradient
// dW[co][tap][ci] = sum_pix dy[pix][co] * x[pix + tap shift][ci] over 8 x 16-pixel tiles (the
// K chunks): a workgroup owns (pixel split, 128-row co tile, 32-channel ci block) and all 9
// taps — a [128 co] x [9 x 32] block of the weight gradient — and walks its split's pixel
// tiles.  Per tile it stages the dy tile (128 px x 128 co, 32 KB) and the tile's 10 x 18 x 32
// x window (11.5 KB, ONCE for the nine taps) by LDS-DMA into one of two stages, the next tile's
// landing during this tile's MFMAs (144 per wave, 80 / 64 under TS).  Both operands are read transposed
// (ds_read_b64_tr_b16): dy as the MFMA A operand (the generic wgrad's image and swizzle),
// the window as B with pixel p's 16-B chunk c at c ^ (((p >> 1) & 1) << 1 | ((p >> 3) & 1)
// << 2) — conflict-free for the 32 lanes of a read at any tap offset (brute-forced).  That
// swizzle depends on p mod 16 only, so a lane's 16 window addresses (one per p mod 16) are
// computed once and every tap / k32 step / half reads at one of them plus an immediate
// offset: no address VALU in the loop.  4 waves = 2 co halves x 2 ci halves, each wave
// 64 co x (9 taps x 16 ci) = 144 fp32 accumulators per lane; the default tap-split form (TS)
// runs 8 waves, the second four repeating those blocks for taps 5-8 (80 accumulators).  The bias gradient (sum of dy
// over pixels) is one more MFMA per k32 step against a ones operand, by the ci-block-0
// workgroups.  Per split: fp32 slabs [split][Cout][9 Cin] (+ [split][Cout] bias partials)
// summed by conv_wgrad_reduce_kernel in a fixed order.
namespace {
constexpr int GT_R = 8, GT_C = 16;                 // pixel tile
constexpr int GX_W = GT_C + 2, GX_H = GT_R + 2;    // x window
constexpr int GX_PIX = GX_W * GX_H;                // 180 pixels x 32 channels (64-B rows)
constexpr int GX_PIECES = (GX_PIX + 15) / 16;      // 12 LDS-DMA pieces of 16 pixels
constexpr int GX_B = GX_PIECES * 1024;             // 12,288
constexpr int GD_B = 128 * 256;                    // dy tile
constexpr int GD0 = 2 * GX_B;                      // [X0][X1][D0][D1]
constexpr int GSMEM = GD0 + 2 * GD_B;              // 90,112 B
}  // namespace

template <int V> struct ic_t { static constexpr int value = V; };

// 64-B window rows: chunk c of pixel p at c ^ (((p >> 3) & 1) << 1)
__device__ __forceinline__ int xswz(int p) { return ((p >> 3) & 1) << 1; }


// XF: x is read as relu(x * scale + shift) (WgradArgs::xf, the forward's input transform): each
// wave rewrites its own window pieces of the next tile after its DMAs drained at the end of the
// current tile (the loop-top barrier publishes them), the first tile's before the loop.
// TS (tap split): 8 waves, two per SIMD — waves 4..7 repeat waves 0..3's (co half, ci half) roles
// for taps 5..8 while waves 0..3 take taps 0..4 (80 accumulators instead of 144, every output
// still owned by one wave: no cross-wave reduction); the DMA pieces are spread over the 8 waves.
// NG = 3: 12 waves, three per SIMD, one kernel row kh per wave group (48 accumulators); the DMA
// pieces strided over the waves (piece wsa + 12 j).
template <bool BIAS, bool XF = false, int NG = 1>
__global__ __launch_bounds__(NG * 256) void conv_wgrad_win_kernel(WgradArgs a, int64_t x_bytes, int nsplit, int ncb,
                                                                  int nct, int ntile) {
  constexpr bool TS = NG > 1;
  constexpr int NW = 4 * NG;                        // waves
  __shared__ __attribute__((aligned(16))) unsigned char smem[GSMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wsa = __builtin_amdgcn_readfirstlane(tid >> 6);   // 0..NW-1
  const int kq = TS ? wsa >> 2 : 0;                 // TS: tap group (NG 2: taps 0-4 | 5-8; NG 3: row kq)
  const int ws = TS ? wsa & 3 : wsa;
  const int wr = ws >> 1, wc = ws & 1;              // co half, 16-channel half of the 32-channel block
  constexpr int PPW = NG == 3 ? 3 : TS ? 4 : 8, XPW = NG == 3 ? 1 : TS ? 2 : 3;  // dy / x DMA pieces per wave
  // piece ids: contiguous per wave (NG 1, 2), strided (NG 3)
  auto dpiece = [&](int j) { return NG == 3 ? wsa + NW * j : wsa * PPW + j; };
  auto xpiece = [&](int j) { return NG == 3 ? wsa : wsa * XPW + j; };
  const int r = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  // co tile fastest: the nct workgroups sharing a (ci block, split) window stream sit on one XCD
  // (consecutive remapped ids), so x is fetched into one L2 only
  const int ct = r % nct, cb = (r / nct) % ncb, split = r / (ncb * nct);
  const int t0 = (int)((int64_t)split * ntile / nsplit), t1 = (int)((int64_t)(split + 1) * ntile / nsplit);
  const int H = a.g.H, W = a.g.W, Cout = a.g.Cout, Cin = a.g.Cin;
  const int tpr = W / GT_C, tpi = (H / GT_R) * tpr;
  const int NP = 9 * Cin;
  const __amdgpu_buffer_rsrc_t rx = mk_rsrc(a.x, x_bytes);
  const __amdgpu_buffer_rsrc_t rd = mk_rsrc(a.dy, a.M * Cout * 2);
  const bool do_bias = BIAS && cb == 0;
  const int c32 = cb * 32, gi = c32 / a.xgc;
  const int64_t cofs = (int64_t)gi * a.xgs + (c32 - gi * a.xgc);

  // stage tile t into stage b: dy tile rows 2 ws, 2 ws + 1 (pieces j: pixels 4 (j & 3) + lane/16
  // of row 2 ws + j / 4), window pieces 3 ws + j (pixels 16 q + lane / 4).  The empty asm keeps
  // hipcc from hoisting the per-lane constants out of the loop (into spilled registers).
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char *)smem;
  auto issue = [&](int t, int b, bool live) {
    const int img = t / tpi, rem = t - img * tpi;
    const int oh0 = (rem / tpr) * GT_R, ow0 = (rem % tpr) * GT_C;
    int dl = lane >> 4;
    asm volatile("" : "+v"(dl));
    // dy piece P = wsa * PPW + j: tile row P / 4, pixels 4 (P & 3) + lane / 16
    const int64_t dpix = ((int64_t)img * H + oh0) * W + ow0;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int P = dpiece(j);
      if (NG == 3 && P >= 32) continue;               // (NG 3: waves 8-11 stage two dy pieces)
      const int sc = (lane & 15) ^ ((dl << 2) | (P & 3));
      const uint32_t off = (uint32_t)(((dpix + (P >> 2) * W + 4 * (P & 3) + dl) * Cout + ct * 128 + sc * 8) * 2);
      glds16_asm(rd, lds0 + GD0 + b * GD_B + P * 1024, live ? off : OOB, (a.nt & 1) != 0);
    }
    const int64_t xpix = ((int64_t)img * H + oh0 - 1) * W + ow0 - 1;
    int xl = lane >> 2;
    asm volatile("" : "+v"(xl));
#pragma unroll
    for (int j = 0; j < XPW; ++j) {
      if (TS && xpiece(j) >= GX_PIECES) continue;   // (NG 2: waves 6, 7 stage no window piece)
      const int q = xpiece(j);
      const int p = q * 16 + xl;
      const int xr = (p * 3641) >> 16, xc = p - xr * GX_W;       // p / 18, p % 18
      const int ih = oh0 - 1 + xr, iw = ow0 - 1 + xc;
      // (bitwise &: a short-circuit && becomes an exec-masked branch, and at its merge hipcc
      // waits vmcnt(0) before the next ds_read — draining the DMA just issued)
      const bool ok = live & (p < GX_PIX) & ((unsigned)ih < (unsigned)H) & ((unsigned)iw < (unsigned)W);
      const int sc = (lane & 3) ^ xswz(p);
      const uint32_t off = (uint32_t)(((xpix + xr * W + xc) * a.xgc + cofs + sc * 8) * 2);
      glds16_asm(rx, lds0 + b * GX_B + q * 1024, ok ? off : OOB, (a.nt & 2) != 0);
    }
  };

  // XF: the lane's 8 channels are the same in every piece (chunk (lane & 3) ^ xswz(16 q + lane / 4)
  // = (lane & 3) ^ ((lane >> 5) << 1)), so their coefficients stay in registers
  float xsc[8], xsh[8];
  if constexpr (XF) {
    const int lcx = (lane & 3) ^ (((lane >> 5) & 1) << 1);
    const float *xt = a.xf + gi * 2 * a.xgc + (c32 - gi * a.xgc) + lcx * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) { xsc[e] = xt[e]; xsh[e] = xt[a.xgc + e]; }
  }
  auto xform = [&](int t, int b) __attribute__((always_inline)) {
    const int img = t / tpi, rem = t - img * tpi;
    const int oh0 = (rem / tpr) * GT_R, ow0 = (rem % tpr) * GT_C;
    int xl = lane >> 2;
    asm volatile("" : "+v"(xl));
#pragma unroll
    for (int j = 0; j < XPW; ++j) {
      if (TS && xpiece(j) >= GX_PIECES) continue;
      const int q = xpiece(j);
      const int p = q * 16 + xl;
      const int xr = (p * 3641) >> 16, xc = p - xr * GX_W;
      const int ih = oh0 - 1 + xr, iw = ow0 - 1 + xc;
      const bool ok = (p < GX_PIX) & ((unsigned)ih < (unsigned)H) & ((unsigned)iw < (unsigned)W);
      uint4 *ptr = reinterpret_cast<uint4 *>(smem + b * GX_B + q * 1024 + lane * 16);
      const uint4 v = *ptr;
      const unsigned wv[4] = {v.x, v.y, v.z, v.w};
      unsigned o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float z0 = fmaf(__uint_as_float(wv[e] << 16), xsc[2 * e], xsh[2 * e]);
        const float z1 = fmaf(__uint_as_float(wv[e] & 0xffff0000u), xsc[2 * e + 1], xsh[2 * e + 1]);
        o[e] = (unsigned)f2bf(z0 > 0.f ? z0 : 0.f) | ((unsigned)f2bf(z1 > 0.f ? z1 : 0.f) << 16);
      }
      *ptr = ok ? make_uint4(o[0], o[1], o[2], o[3]) : make_uint4(0u, 0u, 0u, 0u);
    }
  };

  // fragment addresses.  A (dy^T, rows k = pixel, cols = co): tr read rows 8g + q (+4 hi)
  // of k32 step ks at + ks * 8192, stage 1 at + GD_B.  B (window): 16 addresses, one per
  // window pixel residue mod 16 (the swizzle depends on bit 3 only); stage 1 at + GX_B.
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  uint32_t aad[2][4];
#pragma unroll
  for (int hi = 0; hi < 2; ++hi)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 8 * g + q4 + 4 * hi, col = wr * 64 + i * 16 + 4 * p4;
      aad[hi][i] = (uint32_t)(GD0 + swz_off(row, col >> 3) + 2 * (col & 7));
    }
  uint32_t xad[16];
  const int pb0 = (g >> 1) * GX_W + 8 * (g & 1) + q4;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int P = pb0 + m;
    xad[m] = (uint32_t)(P * 64 + 16 * ((2 * wc + (p4 >> 1)) ^ xswz(P)) + 8 * (p4 & 1));
  }
  auto trd = [&](uint32_t off) -> cs4 {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) cs4 *)(smem + off));
  };

  const cbf16x8 ones = __builtin_bit_cast(cbf16x8, (__attribute__((ext_vector_type(8))) short){
      0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80});

  // (the last tile issues a dummy stage — every lane out of range, zeros into the idle stage —
  // so no branch sits between the DMA and the fragment reads: at such a merge hipcc waits
  // vmcnt(0) before the first ds_read, draining the next tile's loads)
  if (t0 < t1) {
    issue(t0, 0, true);
    if constexpr (XF) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      xform(t0, 0);
    }
  }

  // the tile loop over taps TB .. TB + NT - 1 (TS: one tap half per wave group, a separate copy
  // of the loop per half so each keeps its accumulators in fixed registers)
  auto run = [&](auto KQ) __attribute__((always_inline)) {
    constexpr int kqc = decltype(KQ)::value;
    constexpr int TB = NG == 3 ? 3 * kqc : 5 * kqc, NT = NG == 3 ? 3 : TS ? (kqc ? 4 : 5) : 9;
    const bool bias_w = do_bias && kqc == 0;
    cf32x4 acc[4][NT];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[i][t] = cf32x4{0.f, 0.f, 0.f, 0.f};
    cf32x4 bacc[2] = {cf32x4{0.f, 0.f, 0.f, 0.f}, cf32x4{0.f, 0.f, 0.f, 0.f}};

    // one loop body for both stages (two bodies made hipcc copy the accumulators between
    // them): the stage's addresses are toggled by +-stage size after each tile
    auto compute = [&]() {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        cbf16x8 af[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const cs4 lo = trd(aad[0][i] + ks * 8192), hi = trd(aad[1][i] + ks * 8192);
          af[i] = __builtin_bit_cast(cbf16x8, (__attribute__((ext_vector_type(8))) short){
                                                  lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
        }
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
          const int t = TB + tt, kh = t / 3, kw = t % 3;
          const int C0 = ks * 2 * GX_W + kh * GX_W + kw, C1 = C0 + 4;
          const cs4 lo = trd(xad[C0 & 15] + (C0 & ~15) * 64);
          const cs4 hi = trd(xad[C1 & 15] + (C1 & ~15) * 64);
          const cbf16x8 bf = __builtin_bit_cast(cbf16x8, (__attribute__((ext_vector_type(8))) short){
                                                    lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, acc[i][tt], 0, 0, 0);
        }
        if (bias_w) {          // co rows wr*64 + 32 wc .. +31 (wave-uniform branch: a runtime index into af -> scratch)
          if (wc == 0) {
            bacc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], ones, bacc[0], 0, 0, 0);
            bacc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], ones, bacc[1], 0, 0, 0);
          } else {
            bacc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2], ones, bacc[0], 0, 0, 0);
            bacc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[3], ones, bacc[1], 0, 0, 0);
          }
        }
      }
    };

    int sd = GD_B, sx = GX_B;          // stage 0 -> 1 address deltas
    for (int t = t0, b = 0; t < t1; ++t, b ^= 1) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      issue(t + 1 < t1 ? t + 1 : t, b ^ 1, t + 1 < t1);
      compute();
      // (transformed after this tile's MFMAs: between its k32 steps measured slower, 948 -> 988 us)
      if constexpr (XF) {
        if (t + 1 < t1) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          xform(t + 1, b ^ 1);
        }
      }
#pragma unroll
      for (int hi = 0; hi < 2; ++hi)
#pragma unroll
        for (int i = 0; i < 4; ++i) aad[hi][i] += sd;
#pragma unroll
      for (int m = 0; m < 16; ++m) xad[m] += sx;
      sd = -sd;
      sx = -sx;
    }

    // slab [split][Cout][9 Cin]: lane holds rows co = 4 (lane>>4) + rr of each 16-row frag, column lane & 15
    float *dst = a.part + (int64_t)split * Cout * NP;
    const int co0 = ct * 128 + wr * 64 + 4 * g;
    const int cl = c32 + wc * 16 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) dst[(int64_t)(co0 + i * 16 + rr) * NP + (TB + tt) * Cin + cl] = acc[i][tt][rr];
    if (bias_w && (lane & 15) == 0)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          a.dbias_part[(int64_t)split * Cout + ct * 128 + wr * 64 + wc * 32 + h * 16 + 4 * g + rr] = bacc[h][rr];
  };
  if constexpr (NG == 3) {
    if (kq == 0) run(ic_t<0>{});
    else if (kq == 1) run(ic_t<1>{});
    else run(ic_t<2>{});
  } else if constexpr (TS) {
    if (kq == 0) run(ic_t<0>{});
    else run(ic_t<1>{});
  } else {
    run(ic_t<0>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int wgrad_win_splits(const WgradArgs &a, int64_t x_bytes) {
  const ConvGeom &g = a.g;
  if (!g_win || g.ks != 3 || g.stride != 1 || g.pad != 1 || g.H % GT_R || g.W % GT_C || g.Ho != g.H || g.Wo != g.W)
    return 0;
  if (g.Cin % 32 || a.xgc % 32 || g.Cout % 128) return 0;
  if (x_bytes >= (int64_t)OOB || a.M * g.Cout * 2 >= (int64_t)OOB) return 0;
  const int64_t ntile = a.M / (GT_R * GT_C);
  const int ncb = g.Cin / 32, nct = g.Cout / 128;
  int G = cu_count();
  if (g_grid_cap > 0 && g_grid_cap < G) G = g_grid_cap;
  int64_t s = G / (ncb * nct);
  if (s < 1) s = 1;
  if (s > ntile) s = ntile;
  return (int)s;
}

// the tap-split 8-wave variant (default): two waves per SIMD hide each other's LDS fragment
// reads behind MFMAs — config 4 1513 -> 1592 frames/s, config 2 3621 -> 3627 (same box,
// profiles/r05/ab/wgrad_tap_split.log); 0 (EWVIT_WGWIN_TS=0): the 4-wave kernel; 2: 12 waves,
// one kernel row per wave group
int g_wgwin_ts = 1;

template <bool BIAS, bool XF, int NG>
static void launch_wgrad_win_t(const WgradArgs &a, int64_t x_bytes, int splits, int ncb, int nct, int ntile, hipStream_t s) {
  const unsigned nwg = (unsigned)(splits * ncb * nct);
  hipLaunchKernelGGL((conv_wgrad_win_kernel<BIAS, XF, NG>), dim3(nwg), dim3(NG * 256),
                     lds_pad(conv_wgrad_win_kernel<BIAS, XF, NG>, GSMEM), s, a, x_bytes, splits, ncb, nct, ntile);
}

bool launch_wgrad_win(const WgradArgs &a_in, int64_t x_bytes, int splits, hipStream_t s) {
  WgradArgs a = a_in;
  a.nt = g_grid_cap > 0 ? (g_win_nt >> 1) & 3 : 0;   // beside the backbone only (see g_win_nt)
  const int ncb = a.g.Cin / 32, nct = a.g.Cout / 128;
  const int ntile = (int)(a.M / (GT_R * GT_C));
  const bool b = a.dbias_part != nullptr, x = a.xf != nullptr;
  auto go = [&](auto TSc) {
    constexpr int T = decltype(TSc)::value;
    if (x && b) launch_wgrad_win_t<true, true, T>(a, x_bytes, splits, ncb, nct, ntile, s);
    else if (x) launch_wgrad_win_t<false, true, T>(a, x_bytes, splits, ncb, nct, ntile, s);
    else if (b) launch_wgrad_win_t<true, false, T>(a, x_bytes, splits, ncb, nct, ntile, s);
    else launch_wgrad_win_t<false, false, T>(a, x_bytes, splits, ncb, nct, ntile, s);
  };
  if (g_wgwin_ts == 2) go(ic_t<3>{});
  else if (g_wgwin_ts) go(ic_t<2>{});
  else go(ic_t<1>{});
  return true;
}

bool launch_win(const FwdArgs &a_in, int64_t src_bytes, bool dgrad, hipStream_t s) {
  FwdArgs a = a_in;
  a.nt = (g_win_nt & 1) && g_grid_cap > 0;   // beside the backbone only (see g_win_nt)
  if (!win_ok(a, dgrad) || src_bytes >= (int64_t)OOB) return false;
  const bool ks = win_ks(a, dgrad);
  const int ntn = ks ? 1 : a.Ncol / 128;
  const int ntiles = (int)(a.M / (WT * WT) * ntn);
  int G = cu_count();
  if (g_grid_cap > 0 && g_grid_cap < G) G = g_grid_cap;
  if (G > ntiles) G = ntiles;
  const int ncb = a.KC / 64;
  const int64_t ob = 2 * (a.ogs ? (a.Ncol / a.ogc - 1) * a.ogs + a.M * a.ogc : a.M * a.Ncol);
  if (ks && a.bwd.part)
    hipLaunchKernelGGL((conv_win_kernel<true, false, false, true, true>), dim3(G), dim3(512), lds_pad(conv_win_kernel<true, false, false, true, true>, SMEM_B), s, a, src_bytes, ob, ntn, ntiles, ncb);
  else if (ks)
    hipLaunchKernelGGL((conv_win_kernel<true, false, false, false, true>), dim3(G), dim3(512), lds_pad(conv_win_kernel<true, false, false, false, true>, SMEM_B), s, a, src_bytes, ob, ntn, ntiles, ncb);
  else if (dgrad && a.bwd.part)
    hipLaunchKernelGGL((conv_win_kernel<true, false, false, true>), dim3(G), dim3(512), lds_pad(conv_win_kernel<true, false, false, true>, SMEM_B), s, a, src_bytes, ob, ntn, ntiles, ncb);
  else if (dgrad)
    hipLaunchKernelGGL((conv_win_kernel<true, false>), dim3(G), dim3(512), lds_pad(conv_win_kernel<true, false>, SMEM_B), s, a, src_bytes, ob, ntn, ntiles, ncb);
  else if (a.xf && a.bn_part)
    hipLaunchKernelGGL((conv_win_kernel<false, true, true>), dim3(G), dim3(512), lds_pad(conv_win_kernel<false, true, true>, SMEM_B), s, a, src_bytes, ob, ntn, ntiles, ncb);
  else if (a.xf)
    hipLaunchKernelGGL((conv_win_kernel<false, false, true>), dim3(G), dim3(512), lds_pad(conv_win_kernel<false, false, true>, SMEM_B), s, a, src_bytes, ob, ntn, ntiles, ncb);
  else if (a.bn_part)
    hipLaunchKernelGGL((conv_win_kernel<false, true>), dim3(G), dim3(512), lds_pad(conv_win_kernel<false, true>, SMEM_B), s, a, src_bytes, ob, ntn, ntiles, ncb);
  else
    hipLaunchKernelGGL((conv_win_kernel<false, false>), dim3(G), dim3(512), lds_pad(conv_win_kernel<false, false>, SMEM_B), s, a, src_bytes, ob, ntn, ntiles, ncb);
  return true;
}

}  // namespace ewvit

extern "C" int ewvit_conv2d_set_wgrad_tap_split(int on) {
  const int prev = ewvit::g_wgwin_ts;
  ewvit::g_wgwin_ts = on == 2 ? 2 : on ? 1 : 0;
  return prev;
}

extern "C" int ewvit_conv2d_set_lds_pad(int on) {
  const int prev = ewvit::g_lds_pad;
  ewvit::g_lds_pad = on ? 1 : 0;
  return prev;
}

// A/B switch: the non-temporal hint on the windowed MWT convs' activation-window DMAs (mask,
// see g_win_nt)
extern "C" int ewvit_conv2d_set_win_nt(int mask) {
  const int prev = ewvit::g_win_nt;
  ewvit::g_win_nt = mask & 7;
  return prev;
}

extern "C" int ewvit_conv2d_set_win(int variant) {
  const int prev = ewvit::g_win;
  ewvit::g_win = variant ? 1 : 0;
  return prev;
}
