// Shared declarations of the conv kernels (conv.hip: the generic implicit-GEMM family;
// convwin.hip: the windowed 3x3 stride-1 kernels of the MWT's big maps).
#pragma once
#include "common.h"

namespace ewvit {

typedef __attribute__((ext_vector_type(8))) __bf16 cbf16x8;
typedef __attribute__((ext_vector_type(4))) float cf32x4;
typedef __attribute__((ext_vector_type(4))) short cs4;

constexpr int CBM = 128, CBN = 128, CBK = 32;

struct ConvGeom {
  int N, H, W, Cin;      // x (fwd) / dx (dgrad) grid
  int Ho, Wo, Cout;      // y / dy grid
  int stride, ks, pad;   // ks 1|3, pad = ks/2
};

// ---------------------------------------------------------------- fwd / dgrad
// A(m, k): m = pixel of the OUTPUT grid of this GEMM (y for fwd, dx for dgrad),
// k = tap * KC + c (KC = Cin for fwd, Cout for dgrad).  B(k, n) = Wp[n][k].
struct FwdArgs {
  const bf16_t *src = nullptr;   // gathered operand: x (fwd) or dy (dgrad), grouped NHWC
  const bf16_t *wp = nullptr;    // packed weights [Ncol][taps][KC]
  const float *bias = nullptr;   // [Ncol] or null
  bf16_t *out = nullptr;         // [M][Ncol], grouped NHWC
  ConvGeom g;
  int64_t M;
  int Ncol, KC;          // GEMM N and per-tap K
  int srcH, srcW;        // spatial size of `src`
  int outH, outW;        // spatial size of the GEMM's output grid
  int sgc, ogc;          // channel group widths of src / out
  int64_t sgs, ogs;      // group strides (elements)
  // optional BatchNorm statistics of the (bf16-rounded) output, LDS-DMA fwd only:
  // per m-tile t and column c, bn_part[t][c] = sum (y - K[c]), bn_part[t][Ncol + c] =
  // sum (y - K[c])^2 with K = bn_shift (or 0); tile 0 copies K to bn_shift_out
  const float *bn_shift = nullptr;
  float *bn_part = nullptr;
  float *bn_shift_out = nullptr;
  // LDS-DMA fwd over a plain NHWC x whose channel count is not a multiple of 64: KC is
  // the per-tap K padded up to 64 (the weights packed with that many input channels)
  // and the staging lanes of channels >= KCr (the real count) read zeros
  int KCr = 0;
  int nt = 0;            // windowed fwd / dgrad: non-temporal hint on the window DMAs
  // optional addend of the output (same layout as out, bf16), added before rounding —
  // the skip connection's gradient folded into the block input's dgrad
  const bf16_t *addend = nullptr;
  // stride-2 3x3 dgrad by output parity class (LDS-DMA kernel): the GEMM rows are the
  // dx pixels (2i + py, 2j + px) of class pc = 2*py + px on an outH x outW grid, and
  // only the class's ntap live taps tapl[] run (dy pixel (i + dh, j + dw)); the
  // epilogue scatters row (n, i, j) to dx pixel (n, 2i + py, 2j + px) of dstH x dstW
  int pc = -1, ntap = 0;
  int tapl[4] = {0, 0, 0, 0};
  int dstH = 0, dstW = 0;
  // optional (LDS-DMA dgrad, plain NHWC dx, uncapped grid): the backward statistics of the
  // BatchNorm(+act) whose output this conv read, summed over the bf16-rounded dx per m-tile
  // (common.h BnBwdStats; bwd.part [m-tiles][2 Ncol])
  BnBwdStats bwd;
  // optional input transform of the windowed fwd (convwin.hip, XF): the conv reads
  // relu(x * xf[g][0][c] + xf[g][1][c]) — a training BatchNorm + ReLU applied by its producer's
  // coefficients (ewvit_bn_coef) — instead of x; channel group g = c / sgc, zero padding after
  // the transform
  const float *xf = nullptr;
  // split K (LDS-DMA 1x1 fwd / dgrad over few tiles, conv.hip launch_glds): work item i is
  // (tile i / ksplit, K-range i % ksplit of nk / ksplit K-tiles), which stores its fp32 partial
  // tile at kpart[split][M][Ncol]; conv_splitk_epi_kernel sums the splits and runs the epilogue
  int ksplit = 1;
  float *kpart = nullptr;
};

typedef __attribute__((address_space(3))) void lds_t;
constexpr uint32_t OOB = 0x80000000u;   // any offset >= num_records reads as zero

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const void *p, int64_t bytes) {
  const uint32_t n = bytes >= (int64_t)OOB ? OOB : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)n, 0x00020000);
}
__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, unsigned char *lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t *)lds, 16, voff, 0, 0, 0);
}
// bijective XCD remap: blocks b, b+8, b+16 ... (one XCD) get consecutive tile ids
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// wait until at most the N youngest vector-memory ops (LDS-DMA pieces) are pending,
// then the workgroup barrier; one asm statement, so hipcc neither drains the DMA
// queue at the barrier nor moves LDS reads across it
template <int N> __device__ __forceinline__ void wait_vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}
// tile kt's pieces landed (L per tile per thread); `rem` younger tiles already issued
// (at most NS-2 of them) may stay in flight across the barrier
template <int L, int NS> __device__ __forceinline__ void wait_tile(int rem) {
  if constexpr (NS >= 4) { if (rem >= 2) { wait_vm_barrier<2 * L>(); return; } }
  if constexpr (NS >= 3) { if (rem >= 1) { wait_vm_barrier<L>(); return; } }
  wait_vm_barrier<0>();
}

// LDS-DMA issued from inline asm: hipcc cannot see these, so it neither waits on them before
// LDS reads (it drains the whole vmcnt queue ahead of any LDS access that may alias a builtin
// DMA) nor counts them; every kernel using them waits with explicit vmcnt counts (wait_tile,
// win_sync).  M0 (the DMA's LDS base) is reserved to hipcc, which sets it before each of its
// own uses; no other M0 user runs in these kernels.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// a buffer resource as four dwords (gfx9 layout: base, base_hi | stride << 16, num_records,
// flags), so the asm operand can be pinned to SGPRs with readfirstlane (hipcc's divergence
// analysis sometimes leaves uniform values in VGPRs, which an "s" operand then rejects)
typedef __attribute__((ext_vector_type(4))) int ci32x4;
__device__ __forceinline__ ci32x4 mk_rsrc4(const void *p, int64_t bytes) {
  const uint32_t n = bytes >= (int64_t)OOB ? OOB : (uint32_t)bytes;
  const uint64_t a = (uint64_t)(uintptr_t)p;
  return ci32x4{(int)(uint32_t)a, (int)((uint32_t)(a >> 32) & 0xffff), (int)n, 0x00020000};
}
__device__ __forceinline__ void glds16_asm(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds), "v"(voff), "s"(r)
               : "memory", "m0");
}
__device__ __forceinline__ void glds16_asm(ci32x4 r, uint32_t lds, uint32_t voff) {
  const ci32x4 rr = {__builtin_amdgcn_readfirstlane(r[0]), __builtin_amdgcn_readfirstlane(r[1]),
                     __builtin_amdgcn_readfirstlane(r[2]), __builtin_amdgcn_readfirstlane(r[3])};
  const uint32_t l = __builtin_amdgcn_readfirstlane(lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(l), "v"(voff), "s"(rr)
               : "memory", "m0");
}
// ... with the non-temporal hint when `nt` (a uniform kernel argument: a scalar branch): the
// windowed MWT convs' activation windows (A/B, ewvit_conv2d_set_win_nt) — streamed once per
// tile, so they need not keep their L2 lines against the concurrent backbone's working set
__device__ __forceinline__ void glds16_asm(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff, bool nt) {
  if (nt)
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds" ::"s"(lds), "v"(voff),
                 "s"(r) : "memory", "m0");
  else
    glds16_asm(r, lds, voff);
}
__device__ __forceinline__ void glds16_asm(ci32x4 r, uint32_t lds, uint32_t voff, bool nt) {
  if (nt) {
    const ci32x4 rr = {__builtin_amdgcn_readfirstlane(r[0]), __builtin_amdgcn_readfirstlane(r[1]),
                       __builtin_amdgcn_readfirstlane(r[2]), __builtin_amdgcn_readfirstlane(r[3])};
    const uint32_t l = __builtin_amdgcn_readfirstlane(lds);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds" ::"s"(l), "v"(voff),
                 "s"(rr) : "memory", "m0");
  } else {
    glds16_asm(r, lds, voff);
  }
}
#pragma clang diagnostic pop

// ---------------------------------------------------------------- wgrad
// A(co, m) = dy[m][co]   -> image Ast[m][co]  (rows of 128 co = 256 B)
// B(m, n') = x[pix(m,tap)][ci] -> image Bst[m][n'] (rows of 128 n' = 256 B)
// 16-B chunk ch of row r lives at 256*r + 16*(ch ^ swz(r)),
// swz(r) = ((r&3)<<2) | ((r>>2)&3)  (T10 image (b): conflict-free tr reads).
struct WgradArgs {
  const bf16_t *x;       // [N, H, W, Cin], grouped (xgc, xgs)
  const bf16_t *dy;      // [N, Ho, Wo, Cout]
  float *part;           // [splits][Cout][taps*Cin]
  float *dbias_part;     // [splits][Cout] partial bias gradients (sum of dy), or null
  ConvGeom g;
  int64_t M;             // N*Ho*Wo
  int64_t mper;          // pixels per split (multiple of 32)
  int xgc;
  int64_t xgs;
  const float *xf = nullptr;  // input transform of the windowed wgrad (FwdArgs::xf; groups of xgc)
  int nt = 0;                 // windowed wgrad: non-temporal hint, 1 the dy tile DMAs, 2 the x windows'
};

__device__ __forceinline__ int swz_off(int r, int ch) {
  return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3)));
}

// the windowed 3x3 stride-1 fwd / dgrad (convwin.hip): true when it ran the shape
bool launch_win(const FwdArgs &a, int64_t src_bytes, bool dgrad, hipStream_t s);
bool win_ok(const FwdArgs &a, bool dgrad);
extern int g_win;   // 1: the windowed kernels take the shapes they accept (default), 0: never
// the windowed 3x3 stride-1 weight gradient (convwin.hip): pixel splits it would use for this
// shape (0 = it does not take the shape), and the launch (slabs [splits][Cout][9*Cin] +
// bias partials [splits][Cout] for conv_wgrad_reduce_kernel)
int wgrad_win_splits(const WgradArgs &a, int64_t x_bytes);
bool launch_wgrad_win(const WgradArgs &a, int64_t x_bytes, int splits, hipStream_t s);

}  // namespace ewvit
