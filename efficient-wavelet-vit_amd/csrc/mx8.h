// MXFP8 operands for v_mfma_scale_f32_16x16x128_f8f6f4 (gfx950): OCP e4m3fn elements with one
// E8M0 scale per 32 consecutive K elements of a row (the OCP MX block), fp32 accumulation — the
// fp8 form of the token GEMMs (BASELINE configs[4]).  The block scale is local to 32 elements,
// so no per-tensor amax pass exists anywhere: activations are quantized by the kernel that forms
// their fragments, weights once per step by the weight pack.
//
// Operand lane map of the 16 x 16 x 128 form, measured with exact data (tools/mx8_probe.hip,
// tools/mx8_scale_map.hip): lane l = 16 g + r holds row (A) / column (B) r, K elements
// [16 g, 16 g + 16) in bytes 0..15 and [64 + 16 g, 64 + 16 g + 16) in bytes 16..31; the scale VGPR
// of lane 16 b + r (byte 0, op_sel 0) is the E8M0 scale of row / column r's K block b =
// [32 b, 32 b + 32).  So block b's 32 elements sit in lane groups 2 (b & 1) and 2 (b & 1) + 1
// (16 each, bytes 16 (b >> 1) ..), and its scale in lane group b.
#pragma once
#include "common.h"

namespace ewvit {

typedef __attribute__((ext_vector_type(8))) int mx_v8i;
typedef __attribute__((ext_vector_type(4))) float mx_vf4;

// the K offsets (within a 128-wide K step) of a lane's two 16-element runs
__device__ __forceinline__ int mx_k0(int lane) { return 16 * (lane >> 4); }
__device__ __forceinline__ int mx_k1(int lane) { return 64 + 16 * (lane >> 4); }

// biased E8M0 exponent e of the smallest power of two 2^X with amax <= 448 * 2^X (so every
// v * 2^-X is within e4m3's range and the block maximum lands in (224, 448]); 127 (scale 1) for
// an all-zero block.  Exact: from the bits of amax (448 = 1.75 * 2^8).
__device__ __forceinline__ int mx_exp(float amax) {
  const unsigned b = __float_as_uint(amax);
  if (amax == 0.f) return 127;
  const int ea = (int)((b >> 23) & 255) - 127;
  const int x = ea - 8 + ((b & 0x7fffffu) > 0x600000u ? 1 : 0);
  const int e = x + 127;
  return e < 1 ? 1 : (e > 253 ? 253 : e);
}
// 2^-X for a biased exponent e (exact power of two)
__device__ __forceinline__ float mx_inv_scale(int e) { return __uint_as_float((unsigned)(254 - e) << 23); }

// 16 floats scaled by s -> 4 dwords of e4m3 (round to nearest even; |v s| <= 448 by
// construction of s, so no saturation), element j in byte j % 4 of dword j / 4
__device__ __forceinline__ void mx_cvt16(const float *v, float s, int *d) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * q] * s, v[4 * q + 1] * s, 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * q + 2] * s, v[4 * q + 3] * s, w, true);
    d[q] = w;
  }
}
__device__ __forceinline__ float mx_amax16(const float *v) {
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) m = fmaxf(m, fabsf(v[j]));
  return m;
}

struct MxFrag {
  mx_v8i d;
  int sc;        // E8M0 scale of block (lane >> 4) of this lane's row / column
};

// An operand fragment quantized in registers: v[0..15] = the lane's row at K offsets
// mx_k0(lane) .., v[16..31] at mx_k1(lane) .. (zeros for rows past the matrix).  The two lanes
// holding one block (lane groups 2c, 2c + 1) share their maxima; lane group b then takes block
// b's scale from lane group 2 (b & 1) (byte b >> 1 of its pair of exponents).
__device__ __forceinline__ MxFrag mx_quant(const float *v) {
  const int lane = threadIdx.x & 63;
  float m0 = mx_amax16(v), m1 = mx_amax16(v + 16);
  m0 = fmaxf(m0, __shfl_xor(m0, 16, 64));
  m1 = fmaxf(m1, __shfl_xor(m1, 16, 64));
  const int e0 = mx_exp(m0), e1 = mx_exp(m1);
  MxFrag f;
  int d[8];
  mx_cvt16(v, mx_inv_scale(e0), d);
  mx_cvt16(v + 16, mx_inv_scale(e1), d + 4);
#pragma unroll
  for (int q = 0; q < 8; ++q) f.d[q] = d[q];
  const int h = lane >> 4;
  const int got = __shfl(e0 | (e1 << 8), ((h & 1) << 5) | (lane & 15), 64);
  f.sc = (got >> (8 * (h >> 1))) & 255;
  return f;
}

// acc += A_frag . B_frag with both block scales (e4m3 x e4m3)
__device__ __forceinline__ mx_vf4 mx_mma(const MxFrag &a, const MxFrag &b, mx_vf4 c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a.d, b.d, c, 0, 0, 0, a.sc, 0, b.sc);
}

// A pre-quantized operand row (the weight packs): bytes of row r at K offsets k0 .. k0 + 15 and
// k1 .. k1 + 15 of the 128-wide step, and its scale byte for block (lane >> 4)
__device__ __forceinline__ MxFrag mx_load(const uint8_t *row, int kstep, const uint8_t *srow) {
  const int lane = threadIdx.x & 63;
  const uint4 a = *reinterpret_cast<const uint4 *>(row + kstep + mx_k0(lane));
  const uint4 b = *reinterpret_cast<const uint4 *>(row + kstep + mx_k1(lane));
  MxFrag f;
  f.d[0] = (int)a.x; f.d[1] = (int)a.y; f.d[2] = (int)a.z; f.d[3] = (int)a.w;
  f.d[4] = (int)b.x; f.d[5] = (int)b.y; f.d[6] = (int)b.z; f.d[7] = (int)b.w;
  f.sc = srow[kstep / 32 + (lane >> 4)];
  return f;
}

// Block-quantize 32 consecutive values (one MX block) for a pack: the exponent byte and the 32
// e4m3 bytes (as 8 dwords)
__device__ __forceinline__ int mx_quant_block(const float *v, int *d) {
  const int e = mx_exp(fmaxf(mx_amax16(v), mx_amax16(v + 16)));
  const float s = mx_inv_scale(e);
  mx_cvt16(v, s, d);
  mx_cvt16(v + 16, s, d + 4);
  return e;
}

}  // namespace ewvit
