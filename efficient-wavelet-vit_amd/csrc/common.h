// Shared device/host helpers for the ewvit HIP library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <cstdarg>

#include "../../include/ewvit.h"

// the non-temporal cache hint on the rest of the MWT branch's streaming traffic (the windowed
// convs' output stores and BN-input loads, the separable conv, the ReLU BatchNorm passes) on top
// of the window DMAs' (convwin.hip g_win_nt, on): 0 (default).  Measured with it compiled in:
// config 2 3577-3583 vs 3626-3630 frames/s without any MWT hint, three interleaved same-box
// rounds (profiles/r06/ab/mwt_nt.log) — the backbone reads those maps' neighbours back through
// L2 sooner than the hint assumes
#ifndef EWVIT_MWT_NT
#define EWVIT_MWT_NT 0
#endif

namespace ewvit {

// ---------------------------------------------------------------- errors
void set_error(const char *fmt, ...);

#define EWVIT_CHECK_ARG(cond, ...)                \
  do {                                            \
    if (!(cond)) {                                \
      ::ewvit::set_error(__VA_ARGS__);            \
      return EWVIT_EINVAL;                        \
    }                                             \
  } while (0)

inline int launch_status(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------- bf16
typedef unsigned short bf16_t;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}
// round-to-nearest-even; NaN stays NaN (hipcc lowers the plain cast to v_cvt_pk_bf16_f32)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

template <int DT> struct Elem;
template <> struct Elem<EWVIT_F32> {
  typedef float T;
  __device__ __forceinline__ static float load(const void *p, int64_t i) {
    return reinterpret_cast<const float *>(p)[i];
  }
  __device__ __forceinline__ static void store(void *p, int64_t i, float v) {
    reinterpret_cast<float *>(p)[i] = v;
  }
};
template <> struct Elem<EWVIT_BF16> {
  typedef bf16_t T;
  __device__ __forceinline__ static float load(const void *p, int64_t i) {
    return bf2f(reinterpret_cast<const bf16_t *>(p)[i]);
  }
  __device__ __forceinline__ static void store(void *p, int64_t i, float v) {
    reinterpret_cast<bf16_t *>(p)[i] = f2bf(v);
  }
};

__device__ __forceinline__ float load_dt(const void *p, int64_t i, int dt) {
  return dt == EWVIT_F32 ? reinterpret_cast<const float *>(p)[i]
                         : bf2f(reinterpret_cast<const bf16_t *>(p)[i]);
}
__device__ __forceinline__ void store_dt(void *p, int64_t i, float v, int dt) {
  if (dt == EWVIT_F32)
    reinterpret_cast<float *>(p)[i] = v;
  else
    reinterpret_cast<bf16_t *>(p)[i] = f2bf(v);
}

// ---------------------------------------------------------------- RNG
// Counter-based hash (splitmix64 finaliser) for dropout: keep(seed, i) is a
// pure function, so backward regenerates the forward mask without storing it.
// The effective seed of a launch is seed + *seed_offset * golden (seed_offset: a
// device int64 advanced once per training step, or null), so a launch recorded
// into a HIP graph draws a fresh mask on every replay.
__device__ __forceinline__ uint64_t step_seed(uint64_t seed, const int64_t *seed_offset) {
  return seed_offset ? seed + 0xD1B54A32D192ED03ull * (uint64_t)(*seed_offset) : seed;
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t i) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (i + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// Cross-lane sums on DPP / v_permlane*_swap (VALU) instead of ds_bpermute: every
// lane of the group ends with the group's sum.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// the 16 lanes of a DPP row (lanes 16r .. 16r+15)
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_mov<0xB1>(v);     // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);     // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);    // row_half_mirror
  v += dpp_mov<0x140>(v);    // row_mirror
  return v;
}
// lanes l, l^16, l^32, l^48 (the 4 rows of the wave)
__device__ __forceinline__ float rows_sum4(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  v = __int_as_float(a[0]) + __int_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(b[0]) + __int_as_float(b[1]);
}
__device__ __forceinline__ float wave_sum(float v) { return rows_sum4(row_sum16(v)); }
// the same butterfly with max (every lane ends with the wave's maximum)
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x141>(v));
  v = fmaxf(v, dpp_mov<0x140>(v));
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  v = fmaxf(__int_as_float(a[0]), __int_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return fmaxf(__int_as_float(b[0]), __int_as_float(b[1]));
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// derivative of a BatchNorm's activation at its pre-activation z (act 1 ReLU, 2 SiLU, else
// identity) — the same operations as batchnorm.hip's act_grad, so producers that sum the
// backward statistics in their epilogue round exactly as bn_bwd_reduce_kernel would
__device__ __forceinline__ float bn_act_grad(int act, float z) {
  if (act == 1) return z > 0.f ? 1.f : 0.f;
  if (act == 2) {
    const float s = __builtin_amdgcn_rcpf(1.f + __expf(-z));
    return s * (1.f + z * (1.f - s));
  }
  return 1.f;
}

// BatchNorm backward statistics left by the kernel that produces the BN output's gradient
// (the consumer conv's input gradient): per partial row t and channel c, part[t][c] = sum g,
// part[t][C + c] = sum g * xhat over the producer's tile rows, with xhat = (x - mean) * invstd
// (x: the BN input, same layout as the gradient), g = d * act'(xhat * gamma + beta) (act) or
// g = d * rscale[row / hw] (rscale: the drop-path factor of the MBConv tail); what
// bn_bwd_dx_kernel finalises from (ewvit_bn_bwd_partials)
struct BnBwdStats {
  float *part = nullptr;
  const bf16_t *x = nullptr;
  const float *mean = nullptr, *invstd = nullptr, *gamma = nullptr, *beta = nullptr, *rscale = nullptr;
  int act = 0, hw = 1;
  int64_t grows = 0;   // rows per BatchNorm row group (consecutive batch slices with their own
                       // statistics: mean / invstd [group][C]); 0 = one group
};

inline bool dtype_ok(int dt) { return dt == EWVIT_F32 || dt == EWVIT_BF16; }

// workgroup cap of the big-grid launches (abi.hip, ewvit_set_grid_cap); 0 = none; per host thread
extern thread_local int g_grid_cap;

}  // namespace ewvit
