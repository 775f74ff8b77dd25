// Shared device/host helpers for the ewvit HIP library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <cstdarg>

#include "../../include/ewvit.h"

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

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

inline bool dtype_ok(int dt) { return dt == EWVIT_F32 || dt == EWVIT_BF16; }

}  // namespace ewvit
