// Deferred weight-gradient reductions.
//
// The backbone's split-K weight gradients (1x1 / LDS-DMA kernels, conv.hip) and the depthwise
// backward (depthwise.hip) leave fp32 partial slabs that a small reduce kernel sums into dW:
// ~110 launches of 5 us per backbone backward pass, each a kernel boundary on the critical
// path.  A caller that knows nothing reads dW before the end of the backward pass (the
// gradient-slot case, ewvit/conv.py) marks the next such call "defer" (ewvit_reduce_defer_next):
// its reduce is queued per stream instead of launched, and the NEXT weight-gradient launch on
// that stream runs it in extra workgroups ahead of its own tiles (RedJobs, at most 2 jobs); what
// is still queued at the end runs in ewvit_reduce_flush.  Same code, same summation order:
// bit-identical to the separate reduce launches.
#pragma once
#include "common.h"

namespace ewvit {

// the destination layout of a conv dW: element (co, ci, tap) at co*s_co + ci*s_ci + tap*s_tap,
// only ci < cin stored (the parameter's own strides and real input channels)
struct WOut {
  int64_t s_co, s_ci, s_tap;
  int cin;
};

struct RedJob {
  const float *part = nullptr;
  float *dw = nullptr;
  int64_t n = 0;          // outputs: Cout * taps * Cin (conv) or C * 9 (depthwise)
  int kind = 0;           // 0 none, 1 conv split-K reduce, 2 depthwise slab reduce
  int Cin = 0, taps = 0, splits = 0, accumulate = 0, T = 1, nblk = 0;
  WOut wo{};
};
struct RedJobs {
  RedJob j[2];
  int nblk = 0;           // extra workgroups in all (a multiple of 8: the host's XCD remap)
};

// dW[co][ci][tap] (= or +=) sum over splits of part[s][co][tap*Cin + ci] (no bias).  T lanes of
// a wave share one 4-element output (T = splits fan-in, a power of two <= 64): lane l sums
// splits l, l+T, ... (4 loads in flight), then an xor tree over the T lanes — fixed order.
__device__ __forceinline__ void wgrad_reduce_block(const float *__restrict__ part, float *__restrict__ dw,
                                                   int Cin, int taps, int splits, int accumulate, WOut wo, int T,
                                                   int64_t n, int blk) {
  const int tid = threadIdx.x;
  const int64_t NP = taps * (int64_t)Cin;
  const int sl = tid & (T - 1);
  const int64_t i = ((int64_t)blk * (256 / T) + tid / T) * 4;
  const bool ok = i < n;
  const int64_t ii = ok ? i : 0;
  float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0, s2 = s0, s3 = s0;
  int k = sl;
  for (; k + 3 * T < splits; k += 4 * T) {
    const float4 a = *reinterpret_cast<const float4 *>(part + (int64_t)k * n + ii);
    const float4 b = *reinterpret_cast<const float4 *>(part + (int64_t)(k + T) * n + ii);
    const float4 c = *reinterpret_cast<const float4 *>(part + (int64_t)(k + 2 * T) * n + ii);
    const float4 d = *reinterpret_cast<const float4 *>(part + (int64_t)(k + 3 * T) * n + ii);
    s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
    s1.x += b.x; s1.y += b.y; s1.z += b.z; s1.w += b.w;
    s2.x += c.x; s2.y += c.y; s2.z += c.z; s2.w += c.w;
    s3.x += d.x; s3.y += d.y; s3.z += d.z; s3.w += d.w;
  }
  for (; k < splits; k += T) {
    const float4 a = *reinterpret_cast<const float4 *>(part + (int64_t)k * n + ii);
    s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
  }
  float r[4] = {(s0.x + s1.x) + (s2.x + s3.x), (s0.y + s1.y) + (s2.y + s3.y),
                (s0.z + s1.z) + (s2.z + s3.z), (s0.w + s1.w) + (s2.w + s3.w)};
  for (int o = T >> 1; o >= 1; o >>= 1)
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] += __shfl_xor(r[e], o, 64);
  if (!ok || sl != 0) return;
  const int co = (int)(i / NP);
  const int np = (int)(i % NP);
  const int tap = np / Cin, ci = np % Cin;
  const int64_t o = co * wo.s_co + ci * wo.s_ci + tap * wo.s_tap;
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (ci + e < wo.cin) dw[o + e * wo.s_ci] = accumulate ? dw[o + e * wo.s_ci] + r[e] : r[e];
}

// Sum the per-block depthwise slabs [slabs][n]: block = 64 outputs x 4 slab groups (one wave
// each, 4 loads in flight), the 4 groups added through LDS `red` (256 floats) in fixed order.
// Called by the whole block (it synchronises).
__device__ __forceinline__ void dw_slab_reduce_block(const float *__restrict__ part, float *__restrict__ dw, int64_t n,
                                                     int slabs, int accumulate, int blk, float *red) {
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t i = (int64_t)blk * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (i < n) {
    int k = g;
    for (; k + 12 < slabs; k += 16) {
      s0 += part[(int64_t)k * n + i];
      s1 += part[(int64_t)(k + 4) * n + i];
      s2 += part[(int64_t)(k + 8) * n + i];
      s3 += part[(int64_t)(k + 12) * n + i];
    }
    for (; k < slabs; k += 4) s0 += part[(int64_t)k * n + i];
  }
  red[g * 64 + lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (g == 0 && i < n) {
    const float t = (red[lane] + red[64 + lane]) + (red[128 + lane] + red[192 + lane]);
    dw[i] = accumulate ? dw[i] + t : t;
  }
}

// host side of a job: its workgroups (256 threads each)
inline int red_job_blocks(const RedJob &j) {
  if (j.kind == 1) return (int)((j.n / 4 * j.T + 255) / 256);
  if (j.kind == 2) return (int)((j.n + 63) / 64);
  return 0;
}

// extra workgroup b (< r.nblk) of a host kernel: its part of job 0 or job 1 (or nothing: the
// round-up to 8).  `red`: 256 floats of LDS (the host's own buffer, unused by these blocks).
__device__ __forceinline__ void run_red_jobs(const RedJobs &r, int b, float *red) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const RedJob &j = r.j[q];
    if (b < j.nblk) {
      if (j.kind == 1) wgrad_reduce_block(j.part, j.dw, j.Cin, j.taps, j.splits, j.accumulate, j.wo, j.T, j.n, b);
      else if (j.kind == 2) dw_slab_reduce_block(j.part, j.dw, j.n, j.splits, j.accumulate, b, red);
      return;
    }
    b -= j.nblk;
  }
}

// ---- host registry (conv.hip): per-stream FIFO of deferred jobs
bool reduce_take_defer();                         // consume this thread's "defer the next reduce" mark
void reduce_defer(hipStream_t s, const RedJob &j);
RedJobs reduce_take_jobs(hipStream_t s);          // up to 2 oldest jobs of stream s (nblk 0: none)

}  // namespace ewvit
