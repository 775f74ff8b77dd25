// Map which A-scale lane of v_mfma_scale_f32_16x16x128_f8f6f4 scales which (row, k-run) of A:
// A = 1 everywhere, B column c = (lane group g = c & 3, elements 8 (c >> 2) .. + 8) ones; wave L
// sets A scale 2^1 on lane L only (B scales 1): C[i][c] = 16 where lane L's scale applies.
//   hipcc --offload-arch=gfx950 -O2 tools/mx8_scale_map.hip -o tools/mx8_scale_map
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef __attribute__((ext_vector_type(8))) int v8i;
typedef __attribute__((ext_vector_type(4))) float vf4;
__global__ void k(float *out, int which) {
  const int l = threadIdx.x, L = blockIdx.x;
  v8i a, b;
  const int one = 0x38;                        // e4m3 1.0
  for (int d = 0; d < 8; ++d) a[d] = one | (one << 8) | (one << 16) | (one << 24);
  const int c = l & 15, g = c & 3, q = c >> 2;
  for (int d = 0; d < 8; ++d) b[d] = ((l >> 4) == g && (d >> 1) == q) ? (one | (one << 8) | (one << 16) | (one << 24)) : 0;
  const int base = 127 | (100 << 8) | (100 << 16) | (100 << 24);
  int sa = base, sb = base;
  if (which == 0 && l == L) sa = 128 | (100 << 8) | (100 << 16) | (100 << 24);
  if (which == 1 && l == L) sb = 128 | (100 << 8) | (100 << 16) | (100 << 24);
  vf4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sa, 0, sb);
  for (int r = 0; r < 4; ++r) out[L * 256 + ((l >> 4) * 4 + r) * 16 + (l & 15)] = acc[r];
}
int main() {
  float *d;
  hipMalloc(&d, 64 * 256 * 4);
  std::vector<float> h(64 * 256);
  for (int which = 0; which < 2; ++which) {
    hipLaunchKernelGGL(k, dim3(64), dim3(64), 0, 0, d, which);
    hipMemcpy(h.data(), d, 64 * 256 * 4, hipMemcpyDeviceToHost);
    printf("%s scale lane -> (row, part g.q) cells != 8 (value)\n", which ? "B" : "A");
    for (int L = 0; L < 64; ++L) {
      printf("L%2d:", L);
      int n = 0;
      for (int i = 0; i < 16; ++i)
        for (int c = 0; c < 16; ++c) {
          const float v = h[L * 256 + i * 16 + c];
          if (v != 8.f) {
            if (n < 12) printf(" (%d,%d.%d)=%g", i, c & 3, c >> 2, v);
            ++n;
          }
        }
      printf("  [%d cells]\n", n);
    }
  }
  return 0;
}
