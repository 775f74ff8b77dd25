// Probe of v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3 operands (gfx950): checks the lane map
// the MX kernels assume — lane l holds A[row l & 15][k = 32 (l >> 4) + j] and B[k = 32 (l >> 4)
// + j][col l & 15] in byte j of its 8 dwords, and the E8M0 scale in byte 0 of its scale VGPR
// applies to that lane's 32 values (2^(e - 127)) — with exact integer data.
//   hipcc --offload-arch=gfx950 -O2 tools/mx8_probe.hip -o tools/mx8_probe && ./tools/mx8_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

typedef __attribute__((ext_vector_type(8))) int v8i;
typedef __attribute__((ext_vector_type(4))) float vf4;

__global__ void probe(const v8i *a, const v8i *b, const int *sa, const int *sb, float *c) {
  const int l = threadIdx.x;
  vf4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa[l], 0, sb[l]);
  for (int r = 0; r < 4; ++r) c[((l >> 4) * 4 + r) * 16 + (l & 15)] = acc[r];
}

// small integers -8..8 and +-448 encode exactly in e4m3fn
static uint8_t enc(int v) {
  if (v == 0) return 0;
  uint8_t s = v < 0 ? 0x80 : 0;
  int a = std::abs(v);
  int e = 0;
  while ((a >> (e + 1)) > 0) ++e;            // a in [2^e, 2^(e+1))
  int m = e >= 3 ? (a >> (e - 3)) & 7 : (a << (3 - e)) & 7;
  return s | (uint8_t)(((e + 7) << 3) | m);
}

int main() {
  const int M = 16, N = 16, K = 128;
  int fails = 0;
  for (int trial = 0; trial < 3; ++trial) {
    std::vector<int> A(M * K), B(K * N);
    srand(11 + trial);
    for (auto &x : A) x = rand() % 17 - 8;
    for (auto &x : B) x = rand() % 17 - 8;
    if (trial == 2) { A[5 * K + 77] = 448; B[77 * N + 3] = -448; }
    std::vector<int> ea(64), eb(64);
    for (int l = 0; l < 64; ++l) {
      ea[l] = trial == 0 ? 127 : 127 + (l % 5) - 2;
      eb[l] = trial == 0 ? 127 : 127 + ((l * 7) % 3) - 1;
    }
    std::vector<int> pa(64 * 8, 0), pb(64 * 8, 0);
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 32; ++j) {
        const int k = 32 * (l >> 4) + j;
        pa[l * 8 + j / 4] |= (int)enc(A[(l & 15) * K + k]) << (8 * (j % 4));
        pb[l * 8 + j / 4] |= (int)enc(B[k * N + (l & 15)]) << (8 * (j % 4));
      }
    std::vector<double> ref(M * N, 0.0);
    for (int i = 0; i < M; ++i)
      for (int jj = 0; jj < N; ++jj)
        for (int k = 0; k < K; ++k) {
          const int g = k / 32;
          ref[i * N + jj] += (double)A[i * K + k] * B[k * N + jj] * std::ldexp(1.0, ea[g * 16 + i] - 127) *
                             std::ldexp(1.0, eb[g * 16 + jj] - 127);
        }
    v8i *da, *db;
    int *dsa, *dsb;
    float *dc;
    hipMalloc(&da, 64 * 32); hipMalloc(&db, 64 * 32); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256);
    hipMalloc(&dc, M * N * 4);
    hipMemcpy(da, pa.data(), 64 * 32, hipMemcpyHostToDevice);
    hipMemcpy(db, pb.data(), 64 * 32, hipMemcpyHostToDevice);
    hipMemcpy(dsa, ea.data(), 256, hipMemcpyHostToDevice);
    hipMemcpy(dsb, eb.data(), 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dc);
    std::vector<float> c(M * N);
    hipMemcpy(c.data(), dc, M * N * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < M * N; ++i)
      if ((double)c[i] != ref[i]) {
        if (bad < 4) printf("trial %d: C[%d][%d] = %g, expected %g\n", trial, i / N, i % N, c[i], ref[i]);
        ++bad;
      }
    printf("trial %d: %d / %d mismatches\n", trial, bad, M * N);
    fails += bad;
    hipFree(da); hipFree(db); hipFree(dsa); hipFree(dsb); hipFree(dc);
  }
  printf(fails ? "MX8 PROBE FAILED\n" : "MX8 PROBE OK\n");
  return fails ? 1 : 0;
}
