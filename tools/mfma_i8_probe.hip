// Operand lane map of v_mfma_i32_16x16x64_i8 on gfx950, checked with exact
// integer data (cdna_hip_programming.md: "Other dtypes: check the map with
// exact integer data before relying on it").  Candidate maps for the 16 i8
// elements j of lane l (g = l >> 4):
//   H1: A[m = l & 15][k = 16 g + j],               B[k = 16 g + j][n = l & 15]
//   H2: A[m = l & 15][k = 8 g + j (j < 8), 32 + 8 g + j - 8 (j >= 8)], B alike
// The product of random A, B is compared with both; prints the map that matches.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_i8_probe.hip -o bin/mfma_i8_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void probe(const int* a, const int* b, int* d) {
  const int l = threadIdx.x;
  v4i av, bv;
  for (int i = 0; i < 4; ++i) {
    av[i] = a[l * 4 + i];
    bv[i] = b[l * 4 + i];
  }
  i32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) d[l * 4 + r] = c[r];
}

static int kmap(int h, int l, int j) {
  const int g = l >> 4;
  return h == 1 ? 16 * g + j : (j < 8 ? 8 * g + j : 32 + 8 * g + j - 8);
}

int main() {
  std::vector<signed char> A(16 * 64), B(64 * 16);  // A[m][k], B[k][n]
  srand(7);
  for (auto& v : A) v = (signed char)(rand() % 255 - 127);
  for (auto& v : B) v = (signed char)(rand() % 255 - 127);
  long ref[16][16] = {};
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n)
      for (int k = 0; k < 64; ++k) ref[m][n] += (long)A[m * 64 + k] * B[k * 16 + n];
  int* da;
  int* db;
  int* dd;
  hipMalloc(&da, 1024);
  hipMalloc(&db, 1024);
  hipMalloc(&dd, 1024);
  for (int h = 1; h <= 2; ++h) {
    std::vector<signed char> pa(1024), pb(1024);
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 16; ++j) {
        const int k = kmap(h, l, j);
        pa[l * 16 + j] = A[(l & 15) * 64 + k];
        pb[l * 16 + j] = B[k * 16 + (l & 15)];
      }
    hipMemcpy(da, pa.data(), 1024, hipMemcpyHostToDevice);
    hipMemcpy(db, pb.data(), 1024, hipMemcpyHostToDevice);
    probe<<<1, 64>>>(da, db, dd);
    std::vector<int> d(256);
    hipMemcpy(d.data(), dd, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        const int n = l & 15, m = 4 * (l >> 4) + r;  // C/D: col = lane & 15, row = 4 g + r
        bad += d[l * 4 + r] != ref[m][n];
      }
    printf("H%d: %d of 256 results differ\n", h, bad);
  }
  return 0;
}
