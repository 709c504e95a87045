// Issue rate of the f16 MFMA shapes on one SIMD: v_mfma_f32_16x16x32_f16 vs
// v_mfma_f32_16x16x16_f16 (and 32x32x16 for scale).  Question: does a K = 16
// step cost half a K = 32 step?  If so, a 46-wide Toeplitz window (K = 31 +
// 15) fits 32 + 16 instead of 2 x 32 (blur_sep.hip's passes, 25 % fewer MFMA
// cycles).
//
//   hipcc --offload-arch=gfx950 -O3 -o bin/mfma_rate tools/mfma_rate.hip
//   bin/mfma_rate
//
// One wave per SIMD on every CU (4 waves per workgroup, one workgroup per CU),
// 8 independent accumulators per wave (no dependency stalls), timed by events;
// cycles are quoted against the 16x16x32 form's documented 16 cycles.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));   \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

// The MFMAs are inline asm on fixed accumulators: the builtins let the
// compiler shuffle accumulators between AGPRs every iteration.
template <int KIND>
__global__ __launch_bounds__(256) void k_rate(float* out, int iters, float seed) {
  const _Float16 s = (_Float16)(seed + threadIdx.x * 1e-3f);
  if constexpr (KIND == 2) {
    f16v acc[4] = {};
    h8 a = {s, s, s, s, s, s, s, s};
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %1, %0" : "+v"(acc[k]) : "v"(a));
    float t = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < 16; ++j) t += acc[k][j];
    out[blockIdx.x * 256 + threadIdx.x] = t;
  } else {
    f4 acc[8] = {};
    h8 a8 = {s, s, s, s, s, s, s, s};
    h4 a4 = {s, s, s, s};
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if constexpr (KIND == 0) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %1, %0" : "+v"(acc[k]) : "v"(a8));
        else asm volatile("v_mfma_f32_16x16x16_f16 %0, %1, %1, %0" : "+v"(acc[k]) : "v"(a4));
      }
    float t = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[blockIdx.x * 256 + threadIdx.x] = t;
  }
}

int main() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  float* out = nullptr;
  CK(hipMalloc(&out, (size_t)cus * 256 * sizeof(float)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 20000;
  const char* names[3] = {"16x16x32_f16", "16x16x16_f16", "32x32x16_f16"};
  const int per_iter[3] = {8, 8, 4};
  double ms_k[3] = {0, 0, 0};
  for (int rep = 0; rep < 3; ++rep)
    for (int kind = 0; kind < 3; ++kind) {
      auto launch = [&]() {
        if (kind == 0) k_rate<0><<<cus, 256>>>(out, iters, 1.0f);
        else if (kind == 1) k_rate<1><<<cus, 256>>>(out, iters, 1.0f);
        else k_rate<2><<<cus, 256>>>(out, iters, 1.0f);
      };
      launch();
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep == 0 || ms < ms_k[kind]) ms_k[kind] = ms;
    }
  // per-SIMD time per MFMA, and cycles scaled so 16x16x32 reads its documented 16
  const double ns0 = ms_k[0] * 1e6 / ((double)iters * per_iter[0]);
  for (int kind = 0; kind < 3; ++kind) {
    const double ns = ms_k[kind] * 1e6 / ((double)iters * per_iter[kind]);
    std::printf("{\"mfma\": \"%s\", \"ms\": %.3f, \"ns_per_mfma_per_simd\": %.3f, \"cycles_vs_16x16x32_at_16\": %.2f}\n",
                names[kind], ms_k[kind], ns, 16.0 * ns / ns0);
  }
  CK(hipFree(out));
  return 0;
}
