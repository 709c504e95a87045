// Probe: v_cvt_pk_u8_f32 saturates to [0,255] and rounds half-to-even on gfx950
// (measured: -5->0, 0.5->0, 1.5->2, 2.5->2, 254.5->254, 256->255, 1e9->255).
//   hipcc --offload-arch=gfx950 -o bin/cvt_probe tools/cvt_probe.hip && bin/cvt_probe
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* in, unsigned* out, int n) {
  int i = threadIdx.x;
  if (i < n) out[i] = __builtin_amdgcn_cvt_pk_u8_f32(in[i], 0, 0u);
}
int main() {
  float h[] = {-5.f, -0.4f, -0.6f, 0.5f, 1.5f, 2.5f, 254.5f, 255.4f, 255.6f, 256.f, 300.f, 1e9f, -1e9f, 127.5f};
  const int n = sizeof(h) / sizeof(h[0]);
  float* d; unsigned* o; unsigned r[n];
  hipMalloc(&d, sizeof h); hipMalloc(&o, sizeof r);
  hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, o, n);
  hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i) printf("%g -> %u\n", h[i], r[i]);
  return 0;
}
