// f32 -> f16 hi + lo splits on gfx950: masked hi + cvt lo (round 2/3 blur)
// against cvt_pkrtz hi + v_fma_mix lo.  Prints how often the two differ and
// the largest |hi + lo - x| / |x| of each.
//   hipcc --offload-arch=gfx950 -O2 tools/split_probe.hip -o bin/split_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 half2v __attribute__((ext_vector_type(2)));

__global__ void probe(const float* x, unsigned* out, int n) {
  const int i = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (i + 1 >= n) return;
  const float a = x[i], b = x[i + 1];
  // method 0
  const float ha = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, a) & 0xFFFFE000u);
  const float hb = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, b) & 0xFFFFE000u);
  const half2v h0 = {(_Float16)ha, (_Float16)hb};
  const half2v l0 = {(_Float16)(a - ha), (_Float16)(b - hb)};
  // method 1
  const unsigned h1 = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_pkrtz(a, b));
  unsigned l1;
  asm volatile("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(l1) : "v"(a), "v"(h1));
  asm volatile("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l1) : "v"(b), "v"(h1));
  out[4 * (i / 2) + 0] = __builtin_bit_cast(unsigned, h0);
  out[4 * (i / 2) + 1] = __builtin_bit_cast(unsigned, l0);
  out[4 * (i / 2) + 2] = h1;
  out[4 * (i / 2) + 3] = l1;
}

static float h2f(unsigned short h) {
  _Float16 v;
  __builtin_memcpy(&v, &h, 2);
  return (float)v;
}

int main() {
  const int n = 1 << 22;
  std::vector<float> x(n);
  srand(3);
  for (int i = 0; i < n; ++i) x[i] = (float)rand() / RAND_MAX * 255.0f * ((i & 7) ? 1.0f : 1e-3f);
  float* dx;
  unsigned* dout;
  hipMalloc(&dx, n * 4);
  hipMalloc(&dout, n * 8);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  probe<<<n / 2 / 256, 256>>>(dx, dout, n);
  std::vector<unsigned> o(n * 2);
  hipMemcpy(o.data(), dout, n * 8, hipMemcpyDeviceToHost);
  long dh = 0, dl = 0;
  double e0 = 0, e1 = 0;
  for (int p = 0; p < n / 2; ++p)
    for (int k = 0; k < 2; ++k) {
      const double xv = x[2 * p + k];
      const unsigned short H0 = o[4 * p] >> (16 * k), L0 = o[4 * p + 1] >> (16 * k);
      const unsigned short H1 = o[4 * p + 2] >> (16 * k), L1 = o[4 * p + 3] >> (16 * k);
      dh += H0 != H1;
      dl += L0 != L1;
      if (xv > 0) {
        e0 = fmax(e0, fabs(h2f(H0) + (double)h2f(L0) - xv) / xv);
        e1 = fmax(e1, fabs(h2f(H1) + (double)h2f(L1) - xv) / xv);
      }
      if ((dh + dl) && (dh + dl) < 4 && (H0 != H1 || L0 != L1))
        printf("x=%.9g  mask: %04x %04x  pkrtz/mix: %04x %04x\n", xv, H0, L0, H1, L1);
    }
  printf("hi differ %ld, lo differ %ld of %d; max rel err mask %.3g, pkrtz/mix %.3g\n", dh, dl, n, e0, e1);
  return 0;
}
