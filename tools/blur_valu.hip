// Separable-VALU comparator for blur:31 ("benchmark both and
// report honestly").  No matrix cores: every tap is a v_fma_f32.
//
//   hipcc --offload-arch=gfx950 -O3 -o bin/blur_valu tools/blur_valu.hip
//   bin/blur_valu [W H iters]          (default 16384 16384 20, RGB u8)
//
// A thread owns 4 consecutive pixels of one channel and walks down a band of
// rows.  Per input row it loads the 108 bytes covering its 34-pixel
// horizontal reach (7 dwordx4, L1/L2 hits for the neighbours' overlap),
// converts the 34 bytes of its channel with v_cvt_f32_ubyteN, forms 4
// horizontal sums (symmetric taps: 15 adds + 16 FMAs each) and scatters them into a 31-row ring of
// pending vertical sums (31 FMAs each, ring slots compile-time: the row loop
// is unrolled by 31).  Per output value: ~8.5 conversions + 31 horizontal +
// 31 vertical VALU ops.
// Borders: constant 0 (zero margins), verified against a float64 host
// reference on a small frame first.  The production kernel is the
// separable MFMA one (csrc/hip/blur_sep.hip); this tool only times the
// alternative.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));   \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

constexpr int K = 31, R = 15, BAND = 62;  // BAND: a multiple of 31 keeps the ring aligned
constexpr int MX = 64;                    // x-margin bytes each side (>= 48 left, >= 64 right reach)
constexpr int MY = R;                     // zero rows above and below

__constant__ float c_w[R + 1];  // taps 0 .. 15 of the symmetric 1-D Gaussian (h = v)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int CH>
__device__ __forceinline__ void band(const unsigned char* __restrict__ in, unsigned char* __restrict__ out,
                                     long pitch, int W, int H, int x0, int y0) {
  float acc[K][4];
#pragma unroll
  for (int s = 0; s < K; ++s)
#pragma unroll
    for (int p = 0; p < 4; ++p) acc[s][p] = 0.f;
  const int nrows = min(BAND, H - y0) + 2 * R;  // input rows y0 - R .. y0 + n + R - 1
  // row i's 108-byte window starts 48 bytes left of pixel x0 (dword aligned: 3 x0 = 12 k)
  const unsigned char* col = in + (long)(3 * x0 - 48);
  for (int base = 0; base < nrows; base += K) {
#pragma unroll
    for (int u = 0; u < K; ++u) {
      const int i = base + u;  // input row y0 - R + i
      if (i >= nrows) break;
      const u32x4* src = reinterpret_cast<const u32x4*>(col + (long)(y0 - R + i) * pitch);
      unsigned int d[28];
#pragma unroll
      for (int q = 0; q < 7; ++q) {
        const u32x4 t = src[q];
        d[4 * q] = t.x;
        d[4 * q + 1] = t.y;
        d[4 * q + 2] = t.z;
        if (4 * q + 3 < 28) d[4 * q + 3] = t.w;
      }
      float val[34];
#pragma unroll
      for (int j = 0; j < 34; ++j) {
        const int b = 3 * j + 3 + CH;  // byte of pixel x0 - 15 + j, channel CH
        val[j] = (float)((d[b >> 2] >> (8 * (b & 3))) & 0xffu);
      }
      float h4[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        // symmetric taps (a Gaussian): 15 adds + 16 FMAs
        float s = c_w[R] * val[p + R];
#pragma unroll
        for (int t = 0; t < R; ++t) s = __builtin_fmaf(c_w[t], val[p + t] + val[p + K - 1 - t], s);
        h4[p] = s;
      }
      // band coordinates: input row i (frame row y0 - R + i) feeds output o =
      // i - t (frame row y0 + o) with weight v[t]
#pragma unroll
      for (int t = 0; t < K; ++t) {
        const int slot = ((u - t) % K + K) % K;  // output o = i - t, slot o mod 31
#pragma unroll
        for (int p = 0; p < 4; ++p) acc[slot][p] = __builtin_fmaf(c_w[t < R ? t : K - 1 - t], h4[p], acc[slot][p]);
      }
      const int o = i - (K - 1);  // output complete after its last tap (t = 30)
      if (o >= 0) {
        const int slot = ((u - (K - 1)) % K + K) % K;
        unsigned char* dst = out + (long)(y0 + o) * pitch + 3 * x0 + CH;
        if (y0 + o < H) {
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            if (x0 + p < W) {
              const unsigned int pk = __builtin_amdgcn_cvt_pk_u8_f32(acc[slot][p], 0, 0u);
              dst[3 * p] = (unsigned char)pk;
            }
          }
        }
      }
      // the slot of output i - 30 is done (stored, or above the band): reuse it
      const int done = ((u - (K - 1)) % K + K) % K;
#pragma unroll
      for (int p = 0; p < 4; ++p) acc[done][p] = 0.f;
    }
  }
}

__global__ __launch_bounds__(256) void k_blur_valu(const unsigned char* in, unsigned char* out, long pitch, int W,
                                                   int H) {
  const int x0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (x0 >= W) return;
  const int y0 = blockIdx.y * BAND;
  switch (blockIdx.z) {
    case 0: band<0>(in, out, pitch, W, H, x0, y0); break;
    case 1: band<1>(in, out, pitch, W, H, x0, y0); break;
    default: band<2>(in, out, pitch, W, H, x0, y0); break;
  }
}

static std::vector<double> gauss() {
  const double sigma = 0.3 * ((K - 1) * 0.5 - 1) + 0.8;
  std::vector<double> g(K);
  double s = 0;
  for (int i = 0; i < K; ++i) s += g[i] = std::exp(-(double)(i - R) * (i - R) / (2 * sigma * sigma));
  for (auto& x : g) x /= s;
  return g;
}

struct Frame {
  int W, H;
  long pitch;
  unsigned char *din, *dout;  // allocation origins; the frame starts MY rows + MX bytes in
  size_t bytes;
  unsigned char* in() const { return din + MY * pitch + MX; }
  unsigned char* out() const { return dout + MY * pitch + MX; }
};

static Frame make(int W, int H) {
  Frame f{W, H, 0, nullptr, nullptr, 0};
  f.pitch = ((long)3 * W + 2 * MX + 255) / 256 * 256;
  f.bytes = (size_t)f.pitch * (H + 2 * MY + 1);
  CK(hipMalloc(&f.din, f.bytes));
  CK(hipMalloc(&f.dout, f.bytes));
  CK(hipMemset(f.din, 0, f.bytes));
  CK(hipMemset(f.dout, 0, f.bytes));
  return f;
}

static void launch(const Frame& f) {
  dim3 grid((f.W / 4 + 255) / 256, (f.H + BAND - 1) / BAND, 3);
  k_blur_valu<<<grid, 256>>>(f.in(), f.out(), f.pitch, f.W, f.H);
  CK(hipGetLastError());
}

int main(int argc, char** argv) {
  const int W = argc > 1 ? std::atoi(argv[1]) : 16384, H = argc > 2 ? std::atoi(argv[2]) : 16384;
  const int iters = argc > 3 ? std::atoi(argv[3]) : 20;
  const auto g = gauss();
  float gf[R + 1];
  for (int i = 0; i <= R; ++i) gf[i] = (float)g[i];
  CK(hipMemcpyToSymbol(HIP_SYMBOL(c_w), gf, sizeof gf));

  {  // correctness on a small frame against a float64 host reference (zero border)
    const int w = 300, h = 77;
    Frame f = make(w, h);
    std::vector<unsigned char> img((size_t)3 * w * h);
    unsigned s = 12345;
    for (auto& b : img) b = (unsigned char)((s = s * 1103515245u + 12345u) >> 24);
    CK(hipMemcpy2D(f.in(), f.pitch, img.data(), 3 * w, 3 * w, h, hipMemcpyHostToDevice));
    launch(f);
    std::vector<unsigned char> got((size_t)3 * w * h);
    CK(hipMemcpy2D(got.data(), 3 * w, f.out(), f.pitch, 3 * w, h, hipMemcpyDeviceToHost));
    int bad = 0, off1 = 0;
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x)
        for (int c = 0; c < 3; ++c) {
          double sum = 0;
          for (int dy = -R; dy <= R; ++dy)
            for (int dx = -R; dx <= R; ++dx) {
              const int yy = y + dy, xx = x + dx;
              if (yy < 0 || yy >= h || xx < 0 || xx >= w) continue;
              sum += g[dy + R] * g[dx + R] * img[((size_t)yy * w + xx) * 3 + c];
            }
          const int ref = (int)std::lrint(std::fmin(255.0, std::fmax(0.0, sum)));
          const int d = std::abs((int)got[((size_t)y * w + x) * 3 + c] - ref);
          bad += d > 1;
          off1 += d == 1;
        }
    std::printf("{\"check\": \"blur_valu 300x77 vs float64\", \"bad\": %d, \"off_by_one\": %d}\n", bad, off1);
    CK(hipFree(f.din));
    CK(hipFree(f.dout));
    if (bad) return 2;
  }

  Frame f = make(W, H);
  CK(hipMemset(f.din, 0x5a, f.bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) launch(f);
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch(f);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  std::printf("{\"kernel\": \"blur_valu\", \"shape\": \"%dx%dx3\", \"ms\": %.4f, \"mpx_s\": %.1f}\n", W, H, ms,
              (double)W * H / (ms * 1e3));
  return 0;
}
