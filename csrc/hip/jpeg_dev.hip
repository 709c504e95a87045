// JPEG pixel stages on the GPU: the host keeps the entropy coding (Huffman is
// a sequential bit stream per restart interval, csrc/core/jpeg.cpp) and the
// device does the arithmetic -- IDCT, chroma upsampling and YCbCr -> RGB on
// decode; colour conversion, chroma subsampling, forward DCT and quantisation
// on encode.  The reference decodes and encodes with OpenCV on the CPU
// (cv::imread / imwrite, kernel.cu:110,236); here a JPEG frame lands in (or
// leaves from) device memory with only its coefficients crossing the link
// (int16 per sample: the same bytes as RGB for 4:2:0).
//
// Numerics follow the host stages operation for operation (float basis
// products in the same order, the same integer upsampling filter), so the two
// paths agree to within one level (the device may fuse a multiply-add).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "stripe/image.h"
#include "stripe/kernels.h"

namespace stripe {

namespace dev {

__constant__ float kJpegBasis[64];  // basis[x * 8 + u] = C(u)/2 cos((2x+1) u pi / 16)
__constant__ int kJpegZigzag[64];   // zigzag index -> natural index

__device__ __forceinline__ uint8_t jpeg_u8(float v) {
  const float r = __builtin_rintf(v);  // round half to even, like lrintf on the host
  return (uint8_t)fminf(255.f, fmaxf(0.f, r));
}

// One wave per 8x8 block (lane = row * 8 + column), four blocks per workgroup:
// row pass tmp[v][x] = sum_u B[x][u] F[v][u], column pass out[y][x] =
// sum_v B[y][v] tmp[v][x], both through LDS.
__global__ __launch_bounds__(256) void k_jpeg_idct(const int16_t* __restrict__ coef, int64_t nblocks, int bw,
                                                   uint8_t* __restrict__ plane, int64_t ps) {
  __shared__ float f[4][64];
  __shared__ float t[4][64];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + w;
  const bool ok = b < nblocks;
  f[w][l] = ok ? (float)coef[b * 64 + l] : 0.f;
  __syncthreads();
  const int r = l >> 3, c = l & 7;
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += kJpegBasis[c * 8 + u] * f[w][r * 8 + u];
  t[w][l] = s;
  __syncthreads();
  float o = 0.f;
#pragma unroll
  for (int v = 0; v < 8; ++v) o += kJpegBasis[r * 8 + v] * t[w][v * 8 + c];
  if (ok) {
    const int64_t by = b / bw, bx = b % bw;
    plane[(by * 8 + r) * ps + bx * 8 + c] = jpeg_u8(o + 128.f);
  }
}

struct JpegPlaneRef {
  const uint8_t* p;
  int64_t ps;
  int cw, ch, fx, fy;
};

// sample (x, y) of an upsampled component: the host's filter (jpeg.cpp
// upsample): 2:1 ratios by the triangle filter with clamped neighbours and
// alternating rounding biases, others by replication
__device__ __forceinline__ int jpeg_sample(const JpegPlaneRef& q, int x, int y) {
  auto at = [&](int xx, int yy) -> int { return q.p[(int64_t)yy * q.ps + xx]; };
  if (q.fx == 1 && q.fy == 1) return at(x, y);
  if ((q.fx == 1 || q.fx == 2) && (q.fy == 1 || q.fy == 2)) {
    const int iy = y / q.fy;
    const int ny = (y % 2 == 0) ? max(0, iy - 1) : min(q.ch - 1, iy + 1);
    auto cs = [&](int i) -> int { return q.fy == 2 ? 3 * at(i, iy) + at(i, ny) : at(i, iy); };
    const bool v4 = q.fy == 2;
    if (q.fx == 1) return v4 ? (cs(x) + 1 + (y & 1)) >> 2 : cs(x);
    const int sh = v4 ? 4 : 2, b0 = v4 ? 8 : 1, b1 = v4 ? 7 : 2;
    const int ix = x >> 1, c = cs(ix);
    if ((x & 1) == 0) return (3 * c + cs(max(0, ix - 1)) + b0) >> sh;
    return (3 * c + cs(min(q.cw - 1, ix + 1)) + b1) >> sh;
  }
  return at(min(q.cw - 1, x / q.fx), min(q.ch - 1, y / q.fy));
}

// one thread per output pixel: upsample every component, convert, store
// interleaved RGB (or gray) rows of `pitch` bytes
__global__ __launch_bounds__(256) void k_jpeg_color(JpegPlaneRef c0, JpegPlaneRef c1, JpegPlaneRef c2, int nc,
                                                    bool rgb, int W, int H, uint8_t* __restrict__ dst, int64_t pitch) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)W * H) return;
  const int y = (int)(i / W), x = (int)(i % W);
  uint8_t* o = dst + (int64_t)y * pitch + (int64_t)x * nc;
  const int Y = jpeg_sample(c0, x, y);
  if (nc == 1) {
    o[0] = (uint8_t)Y;
    return;
  }
  const int U = jpeg_sample(c1, x, y), V = jpeg_sample(c2, x, y);
  if (rgb) {
    o[0] = (uint8_t)Y;
    o[1] = (uint8_t)U;
    o[2] = (uint8_t)V;
    return;
  }
  const float yy = (float)Y, cb = (float)U - 128.f, cr = (float)V - 128.f;
  o[0] = jpeg_u8(yy + 1.402f * cr);
  o[1] = jpeg_u8(yy - 0.344136f * cb - 0.714136f * cr);
  o[2] = jpeg_u8(yy + 1.772f * cb);
}

// encode: level-shifted luma (or gray) / centred, box-averaged chroma planes
// of MCU-padded size from an interleaved source (edge pixels replicated)
__global__ __launch_bounds__(256) void k_jpeg_planes(const uint8_t* __restrict__ src, int64_t pitch, int W, int H,
                                                     int nc, int comp, int f, int ps, int rows,
                                                     float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)ps * rows) return;
  const int y = (int)(i / ps), x = (int)(i % ps);
  auto px = [&](int xx, int yy, int c) -> float {
    xx = min(W - 1, xx);
    yy = min(H - 1, yy);
    return (float)src[(int64_t)yy * pitch + (int64_t)xx * nc + c];
  };
  if (comp == 0) {
    const float v = nc == 1 ? px(x, y, 0) : 0.299f * px(x, y, 0) + 0.587f * px(x, y, 1) + 0.114f * px(x, y, 2);
    out[i] = v - 128.f;
    return;
  }
  float acc = 0.f;
  for (int dy = 0; dy < f; ++dy)
    for (int dx = 0; dx < f; ++dx) {
      const int sx = x * f + dx, sy = y * f + dy;
      const float r = px(sx, sy, 0), g = px(sx, sy, 1), b = px(sx, sy, 2);
      acc += comp == 1 ? -0.168736f * r - 0.331264f * g + 0.5f * b : 0.5f * r - 0.418688f * g - 0.081312f * b;
    }
  out[i] = acc / (float)(f * f);
}

// forward DCT + quantisation, one wave per block: F[v][u] = sum_y B[y][v]
// (sum_x B[x][u] f[y][x]); output in zigzag order
__global__ __launch_bounds__(256) void k_jpeg_fdct(const float* __restrict__ plane, int64_t ps, int64_t nblocks,
                                                   int bw, const uint16_t* __restrict__ q,
                                                   int16_t* __restrict__ coef) {
  __shared__ float f[4][64];
  __shared__ float t[4][64];
  __shared__ float F[4][64];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + w;
  const bool ok = b < nblocks;
  const int r = l >> 3, c = l & 7;
  const int64_t by = ok ? b / bw : 0, bx = ok ? b % bw : 0;
  f[w][l] = ok ? plane[(by * 8 + r) * ps + bx * 8 + c] : 0.f;
  __syncthreads();
  float s = 0.f;  // tmp[y = r][u = c]
#pragma unroll
  for (int x = 0; x < 8; ++x) s += kJpegBasis[x * 8 + c] * f[w][r * 8 + x];
  t[w][l] = s;
  __syncthreads();
  float o = 0.f;  // F[v = r][u = c]
#pragma unroll
  for (int y = 0; y < 8; ++y) o += kJpegBasis[y * 8 + r] * t[w][y * 8 + c];
  F[w][l] = o;
  __syncthreads();
  if (ok) {
    const int z = kJpegZigzag[l];  // lane l writes zigzag slot l
    coef[b * 64 + l] = (int16_t)__builtin_rintf(F[w][z] / (float)q[z]);
  }
}

}  // namespace dev

namespace {

void upload_jpeg_constants() {
  // once per device (several host threads may decode / encode at once)
  static std::mutex mu;
  static bool done[64] = {};
  int d = 0;
  HIP_CHECK(hipGetDevice(&d));
  std::lock_guard<std::mutex> lk(mu);
  if (d < 64 && done[d]) return;
  float B[64];
  for (int x = 0; x < 8; ++x)
    for (int u = 0; u < 8; ++u)
      B[x * 8 + u] = (float)((u == 0 ? std::sqrt(0.5) : 1.0) * 0.5 * std::cos((2 * x + 1) * u * M_PI / 16.0));
  HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(dev::kJpegBasis), B, sizeof B));
  HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(dev::kJpegZigzag), jpeg_zigzag(), 64 * sizeof(int)));
  if (d < 64) done[d] = true;
}

unsigned blocks_for(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

}  // namespace

namespace {
// STRIPE_JPEG_PIN=0 keeps the pageable coefficient upload (A/B switch)
bool pin_uploads() {
  static const bool on = [] {
    const char* e = std::getenv("STRIPE_JPEG_PIN");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
}  // namespace

namespace {
// What jpeg_pixels_device holds while its work is queued: page-locked host
// ranges and device buffers.  On the normal path the function releases them
// itself; if anything throws on the way (an allocation, a copy, a launch), the
// destructor waits for the stream (copies from registered pages may still be
// in flight) and then unregisters and frees everything, so no registration
// outlives the host memory it covers and no device buffer leaks.
struct JpegStaging {
  hipStream_t s;
  std::vector<void*> pinned;    // hipHostRegister'ed host ranges
  std::vector<void*> device;    // hipMallocAsync'ed buffers not yet freed
  bool released = false;
  explicit JpegStaging(hipStream_t st) : s(st) {}
  void* alloc(size_t bytes) {
    void* p = nullptr;
    HIP_CHECK(hipMallocAsync(&p, bytes, s));
    device.push_back(p);
    return p;
  }
  void free_async(void* p) {
    HIP_CHECK(hipFreeAsync(p, s));
    device.erase(std::find(device.begin(), device.end(), p));
  }
  // normal path: queue the frees, then (registered pages only) wait for the
  // copies out of them before unregistering
  void release() {
    for (void* p : device) HIP_CHECK(hipFreeAsync(p, s));
    device.clear();
    if (!pinned.empty()) {
      HIP_CHECK(hipStreamSynchronize(s));
      for (void* hp : pinned) (void)hipHostUnregister(hp);
      pinned.clear();
    }
    released = true;
  }
  ~JpegStaging() {
    if (released) return;
    (void)hipStreamSynchronize(s);
    for (void* p : device) (void)hipFree(p);
    for (void* hp : pinned) (void)hipHostUnregister(hp);
    (void)hipGetLastError();  // the error being thrown is the one to report
  }
};
}  // namespace

void jpeg_pixels_device(const JpegCoefs& jc, uint8_t* dst, int64_t pitch, hipStream_t s) {
  const int nc = (int)jc.comps.size();
  STRIPE_CHECK(nc == 1 || nc == 3, "JPEG: 1 or 3 components");
  STRIPE_CHECK(pitch >= (int64_t)jc.W * nc, "JPEG: destination pitch " << pitch << " < row bytes " << jc.W * nc);
  upload_jpeg_constants();
  // large coefficient planes are page-locked for the upload (a pageable copy
  // is staged through the runtime's bounce buffers at a fraction of the link
  // rate); they are unregistered once the copies have run
  JpegStaging st(s);
  std::vector<uint8_t*> planes((size_t)nc, nullptr);
  dev::JpegPlaneRef ref[3] = {};
  for (int ci = 0; ci < nc; ++ci) {
    const JpegCoefs::Comp& c = jc.comps[(size_t)ci];
    const int64_t nb = (int64_t)c.bw * c.bh, ps = (int64_t)c.bw * 8;
    STRIPE_CHECK(c.coef.size() == (size_t)nb * 64, "JPEG: coefficient plane size");
    const size_t cbytes = (size_t)nb * 64 * sizeof(int16_t);
    auto* dcoef = static_cast<int16_t*>(st.alloc(cbytes));
    planes[(size_t)ci] = static_cast<uint8_t*>(st.alloc((size_t)ps * c.bh * 8));
    if (pin_uploads() && cbytes >= ((size_t)8 << 20)) {
      void* hp = const_cast<int16_t*>(c.coef.data());
      if (hipHostRegister(hp, cbytes, hipHostRegisterDefault) == hipSuccess) st.pinned.push_back(hp);
      else (void)hipGetLastError();  // not registrable: the pageable copy below still works
    }
    HIP_CHECK(hipMemcpyAsync(dcoef, c.coef.data(), cbytes, hipMemcpyHostToDevice, s));
    dev::k_jpeg_idct<<<blocks_for(nb, 4), 256, 0, s>>>(dcoef, nb, c.bw, planes[(size_t)ci], ps);
    HIP_CHECK(hipGetLastError());
    st.free_async(dcoef);
    ref[ci] = {planes[(size_t)ci], ps, (jc.W * c.h + jc.hmax - 1) / jc.hmax, (jc.H * c.v + jc.vmax - 1) / jc.vmax,
               jc.hmax / c.h, jc.vmax / c.v};
  }
  const int64_t npx = (int64_t)jc.W * jc.H;
  dev::k_jpeg_color<<<blocks_for(npx, 256), 256, 0, s>>>(ref[0], ref[nc == 3 ? 1 : 0], ref[nc == 3 ? 2 : 0], nc,
                                                          jc.rgb, jc.W, jc.H, dst, pitch);
  HIP_CHECK(hipGetLastError());
  st.release();
}

JpegQuant jpeg_quantise_device(const uint8_t* src, int64_t pitch, int W, int H, int C, int quality, bool subsample,
                               hipStream_t s) {
  STRIPE_CHECK(C == 1 || C == 3, "JPEG: encode needs 1 or 3 channels, got " << C);
  STRIPE_CHECK(W > 0 && H > 0 && W <= 65535 && H <= 65535, "JPEG: image size out of range");
  STRIPE_CHECK(pitch >= (int64_t)W * C, "JPEG: source pitch " << pitch << " < row bytes " << W * C);
  upload_jpeg_constants();
  JpegQuant jq;
  jq.W = W;
  jq.H = H;
  jq.hs = subsample && C == 3 ? 2 : 1;
  jpeg_tables(quality, jq.q[0], jq.q[1]);
  const int mcu = 8 * jq.hs;
  const int mx = (W + mcu - 1) / mcu, my = (H + mcu - 1) / mcu;
  uint16_t* dq = nullptr;
  HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&dq), sizeof jq.q, s));
  HIP_CHECK(hipMemcpyAsync(dq, jq.q, sizeof jq.q, hipMemcpyHostToDevice, s));
  for (int ci = 0; ci < C; ++ci) {
    JpegQuant::Comp c;
    c.f = ci == 0 ? jq.hs : 1;
    c.bw = mx * c.f;
    c.bh = my * c.f;
    const int ps = c.bw * 8, rows = c.bh * 8;
    const int64_t nb = (int64_t)c.bw * c.bh;
    float* plane = nullptr;
    int16_t* dcoef = nullptr;
    HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&plane), (size_t)ps * rows * sizeof(float), s));
    HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&dcoef), (size_t)nb * 64 * sizeof(int16_t), s));
    dev::k_jpeg_planes<<<blocks_for((int64_t)ps * rows, 256), 256, 0, s>>>(src, pitch, W, H, C, ci,
                                                                             ci == 0 ? 1 : jq.hs, ps, rows, plane);
    HIP_CHECK(hipGetLastError());
    dev::k_jpeg_fdct<<<blocks_for(nb, 4), 256, 0, s>>>(plane, ps, nb, c.bw, dq + (ci == 0 ? 0 : 64), dcoef);
    HIP_CHECK(hipGetLastError());
    c.coef.resize((size_t)nb * 64);
    HIP_CHECK(hipMemcpyAsync(c.coef.data(), dcoef, (size_t)nb * 64 * sizeof(int16_t), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipFreeAsync(plane, s));
    HIP_CHECK(hipFreeAsync(dcoef, s));
    jq.comps.push_back(std::move(c));
  }
  HIP_CHECK(hipFreeAsync(dq, s));
  HIP_CHECK(hipStreamSynchronize(s));  // the coefficient downloads land in pageable host memory
  return jq;
}

}  // namespace stripe
