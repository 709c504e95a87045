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

// No multiply-add contraction in this file: every kernel form (per-pixel or
// 16 samples per lane) and the host stages then round each product and sum
// the same way, so the vectorised kernels are bit-identical to the per-pixel
// ones (contraction chose different fma trees in the two forms of the encode
// planes: one quantisation tie in a 61 x 1000 frame flipped)
#pragma clang fp contract(off)

namespace stripe {

namespace dev {

__constant__ float kJpegBasis[64];  // basis[x * 8 + u] = C(u)/2 cos((2x+1) u pi / 16)
__constant__ int kJpegZigzag[64];   // zigzag index -> natural index

__device__ __forceinline__ uint8_t jpeg_u8(float v) {
  const float r = __builtin_rintf(v);  // round half to even, like lrintf on the host
  return (uint8_t)fminf(255.f, fmaxf(0.f, r));
}

// IDCT with a lane per block row: a wave owns 8 blocks (lane = 8 b + r).  A
// lane loads its row's 8 coefficients with one 16-byte load (a block's 128
// bytes by 8 lanes), runs the row pass in registers, trades rows for columns
// through LDS for the column pass, and rows back for the store: one 8-byte
// store of a block row per lane, 8 blocks of a block row side by side (64
// contiguous bytes per image row) instead of a byte store per thread.  Row
// pass tmp[v][x] = sum_u B[x][u] F[v][u], column pass out[y][x] = sum_v
// B[y][v] tmp[v][x], in a fixed order (fp contraction is off in this file).
__global__ __launch_bounds__(256) void k_jpeg_idct8(const int16_t* __restrict__ coef, int64_t nblocks, int bw,
                                                    uint8_t* __restrict__ plane, int64_t ps) {
  __shared__ float tt[4][8][65];   // [wave][block][row * 8 + col], padded against bank conflicts
  __shared__ uint8_t ob[4][8][72];  // [wave][block][row * 9 + col]
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int bl = l >> 3, r = l & 7;
  const int64_t b = ((int64_t)blockIdx.x * 4 + w) * 8 + bl;
  const bool ok = b < nblocks;
  typedef int v4i __attribute__((ext_vector_type(4)));
  v4i raw = {0, 0, 0, 0};
  if (ok) raw = *reinterpret_cast<const v4i*>(coef + b * 64 + r * 8);
  float f[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) f[u] = (float)(int16_t)((uint32_t)raw[u >> 1] >> (16 * (u & 1)));
  // row pass: t[r][c] = sum_u basis[c][u] f[r][u]
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    float sum = 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) sum += kJpegBasis[c * 8 + u] * f[u];
    tt[w][bl][r * 8 + c] = sum;
  }
  __syncthreads();
  // column pass for column c = r of this lane's block: o[x][c] = sum_v basis[x][v] t[v][c]
  const int c = r;
  float tc[8];
#pragma unroll
  for (int v = 0; v < 8; ++v) tc[v] = tt[w][bl][v * 8 + c];
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    float o = 0.f;
#pragma unroll
    for (int v = 0; v < 8; ++v) o += kJpegBasis[x * 8 + v] * tc[v];
    ob[w][bl][x * 9 + c] = jpeg_u8(o + 128.f);
  }
  __syncthreads();
  if (!ok) return;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    lo |= (uint32_t)ob[w][bl][r * 9 + k] << (8 * k);
    hi |= (uint32_t)ob[w][bl][r * 9 + 4 + k] << (8 * k);
  }
  const int64_t by = b / bw, bx = b % bw;
  typedef uint32_t v2u __attribute__((ext_vector_type(2)));
  *reinterpret_cast<v2u*>(plane + (by * 8 + r) * ps + bx * 8) = v2u{lo, hi};
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

// Upsampled samples x0 .. x0 + 15 of one component in output row y, for a
// group inside the frame (x0 + 16 <= W, x0 % 16 == 0): the same filter as
// jpeg_sample, on 8-byte plane loads.  Returns false for sampling ratios other
// than 1 and 2 (the caller then samples pixel by pixel).
__device__ __forceinline__ bool jpeg_row16(const JpegPlaneRef& q, int x0, int y, int (&s)[16]) {
  if (q.fx > 2 || q.fy > 2) return false;
  const int iy = y / q.fy;
  const bool v4 = q.fy == 2;
  const int ny = (y % 2 == 0) ? max(0, iy - 1) : min(q.ch - 1, iy + 1);
  const uint8_t* r0 = q.p + (int64_t)iy * q.ps;
  const uint8_t* r1 = q.p + (int64_t)ny * q.ps;
  // column sums cs(i) = 3 at(i, iy) + at(i, ny) (v4) or at(i, iy), for the
  // plane columns the 16 outputs read
  auto bytes8 = [](const uint8_t* p, int (&o)[8]) __attribute__((always_inline)) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);  // x0 % 16 == 0, pitch % 8 == 0: 8-byte aligned
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = (v.x >> (8 * e)) & 0xFF;
      o[4 + e] = (v.y >> (8 * e)) & 0xFF;
    }
  };
  if (q.fx == 1) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int a[8], b[8];
      bytes8(r0 + x0 + 8 * h, a);
      if (v4) bytes8(r1 + x0 + 8 * h, b);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[8 * h + e] = v4 ? (3 * a[e] + b[e] + 1 + (y & 1)) >> 2 : a[e];
    }
    return true;
  }
  // fx == 2: output x reads plane columns x / 2 and its neighbour
  const int i0 = x0 >> 1;  // 8-byte aligned
  int a[8], b[8];
  bytes8(r0 + i0, a);
  if (v4) bytes8(r1 + i0, b);
  int cs[10];  // columns i0 - 1 .. i0 + 8 (clamped to the plane)
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[1 + e] = v4 ? 3 * a[e] + b[e] : a[e];
  const int il = max(0, i0 - 1), ir = min(q.cw - 1, i0 + 8);
  cs[0] = v4 ? 3 * r0[il] + r1[il] : r0[il];
  cs[9] = v4 ? 3 * r0[ir] + r1[ir] : r0[ir];
  const int sh = v4 ? 4 : 2, b0 = v4 ? 8 : 1, b1 = v4 ? 7 : 2;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int c = cs[1 + (j >> 1)];
    s[j] = (j & 1) == 0 ? (3 * c + cs[j >> 1] + b0) >> sh : (3 * c + cs[2 + (j >> 1)] + b1) >> sh;
  }
  return true;
}

// YCbCr (or RGB / gray) samples -> output bytes, the host conversion's arithmetic.
__device__ __forceinline__ void jpeg_convert(int Y, int U, int V, bool rgb, uint8_t (&o)[3]) {
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

// Decode colour stage: 16 output pixels of one row per lane (2-D grid: blockIdx.y
// = row, no 64-bit index division).  Groups inside the frame read the planes
// with 8-byte loads and store their 16 RGB pixels as three 16-byte stores (or
// one for gray) when the destination rows are 16-byte aligned (ALIGNED); the
// row's last, partial group samples and stores pixel by pixel.  Same samples
// and arithmetic as the per-pixel form: the GPU and host pixels stay identical.
template <bool ALIGNED>
__global__ __launch_bounds__(256) void k_jpeg_color16(JpegPlaneRef c0, JpegPlaneRef c1, JpegPlaneRef c2, int nc,
                                                      bool rgb, int W, uint8_t* __restrict__ dst, int64_t pitch) {
  const int x0 = ((int)blockIdx.x * 256 + (int)threadIdx.x) * 16;
  const int y = (int)blockIdx.y;
  if (x0 >= W) return;
  uint8_t* o = dst + (int64_t)y * pitch + (int64_t)x0 * nc;
  int sy[16], su[16], sv[16];
  bool fast = x0 + 16 <= W && jpeg_row16(c0, x0, y, sy);
  if (fast && nc == 3) fast = jpeg_row16(c1, x0, y, su) && jpeg_row16(c2, x0, y, sv);
  if (!fast) {
    for (int j = 0; j < 16 && x0 + j < W; ++j) {
      const int x = x0 + j;
      const int Y = jpeg_sample(c0, x, y);
      if (nc == 1) {
        o[j] = (uint8_t)Y;
        continue;
      }
      uint8_t px[3];
      jpeg_convert(Y, jpeg_sample(c1, x, y), jpeg_sample(c2, x, y), rgb, px);
      o[3 * j] = px[0];
      o[3 * j + 1] = px[1];
      o[3 * j + 2] = px[2];
    }
    return;
  }
  if (nc == 1) {
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j >> 2] |= (uint32_t)sy[j] << (8 * (j & 3));
    if (ALIGNED) {
      *reinterpret_cast<uint4*>(o) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) o[j] = (uint8_t)sy[j];
    }
    return;
  }
  uint32_t w[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint8_t px[3];
    jpeg_convert(sy[j], su[j], sv[j], rgb, px);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int e = 3 * j + c;  // compile-time byte index after unrolling
      w[e >> 2] |= (uint32_t)px[c] << (8 * (e & 3));
    }
  }
  if (ALIGNED) {
    uint4* o4 = reinterpret_cast<uint4*>(o);
    o4[0] = make_uint4(w[0], w[1], w[2], w[3]);
    o4[1] = make_uint4(w[4], w[5], w[6], w[7]);
    o4[2] = make_uint4(w[8], w[9], w[10], w[11]);
  } else {
#pragma unroll
    for (int e = 0; e < 48; ++e) o[e] = (uint8_t)(w[e >> 2] >> (8 * (e & 3)));
  }
}

// 16 plane samples x0 .. x0 + 15 of row y from an in-frame source block of
// 16 FS pixels x FS rows (NC channels): words of 16-byte row loads, bytes
// picked at compile-time indices (no scratch), the per-element expressions.
template <int NC, int FS, bool ALIGNED>
__device__ __forceinline__ void planes_group(const uint8_t* __restrict__ src, int64_t pitch, int x0, int y, int comp,
                                             float (&v)[16]) {
  constexpr int NW = 16 * FS * NC / 4;  // source words per row
  uint32_t w[FS][NW];
#pragma unroll
  for (int r = 0; r < FS; ++r) {
    const uint8_t* s = src + (int64_t)(y * FS + r) * pitch + (int64_t)x0 * FS * NC;
    if constexpr (ALIGNED) {
#pragma unroll
      for (int q = 0; q < NW / 4; ++q) {
        const uint4 u = reinterpret_cast<const uint4*>(s)[q];
        w[r][4 * q] = u.x;
        w[r][4 * q + 1] = u.y;
        w[r][4 * q + 2] = u.z;
        w[r][4 * q + 3] = u.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < NW; ++q)
        w[r][q] = (uint32_t)s[4 * q] | ((uint32_t)s[4 * q + 1] << 8) | ((uint32_t)s[4 * q + 2] << 16) |
                  ((uint32_t)s[4 * q + 3] << 24);
    }
  }
  auto byte = [&](int r, int e) -> float { return (float)((w[r][e >> 2] >> (8 * (e & 3))) & 0xFFu); };
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (comp == 0) {
      if constexpr (NC == 1) v[j] = byte(0, j) - 128.f;
      else v[j] = (0.299f * byte(0, 3 * j) + 0.587f * byte(0, 3 * j + 1) + 0.114f * byte(0, 3 * j + 2)) - 128.f;
    } else {
      float acc = 0.f;
#pragma unroll
      for (int dy = 0; dy < FS; ++dy)
#pragma unroll
        for (int dx = 0; dx < FS; ++dx) {
          const int e = NC * (j * FS + dx);
          const float r = byte(dy, e), g = byte(dy, e + 1), b = byte(dy, e + 2);
          acc += comp == 1 ? -0.168736f * r - 0.331264f * g + 0.5f * b : 0.5f * r - 0.418688f * g - 0.081312f * b;
        }
      v[j] = acc / (float)(FS * FS);
    }
  }
}

// Encode planes, 16 consecutive plane samples of one row per lane (2-D grid,
// no 64-bit division): a group whose source pixels are all inside the frame
// (no edge replication) reads them as 16-byte row loads (ALIGNED: source rows
// 16-byte aligned) and stores 16 floats as four 16-byte stores; edge groups
// replicate edge pixels element by element.  Each sample is the per-element
// reference expression (luma 0.299 / 0.587 / 0.114 level-shifted; chroma
// box-averaged over f x f) in a fixed order.
template <bool ALIGNED>
__global__ __launch_bounds__(256) void k_jpeg_planes16(const uint8_t* __restrict__ src, int64_t pitch, int W, int H,
                                                       int nc, int comp, int f, int ps,
                                                       float* __restrict__ out) {
  const int x0 = ((int)blockIdx.x * 256 + (int)threadIdx.x) * 16;
  const int y = (int)blockIdx.y;
  if (x0 >= ps) return;
  float* o = out + (int64_t)y * ps + x0;
  auto px = [&](int xx, int yy, int c) -> float {
    xx = min(W - 1, xx);
    yy = min(H - 1, yy);
    return (float)src[(int64_t)yy * pitch + (int64_t)xx * nc + c];
  };
  auto sample = [&](int x) -> float {
    if (comp == 0)
      return (nc == 1 ? px(x, y, 0) : 0.299f * px(x, y, 0) + 0.587f * px(x, y, 1) + 0.114f * px(x, y, 2)) - 128.f;
    float acc = 0.f;
    for (int dy = 0; dy < f; ++dy)
      for (int dx = 0; dx < f; ++dx) {
        const int sx = x * f + dx, sy = y * f + dy;
        const float r = px(sx, sy, 0), g = px(sx, sy, 1), b = px(sx, sy, 2);
        acc += comp == 1 ? -0.168736f * r - 0.331264f * g + 0.5f * b : 0.5f * r - 0.418688f * g - 0.081312f * b;
      }
    return acc / (float)(f * f);
  };
  const int fs = comp == 0 ? 1 : f;  // source pixels per sample, each way
  const bool inside = (x0 + 16) * fs <= W && (y + 1) * fs <= H && x0 + 16 <= ps;
  if (!inside || fs > 2 || (comp != 0 && nc != 3)) {
    for (int j = 0; j < 16 && x0 + j < ps; ++j) o[j] = sample(x0 + j);
    return;
  }
  float v[16];
  if (comp == 0 && nc == 1) planes_group<1, 1, ALIGNED>(src, pitch, x0, y, comp, v);
  else if (comp == 0) planes_group<3, 1, ALIGNED>(src, pitch, x0, y, comp, v);
  else if (fs == 1) planes_group<3, 1, ALIGNED>(src, pitch, x0, y, comp, v);
  else planes_group<3, 2, ALIGNED>(src, pitch, x0, y, comp, v);
  float4* o4 = reinterpret_cast<float4*>(o);  // ps % 8 == 0, x0 % 16 == 0: 64-byte aligned
#pragma unroll
  for (int q = 0; q < 4; ++q) o4[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
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
    dev::k_jpeg_idct8<<<blocks_for(nb, 32), 256, 0, s>>>(dcoef, nb, c.bw, planes[(size_t)ci], ps);
    HIP_CHECK(hipGetLastError());
    st.free_async(dcoef);
    ref[ci] = {planes[(size_t)ci], ps, (jc.W * c.h + jc.hmax - 1) / jc.hmax, (jc.H * c.v + jc.vmax - 1) / jc.vmax,
               jc.hmax / c.h, jc.vmax / c.v};
  }
  const dev::JpegPlaneRef& r1 = ref[nc == 3 ? 1 : 0];
  const dev::JpegPlaneRef& r2 = ref[nc == 3 ? 2 : 0];
  {
    const dim3 grid(blocks_for(blocks_for(jc.W, 16), 256), (unsigned)jc.H);
    if ((uintptr_t)dst % 16 == 0 && pitch % 16 == 0)
      dev::k_jpeg_color16<true><<<grid, 256, 0, s>>>(ref[0], r1, r2, nc, jc.rgb, jc.W, dst, pitch);
    else
      dev::k_jpeg_color16<false><<<grid, 256, 0, s>>>(ref[0], r1, r2, nc, jc.rgb, jc.W, dst, pitch);
  }
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
    const int f = ci == 0 ? 1 : jq.hs;
    {
      const dim3 grid(blocks_for(blocks_for(ps, 16), 256), (unsigned)rows);
      if ((uintptr_t)src % 16 == 0 && pitch % 16 == 0)
        dev::k_jpeg_planes16<true><<<grid, 256, 0, s>>>(src, pitch, W, H, C, ci, f, ps, plane);
      else
        dev::k_jpeg_planes16<false><<<grid, 256, 0, s>>>(src, pitch, W, H, C, ci, f, ps, plane);
    }
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
