// Fused pointwise pass: out = expand?(post(gray?(pre(p)))) on 16 pixels per lane.
//
// Replaces the reference's separate grayscale and contrast launches
// (kernel.cu:31-58, one thread per pixel, scalar u8 loads) with one pass of
// 16-byte vector loads/stores; every per-channel op is a 256-entry LUT held in
// LDS, gray conversion is exact integer arithmetic (gray:ref's double-precision
// per-channel truncation, kernel.cu:40-42, is reproduced with verified
// multiply-shift constants).  Margins are processed like pixels, so the output
// keeps the x-border contract of the next stencil.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "dev_common.h"
#include "stripe/image.h"
#include "stripe/kernels.h"

namespace stripe {
namespace dev {

template <int CIN, int COUT, bool GRAY, bool NT>
__global__ __launch_bounds__(kNT) void k_pointwise(KArgs a, int ngroups, int g0) {
  __shared__ uint8_t lut[512];
  for (int i = threadIdx.x; i < 512; i += kNT) lut[i] = a.luts[i];
  __syncthreads();
  const int g = blockIdx.x * kNT + threadIdx.x;  // 16-pixel group
  if (g >= ngroups) return;
  const int p0 = (g + g0) * 16;  // first pixel (may be negative: margin)
  const int y = a.ry0 + blockIdx.y;
  const uint8_t* src = a.in + (int64_t)y * a.in_pitch + (int64_t)p0 * CIN;
  uint8_t* dst = a.out + (int64_t)y * a.out_pitch + (int64_t)p0 * COUT;

  // load 16 pixels
  uint32_t in[4 * CIN];
#pragma unroll
  for (int q = 0; q < CIN; ++q) {
    const uint4 v = reinterpret_cast<const uint4*>(src)[q];
    in[4 * q + 0] = v.x;
    in[4 * q + 1] = v.y;
    in[4 * q + 2] = v.z;
    in[4 * q + 3] = v.w;
  }
  if (a.has_pre) {
#pragma unroll
    for (int q = 0; q < CIN; ++q) {
      uint32_t t[4] = {in[4 * q], in[4 * q + 1], in[4 * q + 2], in[4 * q + 3]};
      lut16(lut, t);
      in[4 * q] = t[0];
      in[4 * q + 1] = t[1];
      in[4 * q + 2] = t[2];
      in[4 * q + 3] = t[3];
    }
  }
  constexpr int CM = GRAY ? 1 : CIN;  // channels after gray
  uint32_t mid[4 * CM];
  if constexpr (GRAY) {
    uint32_t rgb[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) rgb[i] = in[i];
    uint32_t o[4];
    gray16(a, rgb, o);
#pragma unroll
    for (int i = 0; i < 4; ++i) mid[i] = o[i];
  } else {
#pragma unroll
    for (int i = 0; i < 4 * CM; ++i) mid[i] = in[i];
  }
  if (a.has_post) {
#pragma unroll
    for (int q = 0; q < CM; ++q) {
      uint32_t t[4] = {mid[4 * q], mid[4 * q + 1], mid[4 * q + 2], mid[4 * q + 3]};
      lut16(lut + 256, t);
#pragma unroll
      for (int i = 0; i < 4; ++i) mid[4 * q + i] = t[i];
    }
  }
  uint32_t out[4 * COUT];
  if constexpr (COUT == 3 && CM == 1) {  // expand: pixel p -> bytes 3p..3p+2
#pragma unroll
    for (int b = 0; b < 48; b += 4) {
      uint32_t w = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int p = (b + e) / 3;
        w |= ((mid[p >> 2] >> ((p & 3) * 8)) & 0xFF) << (8 * e);
      }
      out[b >> 2] = w;
    }
  } else {
    static_assert(COUT == CM, "channel mismatch");
#pragma unroll
    for (int i = 0; i < 4 * COUT; ++i) out[i] = mid[i];
  }
  // constant-border margins hold zeros; reflect/replicate margins are processed
  if (a.out_border == (int)Border::Constant && (p0 < 0 || p0 + 16 > a.W)) {
#pragma unroll
    for (int i = 0; i < 4 * COUT; ++i) {
      uint32_t w = out[i];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int p = p0 + (4 * i + e) / COUT;
        if (p < 0 || p >= a.W) w &= ~(0xFFu << (8 * e));
      }
      out[i] = w;
    }
  }
#pragma unroll
  for (int q = 0; q < COUT; ++q) {
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    const u32x4v v = {out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]};
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4v*>(dst) + q);
    else reinterpret_cast<u32x4v*>(dst)[q] = v;
  }
}

// Channel-preserving byte-wise pass (LUT / invert / brightness / contrast on 1
// or 3 channels): the row is a flat byte stream, 16 contiguous bytes per lane,
// so every load/store instruction covers 1 KiB contiguously (the per-pixel
// form above moves 48-byte RGB groups at a 48-byte lane stride) and nt stores
// write whole lines.  Group g covers row bytes [16 (g + g0), +16).
constexpr int kFlatU = 4;  // 16-byte groups per lane (k_pointwise_flat)

template <bool NT>
__global__ __launch_bounds__(kNT) void k_pointwise_flat(KArgs a, int ngroups, int g0, int C) {
  __shared__ uint8_t lut[512];
  for (int i = threadIdx.x; i < 512; i += kNT) lut[i] = a.luts[i];
  const int y = a.ry0 + blockIdx.y;
  const uint8_t* srow = a.in + (int64_t)y * a.in_pitch;
  uint8_t* drow = a.out + (int64_t)y * a.out_pitch;
  // kFlatU groups per lane, kNT apart: the loads are issued before the LUT
  // barrier, so one LUT fill per workgroup is amortised over 4 KiB per wave
  typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
  u32x4v v[kFlatU];
#pragma unroll
  for (int u = 0; u < kFlatU; ++u) {
    const int g = (blockIdx.x * kFlatU + u) * kNT + threadIdx.x;
    if (g < ngroups) v[u] = *reinterpret_cast<const u32x4v*>(srow + (g + g0) * 16);
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kFlatU; ++u) {
    const int g = (blockIdx.x * kFlatU + u) * kNT + threadIdx.x;
    if (g >= ngroups) break;
    const int b0 = (g + g0) * 16;  // first byte (negative: left margin)
    uint32_t t[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
    if (a.has_pre) lut16(lut, t);
    if (a.has_post) lut16(lut + 256, t);
    if (a.out_border == (int)Border::Constant && (b0 < 0 || b0 + 16 > a.W * C)) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int bb = b0 + i;
        if (bb < 0 || bb >= a.W * C) t[i >> 2] &= ~(0xFFu << (8 * (i & 3)));
      }
    }
    const u32x4v o = {t[0], t[1], t[2], t[3]};
    if constexpr (NT) __builtin_nontemporal_store(o, reinterpret_cast<u32x4v*>(drow + b0));
    else *reinterpret_cast<u32x4v*>(drow + b0) = o;
  }
}

// Margin fill: margin byte (m, c) of row y <- pixel border_index(m) of the same row.
// One thread per (row, side, margin pixel): a flat grid over the rows, so a
// launch is rows * 2 * px / 256 busy workgroups (one 256-thread workgroup per
// row left 2/3 of its threads idle and made a 16384-row blur output 16K
// workgroups: 9.6 us).
__global__ __launch_bounds__(kNT) void k_fill_margins(uint8_t* origin, int64_t pitch, int W, int C, int y0, int rows,
                                                      int px, int border) {
  const int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x;
  const int per_row = 2 * px;
  if (i >= (int64_t)rows * per_row) return;
  const int y = y0 + (int)(i / per_row);
  const int q = (int)(i % per_row);
  const int side = q >= px;
  const int k = (side ? q - px : q) + 1;  // 1..px
  const int m = side ? W - 1 + k : -k;
  const int s = border_index_dev(m, W, border);
  uint8_t* row = origin + (int64_t)y * pitch;
  for (int c = 0; c < C; ++c) row[(int64_t)m * C + c] = s < 0 ? 0 : row[(int64_t)s * C + c];
}

__global__ __launch_bounds__(kNT) void k_synth(uint8_t* origin, int64_t pitch, int64_t E, int row0,
                                               uint64_t seed) {
  const int y = blockIdx.y;
  uint8_t* row = origin + (int64_t)y * pitch;
  for (int64_t b = ((int64_t)blockIdx.x * kNT + threadIdx.x) * 4; b < E; b += (int64_t)gridDim.x * kNT * 4) {
    uint32_t w = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (b + e < E) w |= synth_byte(seed, row0 + y, b + e) << (8 * e);
    if (b + 4 <= E) {
      *reinterpret_cast<uint32_t*>(row + b) = w;
    } else {
      for (int e = 0; b + e < E; ++e) row[b + e] = (uint8_t)(w >> (8 * e));
    }
  }
}

// Row copy between pitched buffers (packed staging <-> padded stripe), 16 bytes
// per lane; ALIGNED: both row starts and E are 16-byte multiples.
template <bool ALIGNED>
__global__ __launch_bounds__(kNT) void k_copy_rows(uint8_t* dst, int64_t dpitch, const uint8_t* src, int64_t spitch,
                                                   int64_t E) {
  const int64_t y = blockIdx.y;
  uint8_t* d = dst + y * dpitch;
  const uint8_t* sr = src + y * spitch;
  for (int64_t b = ((int64_t)blockIdx.x * kNT + threadIdx.x) * 16; b < E; b += (int64_t)gridDim.x * kNT * 16) {
    if constexpr (ALIGNED) {
      *reinterpret_cast<uint4*>(d + b) = *reinterpret_cast<const uint4*>(sr + b);
    } else {
      const int64_t n = E - b < 16 ? E - b : 16;
      for (int64_t e = 0; e < n; ++e) d[b + e] = sr[b + e];
    }
  }
}

// Linear device copy, the same-box streaming floor the benchmark record quotes
// beside its headline: one 16-byte chunk per lane, one chunk per thread, a
// grid of n/4096 workgroups that the dispatcher refills (on MI355X this beat
// every grid-stride / persistent shape: 0.2521 ms for 768 MiB = 6.39 TB/s,
// profiles/r4/final/late/membench_768m.txt); nt loads, store policy SAUX.
template <int SAUX>
__global__ __launch_bounds__(kNT) void k_copy_linear(const uint8_t* in, uint8_t* out, uint32_t bytes) {
  const __amdgpu_buffer_rsrc_t ri = make_rsrc(in, bytes);
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(out, bytes);
  typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
  const uint32_t off = ((uint32_t)blockIdx.x * kNT + threadIdx.x) * 16u;  // past `bytes`: masked by the range check
  const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(ri, off, 0, 2);
  __builtin_amdgcn_raw_buffer_store_b128(v, ro, off, 0, SAUX);
}

// Transport check pattern (comm_ring_check): word j of a message tagged `tag`
// is pattern_word(tag, j); fill writes it, check counts the words that differ.
__global__ __launch_bounds__(kNT) void k_pattern_fill(uint32_t* p, int64_t words, uint32_t tag) {
  for (int64_t j = (int64_t)blockIdx.x * kNT + threadIdx.x; j < words; j += (int64_t)gridDim.x * kNT)
    p[j] = pattern_word(tag, (uint64_t)j);
}

__global__ __launch_bounds__(kNT) void k_pattern_check(const uint32_t* p, int64_t words, uint32_t tag,
                                                       unsigned long long* errors) {
  unsigned bad = 0;
  for (int64_t j = (int64_t)blockIdx.x * kNT + threadIdx.x; j < words; j += (int64_t)gridDim.x * kNT)
    bad += p[j] != pattern_word(tag, (uint64_t)j);
  if (bad) atomicAdd(errors, (unsigned long long)bad);
}

}  // namespace dev

void launch_pattern_fill(void* p, int64_t bytes, uint32_t tag, hipStream_t s) {
  const int64_t words = bytes / 4;
  const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>(1, div_up(words, dev::kNT)), 4096);
  dev::k_pattern_fill<<<g, dev::kNT, 0, s>>>(static_cast<uint32_t*>(p), words, tag);
  HIP_CHECK(hipGetLastError());
}

void launch_pattern_check(const void* p, int64_t bytes, uint32_t tag, unsigned long long* errors, hipStream_t s) {
  const int64_t words = bytes / 4;
  const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>(1, div_up(words, dev::kNT)), 4096);
  dev::k_pattern_check<<<g, dev::kNT, 0, s>>>(static_cast<const uint32_t*>(p), words, tag, errors);
  HIP_CHECK(hipGetLastError());
}

CopyRoofline copy_roofline(int device, int64_t bytes, int frames, int reps) {
  STRIPE_CHECK(bytes > 0, "copy roofline: bytes must be positive");
  frames = std::max(1, frames);
  reps = std::max(3, reps);
  HIP_CHECK(hipSetDevice(device));
  const int64_t n = align_up(bytes, 16);
  std::vector<uint8_t*> buf((size_t)2 * frames, nullptr);
  hipStream_t s = nullptr;
  std::vector<hipEvent_t> ev((size_t)reps + 1, nullptr);
  CopyRoofline r;
  auto cleanup = [&]() {
    if (s) (void)hipStreamSynchronize(s);
    for (auto* p : buf)
      if (p) (void)hipFree(p);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (s) (void)hipStreamDestroy(s);
  };
  try {
    for (auto*& p : buf) {
      HIP_CHECK(hipMalloc(&p, (size_t)n));
      HIP_CHECK(hipMemsetAsync(p, 0x5A, (size_t)n, nullptr));
    }
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
    // one buffer descriptor addresses < 2 GiB: larger copies (e.g. a 32768^2
    // RGB frame, 3 GiB) run as back-to-back launches of at most 1 GiB each
    constexpr int64_t kChunk = int64_t(1) << 30;
    r.bytes = n;
    r.frames = frames;
    for (int policy : {0, 16}) {  // default stores; sc1 (write-through) stores
      auto launch = [&](int i) {
        const int f = i % frames;
        for (int64_t o = 0; o < n; o += kChunk) {
          const int64_t len = std::min(kChunk, n - o);
          const unsigned blocks = (unsigned)div_up(len, 16 * dev::kNT);
          if (policy == 0)
            dev::k_copy_linear<0><<<blocks, dev::kNT, 0, s>>>(buf[2 * f] + o, buf[2 * f + 1] + o, (uint32_t)len);
          else
            dev::k_copy_linear<16><<<blocks, dev::kNT, 0, s>>>(buf[2 * f] + o, buf[2 * f + 1] + o, (uint32_t)len);
        }
      };
      for (int i = 0; i < 2 * frames + 2; ++i) launch(i);
      HIP_CHECK(hipGetLastError());
      // per-copy device time: an event between consecutive copies
      HIP_CHECK(hipEventRecord(ev[0], s));
      for (int i = 0; i < reps; ++i) {
        launch(i);
        HIP_CHECK(hipEventRecord(ev[(size_t)i + 1], s));
      }
      HIP_CHECK(hipEventSynchronize(ev[(size_t)reps]));
      std::vector<float> t((size_t)reps);
      for (int i = 0; i < reps; ++i) HIP_CHECK(hipEventElapsedTime(&t[(size_t)i], ev[(size_t)i], ev[(size_t)i + 1]));
      std::sort(t.begin(), t.end());
      const double med = t[t.size() / 2];
      // back-to-back copies, events at the two ends only (what a host clock
      // around a burst of steps sees)
      HIP_CHECK(hipEventRecord(ev[0], s));
      for (int i = 0; i < reps; ++i) launch(i);
      HIP_CHECK(hipEventRecord(ev[1], s));
      HIP_CHECK(hipEventSynchronize(ev[1]));
      float burst = 0;
      HIP_CHECK(hipEventElapsedTime(&burst, ev[0], ev[1]));
      const double bm = burst / reps;
      if (r.event_ms <= 0 || med < r.event_ms) {
        r.event_ms = med;
        r.policy = policy;
      }
      if (r.burst_ms <= 0 || bm < r.burst_ms) r.burst_ms = bm;
    }
  } catch (...) {
    cleanup();
    throw;
  }
  cleanup();
  return r;
}

namespace dev {
struct CopyMultiArgs {
  CopyDesc d[kCopyMultiMax];
};
// blockIdx.y: the copy; 16-byte chunks when both ends are 16-byte aligned
__global__ __launch_bounds__(kNT) void k_copy_multi(CopyMultiArgs a) {
  const CopyDesc c = a.d[blockIdx.y];
  const bool al = ((uintptr_t)c.src % 16 == 0) && ((uintptr_t)c.dst % 16 == 0);
  const int64_t n16 = al ? c.bytes / 16 : 0;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n16; i += (int64_t)gridDim.x * kNT)
    reinterpret_cast<uint4*>(c.dst)[i] = reinterpret_cast<const uint4*>(c.src)[i];
  for (int64_t b = 16 * n16 + (int64_t)blockIdx.x * kNT + threadIdx.x; b < c.bytes; b += (int64_t)gridDim.x * kNT)
    c.dst[b] = c.src[b];
}
}  // namespace dev

void launch_copy_multi(const CopyDesc* d, int n, hipStream_t s) {
  for (int k = 0; k < n; k += kCopyMultiMax) {
    dev::CopyMultiArgs a{};
    const int m = std::min(kCopyMultiMax, n - k);
    int64_t big = 0;
    for (int i = 0; i < m; ++i) {
      a.d[i] = d[k + i];
      big = std::max(big, d[k + i].bytes);
    }
    if (big <= 0) continue;
    const unsigned gx = (unsigned)std::min<int64_t>(div_up(big, 16 * dev::kNT), 64);
    dev::k_copy_multi<<<dim3(gx, (unsigned)m), dev::kNT, 0, s>>>(a);
    HIP_CHECK(hipGetLastError());
  }
}

void launch_copy_rows(uint8_t* dst, int64_t dpitch, const uint8_t* src, int64_t spitch, int64_t E, int rows,
                      hipStream_t s) {
  if (rows <= 0 || E <= 0) return;
  const bool aligned = ((uintptr_t)dst % 16 == 0) && ((uintptr_t)src % 16 == 0) && dpitch % 16 == 0 &&
                       spitch % 16 == 0 && E % 16 == 0;
  const unsigned gx = (unsigned)std::min<int64_t>(div_up(E, 16 * dev::kNT), 64);
  (void)hipGetLastError();
  if (aligned) dev::k_copy_rows<true><<<dim3(gx, (unsigned)rows), dev::kNT, 0, s>>>(dst, dpitch, src, spitch, E);
  else dev::k_copy_rows<false><<<dim3(gx, (unsigned)rows), dev::kNT, 0, s>>>(dst, dpitch, src, spitch, E);
  HIP_CHECK(hipGetLastError());
}

void launch_pointwise(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s) {
  dev::KArgs a{};
  a.in = L.in;
  a.out = L.out;
  a.luts = pc.luts;
  a.in_pitch = L.in_pitch;
  a.out_pitch = L.out_pitch;
  a.W = L.W;
  a.E = L.W * p.cout;
  a.out_border = (int)p.out_margin_border;
  a.has_pre = p.pro.has_pre;
  a.has_post = p.pro.has_post;
  const GrayParams gp = gray_params(p.pro.gmode);
  a.gmode = gp.mode;
  for (int c = 0; c < 3; ++c) {
    a.gmul[c] = gp.mult[c];
    a.gshift[c] = gp.shift[c];
  }
  const int px = std::min(p.out_margin_px, kMaxRadius);
  const int g0 = px > 0 ? -1 : 0;  // one 16-pixel group of left margin
  const int ngroups = (int)div_up(L.W + px, 16) - g0;
  const int n0_rows = std::max(0, L.ry[1] - L.ry[0]);
  const int n1_rows = L.nrange > 1 ? std::max(0, L.ry[3] - L.ry[2]) : 0;
  for (int r = 0; r < L.nrange; ++r) {
    const int y0 = L.ry[2 * r], y1 = L.ry[2 * r + 1];
    if (y1 <= y0) continue;
    a.ry0 = y0;
    dim3 grid((unsigned)div_up(ngroups, dev::kNT), (unsigned)(y1 - y0));
    const bool gray = p.pro.gray;
    // nt stores when the pass streams more than the Infinity Cache (as the
    // stencil kernels; a smaller set is read back from the cache by the next
    // pass) and only for 1-channel output, where one store instruction covers
    // 1 KiB contiguously: the 3-channel store pattern (16 B per lane at a 48 B
    // stride) writes partial lines that nt sends to HBM unmerged (16K RGB
    // invert 0.295 -> 0.322 ms with nt; 16K gray:ref 0.192 -> 0.184 ms)
    bool nt = p.cout == 1 && (int64_t)(n0_rows + n1_rows) * L.W * (p.cin + p.cout) > dev::kNtMinBytes;
    if (const char* e = std::getenv("STRIPE_NT")) nt = std::atoi(e) != 0;
    // A/B knob, off: capping the resident workgroups of channel-changing passes
    // (STRIPE_PWG_WGS, LDS reservation) only slows them - 16K gray:ref 0.187 ms
    // uncapped, 0.212 at 4 per CU, 0.284 at 2 (profiles/r2d/pw_wgs_ab.txt)
    static const int pwg_wgs = [] {
      const char* e = std::getenv("STRIPE_PWG_WGS");
      return e ? std::atoi(e) : 0;
    }();
    size_t resg = 0;
    if (pwg_wgs > 0 && (int64_t)(n0_rows + n1_rows) * L.W * (p.cin + p.cout) > dev::kNtMinBytes) {
      int dev = 0, lds_cu = 0;
      HIP_CHECK(hipGetDevice(&dev));
      HIP_CHECK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev));
      resg = (size_t)lds_cu / (size_t)(pwg_wgs + 1) + 1024 - 512;
    }
    auto go = [&](auto k_nt, auto k_t) {
      if (nt) k_nt<<<grid, dev::kNT, resg, s>>>(a, ngroups, g0);
      else k_t<<<grid, dev::kNT, resg, s>>>(a, ngroups, g0);
    };
    if (p.cin == p.cout && !gray) {
      // byte-wise: flat 16-byte groups from the left margin to the right one
      const int C = p.cin;
      const int gb0 = -(int)div_up(px * C, 16);
      const int ngb = (int)div_up((L.W + px) * C, 16) - gb0;
      const bool ntf = (int64_t)(n0_rows + n1_rows) * L.W * 2 * C > dev::kNtMinBytes &&
                       !(std::getenv("STRIPE_NT") && std::atoi(std::getenv("STRIPE_NT")) == 0);
      const dim3 gridf((unsigned)div_up(ngb, dev::kNT * dev::kFlatU), (unsigned)(y1 - y0));
      // streaming flat passes: at most 3 resident workgroups per CU (an LDS
      // reservation the kernel never touches; fewer concurrent streams against
      // HBM: 16K RGB invert 0.287 -> 0.269 ms, brightness 0.290 -> 0.268,
      // profiles/r2d/pw_wgs_ab.txt); STRIPE_PW_WGS overrides (0 = no cap)
      static const int pw_wgs = [] {
        const char* e = std::getenv("STRIPE_PW_WGS");
        return e ? std::atoi(e) : 3;
      }();
      size_t res = 0;
      if (pw_wgs > 0 && ntf) {
        int dev = 0, lds_cu = 0;
        HIP_CHECK(hipGetDevice(&dev));
        HIP_CHECK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev));
        res = (size_t)lds_cu / (size_t)(pw_wgs + 1) + 1024 - 512;  // minus the kernel's 512-byte LUT
      }
      if (ntf) dev::k_pointwise_flat<true><<<gridf, dev::kNT, res, s>>>(a, ngb, gb0, C);
      else dev::k_pointwise_flat<false><<<gridf, dev::kNT, 0, s>>>(a, ngb, gb0, C);
    } else if (p.cin == 3 && p.cout == 1 && gray)
      go(dev::k_pointwise<3, 1, true, true>, dev::k_pointwise<3, 1, true, false>);
    else if (p.cin == 3 && p.cout == 3 && gray)
      go(dev::k_pointwise<3, 3, true, true>, dev::k_pointwise<3, 3, true, false>);
    else if (p.cin == 1 && p.cout == 3 && !gray)
      go(dev::k_pointwise<1, 3, false, true>, dev::k_pointwise<1, 3, false, false>);
    else
      fail("pointwise: unsupported channel combination " + std::to_string(p.cin) + "->" + std::to_string(p.cout));
    HIP_CHECK(hipGetLastError());
  }
}

void launch_fill_margins(uint8_t* origin, int64_t pitch, int W, int C, int y0, int y1, int px, Border b,
                         hipStream_t s) {
  if (px <= 0 || y1 <= y0) return;
  STRIPE_CHECK(px <= margin_pixels(C), "margin of " << px << " px does not fit");
  (void)hipGetLastError();
  const int64_t n = (int64_t)(y1 - y0) * 2 * px;
  dev::k_fill_margins<<<dim3((unsigned)div_up(n, dev::kNT)), dev::kNT, 0, s>>>(origin, pitch, W, C, y0, y1 - y0, px,
                                                                               (int)b);
  HIP_CHECK(hipGetLastError());
}

void launch_synth(uint8_t* origin, int64_t pitch, int W, int C, int row0, int rows, uint64_t seed,
                  int margin_px, Border b, hipStream_t s) {
  if (rows <= 0) return;
  const int64_t E = (int64_t)W * C;
  const unsigned gx = (unsigned)std::min<int64_t>(div_up(E, 4 * dev::kNT), 64);
  (void)hipGetLastError();
  dev::k_synth<<<dim3(gx, (unsigned)rows), dev::kNT, 0, s>>>(origin, pitch, E, row0, seed);
  HIP_CHECK(hipGetLastError());
  launch_fill_margins(origin, pitch, W, C, 0, rows, margin_px, b, s);
}

}  // namespace stripe
