// Device helpers shared by the stripe kernels (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "stripe/common.h"

namespace stripe {
namespace dev {

constexpr int kNT = 256;  // threads per workgroup (4 waves)

// Kernel argument block (by value, scalar registers).
struct KArgs {
  const uint8_t* in;
  uint8_t* out;
  const uint8_t* luts;      // [pre | post | epi] 256 B each
  const uint8_t* zero_row;  // origin of a zero row (Constant y-border)
  int64_t in_pitch, out_pitch;
  int W;          // pixels
  int E;          // output row bytes (W * cmid for stencils, W * cout for pointwise)
  int rows;       // local rows
  int row0, Hg;   // border geometry
  int border;     // Border enum
  int ry0, ry1, ry2, ry3;  // output row ranges [ry0,ry1) U [ry2,ry3)
  int band;       // rows per wave task
  int nb0;        // bands covering range 0
  int ntx;        // wave tiles per row (stencil kernels)
  int nbands;     // bands over both ranges
  int out_px;     // x-margin pixels to maintain on the output
  int out_border; // border mode encoded in those margins
  int has_pre, has_post, has_epi;
  // post LUT as an affine map clamp((post_a * v + post_b) >> post_k, 0, 255)
  // (exact for every v, found by the host; 0: use the table)
  int post_aff, post_a, post_b, post_k;
  int gmode;      // 0 bt601, 1 ref
  uint32_t gmul[3];
  int gshift[3];
  int cin;        // pointwise: input channels
  int nxcd;       // > 1: XCD-aware workgroup remap over this many L2 domains
  // buffer-descriptor view (stencil kernels): offsets of the origins in the
  // allocations; every hot-loop load/store is a raw buffer op whose range check
  // masks inactive lanes (no divergent branches around memory ops, so hipcc's
  // vmcnt bookkeeping stays exact and prefetched rows stay in flight)
  const uint8_t* in_base;
  uint8_t* out_base;
  uint32_t in_bytes, in_org, in_zero;
  uint32_t out_bytes, out_org;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

constexpr uint32_t kOOB = 0x80000000u;  // lane offset bias that fails the range check

// Cache-policy (aux) bits of the stencil hot-loop buffer ops (gfx950: 1 = sc0,
// 2 = nt, 16 = sc1).  Loads keep the default policy: halo rows are re-read by
// the neighbouring band (nt loads measured 12-15 % slower on a 16K RGB frame).
// Stores use nt when a pass streams more than the 256 MiB Infinity Cache
// (launch_stencil picks the kernel instance).
constexpr int kLoadAux = 0;
constexpr int kNtAux = 2;
constexpr int64_t kNtMinBytes = 224ll << 20;
// resident workgroups per CU of nt-store (HBM-streaming) stencil launches
constexpr int kNtWgsSep = 2;     // separable (k_sep)
constexpr int kNtWgsDirect = 3;  // direct (k_direct) without a gray prologue
constexpr int kXcdCount = 8;  // MI355X: 8 XCDs of 32 CUs, one L2 each

__device__ __forceinline__ int border_index_dev(int i, int n, int b) {
  if (i >= 0 && i < n) return i;
  if (b == (int)Border::Constant) return -1;
  if (b == (int)Border::Replicate) return i < 0 ? 0 : n - 1;
  if (n == 1) return 0;
  const int period = 2 * (n - 1);
  int j = i % period;
  if (j < 0) j += period;
  return j < n ? j : period - j;
}

// Input row pointer for local row y with the global-edge border applied (scalar).
__device__ __forceinline__ const uint8_t* in_row(const KArgs& a, int y) {
  int g = a.row0 + y;
  if (g < 0 || g >= a.Hg) {
    const int m = border_index_dev(g, a.Hg, a.border);
    if (m < 0) return a.zero_row;
    g = m;
  }
  return a.in + (int64_t)(g - a.row0) * a.in_pitch;
}

// Byte offset (in the input allocation) of local row y's origin, global-edge
// border applied (scalar; no memory access).
__device__ __forceinline__ uint32_t in_row_off(const KArgs& a, int y) {
  int g = a.row0 + y;
  if (g < 0 || g >= a.Hg) {
    const int m = border_index_dev(g, a.Hg, a.border);
    if (m < 0) return a.in_zero;
    g = m;
  }
  return a.in_org + (uint32_t)((int64_t)(g - a.row0) * a.in_pitch);
}

// True when input rows [y0, y1] of this wave's band need no border remap: the
// hot loop then computes row offsets without the remap's scalar branch tree
// (three scalar branches and the remap per row otherwise).
__device__ __forceinline__ bool rows_inside(const KArgs& a, int y0, int y1) {
  return a.row0 + y0 >= 0 && a.row0 + y1 < a.Hg;
}

// Offset of the input row feeding step y + ahead of a band ending at ye (rows
// past the band re-read its last input row).  `inner` (wave-uniform): the
// band's rows need no border remap (rows_inside) -> straight-line scalar math,
// no branch tree; the remap stays for the edge bands.
__device__ __forceinline__ uint32_t ahead_row_off(const KArgs& a, bool inner, int y, int ahead, int ye, int R,
                                                  uint32_t last_row) {
  if (inner) return a.in_org + (uint32_t)(min(y + ahead, ye - 1) + R) * (uint32_t)a.in_pitch;
  return y + ahead < ye ? in_row_off(a, y + ahead + R) : last_row;
}

// Bijective XCD-aware remap of the workgroup index: the hardware hands
// consecutive workgroups to the XCDs round-robin (blockIdx % 8 shares an L2),
// so logical workgroup ranges are made contiguous per XCD: vertically /
// horizontally adjacent tiles (which share halo rows / window bytes) then meet
// in one L2 (cdna_hip_programming.md T1).
__device__ __forceinline__ int xcd_remap(int bid, int nwg, int nxcd) {
  if (nxcd <= 1 || nwg < nxcd) return bid;
  const int q = nwg / nxcd, r = nwg % nxcd;
  const int x = bid % nxcd, slot = bid / nxcd;
  return x * q + min(x, r) + slot;
}

// Row range of workgroup row `by`.
__device__ __forceinline__ void band_range(const KArgs& a, int by, int& ys, int& ye) {
  if (by < a.nb0) {
    ys = a.ry0 + by * a.band;
    ye = min(ys + a.band, a.ry1);
  } else {
    ys = a.ry2 + (by - a.nb0) * a.band;
    ye = min(ys + a.band, a.ry3);
  }
}

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&d)[4], int j) {
  return (d[j >> 2] >> ((j & 3) * 8)) & 0xFFu;
}

__device__ __forceinline__ uint32_t pack4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return a | (b << 8) | (c << 16) | (d << 24);
}

// Gray of one pixel (semantic R, G, B).
__device__ __forceinline__ uint32_t gray_dev(const KArgs& a, uint32_t r, uint32_t g, uint32_t b) {
  if (a.gmode == 1)
    return ((r * a.gmul[0]) >> a.gshift[0]) + ((g * a.gmul[1]) >> a.gshift[1]) +
           ((b * a.gmul[2]) >> a.gshift[2]);
  return (r * 4899u + g * 9617u + b * 1868u + 8192u) >> 14;
}

// 16 RGB pixels (48 bytes) -> 16 gray bytes (4 dwords).
__device__ __forceinline__ void gray16(const KArgs& a, const uint32_t (&rgb)[12], uint32_t (&o)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int p = q * 4 + e;
      const int b0 = 3 * p;
      const uint32_t r = (rgb[b0 >> 2] >> ((b0 & 3) * 8)) & 0xFF;
      const uint32_t g = (rgb[(b0 + 1) >> 2] >> (((b0 + 1) & 3) * 8)) & 0xFF;
      const uint32_t bl = (rgb[(b0 + 2) >> 2] >> (((b0 + 2) & 3) * 8)) & 0xFF;
      v[e] = gray_dev(a, r, g, bl);
    }
    o[q] = pack4(v[0], v[1], v[2], v[3]);
  }
}

__device__ __forceinline__ void lut16(const uint8_t* lut, uint32_t (&o)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t w = o[q];
    o[q] = pack4(lut[w & 0xFF], lut[(w >> 8) & 0xFF], lut[(w >> 16) & 0xFF], lut[w >> 24]);
  }
}

// Store 16 output bytes at row + cb; only bytes < E (straddling chunk is split).
// Static byte indices only (a dynamic index would put `o` in scratch).
__device__ __forceinline__ void store_chunk(uint8_t* row, int cb, int E, const uint32_t (&o)[4]) {
  if (cb + 16 <= E) {
    *reinterpret_cast<uint4*>(row + cb) = make_uint4(o[0], o[1], o[2], o[3]);
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (cb + j < E) row[cb + j] = (uint8_t)byte_of(o, j);
  }
}

// True for lanes whose chunk needs the cold path (straddles E or feeds margins).
template <int C>
__device__ __forceinline__ bool edge_lane(int cb, int E, int px) {
  const int reach = (px + 1) * C;
  return cb + 16 > E || (px > 0 && (cb < reach || cb + 16 > E - reach));
}

}  // namespace dev
}  // namespace stripe
