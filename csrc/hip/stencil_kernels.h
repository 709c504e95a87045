// Stencil kernels (k_sep, k_direct) and their launch templates, shared by
// the instantiation units stencil_inst_*.hip (one group of filters each, so
// the ~440 kernel instances compile in parallel) and stencil.hip.
#pragma once

// Integer stencil passes with fused pointwise prologue/epilogue (gfx950).
//
// Reference: embossKernel (kernel.cu:64-94) - one thread per pixel, in place
// (racy, Q1), runtime-indexed private weight arrays, off-by-one bounds (Q2), and
// separate gray/contrast launches before it.  Here:
//   * every wave works on its own tile: 64 lanes x 16 bytes = a 1 KiB row segment
//     (62 output chunks + one halo chunk each side) marching down a band of rows;
//     waves never wait for each other (no workgroup barrier in the hot loop), and
//     1 KiB tiles quantise wide rows finely (8192 gray: 9 tiles for 8.3 of work);
//   * each lane loads its 16-byte chunk of every input row once (buffer dwordx4,
//     two rows in flight), applies the fused prologue (gray / LUT) in registers;
//   * separable filters: vertical taps in registers as packed-u16 adds - the
//     binomial Gaussians as a cascade of K-1 two-tap sums (no row ring) - the
//     neighbour lanes' vertical sums by DPP wave shifts, the horizontal taps as
//     packed-u16 multiply-adds on v_alignbyte-shifted pairs;
//   * non-separable filters: a K-row register ring of prologue-applied rows, the
//     neighbour lanes' edge dwords by DPP; taps are compile-time literals (zero
//     taps vanish);
//   * every hot-loop load/store is an unconditional raw buffer op; inactive lanes
//     get an offset that fails the descriptor range check (no divergent branches
//     around memory ops -> exact vmcnt, prefetches survive the barriers);
//   * out-of-place and deterministic; the x-border comes from the buffer margins,
//     the y-border from a scalar row remap; edge waves rewrite the output margins
//     after their band (one vmcnt(0) per band).

#include <cstdlib>

#include "dev_common.h"
#include "stripe/kernels.h"
#include "stripe/stencil_defs.h"

#include <map>
#include <mutex>
#include <tuple>

namespace stripe {
namespace dev {

constexpr int kW = 64;               // lanes per wave (one tile)
constexpr int kWaves = kNT / kW;     // independent wave tiles per workgroup
constexpr int kOutChunks = kW - 2;   // output chunks per wave tile

// Orders this wave's LDS writes before its later LDS reads of other lanes' data
// (LDS ops of one wave execute in order; this only stops compiler reordering).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct WaveTask {
  int wave;   // wave index within the workgroup (scalar)
  int lane;
  int xt;     // tile column
  int ys, ye; // rows
  bool valid;
  int dir = 1;  // 1: rows ys .. ye - 1 top-down; -1: bottom-up (kRuns launches)
};

// Task w of a pass: tile column w mod ntx of band w / ntx (band-major).
__device__ __forceinline__ WaveTask task_at(const KArgs& a, int w) {
  WaveTask t;
  t.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  t.lane = threadIdx.x & 63;
  t.xt = w % a.ntx;
  const int bt = w / a.ntx;
  t.valid = bt < a.nbands;
  t.ys = t.ye = 0;
  if (t.valid) {
    band_range(a, bt, t.ys, t.ye);
    t.valid = t.ys < t.ye;
  }
  return t;
}

// kRuns task: a workgroup = kWaves adjacent tile columns of one band, as in
// the one-task launch, but the workgroups dispatched to one XCD (blockIdx % 8)
// walk down runs of kRunLen bands of one column group, consecutive bands one
// dispatch slot (8 workgroups) apart, even bands bottom-up and odd bands
// top-down: the two readers of a boundary's halo rows run on one XCD and read
// them at the same moment (both first or both last), so one of the two reads
// is an L2 hit.  Runs are dealt to the XCDs round-robin (balanced); only every
// kRunLen-th boundary is still read twice through the fabric.
constexpr int kRunLen = 8;
__device__ __forceinline__ WaveTask runs_task(const KArgs& a) {
  WaveTask t;
  t.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  t.lane = threadIdx.x & 63;
  const int b = (int)blockIdx.x;
  const int x = b % kXcdCount, j = b / kXcdCount;
  const int g = (j / kRunLen) * kXcdCount + x;  // global run
  const int ncg = (a.ntx + kWaves - 1) / kWaves;  // column groups
  const int cg = g % ncg;
  const int bt = (g / ncg) * kRunLen + j % kRunLen;
  t.xt = kWaves * cg + t.wave;
  t.valid = bt < a.nbands && t.xt < a.ntx;
  t.ys = t.ye = 0;
  if (t.valid) {
    band_range(a, bt, t.ys, t.ye);
    t.valid = t.ys < t.ye;
  }
  t.dir = (bt & 1) ? 1 : -1;
  return t;
}
// grid of a kRuns launch: every run of every column group
inline int64_t runs_grid(int ntx, int nbands) {
  const int64_t ncg = (ntx + kWaves - 1) / kWaves;
  const int64_t nruns = ncg * ((nbands + kRunLen - 1) / kRunLen);
  return (int64_t)kXcdCount * kRunLen * ((nruns + kXcdCount - 1) / kXcdCount);
}

// The task of this wave in a one-task-per-wave launch (XCD-aware workgroup order).
template <int NW = kWaves>
__device__ __forceinline__ WaveTask wave_task(const KArgs& a) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  return task_at(a, xcd_remap((int)blockIdx.x, (int)gridDim.x, a.nxcd) * NW + wave);
}

enum { PRO_NONE = 0, PRO_LUT = 1, PRO_GRAY = 2, PRO_GRAYLUT = 3 };
// PRO_GRAY: arithmetic gray (bt601 fixed point); PRO_GRAYLUT: gray:ref (three
// truncated per-channel terms, gray_ref_pairs) with its post LUT applied to the
// u16 lanes directly.  Both read 48 RGB bytes per lane.
constexpr bool is_gray(int pro) { return pro == PRO_GRAY || pro == PRO_GRAYLUT; }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

typedef short i16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ i16x2 as_i16x2(uint32_t x) { return __builtin_bit_cast(i16x2, x); }
__device__ __forceinline__ uint32_t as_u32(i16x2 x) { return __builtin_bit_cast(uint32_t, x); }

// The lane's raw input bytes of one row: 16 bytes, or 48 for a gray prologue
// (16 RGB pixels).  Loads are issued by load_raw and the prologue (gray / LUT)
// is applied by cook when the row is consumed, so prefetched rows stay in
// flight instead of being waited for at the load (a LUT or gray conversion at
// the load site forces an s_waitcnt there).
template <int PRO>
struct RawChunk {
  uint32_t d[is_gray(PRO) ? 12 : 4];
};

template <int PRO>
__device__ __forceinline__ void load_raw(__amdgpu_buffer_rsrc_t rin, uint32_t row_off, uint32_t lane_off,
                                         RawChunk<PRO>& r) {
  if constexpr (is_gray(PRO)) {
    const uint32_t off = row_off + lane_off;  // lane_off already scaled by 3
    const u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, kLoadAux);
    const u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(rin, off + 16, 0, kLoadAux);
    const u32x4 v2 = __builtin_amdgcn_raw_buffer_load_b128(rin, off + 32, 0, kLoadAux);
    r.d[0] = v0.x; r.d[1] = v0.y; r.d[2] = v0.z; r.d[3] = v0.w;
    r.d[4] = v1.x; r.d[5] = v1.y; r.d[6] = v1.z; r.d[7] = v1.w;
    r.d[8] = v2.x; r.d[9] = v2.y; r.d[10] = v2.z; r.d[11] = v2.w;
  } else {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rin, row_off + lane_off, 0, kLoadAux);
    r.d[0] = v.x; r.d[1] = v.y; r.d[2] = v.z; r.d[3] = v.w;
  }
}

// gray:ref (kernel.cu:40-42: per-channel truncated products, summed); the
// sum (<= 254) and the optional post LUT land straight in the u16 fields the
// stencil arithmetic uses, so there is no byte packing / unpacking.
template <int N>
__device__ __forceinline__ uint32_t byte_at(const uint32_t (&d)[N], int j) {
  return (d[j >> 2] >> ((j & 3) * 8)) & 0xFFu;
}

__device__ __forceinline__ void gray_ref_pairs(const KArgs& a, const uint32_t (&d)[12], const uint8_t* luts,
                                               uint32_t (&u)[8]) {
  // the exact terms as 24-bit multiply + shift (find_trunc_magic): no LDS
  // traffic for them.  As 48 table lookups per row they kept the LDS 65 % busy
  // on the 16K RGB reference pipeline, half of it bank conflicts (random pixel
  // bytes).  Then all 16 sums, then (one uniform branch) the 16 post-LUT
  // lookups: one LDS round trip per row.
  uint32_t g[16];
  const uint32_t m0 = a.gmul[0] & 0xFFFFFFu, m1 = a.gmul[1] & 0xFFFFFFu, m2 = a.gmul[2] & 0xFFFFFFu;
#pragma unroll
  for (int px = 0; px < 16; ++px)
    g[px] = ((byte_at(d, 3 * px) * m0) >> a.gshift[0]) + ((byte_at(d, 3 * px + 1) * m1) >> a.gshift[1]) +
            ((byte_at(d, 3 * px + 2) * m2) >> a.gshift[2]);
  if (a.has_post && !a.post_aff) {
#pragma unroll
    for (int px = 0; px < 16; ++px) g[px] = luts[256 + g[px]];
  }
#pragma unroll
  for (int pp = 0; pp < 8; ++pp) u[pp] = g[2 * pp] | (g[2 * pp + 1] << 16);
  if (a.has_post && a.post_aff) {
    // affine post map (contrast, brightness, invert ...) in packed i16: 4 VALU
    // per pixel pair instead of 2 dependent LDS lookups (random bytes index
    // the table: bank conflicts and a round trip the wave waits for)
    const short ma = (short)a.post_a, mb = (short)a.post_b;
    const i16x2 sh = {(short)a.post_k, (short)a.post_k};
#pragma unroll
    for (int pp = 0; pp < 8; ++pp) {
      i16x2 t = as_i16x2(u[pp]) * ma + mb;
      t = t >> sh;
      t = __builtin_elementwise_max(t, (i16x2)(short)0);
      u[pp] = as_u32(__builtin_elementwise_min(t, (i16x2)(short)255));
    }
  }
}

// Prologue: the 16 output-channel bytes of a raw chunk.
template <int PRO>
__device__ __forceinline__ void cook(const KArgs& a, const RawChunk<PRO>& r, const uint8_t* lut_post,
                                     uint32_t (&o)[4]) {
  if constexpr (PRO == PRO_GRAYLUT) {
    uint32_t u[8];
    gray_ref_pairs(a, r.d, lut_post - 256, u);
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = __builtin_amdgcn_perm(u[2 * q + 1], u[2 * q], 0x06040200u);
  } else if constexpr (PRO == PRO_GRAY) {
    gray16(a, r.d, o);
    if (a.has_post) lut16(lut_post, o);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = r.d[q];
    if constexpr (PRO == PRO_LUT) lut16(lut_post, o);
  }
}

// Load + prologue in one step (rows that are consumed right away).
template <int PRO>
__device__ __forceinline__ void load_chunk(const KArgs& a, __amdgpu_buffer_rsrc_t rin, uint32_t row_off,
                                           uint32_t lane_off, const uint8_t* lut_post, uint32_t (&o)[4]) {
  RawChunk<PRO> r;
  load_raw<PRO>(rin, row_off, lane_off, r);
  cook<PRO>(a, r, lut_post, o);
}

template <int PRO>
__device__ __forceinline__ void load_luts(const KArgs& a, uint8_t* lds) {
  for (int i = threadIdx.x; i < 768; i += (int)blockDim.x) lds[i] = a.luts[i];
}

// Legacy skip border (kernel.cu:83 interior-only bounds): bytes of pixels in the
// skip region keep the prologue value.  The column part of the region is fixed
// per lane, so skip_cols builds the lane's byte mask once per band (bits set:
// the stencil output is kept); the row part is one scalar test per row, and the
// merge is 4 bit-selects per row (was 16 compare/selects per row, and the
// per-row scalar bounds spilled SGPRs in every SKIP instance).
template <int C>
__device__ __forceinline__ void skip_cols(const KArgs& a, int cb, int R, uint32_t (&keep)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t m = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int x = (cb + 4 * q + e) / C;
      m |= (x > R && x < a.W - R) ? (0xFFu << (8 * e)) : 0u;
    }
    keep[q] = m;
  }
}

__device__ __forceinline__ void apply_skip(const KArgs& a, int gy, int R, const uint32_t (&keep)[4],
                                           const uint32_t (&center)[4], uint32_t (&o)[4]) {
  const bool row_skip = gy <= R || gy >= a.Hg - R;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t m = row_skip ? 0u : keep[q];
    o[q] = (o[q] & m) | (center[q] & ~m);
  }
}

// First stencil byte of wave tile xt (tb bytes a tile) of a row.  The row's
// last tile starts early enough to hold every byte its right margins copy:
// with a plain grid, a last tile shorter than the margin reach ((px + 1) C
// bytes) would copy pixels the tile before it stores -- another wave,
// unordered with it (e.g. 333-pixel RGB rows: 999 bytes, a 7-byte last tile).
// It then overlaps its neighbour, and both store the same values there.
template <int C>
__device__ __forceinline__ int tile_base(const KArgs& a, int xt, int tb) {
  const int b = xt * tb;
  if (xt == 0 || xt != a.ntx - 1 || a.out_px == 0) return b;
  return min(b, (a.E - (a.out_px + 1) * C) & ~15);
}

// After a band: the row's edge waves rewrite the x-margins of their output
// rows (margin pixel m <- pixel border_index(m) of the same row).  A margin
// byte's writer must follow the store of its source byte and the store of the
// row's last chunk, whose 16 bytes reach past the row into the right margin:
// the edge tile makes both (tile_base), so vmcnt(0) orders them; the reads
// use sc0 (L2) so they see them.
// C: stencil channels (the wave tiling covers W * C bytes); CO: output bytes
// per pixel (3 for a fused expand of a 1-channel stencil, else C).
template <int C, int CO = C>
__device__ __forceinline__ void band_margins(const KArgs& a, const WaveTask& t) {
  const int px = a.out_px;
  if (px == 0) return;
  const bool left = t.xt == 0;
  const bool right = t.xt == a.ntx - 1;
  if (!left && !right) return;
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this band's stores are done
  const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.out_base, a.out_bytes);
  const int nb = px * CO;  // margin bytes per side
  const int per_row = 2 * nb;
  for (int i = t.lane; i < (t.ye - t.ys) * per_row; i += kW) {
    const int y = t.ys + i / per_row;
    const int q = i % per_row;
    const int side = q >= nb;
    const int k = (side ? q - nb : q) / CO + 1;
    const int c = (side ? q - nb : q) % CO;
    if ((side == 0 && !left) || (side == 1 && !right)) continue;
    const int m = side ? a.W - 1 + k : -k;
    const int src = border_index_dev(m, a.W, a.out_border);
    const uint32_t row = a.out_org + (uint32_t)((int64_t)y * a.out_pitch);
    uint8_t v = 0;
    if (src >= 0) v = __builtin_amdgcn_raw_buffer_load_b8(rout, row + src * CO + c, 0, 1);
    __builtin_amdgcn_raw_buffer_store_b8(v, rout, row + m * CO + c, 0, 0);
  }
}

// v_perm selector of output dword k of an expanded chunk: its bytes are
// stencil bytes (4k + i) / 3, taken from source dwords q = (4k/3)/4 and q + 1.
constexpr uint32_t expand_sel(int k) {
  uint32_t s = 0;
  const int q = (4 * k / 3) / 4;
  for (int i = 0; i < 4; ++i) s |= (uint32_t)((4 * k + i) / 3 - 4 * q) << (8 * i);
  return s;
}

// Output store of one row of a wave tile.  Plain: each lane stores its 16-byte
// chunk at row + L.off[0] (kOOB-biased lanes are masked by the range check).
// EXP (fused `expand` epilogue): a lane's 16 gray bytes become 48 bytes of 3
// equal channels (12 v_perm).  Stored in place they would be three 16-byte
// stores at a 48-byte lane stride (each instruction touching 3x the cache lines
// of a contiguous one); instead the wave re-tiles them through LDS (3 KiB per
// wave: 3 ds_write_b128 at the 48-byte stride, conflict-free per 8 lanes, and
// 3 contiguous ds_read_b128) so store j writes chunk 64j + lane of the tile's
// 3072 contiguous output bytes.
struct OutLanes {
  uint32_t off[3];  // per-lane offset from the row start (kOOB: not stored)
};

template <bool EXP>
__device__ __forceinline__ OutLanes out_lanes(const KArgs& a, int lane, int cb0) {
  OutLanes L;
  if constexpr (!EXP) {
    const int cb = cb0 + 16 * lane;
    L.off[0] = lane >= 1 && lane <= kW - 2 && cb < a.E ? (uint32_t)cb : kOOB;
    L.off[1] = L.off[2] = kOOB;
  } else {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int c = kW * j + lane;  // output chunk of the tile
      const int s = c / 3;          // lane that computed it
      L.off[j] = s >= 1 && s <= kW - 2 && cb0 + 16 * s < a.E ? (uint32_t)(3 * cb0 + 16 * c) : kOOB;
    }
  }
  return L;
}

template <bool EXP, int SAUX>
__device__ __forceinline__ void store_out(const uint32_t (&o)[4], __amdgpu_buffer_rsrc_t rout, bool valid,
                                          uint32_t row, const OutLanes& L, uint4* xb, int lane) {
  if constexpr (!EXP) {
    const u32x4 ov = {o[0], o[1], o[2], o[3]};
    __builtin_amdgcn_raw_buffer_store_b128(ov, rout, valid ? row + L.off[0] : kOOB, 0, SAUX);
  } else {
#pragma unroll
    for (int j = 0; j < 3; ++j) {  // 4 live dwords at a time
      uint32_t e[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 4 * j + i, q = (4 * k / 3) / 4;
        e[i] = __builtin_amdgcn_perm(o[q < 3 ? q + 1 : 3], o[q], expand_sel(k));
      }
      xb[3 * lane + j] = make_uint4(e[0], e[1], e[2], e[3]);
    }
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const uint4 v = xb[kW * j + lane];
      const u32x4 ov = {v.x, v.y, v.z, v.w};
      __builtin_amdgcn_raw_buffer_store_b128(ov, rout, valid ? row + L.off[j] : kOOB, 0, SAUX);
    }
    wave_lds_sync();  // reads done before the next row's writes (program order)
  }
}

// ------------------------------------------------------------------------------
// Separable filters (gaussian3/5/7, box3/5)
// ------------------------------------------------------------------------------
__device__ __forceinline__ void unpack16(const uint32_t (&r)[4], uint32_t (&p)[8]) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    p[2 * d] = __builtin_amdgcn_perm(0u, r[d], 0x0c010c00u);      // (b0, b1)
    p[2 * d + 1] = __builtin_amdgcn_perm(0u, r[d], 0x0c030c02u);  // (b2, b3)
  }
}

// Prologue straight to the unpacked u16-pair form of the stencil arithmetic.
template <int PRO>
__device__ __forceinline__ void cook_pairs(const KArgs& a, const RawChunk<PRO>& r, const uint8_t* luts,
                                           uint32_t (&u)[8]) {
  if constexpr (PRO == PRO_GRAYLUT) {
    gray_ref_pairs(a, r.d, luts, u);
  } else {
    uint32_t c[4];
    cook<PRO>(a, r, luts + 256, c);
    unpack16(c, u);
  }
}

template <class F>
struct SepTraits {
  static constexpr int gsum() {
    int s = 0;
    for (int i = 0; i < F::K; ++i) s += F::g(i);
    return s;
  }
  static constexpr int log2div() {
    int l = 0;
    while ((1 << l) < F::DIV) ++l;
    return (1 << l) == F::DIV ? l : -1;
  }
  // horizontal sums (+ rounding) fit 16 bits and the division is a shift
  static constexpr bool H16 = log2div() >= 0 && gsum() * gsum() * 255 + F::DIV / 2 < 65536;
  // binomial H16 filters: the rounding term DIV/2 rides on the vertical sums
  // (+DIV/2/gsum on each, summed gsum times by the horizontal taps), added by
  // the cascade's last stage as a third operand (v_add3_u32: the packed u16
  // fields never carry, every partial sum is < 2^16)
  static constexpr bool FOLD = H16 && F::BINOM && (F::DIV / 2) % gsum() == 0;
  static constexpr uint32_t kFold = FOLD ? (uint32_t)(F::DIV / 2 / gsum()) * 0x00010001u : 0u;
  static constexpr bool SYM = [] {
    for (int i = 0; i < F::K; ++i)
      if (F::g(i) != F::g(F::K - 1 - i)) return false;
    return true;
  }();
};

// u16 pair (v[k], v[k+1]) of the window (k: u16 index, compile-time after unroll)
template <int WDW>
__device__ __forceinline__ uint32_t pair_at(const uint32_t (&w)[WDW], int k) {
  return (k & 1) ? __builtin_amdgcn_alignbyte(w[(k + 1) >> 1], w[(k - 1) >> 1], 2) : w[k >> 1];
}

// op(pair at base - d, pair at base + d) for an even base (a symmetric tap
// pair, op = packed add, or sub for antisymmetric taps).  For odd d both pairs
// straddle dwords; applying op to the whole dwords first and extracting the
// pair once gives the same fields (the ops are per 16-bit half), and the dword
// op w[j] op w[j + d] is the same for neighbouring output pairs, so the
// unrolled horizontal loop shares it: one op + one alignbyte per output pair
// instead of two alignbytes + one op.
template <class Op, int WDW>
__device__ __forceinline__ uint32_t sym_pair(const uint32_t (&w)[WDW], int base, int d, Op op) {
  if ((d & 1) == 0) return op(w[(base + d) >> 1], w[(base - d) >> 1]);
  const uint32_t lo = op(w[(base + d - 1) >> 1], w[(base - d - 1) >> 1]);
  const uint32_t hi = op(w[(base + d + 1) >> 1], w[(base - d + 1) >> 1]);
  return __builtin_amdgcn_alignbyte(hi, lo, 2);
}
struct PkAddU16 {
  __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return as_u32(as_u16x2(a) + as_u16x2(b)); }
};
struct PkSubI16 {  // a - b per field
  __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return as_u32(as_i16x2(a) - as_i16x2(b)); }
};

// Vertical filter state.  Binomial filters: cascade of K-1 two-tap sums
// s_k[y] = s_{k-1}[y] + s_{k-1}[y-1] (K-1 state rows); others: the last K rows.
template <class F>
struct VState {
  static constexpr int NS = F::BINOM ? F::K - 1 : F::SOBEL ? 2 : F::K;
  uint32_t s[NS][8];
};

// Sobel: push one row; `sm` = r0 + 2 r1 + r2 (smoothing, u16) and `df` = r2 - r0
// (difference, i16) of the row above it.  State: the two previous rows.
template <class F>
__device__ __forceinline__ void vpush_sobel(const uint32_t (&row)[8], const VState<F>& prev, VState<F>& next,
                                            uint32_t (&sm)[8], uint32_t (&df)[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    next.s[0][k] = prev.s[1][k];
    next.s[1][k] = row[k];
    const u16x2 r0 = as_u16x2(prev.s[0][k]), r1 = as_u16x2(prev.s[1][k]), r2 = as_u16x2(row[k]);
    sm[k] = as_u32(r0 + r2 + (r1 << (unsigned short)1));
    df[k] = as_u32(as_i16x2(row[k]) - as_i16x2(prev.s[0][k]));
  }
}

// Push one unpacked row; `v` receives the vertical sums of the row R above it.
template <class F>
__device__ __forceinline__ void vpush(const uint32_t (&row)[8], const VState<F>& prev, VState<F>& next,
                                      uint32_t (&v)[8]) {
  if constexpr (F::BINOM) {
    constexpr uint32_t kf = SepTraits<F>::kFold;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint32_t cur = row[k];
#pragma unroll
      for (int st = 0; st < F::K - 1; ++st) {
        next.s[st][k] = cur;
        if (kf != 0 && st == F::K - 2)  // fields stay < 2^16: no carry between them
          asm("v_add3_u32 %0, %1, %2, %3" : "=v"(cur) : "v"(cur), "v"(prev.s[st][k]), "s"(kf));
        else
          cur = as_u32(as_u16x2(cur) + as_u16x2(prev.s[st][k]));
      }
      v[k] = cur;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int i = 0; i < F::K - 1; ++i) next.s[i][k] = prev.s[i + 1][k];
      next.s[F::K - 1][k] = row[k];
      u16x2 acc = as_u16x2(next.s[0][k]) * (unsigned short)F::g(0);
#pragma unroll
      for (int i = 1; i < F::K; ++i) acc += as_u16x2(next.s[i][k]) * (unsigned short)F::g(i);
      v[k] = as_u32(acc);
    }
  }
}

// The horizontal window of a lane's vertical sums: window dword i is logical
// dword i - WLO/2 of the lane's 8 (negative: the left lane's, >= 8: the right
// lane's), fetched by DPP wave shifts (wave_shr:1 / wave_shl:1); lanes 0 and 63
// get zeros for the missing side (their outputs are never stored).
template <int WLO, int WDW>
__device__ __forceinline__ void dpp_window(const uint32_t (&v)[8], uint32_t (&w)[WDW]) {
#pragma unroll
  for (int i = 0; i < WDW; ++i) {
    const int g = i - WLO / 2;
    if (g < 0) w[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[8 + g], 0x138, 0xf, 0xf, false);
    else if (g >= 8) w[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[g - 8], 0x130, 0xf, 0xf, false);
    else w[i] = v[g];
  }
}

// Horizontal pass of an H16 separable filter (SepTraits::H16): the lane's 16
// output bytes from its window of vertical sums (dpp_window).
template <int C, class F, int WLO, int WDW>
__device__ __forceinline__ void sep_h16_out(const uint32_t (&w)[WDW], uint32_t (&o)[4]) {
  using T = SepTraits<F>;
  constexpr int R = F::R, K = F::K;
  uint32_t h[8];
#pragma unroll
  for (int pp = 0; pp < 8; ++pp) {
    u16x2 sacc;
    if constexpr (T::SYM && F::g(0) == 1) {
      // mirrored taps share a weight: (x[-i] + x[+i]) * g, outermost pair
      // (weight 1) first, centre last: 2R ops per output pair.  Plain u32
      // arithmetic on the packed pair is exact (H16: every partial sum and
      // product is < 2^16, so nothing crosses into the high field), which
      // turns power-of-two weights into one v_lshl_add_u32.
      auto madd = [](uint32_t s, uint32_t acc, int g) __attribute__((always_inline)) {
        if ((g & (g - 1)) == 0) {
          int k = 0;
          while ((1 << k) < g) ++k;
          return (s << k) + acc;
        }
        return as_u32(as_u16x2(s) * (unsigned short)g + as_u16x2(acc));
      };
      uint32_t acc = sym_pair(w, WLO + 2 * pp, R * C, PkAddU16{});
#pragma unroll
      for (int i = 1; i < R; ++i) acc = madd(sym_pair(w, WLO + 2 * pp, (R - i) * C, PkAddU16{}), acc, F::g(i));
      acc = madd(pair_at(w, WLO + 2 * pp), acc, F::g(R));
      sacc = as_u16x2(acc);
      if constexpr (!T::FOLD) sacc += (u16x2)(unsigned short)(F::DIV / 2);
    } else {
      sacc = (u16x2)(unsigned short)(F::DIV / 2);
#pragma unroll
      for (int i = 0; i < K; ++i)
        sacc += as_u16x2(pair_at(w, WLO + 2 * pp + (i - R) * C)) * (unsigned short)F::g(i);
    }
    if constexpr (T::log2div() != 8) sacc = sacc >> (unsigned short)T::log2div();
    h[pp] = as_u32(sacc);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
    o[q] = T::log2div() == 8 ? __builtin_amdgcn_perm(h[2 * q + 1], h[2 * q], 0x07050301u)
                             : __builtin_amdgcn_perm(h[2 * q + 1], h[2 * q], 0x06040200u);
}

// One wave task (a band of rows of one tile column) of a separable filter.
template <int C, class F, int PRO, bool SKIP, int SAUX, bool EXP>
__device__ __forceinline__ void sep_task(const KArgs& a, const WaveTask& t, const uint8_t* luts, uint4* xb) {
  static_assert(!EXP || C == 1, "expand epilogue needs a 1-channel stencil");
  constexpr int R = F::R, K = F::K;
  constexpr int WLO = (R * C <= 8) ? 8 : 16;  // u16 window start (relative to chunk)
  constexpr int WDW = (2 * WLO + 16) / 2;     // window dwords
  constexpr int CIN = is_gray(PRO) ? 3 : 1;  // input bytes per output byte
  using T = SepTraits<F>;
  const int lane = t.lane;
  const int ys = t.ys, ye = t.ye;
  // rows are stepped in logical order y = ys .. ye - 1; a bottom-up task
  // (t.dir < 0) maps logical row y to physical row ys + ye - 1 - y.  The
  // vertical taps are symmetric (sobel's difference taps flip sign under a
  // magnitude), so the outputs are the same bits in either direction.
  constexpr bool kRev = SepTraits<F>::SYM;  // kRuns instances only (static_assert there)
  const int pbase = kRev && t.dir < 0 ? ys + ye - 1 : 0;
  const int psign = kRev && t.dir < 0 ? -1 : 1;
  auto phys = [&](int y) __attribute__((always_inline)) { return pbase + psign * y; };
  const int cb = tile_base<C>(a, t.xt, kOutChunks * 16) - 16 + lane * 16;
  const uint32_t lane_in = cb < a.E + 16 ? (uint32_t)(cb * CIN) : kOOB;
  const OutLanes lout = out_lanes<EXP>(a, lane, cb - 16 * lane);
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in_base, a.in_bytes);
  const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.out_base, a.out_bytes);
  const uint32_t last_row = in_row_off(a, phys(ye - 1 + R));
  // @skip: the prologue bytes of the last 4 input rows (slot (r - ys) mod 4),
  // so an output row's centre bytes come from registers, not a second load
  constexpr int kRing = SKIP ? 4 : 1;
  static_assert(!SKIP || R < kRing, "skip centre ring too short");
  uint32_t cen[kRing][4];
  uint32_t keep[SKIP ? 4 : 1];
  if constexpr (SKIP) skip_cols<C>(a, cb, R, keep);
  auto keep_centre = [&](const uint32_t (&u)[8], uint32_t (&c)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) c[q] = __builtin_amdgcn_perm(u[2 * q + 1], u[2 * q], 0x06040200u);
  };

  VState<F> sa, sb;
#pragma unroll
  for (int i = 0; i < VState<F>::NS; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) sa.s[i][k] = 0;
  uint32_t vdummy[8];
#pragma unroll
  for (int i = 0; i < K - 1; ++i) {  // prime with rows ys-R .. ys+R-1
    uint32_t u[8];
    RawChunk<PRO> rr;
    load_raw<PRO>(rin, in_row_off(a, phys(ys - R + i)), lane_in, rr);
    cook_pairs<PRO>(a, rr, luts, u);
    if constexpr (SKIP) {
      if (i >= R) keep_centre(u, cen[(i - R) % kRing]);
    }
    if constexpr (F::SOBEL) {
      if (i & 1) vpush_sobel<F>(u, sb, sa, vdummy, vdummy);
      else vpush_sobel<F>(u, sa, sb, vdummy, vdummy);
    } else {
      if (i & 1) vpush<F>(u, sb, sa, vdummy);
      else vpush<F>(u, sa, sb, vdummy);
    }
  }
  // kPF rows in flight per lane (memory-level parallelism is what this streaming
  // kernel is bound by); loads past the band re-read its last input row
  // (unconditional: no branch around the load)
  // (a gray prologue reads 48 bytes per row: 2 rows give more bytes in flight
  // than 4 plain rows, at 24 fewer registers; 6 or 8 plain rows ran 2-11 %
  // slower on warm N=8 shares and no faster on 16K frames, profiles/r6/kpf/)
  constexpr int kPF = is_gray(PRO) ? 2 : 4;
  RawChunk<PRO> nx[kPF];
#pragma unroll
  for (int i = 0; i < kPF; ++i)
    load_raw<PRO>(rin, ys + i < ye ? in_row_off(a, phys(ys + i + R)) : last_row, lane_in, nx[i]);

  const bool inner = rows_inside(a, ys - R, ye - 1 + R);
  // input row feeding step y + kPF (ahead_row_off, through phys)
  auto ahead_off = [&](int y) __attribute__((always_inline)) -> uint32_t {
    if (inner) return a.in_org + (uint32_t)phys(min(y + kPF, ye - 1) + R) * (uint32_t)a.in_pitch;
    return y + kPF < ye ? in_row_off(a, phys(y + kPF + R)) : last_row;
  };
  // (i: the step's index in its unrolled group; the group starts at a multiple
  // of kRing rows past ys, so ring slots are compile-time)
  auto row_step = [&](int y, int i, const VState<F>& prev, VState<F>& next, RawChunk<PRO>& nb, bool valid) {
    uint32_t u[8], vv[8], dd[8];
    cook_pairs<PRO>(a, nb, luts, u);
    load_raw<PRO>(rin, ahead_off(y), lane_in, nb);
    if constexpr (SKIP) keep_centre(u, cen[(i + R) % kRing]);  // input row y + R
    if constexpr (F::SOBEL) {
      vpush_sobel<F>(u, prev, next, vv, dd);
    } else {
      vpush<F>(u, prev, next, vv);
    }
    // lanes 0 and 63 (halo chunks) compute garbage and their store is masked
    // neighbour lanes' vertical sums by DPP wave shifts (no LDS round trip, no
    // wave sync; 5 % faster on gray stripes than an LDS row, profiles/r2d/sep_dpp_ab.txt)
    uint32_t w[WDW];
    uint32_t wd[F::SOBEL ? WDW : 1];
    dpp_window<WLO, WDW>(vv, w);
    if constexpr (F::SOBEL) dpp_window<WLO, WDW>(dd, wd);
    uint32_t o[4];
    if constexpr (F::SOBEL) {
      // Gx = S[x+C] - S[x-C], Gy = D[x-C] + 2 D[x] + D[x+C], out = min(|Gx| + |Gy|, 255)
      uint32_t h[8];
#pragma unroll
      for (int pp = 0; pp < 8; ++pp) {
        const i16x2 gx = as_i16x2(sym_pair(w, WLO + 2 * pp, C, PkSubI16{}));
        const i16x2 gy = as_i16x2(sym_pair(wd, WLO + 2 * pp, C, PkAddU16{})) +
                         (as_i16x2(pair_at(wd, WLO + 2 * pp)) << (short)1);
        if constexpr (F::L2) {
          // min(round(sqrt(n)), 255), n = gx^2 + gy^2, exactly, in f32: only
          // n <= 65536 matters (a larger root saturates), n is exact in f32, and
          // there sqrt(n) stays >= 0.25 / (2 * 256.5) ~ 4.9e-4 away from every
          // k + 1/2 (|n - (k + 1/2)^2| >= 1/4), far beyond v_sqrt_f32's 1 ulp
          // (3e-5 at 256): rounding the f32 root to nearest is exact (no ties).
          // (Integer corrections of a truncated root cost 2.7x this pass's time.)
          uint32_t hv[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const float fx = (float)gx[e], fy = (float)gy[e];
            const float n = __builtin_fminf(__builtin_fmaf(fx, fx, fy * fy), 65536.0f);
            hv[e] = min((uint32_t)__builtin_rintf(__builtin_amdgcn_sqrtf(n)), 255u);
          }
          h[pp] = hv[0] | (hv[1] << 16);
        } else {
          const i16x2 m = __builtin_elementwise_max(gx, -gx) + __builtin_elementwise_max(gy, -gy);
          h[pp] = as_u32(__builtin_elementwise_min(m, (i16x2)(short)255));
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = __builtin_amdgcn_perm(h[2 * q + 1], h[2 * q], 0x06040200u);
    } else if constexpr (T::H16) {
      sep_h16_out<C, F, WLO, WDW>(w, o);
    } else {
      uint32_t ob[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        uint32_t hs = 0;
#pragma unroll
        for (int i = 0; i < K; ++i) {
          const int k = WLO + j + (i - R) * C;
          hs += (uint32_t)F::g(i) * ((w[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu);
        }
        ob[j] = (hs + F::DIV / 2) / F::DIV;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = pack4(ob[4 * q], ob[4 * q + 1], ob[4 * q + 2], ob[4 * q + 3]);
    }
    if constexpr (SKIP) apply_skip(a, a.row0 + phys(y), R, keep, cen[i % kRing], o);
    if (a.has_epi) lut16(luts + 512, o);
    // rows past the band (tail of the 4-row group) are computed but not stored
    store_out<EXP, SAUX>(o, rout, valid, a.out_org + (uint32_t)((int64_t)phys(y) * a.out_pitch), lout, xb, lane);
  };

  // rows go in groups of kG with no branch around any step, ping-ponging the
  // filter state so no register copies are needed
  constexpr bool live_in_b = ((K - 1) & 1) != 0;
  constexpr int kG = kPF > kRing ? kPF : kRing;  // multiple of both
  static_assert(kG % kPF == 0 && kG % kRing == 0, "row group must cover the prefetch and ring periods");
  for (int y = ys; y < ye; y += kG) {
#pragma unroll
    for (int i = 0; i < kG; i += 2) {
      if (live_in_b) {
        row_step(y + i, i, sb, sa, nx[i % kPF], y + i < ye);
        row_step(y + i + 1, i + 1, sa, sb, nx[(i + 1) % kPF], y + i + 1 < ye);
      } else {
        row_step(y + i, i, sa, sb, nx[i % kPF], y + i < ye);
        row_step(y + i + 1, i + 1, sb, sa, nx[(i + 1) % kPF], y + i + 1 < ye);
      }
    }
  }
  band_margins<C, EXP ? 3 : C>(a, t);
}

// Separable filter kernel.  MODE picks how waves get their tasks:
//   kOneTask  one band of one tile column per wave (the hardware dispatcher
//             refills the CUs as workgroups retire);
//   kRuns     one task per wave, XCD-local runs of bands in alternating
//             directions (runs_task; PassLaunch::order = 1).
// Round 5's other task modes (tail bands, a persistent work queue, stacked
// bands per workgroup) and the per-wave timeline were measured slower and
// live in tools/sepx_modes.h with the study that measured them.  4-wave
// workgroups: one- and two-wave workgroups at the same waves per CU were
// 4-7 % slower (profiles/r5/cold/sepx_wg_*.txt).
// (skip border + expand epilogue, a rare combination: 2 VGPRs over the 128 of
// 4 waves/SIMD with the gray prologue -> 3 waves rather than a scratch spill)
enum KMode { kOneTask = 0, kRuns = 4 };
template <int C, class F, int PRO, bool SKIP, int SAUX, bool EXP = false, int MODE = kOneTask>
__global__ __launch_bounds__(kNT, (F::K >= 7 ? 2 : (SKIP && EXP ? 3 : 4))) void k_sep(KArgs a) {
  static_assert(MODE == kOneTask || MODE == kRuns, "k_sep task modes: kOneTask, kRuns");
  static_assert(MODE != kRuns || SepTraits<F>::SYM, "a bottom-up band needs symmetric vertical taps");
  __shared__ __attribute__((aligned(16))) uint4 xbuf[EXP ? kWaves : 1][EXP ? 3 * kW : 1];
  __shared__ uint8_t luts[768];
  if (PRO != PRO_NONE || a.has_epi) {
    load_luts<PRO>(a, luts);
    __syncthreads();
  }
  const WaveTask t = MODE == kRuns ? runs_task(a) : wave_task(a);
  if (t.valid) sep_task<C, F, PRO, SKIP, SAUX, EXP>(a, t, luts, xbuf[EXP ? t.wave : 0]);
}

// ------------------------------------------------------------------------------
// Gray sobel (|Gx| + |Gy|, saturated) on row pairs
// ------------------------------------------------------------------------------
// k_sep packs two horizontally adjacent pixels into a u16 pair, so every
// horizontal tap of a row needs a v_alignbit for the odd neighbour (~160 VALU
// a row).  Here a dword holds one pixel of two consecutive rows (y, y + 1):
// the vertical smoothing / difference of both output rows is one packed op,
// a pixel's horizontal neighbours are whole registers (the lane edges by DPP
// wave shifts), and a step emits two rows (~122 VALU a row).  Same task
// mapping, lane layout and stores as k_sep<1, Sobel, PRO_NONE>; bit-identical.
// Pixel j of a lane (byte j of its 16-byte chunk) of rows a, b as a u16 pair.
__device__ __forceinline__ uint32_t rows_pair(const u32x4& ra, const u32x4& rb, int j) {
  const uint32_t k = (uint32_t)(j & 3);
  return __builtin_amdgcn_perm(rb[j >> 2], ra[j >> 2], k | 0x0C00u | ((4u + k) << 16) | 0x0C000000u);
}

// Two output rows (y, y + 1) from rows y - 1 .. y + 2: r0 = row y, r1 = y + 1,
// r2 = y + 2; A[j] holds (r(y - 1), r(y)) on entry and (r(y + 1), r(y + 2))
// on return; o0 / o1 are the lane's 16 output bytes of rows y / y + 1.
// se / de: the vertical sum / difference pair of the pixel beyond the wave's
// edge (lane 0: the left neighbour, lane 63: the right one; 0 when the wave's
// outer lanes are halo lanes).
__device__ __forceinline__ void sobel_rp_step(const u32x4& r0, const u32x4& r1, const u32x4& r2, uint32_t (&A)[16],
                                              uint32_t (&o0)[4], uint32_t (&o1)[4], uint32_t se = 0,
                                              uint32_t de = 0) {
  uint32_t S[18], D[18];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t mid = rows_pair(r0, r1, j);  // (r(y), r(y + 1))
    const uint32_t b = rows_pair(r1, r2, j);    // (r(y + 1), r(y + 2))
    // vertical [1 2 1] of rows y, y + 1: halves <= 1020, no carry across
    S[j + 1] = A[j] + b + (mid << 1);
    D[j + 1] = as_u32(as_i16x2(b) - as_i16x2(A[j]));  // [-1 0 1]
    A[j] = b;
  }
  // neighbours across the lane edges: lane l - 1's last pixel, lane l + 1's
  // first (wave shifts; lanes 0 / 63 keep se / de)
  S[0] = (uint32_t)__builtin_amdgcn_update_dpp((int)se, (int)S[16], 0x138, 0xf, 0xf, false);
  D[0] = (uint32_t)__builtin_amdgcn_update_dpp((int)de, (int)D[16], 0x138, 0xf, 0xf, false);
  S[17] = (uint32_t)__builtin_amdgcn_update_dpp((int)se, (int)S[1], 0x130, 0xf, 0xf, false);
  D[17] = (uint32_t)__builtin_amdgcn_update_dpp((int)de, (int)D[1], 0x130, 0xf, 0xf, false);
  // horizontal [1 2 1] of D as two pair sums shared by neighbouring pixels
  i16x2 T[17];
#pragma unroll
  for (int j = 0; j < 17; ++j) T[j] = as_i16x2(D[j]) + as_i16x2(D[j + 1]);
  uint32_t mg[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const i16x2 gx = as_i16x2(S[j + 2]) - as_i16x2(S[j]);
    const i16x2 gy = T[j] + T[j + 1];
    const i16x2 mm = __builtin_elementwise_max(gx, -gx) + __builtin_elementwise_max(gy, -gy);
    mg[j] = as_u32(__builtin_elementwise_min(mm, (i16x2)(short)255));
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t p01 = __builtin_amdgcn_perm(mg[4 * q + 1], mg[4 * q], 0x06020400u);
    const uint32_t p23 = __builtin_amdgcn_perm(mg[4 * q + 3], mg[4 * q + 2], 0x06020400u);
    o0[q] = __builtin_amdgcn_perm(p23, p01, 0x05040100u);  // row y
    o1[q] = __builtin_amdgcn_perm(p23, p01, 0x07060302u);  // row y + 1
  }
}

// PB = 0: rows streamed two steps ahead (any band height).  PB > 0: the band
// is PB rows and all PB + 2 input rows are requested up front, so a wave
// waits for one memory round trip, not one per step (a short-lived wave's
// life is mostly those waits: profiles/r5/cfg3/README.md).
// WIDE: 1 KiB tiles, every lane an output lane; the two pixels beyond the
// tile come from one extra dword load per row (lanes 0-31 the left
// neighbour's dword, 32-63 the right one's) and enter the wave shifts as their
// `old` value.  8192-wide gray rows are then 8 tiles instead of 9 (the ninth
// 26 % used): 4096 waves at 4-row bands, 4 per SIMD instead of 4-5.
template <int SAUX, int PB = 0, bool WIDE = false>
__global__ __launch_bounds__(kNT, 4) void k_sobel_rp(KArgs a) {
  const WaveTask t = wave_task(a);
  if (!t.valid) return;
  const int lane = t.lane;
  const int ys = t.ys, ye = t.ye;
  constexpr int kTile = WIDE ? kW * 16 : kOutChunks * 16;  // output bytes per wave row
  const int cb0 = tile_base<1>(a, t.xt, kTile) - (WIDE ? 0 : 16);
  const int cb = cb0 + lane * 16;
  const uint32_t lane_in = cb < a.E + 16 ? (uint32_t)cb : kOOB;
  OutLanes lout;
  if constexpr (WIDE) {
    lout.off[0] = cb < a.E ? (uint32_t)cb : kOOB;
    lout.off[1] = lout.off[2] = kOOB;
  } else {
    lout = out_lanes<false>(a, lane, cb0);
  }
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in_base, a.in_bytes);
  const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.out_base, a.out_bytes);
  // rows past the band's lower halo row (ye) re-read it: they feed unstored outputs
  auto load = [&](int y) __attribute__((always_inline)) {
    return __builtin_amdgcn_raw_buffer_load_b128(rin, in_row_off(a, min(y, ye)) + lane_in, 0, kLoadAux);
  };
  // the edge pixels' dwords (WIDE): byte 3 of the dword before the tile for
  // lanes < 32, byte 0 of the one after it for lanes >= 32 (x-margins hold the
  // border pixels; past the row's right margin nothing is needed)
  const int eo = lane < 32 ? cb0 - 4 : cb0 + kTile;
  const uint32_t e_in = eo < a.E + 16 ? (uint32_t)eo : kOOB;
  const uint32_t ek = lane < 32 ? 3u : 0u;
  const uint32_t esel = ek | 0x0C00u | ((4u + ek) << 16) | 0x0C000000u;  // (byte of row a, byte of row b) as u16s
  auto load_e = [&](int y) __attribute__((always_inline)) {
    return WIDE ? __builtin_amdgcn_raw_buffer_load_b32(rin, in_row_off(a, min(y, ye)) + e_in, 0, kLoadAux) : 0u;
  };
  uint32_t Ae = 0;  // edge pair (r(y - 1), r(y))
  auto edge = [&](uint32_t e0, uint32_t e1, uint32_t e2, uint32_t& se, uint32_t& de) __attribute__((always_inline)) {
    if constexpr (WIDE) {
      const uint32_t me = __builtin_amdgcn_perm(e1, e0, esel);
      const uint32_t be = __builtin_amdgcn_perm(e2, e1, esel);
      se = Ae + be + (me << 1);
      de = as_u32(as_i16x2(be) - as_i16x2(Ae));
      Ae = be;
    } else {
      se = de = 0;
    }
  };
  auto store2 = [&](int y, const uint32_t (&o0)[4], const uint32_t (&o1)[4]) __attribute__((always_inline)) {
    store_out<false, SAUX>(o0, rout, y < ye, a.out_org + (uint32_t)((int64_t)y * a.out_pitch), lout, nullptr, lane);
    store_out<false, SAUX>(o1, rout, y + 1 < ye, a.out_org + (uint32_t)((int64_t)(y + 1) * a.out_pitch), lout,
                           nullptr, lane);
  };
  // A[j] = (r(y - 1), r(y)) of the current step y (the previous step's B)
  uint32_t A[16];
  if constexpr (PB > 0) {
    u32x4 R[PB + 2];     // rows ys - 1 .. ys + PB
    uint32_t Ee[PB + 2];  // their edge dwords
#pragma unroll
    for (int k = 0; k < PB + 2; ++k) {
      R[k] = load(ys - 1 + k);
      Ee[k] = load_e(ys - 1 + k);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) A[j] = rows_pair(R[0], R[1], j);
    if constexpr (WIDE) Ae = __builtin_amdgcn_perm(Ee[1], Ee[0], esel);
#pragma unroll
    for (int st = 0; st < PB / 2; ++st) {
      uint32_t o0[4], o1[4], se, de;
      edge(Ee[2 * st + 1], Ee[2 * st + 2], Ee[2 * st + 3], se, de);
      sobel_rp_step(R[2 * st + 1], R[2 * st + 2], R[2 * st + 3], A, o0, o1, se, de);
      store2(ys + 2 * st, o0, o1);
    }
  } else {
    u32x4 r0;  // row y
    uint32_t e0;
    {
      const u32x4 rm = load(ys - 1);
      r0 = load(ys);
      const uint32_t em = load_e(ys - 1);
      e0 = load_e(ys);
#pragma unroll
      for (int j = 0; j < 16; ++j) A[j] = rows_pair(rm, r0, j);
      if constexpr (WIDE) Ae = __builtin_amdgcn_perm(e0, em, esel);
    }
    // rows y + 1, y + 2 of this step and of the next one in flight
    u32x4 nx[2][2];
    uint32_t ne[2][2];
    nx[0][0] = load(ys + 1);
    nx[0][1] = load(ys + 2);
    nx[1][0] = load(ys + 3);
    nx[1][1] = load(ys + 4);
    ne[0][0] = load_e(ys + 1);
    ne[0][1] = load_e(ys + 2);
    ne[1][0] = load_e(ys + 3);
    ne[1][1] = load_e(ys + 4);
    auto step = [&](int y, u32x4 (&cur)[2], uint32_t (&ce)[2]) __attribute__((always_inline)) {
      const u32x4 r1 = cur[0], r2 = cur[1];
      const uint32_t e1 = ce[0], e2 = ce[1];
      cur[0] = load(y + 5);  // the step after next
      cur[1] = load(y + 6);
      ce[0] = load_e(y + 5);
      ce[1] = load_e(y + 6);
      uint32_t o0[4], o1[4], se, de;
      edge(e0, e1, e2, se, de);
      sobel_rp_step(r0, r1, r2, A, o0, o1, se, de);
      store2(y, o0, o1);
      r0 = r2;
      e0 = e2;
    };
    for (int y = ys; y < ye; y += 4) {
      step(y, nx[0], ne[0]);
      step(y + 2, nx[1], ne[1]);
    }
  }
  band_margins<1, 1>(a, t);
}

// ------------------------------------------------------------------------------
// Direct (non-separable) filters: emboss3/5, sharpen, laplace
// ------------------------------------------------------------------------------
// The last K input rows live in registers, unpacked to u16 pairs and extended
// by the neighbour lanes' edge dwords (DPP wave shifts: no LDS, no wave sync);
// every tap is one packed i16 multiply-add per two outputs (|sum| <= 17*255).
// The y loop is unrolled K times so the register ring is indexed statically,
// and the K raw rows of the next round are in flight meanwhile.
template <int NX>
__device__ __forceinline__ void extend_row(const uint32_t (&u)[8], uint32_t (&e)[8 + 2 * NX]) {
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    // lane l gets lane l-1's dword (wave_shr:1) / lane l+1's (wave_shl:1); the
    // halo lanes 0 and 63 receive zeros and their outputs are never stored
    e[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u[8 - NX + i], 0x138, 0xf, 0xf, false);
    e[NX + 8 + i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u[i], 0x130, 0xf, 0xf, false);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) e[NX + i] = u[i];
}

template <int C, class F, int PRO, bool SKIP, int SAUX, bool EXP = false>
__global__ __launch_bounds__(kNT, (F::K >= 5 ? 3 : 4)) void k_direct(KArgs a) {
  static_assert(!EXP || C == 1, "expand epilogue needs a 1-channel stencil");
  constexpr int R = F::R, K = F::K;
  constexpr int NX = (R * C + 1) / 2;  // neighbour dwords per side
  constexpr int NE = 8 + 2 * NX;       // extended row dwords
  constexpr int CIN = is_gray(PRO) ? 3 : 1;
  __shared__ uint8_t luts[768];
  if (PRO != PRO_NONE || a.has_epi) {
    load_luts<PRO>(a, luts);
    __syncthreads();
  }
  const WaveTask t = wave_task(a);
  if (!t.valid) return;
  const int lane = t.lane;
  const int ys = t.ys, ye = t.ye;
  const int cb = tile_base<C>(a, t.xt, kOutChunks * 16) - 16 + lane * 16;
  const uint32_t lane_in = cb < a.E + 16 ? (uint32_t)(cb * CIN) : kOOB;
  const OutLanes lout = out_lanes<EXP>(a, lane, cb - 16 * lane);
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in_base, a.in_bytes);
  const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.out_base, a.out_bytes);
  const uint32_t last_row = in_row_off(a, ye - 1 + R);
  __shared__ __attribute__((aligned(16))) uint4 xbuf[EXP ? kWaves : 1][EXP ? 3 * kW : 1];
  uint4* xb = xbuf[EXP ? t.wave : 0];

  uint32_t keep[SKIP ? 4 : 1];
  if constexpr (SKIP) skip_cols<C>(a, cb, R, keep);
  uint32_t ring[K][NE];  // slot of input row r: (r - (ys - R)) mod K
  auto push = [&](const RawChunk<PRO>& raw, uint32_t (&slot)[NE]) __attribute__((always_inline)) {
    uint32_t u[8];
    cook_pairs<PRO>(a, raw, luts, u);
    extend_row<NX>(u, slot);
  };
#pragma unroll
  for (int i = 0; i < K - 1; ++i) {  // rows ys-R .. ys+R-1
    RawChunk<PRO> r;
    load_raw<PRO>(rin, in_row_off(a, ys - R + i), lane_in, r);
    push(r, ring[i]);
  }
  RawChunk<PRO> nx[K];  // row y + o + R for the step o of the current round
#pragma unroll
  for (int o = 0; o < K; ++o) load_raw<PRO>(rin, ys + o < ye ? in_row_off(a, ys + o + R) : last_row, lane_in, nx[o]);

  const bool inner = rows_inside(a, ys - R, ye - 1 + R);
  for (int y = ys; y < ye; y += K) {
#pragma unroll
    for (int o = 0; o < K; ++o) {
      const int yy = y + o;
      push(nx[o], ring[(o + K - 1) % K]);
      load_raw<PRO>(rin, ahead_row_off(a, inner, yy, K, ye, R, last_row), lane_in, nx[o]);
      uint32_t h[8];
#pragma unroll
      for (int pp = 0; pp < 8; ++pp) {
        i16x2 acc = {0, 0};
#pragma unroll
        for (int dy = 0; dy < K; ++dy)
#pragma unroll
          for (int dx = 0; dx < K; ++dx) {
            constexpr int unused = 0;
            (void)unused;
            const int w = F::w(dy, dx);
            if (w == 0) continue;
            const i16x2 v = as_i16x2(pair_at(ring[(o + dy) % K], 2 * NX + 2 * pp + (dx - R) * C));
            if (w == 1) acc += v;
            else if (w == -1) acc -= v;
            else acc += v * (short)w;
          }
        acc = __builtin_elementwise_max(acc, (i16x2)(short)0);
        h[pp] = as_u32(__builtin_elementwise_min(acc, (i16x2)(short)255));
      }
      uint32_t o4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) o4[q] = __builtin_amdgcn_perm(h[2 * q + 1], h[2 * q], 0x06040200u);
      if constexpr (SKIP) {
        uint32_t center[4];
        const uint32_t(&cr)[NE] = ring[(o + R) % K];
#pragma unroll
        for (int q = 0; q < 4; ++q) center[q] = __builtin_amdgcn_perm(cr[NX + 2 * q + 1], cr[NX + 2 * q], 0x06040200u);
        apply_skip(a, a.row0 + yy, R, keep, center, o4);
      }
      if (a.has_epi) lut16(luts + 512, o4);
      store_out<EXP, SAUX>(o4, rout, yy < ye, a.out_org + (uint32_t)((int64_t)yy * a.out_pitch), lout, xb, lane);
    }
  }
  band_margins<C, EXP ? 3 : C>(a, t);
}

// ------------------------------------------------------------------------------
// dispatch
// ------------------------------------------------------------------------------
// Resident workgroups per device for a kernel (occupancy x CUs), cached.
inline int resident_slots(const void* fn) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> cache;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({fn, dev});
  if (it != cache.end()) return it->second;
  int per_cu = 0, cus = 0;
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kNT, 0));
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int slots = std::max(1, per_cu) * std::max(1, cus);
  cache[{fn, dev}] = slots;
  return slots;
}

// Launch geometry: band height a multiple of 4 (rows are stepped in groups of 4).
// Default band height: short bands keep the rows all resident workgroups touch
// at once in a compact window (measured on MI355X, 16384-wide RGB: gaussian5
// 0.323 ms/pass at 12 rows vs 0.370 ms with one tall band per workgroup, which
// spreads the concurrent streams over the whole frame); the engine's autotuner
// can override per shape.
// XCD-aware workgroup remap (xcd_remap): the caller sets a.nxcd (launch_stencil:
// on for passes whose working set stays in the Infinity Cache, where halo rows
// shared by vertically adjacent bands become L2 hits); STRIPE_XCD=<n> forces it
// (0 = off) for A/B runs.
inline int env_nxcd() {
  static const int v = [] {
    const char* e = std::getenv("STRIPE_XCD");
    return e ? std::atoi(e) : -1;
  }();
  return v;
}

inline void plan_bands(KArgs& a, dim3& grid, int tiles, int n0, int n1, int band, int R, int slots) {
  (void)slots;
  if (env_nxcd() >= 0) a.nxcd = env_nxcd();
  if (band <= 0) band = R >= 3 ? 16 : 12;
  band = (int)align_up(band, 4);
  a.band = band;
  a.nb0 = (int)div_up(n0, band);
  a.nbands = a.nb0 + (int)div_up(n1, band);
  a.ntx = tiles;
  grid = dim3((unsigned)div_up((int64_t)tiles * a.nbands, kWaves));
}

// Occupancy cap of the HBM-streaming (nt-store) stencil launches: fewer
// resident waves per SIMD keep fewer concurrent row streams open against HBM
// (16384^2 RGB, band autotune on, profiles/r2d/nt_wgs_ab.txt: separable
// gaussian5 0.311 -> 0.282 ms at 2 workgroups per CU, gaussian3 0.299 -> 0.269,
// sobel 0.315 -> 0.293; direct emboss3 0.300 -> 0.283 at 3; the gray-prologue
// direct kernels read 3 bytes per output byte and gain nothing).  The cap is an
// LDS reservation (dynamic shared memory the kernel never touches) sized so
// only `target` workgroups fit a CU's LDS; STRIPE_NT_WGS overrides the cap of
// HBM-streaming launches (stencil_cap; 0 = no cap).
inline int env_nt_wgs() {
  static const int env = [] {
    const char* e = std::getenv("STRIPE_NT_WGS");
    return e ? std::atoi(e) : -1;
  }();
  return env;
}

inline size_t nt_lds_reserve(const void* fn, int target) {
  if (target <= 0) return 0;
  static std::mutex mu;
  static std::map<std::tuple<const void*, int, int>, size_t> cache;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({fn, dev, target});
  if (it != cache.end()) return it->second;
  int lds_cu = 0;
  HIP_CHECK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev));
  hipFuncAttributes fa{};
  HIP_CHECK(hipFuncGetAttributes(&fa, fn));
  const size_t total = (size_t)lds_cu / (size_t)(target + 1) + 1024;  // target fit, target + 1 do not
  const size_t dyn = total > fa.sharedSizeBytes ? total - fa.sharedSizeBytes : 0;
  cache[{fn, dev, target}] = dyn;
  return dyn;
}

// Occupancy cap of one launch: wgs >= 0 is the engine's choice (its autotuner
// times the caps per pass and box, since the best cap depends on the clock
// and memory behaviour of the box: round-2 driver run);
// wgs < 0 takes the family default, applied to HBM-streaming launches only.
inline int stencil_cap(bool nt, int wgs, int family_default) {
  if (nt && env_nt_wgs() >= 0) return env_nt_wgs();  // A/B runs pin the streaming cap only
  if (wgs >= 0) return wgs;
  return nt ? family_default : 0;
}

template <int C, class F, int PRO, bool EXP = false>
void launch_one(bool skip, bool nt, int wgs, KArgs a, int tiles, int n0, int n1, int band, hipStream_t s,
                int order = 0) {
  using K = void (*)(KArgs);
  dim3 grid;
  if constexpr (F::SEP && PRO == PRO_NONE && !EXP) {
    if constexpr (SepTraits<F>::SYM) {
      if (order == 1) {  // kRuns (runs_task); the remap is its own
        const K fns[4] = {k_sep<C, F, PRO, false, 0, EXP, kRuns>, k_sep<C, F, PRO, false, kNtAux, EXP, kRuns>,
                          k_sep<C, F, PRO, true, 0, EXP, kRuns>, k_sep<C, F, PRO, true, kNtAux, EXP, kRuns>};
        const K fn = fns[2 * skip + nt];
        plan_bands(a, grid, tiles, n0, n1, band, F::R, 0);
        grid = dim3((unsigned)runs_grid(tiles, a.nbands));
        fn<<<grid, kNT, nt_lds_reserve((const void*)fn, stencil_cap(nt, wgs, kNtWgsSep)), s>>>(a);
        return;
      }
    }
  }
  if constexpr (F::SEP && F::SOBEL && C == 1 && PRO == PRO_NONE && !EXP) {
    if constexpr (!F::L2) {
      // gray L1 sobel on row pairs (STRIPE_SOBEL_RP=0: the k_sep form, A/B)
      static const bool rp = [] {
        const char* e = std::getenv("STRIPE_SOBEL_RP");
        return !(e && std::atoi(e) == 0);
      }();
      // 8-row bands request all ten input rows up front (the autotuner's
      // band-8 candidate; full 8192^2 frame 2-3.5 % faster than the best
      // streamed band, profiles/r5/cfg3/README.md); STRIPE_SOBEL_PB=8|12
      // forces bands of that height with up-front loads (A/B)
      static const int pb_env = [] {
        const char* e = std::getenv("STRIPE_SOBEL_PB");
        const int v = e ? std::atoi(e) : -1;
        return v == 0 || v == 8 || v == 12 ? v : -1;
      }();
      // 1 KiB tiles with edge loads (STRIPE_SOBEL_WIDE=0: 62-lane tiles, A/B)
      static const bool wide = [] {
        const char* e = std::getenv("STRIPE_SOBEL_WIDE");
        return !(e && std::atoi(e) == 0);
      }();
      if (rp && !skip) {
        const int pb = pb_env >= 0 ? pb_env : (band == 8 ? 8 : 0);
        const K fns[2][3][2] = {{{k_sobel_rp<0>, k_sobel_rp<kNtAux>},
                                 {k_sobel_rp<0, 8>, k_sobel_rp<kNtAux, 8>},
                                 {k_sobel_rp<0, 12>, k_sobel_rp<kNtAux, 12>}},
                                {{k_sobel_rp<0, 0, true>, k_sobel_rp<kNtAux, 0, true>},
                                 {k_sobel_rp<0, 8, true>, k_sobel_rp<kNtAux, 8, true>},
                                 {k_sobel_rp<0, 12, true>, k_sobel_rp<kNtAux, 12, true>}}};
        const K fn = fns[wide][pb == 8 ? 1 : pb == 12 ? 2 : 0][nt];
        if (pb) band = pb;
        if (wide) tiles = (int)div_up((int64_t)a.E, kW * 16);
        plan_bands(a, grid, tiles, n0, n1, band, F::R, 0);
        fn<<<grid, kNT, nt_lds_reserve((const void*)fn, stencil_cap(nt, wgs, kNtWgsSep)), s>>>(a);
        return;
      }
    }
  }
  if constexpr (F::SEP) {
    const K fns[4] = {k_sep<C, F, PRO, false, 0, EXP>, k_sep<C, F, PRO, false, kNtAux, EXP>,
                      k_sep<C, F, PRO, true, 0, EXP>, k_sep<C, F, PRO, true, kNtAux, EXP>};
    const K fn = fns[2 * skip + nt];
    plan_bands(a, grid, tiles, n0, n1, band, F::R, resident_slots((const void*)fn));
    fn<<<grid, kNT, nt_lds_reserve((const void*)fn, stencil_cap(nt, wgs, kNtWgsSep)), s>>>(a);
  } else {
    const K fns[4] = {k_direct<C, F, PRO, false, 0, EXP>, k_direct<C, F, PRO, false, kNtAux, EXP>,
                      k_direct<C, F, PRO, true, 0, EXP>, k_direct<C, F, PRO, true, kNtAux, EXP>};
    const K fn = fns[2 * skip + nt];
    plan_bands(a, grid, tiles, n0, n1, band, F::R, resident_slots((const void*)fn));
    fn<<<grid, kNT, nt_lds_reserve((const void*)fn, stencil_cap(nt, wgs, is_gray(PRO) ? 0 : kNtWgsDirect)), s>>>(a);
  }
}

template <int PRO, class F>
void launch_gray_out(bool expand, bool skip, bool nt, int wgs, const KArgs& a, int tiles, int n0, int n1, int band,
                     hipStream_t s) {
  if (expand) launch_one<1, F, PRO, true>(skip, nt, wgs, a, tiles, n0, n1, band, s);
  else launch_one<1, F, PRO, false>(skip, nt, wgs, a, tiles, n0, n1, band, s);
}

template <class F>
void launch_filter(const Pass& p, const KArgs& a, int tiles, int n0, int n1, int band, bool nt, int wgs,
                   hipStream_t s, int order) {
  const bool gray = p.pro.gray;
  const bool lut = p.pro.has_post;
  const bool skip = p.border == Border::Skip;
  const bool ex = p.epi_expand;
  if (p.cmid == 3) {
    STRIPE_CHECK(!gray && !ex, "gray prologue / expand epilogue need a 1-channel stencil");
    if (lut) launch_one<3, F, PRO_LUT>(skip, nt, wgs, a, tiles, n0, n1, band, s);
    else launch_one<3, F, PRO_NONE>(skip, nt, wgs, a, tiles, n0, n1, band, s, order);
  } else {
    if (gray && a.gmode == 1) launch_gray_out<PRO_GRAYLUT, F>(ex, skip, nt, wgs, a, tiles, n0, n1, band, s);
    else if (gray) launch_gray_out<PRO_GRAY, F>(ex, skip, nt, wgs, a, tiles, n0, n1, band, s);
    else if (lut) launch_gray_out<PRO_LUT, F>(ex, skip, nt, wgs, a, tiles, n0, n1, band, s);
    else if (!ex) launch_one<1, F, PRO_NONE>(skip, nt, wgs, a, tiles, n0, n1, band, s, order);
    else launch_gray_out<PRO_NONE, F>(ex, skip, nt, wgs, a, tiles, n0, n1, band, s);
  }
}


// Every filter F has launch_filter<F> compiled in exactly one stencil_inst_*.hip.
#define STRIPE_LAUNCH_FILTER_SIG(F) \
  void launch_filter<sdef::F>(const Pass&, const KArgs&, int, int, int, int, bool, int, hipStream_t, int)
#define STRIPE_EXTERN_LAUNCH_FILTER(F) extern template STRIPE_LAUNCH_FILTER_SIG(F);
#define STRIPE_INSTANTIATE_LAUNCH_FILTER(F) template STRIPE_LAUNCH_FILTER_SIG(F);
#define STRIPE_STENCIL_FILTERS(X) \
  X(Emboss3) X(Emboss5) X(Sharpen) X(Laplace) X(Sobel) X(SobelL2) X(Gaussian3) X(Gaussian5) X(Gaussian7) X(Box3) \
  X(Box5)

}  // namespace dev
}  // namespace stripe
