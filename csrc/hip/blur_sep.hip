// Separable large-kernel blur on MFMA (blur:K, K <= 33; SURVEY config 5).
//
// The Gaussian K x K window is rank one, so one output costs two K-tap 1-D
// passes, both run as GEMMs on the matrix cores with the intermediate kept in
// registers (no LDS round trip, no second kernel):
//
//   horizontal  X[16 rows][16 px] = In[16 rows][64-px window] . Th[64][16]
//               per channel: Th is the banded Toeplitz matrix of the 1-D
//               weights; A = the channel's input pixels, staged in LDS as
//               exact f16 planes (RGB de-interleaved while staging).
//   vertical    Out^T[16 px][16 rows] = X^T[16][64 rows] . Tv^T[64][16]
//               X comes straight from the horizontal MFMA's accumulator layout
//               (column on the lane, rows in registers = the A operand of a
//               product that sums over X's rows), and the transposed product
//               leaves each lane with 4 consecutive output pixels of one row
//               (RGB: 12 interleaved bytes, one dwordx3 store).
//
// Precision: u8 inputs are exact in f16 (as subnormals, below); weights and X are split into f16
// hi + lo parts (2 MFMAs for the horizontal pass, 3 for the vertical), so the
// f32 result is within ~1e-5 of the f64 golden (conv
// passes match within 1 LSB, ties only).  The ":lsb" mode (LSB below) takes
// one f16 part of each on the centred input: every output within 1 LSB.
//
// Work: a wave owns a strip of NX 16-pixel tiles x one band of rows (a
// multiple of 32); the NW waves of a workgroup own NW adjacent strips and
// stage their common window cooperatively (NW = 1: every wave its own tile,
// no workgroup barrier).  32 output rows need 64 rows of X; each 32-row X
// pair is consumed as soon as it is made: it finishes the previous output
// group (k-step 1) and starts the next one (k-step 0), so only the running
// f32 sums stay in registers.
//
// Reference parity: the reference has no large-kernel blur (its only float
// work is kernel.cu:39-47's contrast); this is the MFMA showcase of the
// framework, SURVEY §2 "large-kernel conv".
#include "dev_common.h"
#include "stripe/kernels.h"
#include "stripe/trace.h"

#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <vector>

namespace stripe {
namespace dev {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

constexpr int kSepWaves = 4;
constexpr int kSepEntries = 12;          // weight fragments per lane: Bh[2][2], Bv[2][2][2]

struct SepArgs {
  KArgs a;
  const u4* tw;  // [entry][lane] weight fragments (8 halves each)
  int R, L, nstrips;
  int a0, a2;  // group-grid origins of ranges 0 / 1 (global row multiple of 32)
  float bias;  // LSB mode: 128 * sum(h) * sum(v), the x - 128 shift of the input
  float hinit;  // LSB: horizontal accumulator start, -128 * sum(scaled h) * 2^-24 (the centring)
};

__device__ __forceinline__ void sep_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// (x, y) -> f16 hi parts and f16 lo parts of the remainders: x ~ hi + lo to ~2^-21.
// hi keeps the top 11 significant bits (mantissa masked, exact in f16), so the
// remainder needs no f16 round trip.
__device__ __forceinline__ void split_h2(float x, float y, uint32_t& hi, uint32_t& lo) {
  const float hx = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, x) & 0xFFFFE000u);
  const float hy = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, y) & 0xFFFFE000u);
  const half2v h = {(_Float16)hx, (_Float16)hy};
  const half2v l = {(_Float16)(x - hx), (_Float16)(y - hy)};
  hi = __builtin_bit_cast(uint32_t, h);
  lo = __builtin_bit_cast(uint32_t, l);
}

// 4 f32 -> 4 saturated, round-half-even u8 in one dword: v_cvt_pk_u8_f32
// rounds in the MODE rounding mode (nearest-even by default) and saturates to
// [0, 255] itself (tools/cvt_probe.hip on gfx950: -5 -> 0, 2.5 -> 2, 256 -> 255,
// 1e9 -> 255), so no clamp instruction is needed.
__device__ __forceinline__ uint32_t pack_u8x4(f4 v) {
  uint32_t o = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) o = __builtin_amdgcn_cvt_pk_u8_f32(v[r], r, o);
  return o;
}

// Subnormal staging: byte b becomes the f16 bit pattern 0x00bb, the exact
// subnormal b * 2^-24 (the MFMA keeps f16 subnormal inputs), so a pair of
// bytes is ONE v_perm (zero high bytes from selector 0x0C).  The horizontal
// weights are stored scaled by 2^(24 - e) and the vertical ones by 2^e
// (prepare_sep_consts), so X and the output keep their units; the LSB mode's
// x - 128 centring is the horizontal accumulator's start value.  (Round 6:
// replaced (1024 + b) f16 built by a perm and a packed subtract per pair --
// 2.5x the staging VALU; 1-3 % faster on every shape, profiles/r6/subn/.)
// RGB: d0 d1 d2 = R0 G0 B0 R1 | G1 B1 R2 G2 | B2 R3 G3 B3.
__device__ __forceinline__ uint32_t sub_pair(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// 2 f32 -> 2 f16, round to nearest even (the LSB mode's single-part X).
__device__ __forceinline__ uint32_t f32x2_to_h2(float x, float y) {
  const half2v h = {(_Float16)x, (_Float16)y};
  return __builtin_bit_cast(uint32_t, h);
}

// Planar kernel.  A wave owns a strip of NX x-tiles of 16 pixels (all C
// channels) and a band of rows.  Each 32-row X pair is staged into LDS as C
// f16 channel PLANES (RGB is de-interleaved while staging: 6 byte->subnormal
// f16 perms per 4 pixels), so the horizontal Toeplitz product of
// one channel needs a 64-pixel window per 16 outputs: 2 k-steps instead of the
// 4 k-steps a 128-byte interleaved window takes (RGB: 8 horizontal MFMAs per
// 16 output bytes instead of 16, 20 in all instead of 28).  The vertical
// product is unchanged; for RGB a lane ends with 4 consecutive pixels of one
// output row in each channel accumulator, i.e. 12 contiguous interleaved
// bytes: one dwordx3 store.
//
// NW > 1: the NW waves of a workgroup take NW adjacent strips of one band and
// stage their common window once, cooperatively, into a double-buffered tile
// (one LDS barrier per pair): NW strips of PX pixels read NW PX + 48 staged
// pixels per row instead of NW (PX + 48) -- RGB at 2 tiles: 176 instead of 320.
// workgroup size: kSepWaves independent waves, or the NW waves sharing a window
constexpr int blur_threads(int nw) { return 64 * (nw == 1 ? kSepWaves : nw); }

template <int C, int NX_, int NW_ = 1>
struct PlGeom {
  static constexpr int NX = NX_;                     // 16-pixel x-tiles per strip
  static constexpr int NW = NW_;                     // waves (strips) sharing one staged window
  static constexpr int PX = 16 * NX;                 // output pixels per strip
  static constexpr int WPX = NW * PX + 48;           // staged pixels per row: [sx0 - 16, sx0 + NW PX + 32)
  static constexpr int UB = C == 3 ? 12 : 16;        // bytes per staging load (4 RGB / 16 gray pixels)
  static constexpr int UPX = UB / C;                 // pixels per staging load
  static constexpr int U = WPX / UPX;                // loads per staged row
  static constexpr int LANES = 64 * NW;              // lanes staging one window
  static constexpr int LPL = (32 * U + LANES - 1) / LANES;  // loads per lane per 32-row pair
  // plane row bytes: 16 q with q = 2 mod 4.  ds_read_b128 serves a wave in
  // the lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32), and the
  // fragment of lane (m, g) starts at quad q m + g: with q = 2 mod 4 every
  // group hits 16 distinct 4-bank quads (an odd q leaves 3 quads doubled:
  // 44 % of the LDS cycles were bank conflicts with q = 11)
  static constexpr int STRIDE = 16 * ((2 * WPX + 15) / 16 + (((2 - (2 * WPX + 15) / 16) % 4) + 4) % 4);
  static constexpr int PLANE = 32 * STRIDE;
  static constexpr int TILE = C * PLANE;             // LDS bytes of one staged window
  // dynamic LDS per workgroup: one window per wave, or NW = all waves sharing
  // a double-buffered window
  static constexpr int LDS = NW == 1 ? kSepWaves * TILE : 2 * TILE;
  static constexpr int THREADS = blur_threads(NW);  // workgroup size
  static_assert(NW == 1 || NW == 4 || NW == 8, "a shared window spans the whole workgroup");
  static_assert(WPX % UPX == 0, "staged row must be whole loads");
  static_assert(STRIDE % 64 == 32 && STRIDE >= 2 * WPX, "plane stride");
};

// EDGE: the row width is not a multiple of 4 pixels (the last group of a row
// is partial: byte stores); otherwise every group is whole or past the row.
// NX x-tiles per strip, PFD 32-row pairs prefetched ahead, OCC waves per SIMD.
// LSB: the "blur:K:lsb" precision mode -- input centred (x - 128, exact in
// f16), single f16 weights and a single f16 X, the shift added back as the
// accumulators' start value: 8 MFMAs per tile instead of 20, every output
// within 1 LSB of the f64 result (the host bounds the error per weight set and
// keeps the exact kernel when it cannot promise that).
// (launch bounds: OCC waves per SIMD = OCC * 256 / THREADS workgroups per CU)
// (Round 6 measured wave priorities -- the static form for the younger half
// of the 8-wave workgroup, priority over each step's MFMAs -- and stores of
// whole 96-byte row pieces as A/B instances: null or slower, removed;
// profiles/r6/sched/, profiles/r6/blurpst/.)
template <int C, bool EDGE, int NX_, int PFD, int OCC, bool LSB = false, int NW = 1, bool EARLY = true>
__global__ __launch_bounds__(blur_threads(NW), OCC * 256 / blur_threads(NW)) void k_blur_pl(SepArgs sa) {
  using G = PlGeom<C, NX_, NW>;
  constexpr int NX = G::NX;
  const KArgs& a = sa.a;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int sl = NW == 1 ? lane : (int)threadIdx.x;  // staging lane
  int strip, by, sgx;  // strip of this wave, band, first strip of the staged window
  if constexpr (NW == 1) {
    const int task = xcd_remap((int)blockIdx.x, (int)gridDim.x, a.nxcd) * kSepWaves + wave;
    if (task >= sa.nstrips * a.nbands) return;  // wave-uniform
    strip = task % sa.nstrips;
    by = task / sa.nstrips;
    sgx = strip;
  } else {
    const int nsg = (sa.nstrips + NW - 1) / NW;  // strip groups
    const int gt = xcd_remap((int)blockIdx.x, (int)gridDim.x, a.nxcd);
    if (gt >= nsg * a.nbands) return;  // workgroup-uniform: every wave meets every barrier
    by = gt / nsg;
    sgx = (gt % nsg) * NW;
    strip = sgx + wave;  // past the row (last group): computed, never stored
  }
  uint8_t* wl = lds + (NW == 1 ? wave * G::TILE : 0);
  // bands and 32-row groups sit on a grid of global rows (multiples of 32):
  // every output row is summed in the same order whatever the launch's row
  // ranges, so results are independent of the partition, bit for bit
  int base, ys, ye;
  if (by < a.nb0) {
    base = sa.a0 + by * a.band;
    ys = max(base, a.ry0);
    ye = min(base + a.band, a.ry1);
  } else {
    base = sa.a2 + (by - a.nb0) * a.band;
    ys = max(base, a.ry2);
    ye = min(base + a.band, a.ry3);
  }
  const int R = sa.R;

  // ---- weights: Bh[s][hl] (horizontal, 2 k-steps), Bv[q][s][hl] (vertical) ----
  constexpr int NHL = LSB ? 1 : 2;  // weight parts (hi, lo)
  half8 bh[2][NHL], bv[2][2][NHL];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int hl = 0; hl < NHL; ++hl) bh[s][hl] = __builtin_bit_cast(half8, sa.tw[(s * 2 + hl) * 64 + lane]);
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int hl = 0; hl < NHL; ++hl)
        bv[q][s][hl] = __builtin_bit_cast(half8, sa.tw[(4 + q * 4 + s * 2 + hl) * 64 + lane]);

  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in_base, a.in_bytes);
  const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.out_base, a.out_bytes);
  const int lo_ok = max(-R, -a.row0);  // rows addressable without remapping
  const int hi_ok = min(a.rows - 1 + R, a.Hg - 1 - a.row0);
  const int sx = strip * G::PX;   // first output pixel of the strip
  const int wx = sgx * G::PX - 16;  // first staged pixel of the window
  const int m = lane & 15, g = lane >> 4;

  // staging map: load i of a staging lane is unit u = sl + LANES i -> pair
  // row u / U, pixels UPX * (u % U) .. of the staged window.  The (row, unit)
  // pattern repeats every P loads (LANES P = a multiple of U), so only P
  // (row, column) pairs live in registers.
  constexpr int P = [] {
    for (int p = 1; p < G::LPL; ++p)
      if (G::LANES * p % G::U == 0) return p;
    return G::LPL;
  }();
  constexpr int RSTEP = G::LANES * P / G::U;  // pair rows advanced every P loads
  static_assert(P == G::LPL || G::LANES * P % G::U == 0, "staging period");
  int srow[P];
  int scol[P];  // first staged pixel of the unit, relative to the window start
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int u = sl + G::LANES * i;
    srow[i] = u / G::U;
    scol[i] = G::UPX * (u % G::U);
  }
  auto unit_ok = [&](int i) __attribute__((always_inline)) { return srow[i % P] + RSTEP * (i / P) < 32; };
  typedef uint32_t u3 __attribute__((ext_vector_type(3)));
  typedef std::conditional_t<C == 3, u3, u4> unit_t;
  unit_t pf[PFD][G::LPL];
  const int yh0 = base - 16;               // input row of X row 0
  const int ngroups = (ye - base + 31) >> 5;
  // lane part of an interior load's offset: row srow * pitch + window bytes
  uint32_t loff[P];
#pragma unroll
  for (int i = 0; i < P; ++i) loff[i] = (uint32_t)(srow[i] * a.in_pitch + (wx + scol[i]) * C);
  auto load = [&](int i, uint32_t off, auto buf_c) __attribute__((always_inline)) {
    constexpr int B = decltype(buf_c)::value;
    if constexpr (C == 3) pf[B][i] = __builtin_amdgcn_raw_buffer_load_b96(rin, off, 0, 0);
    else pf[B][i] = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, 0);
  };
  auto prefetch = [&](int k, auto buf_c) __attribute__((always_inline)) {
    const int yt = yh0 + 32 * k;
    if (__builtin_expect(yt >= lo_ok && yt + 31 <= hi_ok, 1)) {
      // interior pair (wave-uniform branch): one add per load
      const uint32_t sb = a.in_org + (uint32_t)((int64_t)yt * a.in_pitch);
#pragma unroll
      for (int i = 0; i < G::LPL; ++i) {
        const uint32_t off = sb + (uint32_t)(RSTEP * (i / P) * a.in_pitch) + loff[i % P];
        load(i, unit_ok(i) ? off : kOOB, buf_c);
      }
    } else {
#pragma unroll
      for (int i = 0; i < G::LPL; ++i) {
        // rows beyond the stripe + halo feed only zero weights: clamp, then border-map
        const int y = yt + srow[i % P] + RSTEP * (i / P);
        const uint32_t roff = in_row_off(a, min(max(y, -R), a.rows - 1 + R));
        load(i, unit_ok(i) ? roff + (uint32_t)((wx + scol[i % P]) * C) : kOOB, buf_c);
      }
    }
  };
  auto stage = [&](auto buf_c, uint8_t* wl) __attribute__((always_inline)) {
    constexpr int B = decltype(buf_c)::value;
#pragma unroll
    for (int i = 0; i < G::LPL; ++i) {
      if (!unit_ok(i)) continue;  // idle lanes of the last load (lane-divergent, LDS only)
      const int dst = (srow[i % P] + RSTEP * (i / P)) * G::STRIDE + 2 * scol[i % P];
      if constexpr (C == 3) {
        const uint32_t d0 = pf[B][i].x, d1 = pf[B][i].y, d2 = pf[B][i].z;
        const uint32_t r01 = sub_pair(d1, d0, 0x0C030C00u), r23 = sub_pair(d2, d1, 0x0C050C02u);
        const uint32_t g01 = sub_pair(d1, d0, 0x0C040C01u), g23 = sub_pair(d2, d1, 0x0C060C03u);
        const uint32_t b01 = sub_pair(d1, d0, 0x0C050C02u), b23 = sub_pair(d2, d1, 0x0C070C04u);
        *reinterpret_cast<u2*>(wl + dst) = u2{r01, r23};
        *reinterpret_cast<u2*>(wl + G::PLANE + dst) = u2{g01, g23};
        *reinterpret_cast<u2*>(wl + 2 * G::PLANE + dst) = u2{b01, b23};
      } else {
        const u4 d = pf[B][i];
        const u4 lo = {sub_pair(d.x, d.x, 0x0C010C00u), sub_pair(d.x, d.x, 0x0C030C02u),
                       sub_pair(d.y, d.y, 0x0C010C00u), sub_pair(d.y, d.y, 0x0C030C02u)};
        const u4 hi = {sub_pair(d.z, d.z, 0x0C010C00u), sub_pair(d.z, d.z, 0x0C030C02u),
                       sub_pair(d.w, d.w, 0x0C010C00u), sub_pair(d.w, d.w, 0x0C030C02u)};
        *reinterpret_cast<u4*>(wl + dst) = lo;
        *reinterpret_cast<u4*>(wl + dst + 16) = hi;
      }
    }
  };

  // output columns: a lane's 4 pixels 4g .. 4g + 3 of x-tile i
  uint32_t colok[NX];  // 0: whole group in the row; kOOB: none; else partial (byte stores)
  int npx[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int x = sx + 16 * i + 4 * g;
    npx[i] = min(4, max(0, a.W - x));
    colok[i] = npx[i] == 4 ? 0u : kOOB;
  }
  f4 acc[C][NX][2];  // running vertical sums of the current output group
  // ES (shared double-buffered windows, two pairs prefetched): pair k + 1 is
  // staged into the other window buffer in the middle of step k's tiles, so
  // its conversion VALU and LDS writes run beside step k's MFMAs instead of
  // between the barrier and the first MFMA (buffer (k + 1) & 1 held pair
  // k - 1, whose readers all passed step k's barrier)
  constexpr bool ES = EARLY && NW > 1 && PFD == 2;
  auto step = [&](auto fin_c, auto start_c, auto buf_c, int k) __attribute__((always_inline)) {
    constexpr bool FIN = decltype(fin_c)::value, START = decltype(start_c)::value;
    // the window of pair k: the wave's own tile, or buffer k & 1 of the shared
    // one (written here, read after the barrier; the other buffer's readers of
    // pair k - 1 all passed this pair's barrier before it is written again)
    uint8_t* const wt = NW == 1 ? wl : wl + (k & 1) * G::TILE;
    if constexpr (!ES) stage(buf_c, wt);
    if constexpr (NW == 1) {
      sep_lds_sync();
    } else {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");  // s_waitcnt lgkmcnt(0); loads stay in flight
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    }
    // pair k + PFD exists iff group k + PFD - 1 does (pairs 0 .. ngroups)
    if (START && k + PFD <= ngroups) prefetch(k + PFD, buf_c);
    const int yg = base + 32 * (k - 1);  // first row of the group being finished
    uint32_t rowoff[2];
    if constexpr (FIN) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int y = yg + 16 * q + m;
        rowoff[q] = (y >= ys && y < ye) ? a.out_org + (uint32_t)((int64_t)y * a.out_pitch) : kOOB;
      }
    }
    // Tiles t = C i + c (x-tile i, channel c), software-pipelined: the LDS
    // fragments of tile t + 2 are read and the horizontal MFMAs of tile t + 1
    // issued before tile t's split and vertical MFMAs, so neither the LDS
    // latency nor the MFMA -> VALU dependency of the split stalls the wave.
    constexpr int T = NX * C;
    auto hread = [&](int t, half8 (&f)[2][2]) __attribute__((always_inline)) {
      const int i = t / C, c = t % C;
      const uint8_t* fb = wt + c * G::PLANE + m * G::STRIDE + 2 * ((NW == 1 ? 0 : wave * G::PX) + 16 * i + 8 * g);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        f[0][s] = *reinterpret_cast<const half8*>(fb + 64 * s);
        f[1][s] = *reinterpret_cast<const half8*>(fb + 16 * G::STRIDE + 64 * s);
      }
    };
    // horizontal: X tiles of rows 0..15 and 16..31 of the pair
    auto hmfma = [&](const half8 (&f)[2][2], f4 (&x)[2]) __attribute__((always_inline)) {
      const float x0 = LSB ? sa.hinit : 0.f;
      x[0] = f4{x0, x0, x0, x0};
      x[1] = f4{x0, x0, x0, x0};
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int hl = 0; hl < NHL; ++hl)
#pragma unroll
          for (int h = 0; h < 2; ++h) x[h] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[h][s], bh[s][hl], x[h], 0, 0, 0);
    };
    // finished output bytes of the current x-tile, packed as the channels
    // complete: RGB interleave R0 G0 B0 R1 | G1 B1 R2 G2 | B2 R3 G3 B3 (byte e = 3 px + c)
    uint32_t wo[2][C];
    auto vert = [&](int t, const f4 (&x)[2]) __attribute__((always_inline)) {
      const int i = t / C, c = t % C;
      // accumulator layout -> A operand of the vertical product (k = X row, permuted)
      f4 o4[2], n4[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        o4[q] = acc[c][i][q];
        n4[q] = LSB ? f4{sa.bias, sa.bias, sa.bias, sa.bias} : f4{0.f, 0.f, 0.f, 0.f};
      }
      if constexpr (LSB) {
        const u4 uh = {f32x2_to_h2(x[0][0], x[0][1]), f32x2_to_h2(x[0][2], x[0][3]), f32x2_to_h2(x[1][0], x[1][1]),
                       f32x2_to_h2(x[1][2], x[1][3])};
        const half8 ah = __builtin_bit_cast(half8, uh);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if constexpr (FIN) o4[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bv[q][1][0], o4[q], 0, 0, 0);
          if constexpr (START) n4[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bv[q][0][0], n4[q], 0, 0, 0);
        }
      } else {
        uint32_t h[4], l[4];
        split_h2(x[0][0], x[0][1], h[0], l[0]);
        split_h2(x[0][2], x[0][3], h[1], l[1]);
        split_h2(x[1][0], x[1][1], h[2], l[2]);
        split_h2(x[1][2], x[1][3], h[3], l[3]);
        const u4 uh = {h[0], h[1], h[2], h[3]}, ul = {l[0], l[1], l[2], l[3]};
        const half8 ah = __builtin_bit_cast(half8, uh), al = __builtin_bit_cast(half8, ul);
        // four independent 3-MFMA chains, interleaved
#pragma unroll
        for (int st = 0; st < 3; ++st)
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const half8 av = st == 2 ? al : ah;
            if constexpr (FIN) o4[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv[q][1][st == 1], o4[q], 0, 0, 0);
            if constexpr (START) n4[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv[q][0][st == 1], n4[q], 0, 0, 0);
          }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if constexpr (START) acc[c][i][q] = n4[q];
        if constexpr (FIN) {
          if (c == 0) {
#pragma unroll
            for (int w = 0; w < C; ++w) wo[q][w] = 0;
          }
#pragma unroll
          for (int px = 0; px < 4; ++px) {
            const int e = C * px + c;
            wo[q][e >> 2] = __builtin_amdgcn_cvt_pk_u8_f32(o4[q][px], e & 3, wo[q][e >> 2]);
          }
        }
      }
      if constexpr (FIN) {
        if (c != C - 1) return;
        // lane: pixels 4g .. 4g + 3 of x-tile i in output row yg + 16 q + m
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const uint32_t off = rowoff[q] + (uint32_t)((sx + 16 * i + 4 * g) * C);
          if (!EDGE || npx[i] == 4 || npx[i] == 0 || rowoff[q] == kOOB) {
            if constexpr (C == 3)
              __builtin_amdgcn_raw_buffer_store_b96(u3{wo[q][0], wo[q][1], wo[q][2]}, rout, off | colok[i], 0, 0);
            else
              __builtin_amdgcn_raw_buffer_store_b32(wo[q][0], rout, off | colok[i], 0, 0);
          } else {  // the row's last, partial group (W % 4 != 0): bytes < C W only
#pragma unroll
            for (int e = 0; e < 4 * C; ++e)
              __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(wo[q][e >> 2] >> (8 * (e & 3))), rout,
                                                   e < C * npx[i] ? off + (uint32_t)e : kOOB, 0, 0);
          }
        }
      }
    };
    half8 F[2][2][2];
    f4 X[2][2];
    hread(0, F[0]);
    if (T > 1) hread(1, F[1]);
    hmfma(F[0], X[0]);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      if (t + 1 < T) hmfma(F[(t + 1) & 1], X[(t + 1) & 1]);
      if (t + 2 < T) hread(t + 2, F[t & 1]);
      vert(t, X[t & 1]);
      if constexpr (ES) {
        if (t == (T > 1 ? 1 : 0) && k + 1 <= ngroups)
          stage(std::integral_constant<int, 1 - decltype(buf_c)::value>{}, wl + ((k + 1) & 1) * G::TILE);
      }
    }
    if constexpr (NW == 1) sep_lds_sync();  // fragment reads done before the next pair overwrites the planes
  };
  using T_ = std::integral_constant<bool, true>;
  using F_ = std::integral_constant<bool, false>;
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, PFD - 1>;  // the other prefetch buffer (PFD 2)
  prefetch(0, B0{});
  if constexpr (PFD == 1) {
    step(F_{}, T_{}, B0{}, 0);
    for (int k = 1; k < ngroups; ++k) step(T_{}, T_{}, B0{}, k);
    step(T_{}, F_{}, B0{}, ngroups);
  } else {
    prefetch(1, B1{});  // pair 1 exists: ngroups >= 1
    if constexpr (ES) stage(B0{}, wl);  // pair 0; later pairs are staged a step early
    // pair k sits in buffer k & 1 (static: the loop runs pairs of steps)
    step(F_{}, T_{}, B0{}, 0);
    int k = 1;
    for (; k + 1 < ngroups; k += 2) {
      step(T_{}, T_{}, B1{}, k);
      step(T_{}, T_{}, B0{}, k + 1);
    }
    if (k < ngroups) {  // odd k
      step(T_{}, T_{}, B1{}, k);
      ++k;
    }
    if (k & 1) step(T_{}, F_{}, B1{}, k);
    else step(T_{}, F_{}, B0{}, k);
  }
}


}  // namespace dev

// Weight scaling of the subnormal staging: horizontal weights x 2^kexp,
// vertical x 2^(24 - kexp), kexp the largest shift keeping every scaled
// horizontal weight <= 2^15 (hi + lo parts normal f16, well inside the f16
// range).  False when the vertical weights would then leave that range too
// (max|h| * max|v| > 64: such a sepconv runs on the general conv kernel).
static bool sep_scale(const Pass& p, int* kexp_out) {
  double maxh = 0, maxv = 0;
  for (float w : p.sep_h) maxh = std::max(maxh, std::fabs((double)w));
  for (float w : p.sep_v) maxv = std::max(maxv, std::fabs((double)w));
  int kexp = 24;
  while (kexp > 0 && maxh * std::ldexp(1.0, kexp) > 32768.0) --kexp;
  if (kexp_out) *kexp_out = kexp;
  return maxh * std::ldexp(1.0, kexp) <= 32768.0 && maxv * std::ldexp(1.0, 24 - kexp) <= 32768.0;
}

bool sep_supported(const Pass& p) {
  // planar kernel: 64-pixel horizontal window per 16 outputs (R <= 16) and the
  // 48-byte left reach of the staged window within the buffers' x-margin
  return !p.sep_h.empty() && p.sep_v.size() == p.sep_h.size() && (p.cmid == 1 || p.cmid == 3) && p.R <= 16 &&
         16 * p.cmid <= kMarginBytes && sep_scale(p, nullptr);
}

// Per-lane weight fragments.  Lane l (g = l >> 4, n = l & 15), element j:
//  Bh[s][hl]: window pixel k = 32 s + 8 g + j (window pixel 0 = x-tile start
//             - 16), output pixel n: tap t = k - 16 - n + R when 0 <= t < K.
//  Bv[q][s][hl]: X row hr = 32 s + 16 (j >> 2) + 4 g + (j & 3) (the accumulator
//             order of the A operand), output row 16 q + n of the 32-row group:
//             tap t = hr - 16 - 16 q - n + R.
// Worst-case error (in output LSB) of the LSB mode for 1-D weights h, v: the
// input is centred (|x - 128| <= 128, exact in f16), the weights are rounded
// to f16, X to f16 (relative error <= 2^-11), products and sums in f32.
double sep_lsb_bound(const std::vector<float>& h, const std::vector<float>& v) {
  double sh = 0, dh = 0, sv = 0, dv = 0, svr = 0;
  for (float w : h) {
    sh += std::fabs((double)w);
    dh += std::fabs((double)w - (double)(float)(_Float16)w);
  }
  for (float w : v) {
    sv += std::fabs((double)w);
    dv += std::fabs((double)w - (double)(float)(_Float16)w);
    svr += std::fabs((double)(float)(_Float16)w);
  }
  const double e1 = 128.0 * dh;                 // horizontal weight rounding
  const double xmax = 128.0 * sh + e1;          // |X| of the centred input
  if (xmax >= 60000.0) return 1e30;             // X would leave the f16 range
  const double e2 = xmax * std::ldexp(1.0, -11);  // X rounded to f16
  // + f32 accumulation (K products per pass, 2^-24 each) with a margin
  return svr * (e1 + e2) + dv * 128.0 * sh + 1e-3 + 2.0 * (double)h.size() * std::ldexp(xmax * (1.0 + sv), -24);
}

void prepare_sep_consts(const Pass& p, PassConsts* pc, hipStream_t s) {
  const int K = p.K, R = p.R;
  STRIPE_CHECK(sep_supported(p), "separable blur geometry unsupported (K=" << K << ", C=" << p.cmid << ")");
  // precision mode: 0 = hi + lo splits (exact except ~1e-4 of a tie), 2 = LSB
  // (single f16 parts on the centred input, every output within 1 LSB; kept
  // only when the error bound stays < 0.45 LSB)
  pc->conv_mode = 0;
  if (p.conv_digits == 2) {
    const double bound = sep_lsb_bound(p.sep_h, p.sep_v);
    if (bound < 0.45) {
      pc->conv_mode = 2;
      double sh = 0, sv = 0;
      // the shift back uses the exact weights: only the centred part carries
      // the f16 rounding (random sign, no systematic bias)
      for (float w : p.sep_h) sh += (double)w;
      for (float w : p.sep_v) sv += (double)w;
      pc->conv_bias = 128.0 * sh * sv;
    } else {
      STRIPE_LOG(Info, -1, "blur" << K << " lsb: f16 weights could miss by " << bound << " LSB, using hi + lo parts");
    }
  }
  // subnormal staging: weights scaled by sep_scale's powers of two
  int kexp = 24;
  sep_scale(p, &kexp);
  const float hs = (float)std::ldexp(1.0, kexp), vs = (float)std::ldexp(1.0, 24 - kexp);
  std::vector<_Float16> host((size_t)dev::kSepEntries * 64 * 8, (_Float16)0.f);
  auto put = [&](int e, int lane, int j, float w, int hl) {
    const _Float16 whi = (_Float16)w;
    const _Float16 v = hl == 0 ? whi : (_Float16)(w - (float)whi);
    host[((size_t)e * 64 + lane) * 8 + j] = v;
  };
  for (int lane = 0; lane < 64; ++lane) {
    const int g = lane >> 4, n = lane & 15;
    for (int j = 0; j < 8; ++j) {
      for (int sidx = 0; sidx < 2; ++sidx) {
        const int t = 32 * sidx + 8 * g + j - 16 - n + R;
        const float w = (t >= 0 && t < K) ? p.sep_h[(size_t)t] * hs : 0.f;
        for (int hl = 0; hl < 2; ++hl) put(sidx * 2 + hl, lane, j, w, hl);
      }
      for (int q = 0; q < 2; ++q)
        for (int sidx = 0; sidx < 2; ++sidx) {
          const int hr = 32 * sidx + 16 * (j >> 2) + 4 * g + (j & 3);
          const int t = hr - 16 - 16 * q - n + R;
          const float w = (t >= 0 && t < K) ? p.sep_v[(size_t)t] * vs : 0.f;
          for (int hl = 0; hl < 2; ++hl) put(4 + q * 4 + sidx * 2 + hl, lane, j, w, hl);
        }
    }
  }
  // LSB: X = sum h~ (b - 128) = sum h~ b - 128 sum h~, h~ the (scaled) f16
  // weights the MFMA multiplies: the shift is the accumulator's start value
  double shs = 0;
  for (float w : p.sep_h) shs += (double)(float)(_Float16)(w * hs);
  pc->sep_hinit = -128.0 * shs * std::ldexp(1.0, -24);
  pc->conv_bytes = host.size() * sizeof(_Float16);
  HIP_CHECK(hipMalloc(&pc->conv, pc->conv_bytes));
  HIP_CHECK(hipMemcpyAsync(pc->conv, host.data(), pc->conv_bytes, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipStreamSynchronize(s));
}

// SIMDs of the current device (CUs x 4), cached per device.
static int64_t resident_simds() {
  static thread_local int cached_dev = -1;
  static thread_local int64_t cached = 0;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  if (dev != cached_dev) {
    int cus = 0;
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    cached = (int64_t)std::max(1, cus) * 4;
    cached_dev = dev;
  }
  return cached;
}

void launch_blur_sep(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s) {
  STRIPE_CHECK(pc.conv != nullptr, "blur pass constants not prepared");
  STRIPE_CHECK(L.in_base && L.out_base, "blur launch needs the allocation view (in_base/out_base)");
  STRIPE_CHECK(L.in_bytes > 0 && L.in_bytes < (int64_t)dev::kOOB && L.out_bytes > 0 &&
                   L.out_bytes < (int64_t)dev::kOOB - 65536,
               "stripe buffers must be < 2 GiB - 64 KiB for buffer-descriptor addressing");
  STRIPE_CHECK((L.rebased || (L.in_org >= kMarginBytes && L.out_org >= kMarginBytes)) && L.in_zero >= kMarginBytes,
               "bad origin offsets");
  dev::SepArgs sa{};
  dev::KArgs& a = sa.a;
  a.in = L.in;
  a.out = L.out;
  a.zero_row = L.zero_row;
  a.in_pitch = L.in_pitch;
  a.out_pitch = L.out_pitch;
  a.W = L.W;
  a.E = L.W * p.cmid;
  a.rows = L.rows;
  a.row0 = L.row0;
  a.Hg = L.Hg;
  a.border = (int)p.border;
  a.in_base = L.in_base;
  a.out_base = L.out_base;
  a.in_bytes = (uint32_t)L.in_bytes;
  a.in_org = (uint32_t)L.in_org;
  a.in_zero = (uint32_t)L.in_zero;
  a.out_bytes = (uint32_t)L.out_bytes;
  a.out_org = (uint32_t)L.out_org;
  sa.R = p.R;
  sa.L = 16 * p.cmid;
  // kernel configuration: x-tiles per strip, pairs prefetched ahead, waves per
  // SIMD.  Measured on 16K frames (profiles/r3/blur/kbench.txt): RGB is best at
  // 2 tiles / 1 pair / 2 waves (0.566 ms; 4 or 6 tiles at 1 wave with 2 pairs in
  // flight: 0.586 / 0.649 ms); gray at 16 tiles / 2 pairs / 1 wave (0.213 ms
  // against 0.234 ms at 8 / 1 / 2).  The W % 4 != 0 variant of the wide gray
  // strip spills SGPRs (so does an 8-tile one), so edge frames take 4 tiles.
  // LSB mode (2.5x fewer MFMAs, 24 fewer weight VGPRs): RGB at 4 tiles / 2
  // pairs / 1 wave, 0.40-0.43 ms against 0.55 ms at the exact mode's 2 / 1 / 2
  // (the narrower strip's 2.5x input overfetch now sets the time); gray keeps
  // the exact kernels.
  // Workgroup-shared windows (round-3 A/B runs, profiles/r3/blur/): RGB
  // exact at 2 / 1 / 2 0.556 -> 0.499-0.505 ms with 4 or 8 waves sharing a
  // window; lsb 0.423-0.426 (4 / 2 / 1 per wave) -> 0.418-0.420 (4 waves) ->
  // 0.386-0.393 (8 waves: 304 staged pixels per row for 256 outputs, one
  // 8-wave workgroup per CU with a 2 x 58 KB tile); the N=8 stripe and 16K
  // gray move within noise (gray stays per wave).  W % 4 != 0 frames (16383 x
  // 4099): exact 0.130-0.134 ms with 4 waves vs 0.139-0.142 with 8, lsb
  // 0.113-0.116 vs 0.108-0.110.  Two pairs in flight (PFD = 2, the register
  // prefetch two pairs ahead) on the 8-wave windows: exact 0.494-0.497 ->
  // 0.481-0.491 ms, lsb 0.389-0.391 -> 0.365-0.367, the N=8 stripe's lsb
  // 0.0487 -> 0.0455 (r3_blur_nw8.sh).  Gray on 8-wave windows of 8-tile strips
  // (r3_blur_gray.sh): 16K 0.211-0.212 (16 tiles per wave, 1 wave/SIMD) ->
  // 0.201-0.202 ms, 16384x2048 0.037 -> 0.034.
  struct Cfg {
    int nx, occ, nw;
    void (*fn)(dev::SepArgs);
    size_t lds;
  };
#define STRIPE_BLUR_CFGW(CC, EDGE, NX, PFD, OCC, LSB, NW) \
  Cfg { NX, OCC, NW, dev::k_blur_pl<CC, EDGE, NX, PFD, OCC, LSB, NW>, (size_t)dev::PlGeom<CC, NX, NW>::LDS }
#define STRIPE_BLUR_CFG(CC, EDGE, NX, PFD, OCC, LSB) STRIPE_BLUR_CFGW(CC, EDGE, NX, PFD, OCC, LSB, 1)
  static const Cfg cfgs[2][2][2] = {
      {{STRIPE_BLUR_CFGW(1, false, 8, 1, 2, false, 8), STRIPE_BLUR_CFG(1, true, 4, 1, 2, false)},
       {STRIPE_BLUR_CFGW(3, false, 2, 2, 2, false, 8), STRIPE_BLUR_CFGW(3, true, 2, 1, 2, false, 4)}},
      {{STRIPE_BLUR_CFGW(1, false, 8, 1, 2, false, 8), STRIPE_BLUR_CFG(1, true, 4, 1, 2, false)},  // gray: exact (below)
       {STRIPE_BLUR_CFGW(3, false, 2, 2, 2, true, 8), STRIPE_BLUR_CFGW(3, true, 2, 1, 2, true, 8)}}};
  const bool edge = L.W % 4 != 0;
  // gray frames keep the exact kernel under :lsb (it satisfies the mode and
  // was faster: 16K gray 0.218-0.220 ms exact vs 0.228-0.231 ms lsb at the same
  // 16 / 2 / 1 shape; at one wave per SIMD the shorter MFMA chains expose more
  // latency than they save)
  const bool lsb = pc.conv_mode == 2 && p.cmid == 3;
  sa.bias = (float)pc.conv_bias;
  sa.hinit = (float)pc.sep_hinit;
  sa.tw = reinterpret_cast<const dev::u4*>(pc.conv);
  // A/B variants of the RGB non-edge kernel (STRIPE_BLUR_VARIANT=n): 1 = two
  // independent 4-wave workgroups per CU (NW 4, two pairs in flight), 2 = the
  // same with one pair in flight, 3 = the 8-wave windows staging each pair
  // between the barrier and the MFMAs (round 4's default, EARLY = false).
  // (Round 6: one x-tile per wave with 12 or 16 waves sharing the window, 3-4
  // waves per SIMD at 116-147 registers, was 5-25 % slower, profiles/r6/occ/;
  // an LDS-DMA ring three pairs ahead, one f16 buffer staged between
  // two barriers, was exact but 13-25 % slower, profiles/r6/dma/: removed.)
  // (Three pairs in flight, lsb, 254 registers: 0.376 vs 0.354 ms on 16K,
  // 0.047 vs 0.042 on the stripe, profiles/r5/blur/pfd3_*.txt: removed.)
#define STRIPE_BLUR_LATE(LSB)                                                                        \
  Cfg { 2, 2, 8, dev::k_blur_pl<3, false, 2, 2, 2, LSB, 8, false>, (size_t)dev::PlGeom<3, 2, 8>::LDS }
  static const Cfg variants[2][4] = {
      {STRIPE_BLUR_CFGW(3, false, 2, 2, 2, false, 8), STRIPE_BLUR_CFGW(3, false, 2, 2, 2, false, 4),
       STRIPE_BLUR_CFGW(3, false, 2, 1, 2, false, 4), STRIPE_BLUR_LATE(false)},
      {STRIPE_BLUR_CFGW(3, false, 2, 2, 2, true, 8), STRIPE_BLUR_CFGW(3, false, 2, 2, 2, true, 4),
       STRIPE_BLUR_CFGW(3, false, 2, 1, 2, true, 4), STRIPE_BLUR_LATE(true)}};
#undef STRIPE_BLUR_LATE
  static const int env_variant = [] {
    const char* e = std::getenv("STRIPE_BLUR_VARIANT");
    return e ? std::atoi(e) : 0;
  }();
  const Cfg& cf = (p.cmid == 3 && !edge && env_variant > 0 && env_variant < 4) ? variants[lsb][env_variant]
                                                                               : cfgs[lsb][p.cmid == 3][edge];
#undef STRIPE_BLUR_CFG
#undef STRIPE_BLUR_CFGW
  // strips, rounded up to whole windows when NW waves share one
  sa.nstrips = (int)div_up(L.W, 16 * cf.nx);
  const int64_t nstrips_w = div_up(sa.nstrips, cf.nw) * cf.nw;

  const int n0 = std::max(0, L.ry[1] - L.ry[0]);
  const int n1 = L.nrange > 1 ? std::max(0, L.ry[3] - L.ry[2]) : 0;
  if (n0 + n1 > 0) {
    a.ry0 = L.ry[0];
    a.ry1 = L.ry[0] + n0;
    a.ry2 = n1 ? L.ry[2] : 0;
    a.ry3 = n1 ? L.ry[3] : 0;
    // band = gpb 32-row groups.  A task costs gpb + 1 pair steps (one warm-up
    // pair per band), and the launch runs in rounds of one task per resident
    // wave slot (2 waves per SIMD): pick gpb minimising rounds x (gpb + 1).
    // (Counting SIMDs instead of wave slots left a 16384x2048 RGB stripe at
    // 3072 tasks on 2048 slots: a half-empty second round.)
    // L.band (rows, >= 32) overrides for tuning.
    // 32-row groups from the grid origin of each range (counting a spare
    // group for the offset made a 2048-row stripe 65 groups and the pick 544
    // rows: 0.0613 ms against 0.0593 at 512, r3_blur_band2.sh)
    auto grid0 = [&](int y0) { return y0 - (int)(((int64_t)L.row0 + y0) & 31); };
    sa.a0 = grid0(a.ry0);
    sa.a2 = n1 ? grid0(a.ry2) : 0;
    const int64_t g0 = div_up(a.ry1 - sa.a0, 32), g1 = n1 ? div_up(a.ry3 - sa.a2, 32) : 0;
    const int64_t slots = (int64_t)cf.occ * resident_simds();
    int64_t gpb = 1, best = -1;
    for (int64_t c = 1; c <= 64; ++c) {
      const int64_t tasks = nstrips_w * (div_up(g0, c) + div_up(g1, c));
      const int64_t cost = div_up(tasks, slots) * (c + 1);
      if (best < 0 || cost < best) {
        best = cost;
        gpb = c;
      }
    }
    if (L.band >= 32) gpb = L.band / 32;
    const int band = (int)(32 * gpb);

    a.band = band;
    // XCD-contiguous workgroups when the pass stays in the Infinity Cache (an
    // N=8 stripe): neighbouring windows' shared columns become L2 hits (lsb
    // 16384x2048 RGB 0.0454-0.046 -> 0.0431 ms, exact unchanged; a frame
    // streaming from HBM gains nothing, r3_blur_band2.sh); STRIPE_XCD forces it
    static const int env_xcd = [] {
      const char* e = std::getenv("STRIPE_XCD");
      return e ? std::atoi(e) : -1;
    }();
    const int64_t pass_bytes = (int64_t)(n0 + n1) * L.W * 2 * p.cmid;
    // (the engine's memory policy decides for a cache-cold stripe: L.nt = 1)
    const bool streaming = L.nt >= 0 ? L.nt != 0 : pass_bytes > dev::kNtMinBytes;
    a.nxcd = env_xcd >= 0 ? env_xcd : (streaming ? 0 : dev::kXcdCount);
    a.nb0 = (int)div_up(a.ry1 - sa.a0, band);
    a.nbands = a.nb0 + (n1 ? (int)div_up(a.ry3 - sa.a2, band) : 0);
    const dim3 grid((unsigned)(cf.nw == 1 ? div_up((int64_t)sa.nstrips * a.nbands, dev::kSepWaves)
                                          : nstrips_w / cf.nw * a.nbands));
    // lsb on a cache-resident pass (an N=8 stripe): staging each pair between
    // the barrier and the MFMAs (EARLY = false) is ~2 % faster there (0.0408-
    // 0.0416 vs 0.0420-0.0425 ms), the early staging on streaming frames and in
    // the exact mode (profiles/r5/blur/README.md)
    void (*fn)(dev::SepArgs) = cf.fn;
    if (lsb && !streaming && &cf == &cfgs[1][1][0]) fn = variants[1][3].fn;
    fn<<<grid, 64 * (cf.nw == 1 ? dev::kSepWaves : cf.nw), cf.lds, s>>>(sa);
    HIP_CHECK(hipGetLastError());
  }
  if (p.out_margin_px > 0)
    for (int r = 0; r < L.nrange; ++r)
      launch_fill_margins(L.out, L.out_pitch, L.W, p.cmid, L.ry[2 * r], L.ry[2 * r + 1], p.out_margin_px,
                          p.out_margin_border, s);
}

}  // namespace stripe
